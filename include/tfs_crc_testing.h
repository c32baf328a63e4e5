/*
 * tfs_crc_testing.h -- test, calibration and tuning hooks of libtfs_crc.so.
 *
 * NOT part of the dataserver drop-in boundary (include/tfs_crc.h holds that):
 * these entry points exist for the repository's tests, bench and A/B tools --
 * synthetic data generators, fault injection, scheduler / resident-ring state,
 * the calibration streams of the measurement build, and the toggles that select
 * between measured kernel forms.  A dataserver never needs them; every one has
 * a default that is the product's behaviour.  Same return conventions as
 * tfs_crc.h.
 */
#ifndef TFS_CRC_TESTING_H_
#define TFS_CRC_TESTING_H_

#include "tfs_crc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fill nbytes (multiple of 8) of device memory with the splitmix64 synthetic
 * stream of tfs_amd/synth.py: word i = splitmix64(seed + (first_word+i+1)*GOLDEN). */
int tfs_crc32_synth_fill_device(tfs_crc_ctx* ctx, void* d_dst, uint64_t nbytes, uint64_t seed, uint64_t first_word,
                                void* stream);
/* Write FileInfo{id=first_id+f, offset_=rec_off[f], size_=usize_=len[f]+36, crc_=crc[f]}
 * at d_image + d_rec_off[f] for f < n (device pointers). */
int tfs_crc32_write_headers_device(tfs_crc_ctx* ctx, void* d_image, const uint64_t* d_rec_off, const uint32_t* d_len,
                                   const uint32_t* d_crc, uint64_t first_id, uint32_t n, void* stream);
/* Write unsealed V1 frame headers {flag V1, length = d_body_len[f], type =
 * pcode, version, id = first_id + f, crc 0} at d_base + d_frame_off[f]. */
int tfs_crc32_write_packet_headers_device(tfs_crc_ctx* ctx, void* d_base, const uint64_t* d_frame_off,
                                          const uint32_t* d_body_len, uint32_t n, int32_t pcode, int32_t version,
                                          uint64_t first_id, void* stream);
/* Calibration: stream the bytes without CRC arithmetic.  pattern 0 = coalesced
 * grid-stride over [d_base, d_base+nbytes); pattern 1 = the CRC kernel's
 * per-file lane-segment access pattern over d_desc (len multiple of 1 KiB).
 * Measurement build only (libtfs_crc_measure.so); the product library returns
 * TFS_EXIT_PARAMETER_ERROR. */
int tfs_crc32_membench_device(tfs_crc_ctx* ctx, int pattern, const void* d_base, const tfs_crc_desc* d_desc,
                              uint32_t n, uint64_t nbytes, uint32_t* d_out, unsigned grid, void* stream);
/* Fault injection (tests of the callers' error paths, like the reference's
 * `ds_client send_crc_error`, src/tools/dataserver/ds_client.cpp:522-566): after
 * `skip` more host-memory submissions (batch / verify / submit / scalar /
 * block verify / block compaction / packet calls) the next `count` ones fail with
 * TFS_CRC_EXIT_DEVICE_ERROR before any GPU work.  count = 0 disarms. */
int tfs_crc32_inject_device_error(tfs_crc_ctx* ctx, uint32_t skip, uint32_t count);
/* Test hooks for the scheduler and resident-ring state (tests/test_resident.py):
 * the device addresses and sizes of ctx's scheduler slots and resident-kernel
 * state (NULL before the first resident batch), and a poisoned resident state --
 * every workgroup's count of units done set to `done`, as a stale recycled
 * allocation would hold -- to check that such a batch ends in
 * TFS_CRC_EXIT_DEVICE_ERROR in bounded time instead of hanging. */
int tfs_crc32_debug_state(tfs_crc_ctx* ctx, void** d_sched, uint64_t* sched_bytes, void** d_res_state,
                          uint64_t* res_state_bytes);
int tfs_crc32_debug_poison_resident(tfs_crc_ctx* ctx, uint32_t done);
/* Resident form of the synchronous small batches (tfs_crc32_batch / _verify /
 * the scalar drop-in with <= 256 files read in place from page-locked memory,
 * i.e. every close batch of DataManagement::close_write_file,
 * data_management.cpp:173-236): a kernel that stays on the GPU between batches
 * takes them from a page-locked ring, so a batch costs no launch; it leaves
 * after TFS_CRC_RESIDENT_IDLE_US (200) without work and is relaunched on the
 * next batch.  on = 0 launches every batch instead (also TFS_CRC_RESIDENT=0).
 * Stats: kernel launches made and files taken through the ring so far. */
int tfs_crc32_set_resident(tfs_crc_ctx* ctx, int on);
int tfs_crc32_resident_stats(tfs_crc_ctx* ctx, uint64_t* launches, uint64_t* files);
/* Where the context's resident ring lives: 1 = fine-grained device memory the host
 * writes through the PCIe BAR (the default on a large-BAR device), 0 = page-locked
 * host memory (no large BAR, or TFS_CRC_RESIDENT_VRAM=0 when the context was
 * made), -1 = not set up yet (no resident call so far). */
int tfs_crc32_resident_ring_in_device_memory(tfs_crc_ctx* ctx);
/* Resident-path stamps (measurement build only, libtfs_crc_measure.so; the product
 * returns TFS_EXIT_PARAMETER_ERROR).  tfs_crc32_res_trace, before the context's
 * first resident call: `pinned` (page-locked, 4096 units x 8 u64) receives, per
 * ring unit, the GPU's 100 MHz wall-clock stamps of the poll issue that found the
 * unit published, that poll's return, the unit's words back, the acquire fence
 * done, wave 0's payload loads back and its CRC done (TFS_CRC_RES_NOFENCE=1 at
 * that call: the kernel skips the fence, measurement only).
 * tfs_crc32_res_trace_last: the last synchronous call's host stamps (steady clock
 * ns) {enter, posted, result seen, return}, its first ring unit, whether it went
 * through the ring, and the wall-clock rate in kHz (tools/floor_probe.cpp). */
int tfs_crc32_res_trace(tfs_crc_ctx* ctx, void* pinned);
int tfs_crc32_res_trace_last(tfs_crc_ctx* ctx, uint64_t* out8);
/* Throughput launches (the *_device calls and large host batches: one
 * persistent workgroup per CU) leave the CUs of every resident kernel of their
 * device free while it lives or has had a batch in the last 50 ms, so a close
 * batch never waits for a 10 ms verify or compaction launch and such a launch
 * never waits for the resident kernel's lifetime.  on = 0 uses
 * every CU regardless.  tfs_crc32_throughput_grid: workgroups the next
 * throughput launch of ctx would use. */
int tfs_crc32_set_cu_reserve(tfs_crc_ctx* ctx, int on);
/* Throughput launches of the file kernel (batches of more than 256 files) cut
 * every file longer than 128 KiB into a ragged head and 128 KiB segments that
 * separate waves checksum, then fold the segment CRCs into the file's CRC on the
 * GPU: one wave never streams a long file alone.  Results are
 * identical either way; on = 0 keeps every file on one wave (A/B).  The
 * launch's units -- whole files, heads and segments -- form one list in address
 * order (each file's head, then its segments, then the next file), so the waves
 * walk the image once (round 4; the measurement build's on = 2 is round 3's form,
 * segments appended after all files). */
int tfs_crc32_set_split(tfs_crc_ctx* ctx, int on);
/* Device compaction (tfs_compact_jobs_device, and the block-file compactor that
 * calls it) cuts every live record whose payload is longer than `seg_bytes` into a
 * ragged head and whole seg_bytes payload segments that separate waves copy and
 * checksum, then folds the segment CRCs into the record's CRC and status on the
 * GPU.  seg_bytes: 8192, 16384 or 32768 for every launch; 0 keeps
 * every record on one wave; 1 restores the default: whole records (segments
 * averaged -0.4 % over seven boxes).  Output bytes, CRCs and
 * statuses are identical either way. */
int tfs_crc32_set_compact_segment(tfs_crc_ctx* ctx, uint32_t seg_bytes);
int tfs_crc32_throughput_grid(tfs_crc_ctx* ctx);
/* Scheduler slots: ctx-owned streams bound (the ctx stream, compaction streams,
 * tfs_crc32_stream_create), and launches so far on streams the ctx does not own
 * (each of those takes a pooled slot zeroed on its stream before the kernel). */
int tfs_crc32_sched_stats(tfs_crc_ctx* ctx, uint32_t* owned_streams, uint64_t* foreign_launches);
/* Split / segment plans the ctx holds and their device bytes: one per owned stream
 * that made a throughput launch, and one shared by all launches on streams the ctx
 * does not own (the footprint no longer grows with foreign streams). */
int tfs_crc32_plan_stats(tfs_crc_ctx* ctx, uint32_t* plans, uint64_t* bytes);
/* The latest split throughput launch of ctx (debug/test hook; call it with no
 * other launch of ctx in flight): split launches so far, ext units its plan
 * reserved (`used`: segments of files > 128 KiB; when they do not all fit, the
 * files of the address-ordered prefix that fits in `cap` are split and the rest stay whole),
 * its files, the plan's capacity and the workgroups it ran on.  The launch's
 * work units are files + min(used, cap); it takes dynamic chunked tickets when
 * those units come to >= 16 tickets per wave.  Waits for that
 * launch.  Each owned stream has its own plan, so split launches on different
 * owned streams overlap; launches on foreign streams share one plan. */
int tfs_crc32_split_stats(tfs_crc_ctx* ctx, uint64_t* launches, uint64_t* used, uint32_t* files, uint32_t* cap,
                          uint32_t* grid);

#ifdef __cplusplus
}
#endif
#endif /* TFS_CRC_TESTING_H_ */
