/*
 * tfs_crc.h -- C ABI of the MI355X-native per-file CRC32 integrity path.
 *
 * Drop-in boundary for TFS's dataserver CRC call sites (reference =
 * simonsysu/tfs @ TFS 2.3.0, /root/reference).  Every entry point below names
 * the reference interface it replaces.  Plain C types only (no torch, no HIP
 * types): device pointers and streams are passed as `void*`.
 *
 * Arithmetic: reflected CRC-32, polynomial 0xEDB88320, caller-supplied seed,
 * no pre/post inversion, len <= 0 returns the seed -- bit-identical to
 * tfs::common::Func::crc (src/common/func.cpp:426-435, table
 * src/common/func.h:128-154).  The computation runs on the GPU (hand-written
 * gfx950 kernels in tfs_amd/csrc/); there is no CPU fallback: without a usable
 * device every entry point returns TFS_CRC_EXIT_NO_DEVICE.
 *
 * Return convention (reference src/common/error_msg.h, src/common/cdefine.h):
 *   TFS_SUCCESS (0) on success, negative TFS codes on failure.
 */
#ifndef TFS_CRC_H_
#define TFS_CRC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define TFS_SUCCESS 0                      /* cdefine.h:26 */
#define TFS_EXIT_CHECK_CRC_ERROR (-1010)   /* error_msg.h:35  verify: crc mismatch */
#define TFS_EXIT_PARAMETER_ERROR (-1016)   /* error_msg.h:41  bad argument */
#define TFS_EXIT_DATA_FILE_ERROR (-8013)   /* error_msg.h:149 close: client crc != data crc */
#define TFS_EXIT_FILE_INFO_ERROR (-8016)   /* error_msg.h:152 FileInfo id/flag mismatch */
#define TFS_EXIT_READ_FILE_SIZE_ERROR (-8034) /* error_msg.h:170 record shorter than FileInfo */
#define TFS_EXIT_SYNC_FILE_ERROR (-8038)   /* error_msg.h:174 verify: size mismatch */
/* New codes (outside the reference's -1000..-16008 range): */
#define TFS_CRC_EXIT_DEVICE_ERROR (-20001) /* a HIP call failed; see tfs_crc32_last_error() */
#define TFS_CRC_EXIT_NO_DEVICE (-20002)    /* no usable gfx950 device / kernels not loadable */

/* FileInfo flags, src/dataserver/dataserver_define.h:54-59 */
#define TFS_FI_DELETED 1
#define TFS_FI_INVALID 2
#define TFS_FI_CONCEAL 4

#define TFS_FILEINFO_SIZE 36          /* sizeof(FileInfo), internal.h:432-446, pack(4) */
#define TFS_BLOCK_RESERVER_LENGTH 512 /* physical_block.h:31 */

/* ---- data layouts ---------------------------------------------------- */

/* One file to checksum: `len` bytes at base + offset, starting CRC `seed`
 * (Func::crc's first argument; 0 at every per-file call site,
 * data_file.cpp:190).  16 bytes, naturally aligned. */
typedef struct tfs_crc_desc {
  uint64_t offset;
  uint32_t len;
  uint32_t seed;
} tfs_crc_desc;

/* One file to verify: recomputed Func::crc(0, base+offset, len) must equal
 * `expected` (the stored FileInfo.crc_, sync_backup.cpp:429). 16 bytes. */
typedef struct tfs_crc_vdesc {
  uint64_t offset;
  uint32_t len;
  uint32_t expected;
} tfs_crc_vdesc;

/* FileInfo exactly as stored in a block (src/common/internal.h:432-446). */
#pragma pack(push, 4)
typedef struct tfs_file_info {
  uint64_t id_;
  int32_t offset_;
  int32_t size_;   /* payload + 36 on disk */
  int32_t usize_;
  int32_t modify_time_;
  int32_t create_time_;
  int32_t flag_;
  uint32_t crc_;
} tfs_file_info;
#pragma pack(pop)

/* One index entry of a block (RawMeta, internal.h:535-645): file id, logical
 * data offset of its FileInfo, size incl. the 36-byte header. */
typedef struct tfs_raw_meta {
  uint64_t file_id;
  int32_t offset;
  int32_t size;
} tfs_raw_meta;

typedef struct tfs_crc_ctx tfs_crc_ctx;

/* ---- context ---------------------------------------------------------- */

/* Create a context bound to HIP device `device` (one per GPU; the dataserver
 * owns one per local GPU).  Loads the CRC tables into device memory.
 * Thread-safe to use from many threads (calls are serialised per ctx). */
int tfs_crc32_ctx_create(int device, tfs_crc_ctx** out);
int tfs_crc32_ctx_destroy(tfs_crc_ctx* ctx);
/* Message of the last failure on this ctx (or of the process-wide default ctx
 * when ctx == NULL).  Never NULL. */
const char* tfs_crc32_last_error(const tfs_crc_ctx* ctx);
/* Number of HIP devices visible to this process (0 when none). */
int tfs_crc32_device_count(void);
/* NUMA node of HIP device `device` (its PCI device's sysfs numa_node), -1 when
 * unknown: where a process serving that GPU should keep its threads and
 * page-locked buffers. */
int tfs_crc32_device_numa_node(int device);

/* ---- scalar drop-in --------------------------------------------------- */

/* Replaces `static uint32_t Func::crc(uint32_t crc, const char* data,
 * const int32_t len)` (src/common/func.h:90, func.cpp:426-435).  Host buffer,
 * result by value, len <= 0 returns crc.  Runs on the scalar context: the
 * calling thread's binding (tfs_crc32_bind_thread), else the process default
 * (tfs_crc32_set_default_ctx), else a context on device 0 made on first use.
 *
 * Failure mode: Func::crc has no error channel, so on a device failure
 * tfs_crc32 returns `crc` (the seed) -- a value the caller will usually take
 * for a CRC mismatch.  Every such failure is counted (tfs_crc32_error_count,
 * process-wide, never reset), and the first is reported on stderr.  Call sites
 * that can act on an error -- the packet decode check (base_packet.cpp:141) and
 * the mirror / repair re-CRC (sync_backup.cpp:383,412, file_repair.cpp:142) --
 * use tfs_crc32_e, whose *err (TFS_CRC_EXIT_DEVICE_ERROR / _NO_DEVICE, or
 * TFS_SUCCESS) tells a device fault from a mismatch. */
uint32_t tfs_crc32(uint32_t crc, const char* data, int32_t len);
uint32_t tfs_crc32_e(uint32_t crc, const char* data, int32_t len, int* err);
/* Scalar drop-in failures so far in this process (both forms). */
uint64_t tfs_crc32_error_count(void);
/* Choose the scalar context: for the whole process (NULL = back to device 0's
 * default), or for the calling thread only (a packet worker serving one GPU's
 * blocks binds that group member's context; NULL unbinds).  Destroying a
 * context clears the process default and every thread's binding to it (each
 * thread drops it on its next scalar call, which then uses the process default);
 * binding a context that is not live returns TFS_EXIT_PARAMETER_ERROR.  A scalar
 * call running while another thread destroys its context is the caller's to
 * avoid. */
int tfs_crc32_set_default_ctx(tfs_crc_ctx* ctx);
int tfs_crc32_bind_thread(tfs_crc_ctx* ctx);
/* The context the scalar calls of this thread use (created on first use), or
 * NULL when none can be made. */
tfs_crc_ctx* tfs_crc32_default_ctx(void);

/* Per-context call counters, monotonic from the context's creation, so an
 * integration can see callers that should batch.  A lone host call (one body)
 * shorter than TFS_CRC_LONE_CROSSOVER bytes costs one GPU round trip over PCIe
 * (~4 us up to 80 bytes, 5-7 us above), longer than the reference's host loop takes on
 * it (1.6 ns/byte): such a caller -- a small RPC body checked alone,
 * base_packet.cpp:141 -- should gather its bodies into one tfs_crc32_batch /
 * tfs_packet_verify call.  Scalar calls count on the context they run on. */
#define TFS_CRC_LONE_CROSSOVER 3500 /* round 6: 3,452 B measured on the closing tree with the ring in device memory, 4,437 with it in host memory (bench.py --workload small_bodies) */
typedef struct tfs_crc_stats {
  uint64_t host_calls;         /* synchronous host-memory calls: scalar, get_crc, batch, verify, small packet sets */
  uint64_t host_files;         /* bodies they carried */
  uint64_t lone_calls;         /* of host_calls, those carrying exactly one body */
  uint64_t lone_small_calls;   /* of lone_calls, bodies shorter than TFS_CRC_LONE_CROSSOVER bytes */
  uint64_t lone_small_bytes;   /* the bytes of those bodies */
  uint64_t resident_launches;  /* resident kernel launches (the first and every relaunch) */
  uint64_t resident_files;     /* bodies the resident kernel took */
  uint64_t resident_ring_full; /* batches launched because the resident ring had no room */
} tfs_crc_stats;
int tfs_crc32_stats(tfs_crc_ctx* ctx, tfs_crc_stats* out);

/* Replaces DataFile::get_crc() (src/dataserver/data_file.cpp:168-194):
 * Func::crc(0, data, length).  The reference re-reads payloads > 2 MiB in
 * 2 MiB chunks with a running seed (:183-186); that equals one pass over the
 * whole payload, which is what this computes. */
int tfs_datafile_get_crc(tfs_crc_ctx* ctx, const char* data, int32_t length, uint32_t* out_crc);

/* ---- batch, host memory ----------------------------------------------- */

/* Batched Func::crc over `n` files of a host buffer [base, base+base_len):
 * out_crc[i] = Func::crc(d[i].seed, base + d[i].offset, d[i].len).  A
 * page-locked `base` (tfs_crc32_host_malloc_pinned / hipHostMalloc) is read in
 * place by the kernel (zero-copy, up to 65,536 files); pageable bytes are staged
 * through pinned memory (hipMemcpyAsync) to the GPU.
 * Call sites: data_file.cpp:190 via data_management.cpp:197 (write), batched
 * across concurrent leases. */
int tfs_crc32_batch(tfs_crc_ctx* ctx, const tfs_crc_desc* d, uint32_t n, const void* base, uint64_t base_len,
                    uint32_t* out_crc);

/* Batched verify-on-read: out_crc[i] = Func::crc(0, base+d[i].offset, d[i].len),
 * out_ok[i] = (out_crc[i] == d[i].expected), *n_bad = number of mismatches.
 * Returns TFS_SUCCESS when all match, TFS_EXIT_CHECK_CRC_ERROR when any does
 * not (sync_backup.cpp:429), other negatives on error.  out_crc / out_ok /
 * n_bad may be NULL.  Call sites: sync_backup.cpp:383/412, file_repair.cpp:142,
 * block_console.cpp:570. */
int tfs_crc32_verify(tfs_crc_ctx* ctx, const tfs_crc_vdesc* d, uint32_t n, const void* base, uint64_t base_len,
                     uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad);

/* ---- batch, device-resident ------------------------------------------- */

/* Same as tfs_crc32_batch with every pointer in device memory of ctx's GPU;
 * enqueued on `stream` (a hipStream_t, NULL = ctx's stream); asynchronous:
 * results are valid once the stream reaches this point. */
int tfs_crc32_batch_device(tfs_crc_ctx* ctx, const tfs_crc_desc* d_desc, uint32_t n, const void* d_base,
                           uint32_t* d_out_crc, void* stream);
/* Device-resident verify. d_n_bad (may be NULL) is accumulated into (atomic
 * add), so zero it first.  d_out_crc / d_out_ok may be NULL. */
int tfs_crc32_verify_device(tfs_crc_ctx* ctx, const tfs_crc_vdesc* d_desc, uint32_t n, const void* d_base,
                            uint32_t* d_out_crc, uint8_t* d_out_ok, uint32_t* d_n_bad, void* stream);

/* ---- async host API ---------------------------------------------------- */

typedef struct tfs_crc_ticket {
  uint64_t id;
} tfs_crc_ticket;

/* Enqueue a host-memory verify (as tfs_crc32_verify) and return immediately;
 * the caller keeps d/base/outputs alive and unmodified until tfs_crc32_wait.
 * H2D copy, kernel and D2H copy run on the ctx stream, double-buffered against
 * other in-flight submissions. */
int tfs_crc32_submit_verify(tfs_crc_ctx* ctx, const tfs_crc_vdesc* d, uint32_t n, const void* base,
                            uint64_t base_len, uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad,
                            tfs_crc_ticket* ticket);
/* Block until the ticket's results are in the caller's buffers; returns the
 * status the synchronous call would have returned. */
int tfs_crc32_wait(tfs_crc_ctx* ctx, tfs_crc_ticket ticket);

/* ---- block images ----------------------------------------------------- */

/* Verify-on-read of files stored in a block image (logical data area: offset 0
 * = first FileInfo, i.e. the bytes after the 512-byte BlockPrefix,
 * physical_block.cpp:30-35).  For each meta: read the FileInfo at
 * image+meta.offset, recompute Func::crc(0, payload, meta.size-36) and report
 * per file status[i] in {TFS_SUCCESS, TFS_EXIT_FILE_INFO_ERROR (header id !=
 * meta id), TFS_EXIT_READ_FILE_SIZE_ERROR (meta.size <= 36),
 * TFS_EXIT_SYNC_FILE_ERROR (FileInfo.size_ != meta.size), TFS_EXIT_CHECK_CRC_ERROR}
 * -- the checks of sync_backup.cpp:345-435 / block_console.cpp:543-577 in that
 * order.  d_* variants take device pointers; the host variant reads a page-locked
 * image in place (only the named records cross PCIe) and copies a pageable one. */
int tfs_block_verify(tfs_crc_ctx* ctx, const void* image, uint64_t image_len, const tfs_raw_meta* metas, uint32_t n,
                     uint32_t* out_crc, int32_t* out_status, uint32_t* n_bad);
int tfs_block_verify_device(tfs_crc_ctx* ctx, const void* d_image, uint64_t image_len, const tfs_raw_meta* d_metas,
                            uint32_t n, uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad, void* stream);

/* Compaction with re-CRC (CompactTask::real_compact, src/dataserver/task.cpp:713-836):
 * walk `metas` (sorted by offset, traverse_sorted_segment_meta), skip files
 * whose real flag (flags[i], logic_block.cpp:1273) has FI_DELETED|FI_INVALID,
 * and pack each live file as FileInfo{offset_=w, size_=usize_=payload+36,
 * other fields and crc_ copied} | payload into `dest` (task.cpp:753-798).
 * Adds the verify the reference does not do: recomputed payload CRC ==
 * stored crc_ (crc_ok[i] = 1 ok, 0 mismatch, 2 skipped).  dest_metas receives
 * the RawMeta list of the new block (task.cpp:764-768); *dest_len and
 * *n_live the new data size and file count.  Host buffers; the source block is
 * copied to the GPU, verified and repacked there, and the new block copied
 * back (H<->D included, BASELINE config 4). */
int tfs_block_compact(tfs_crc_ctx* ctx, const void* src_image, uint64_t src_len, const tfs_raw_meta* metas,
                      const int32_t* flags, uint32_t n, void* dest_image, uint64_t dest_cap, tfs_raw_meta* dest_metas,
                      uint8_t* crc_ok, uint64_t* dest_len, uint32_t* n_live);

/* Device-resident compaction data pass (one kernel, one read of every live
 * record): for the live files d_live_metas[0..n) (already filtered and in
 * offset order), re-CRC each payload against its stored crc_ and write
 * FileInfo{offset_ = d_dest_off[i], size_ = usize_ = meta.size, flag_ =
 * d_flags[i], rest copied} | payload at d_dest + d_dest_off[i].  Per-file
 * status as tfs_block_verify, except that an empty file (meta.size == 36) is
 * copied like any other (real_compact does; only meta.size < 36 is
 * TFS_EXIT_READ_FILE_SIZE_ERROR); d_n_bad (may be NULL) accumulated into.  The
 * caller computes d_dest_off (the running sum of live sizes, task.cpp:753-768)
 * and d_dest must hold sum(size).  Several blocks can share one call when
 * their images are concatenated in d_src.  Asynchronous on `stream`. */
int tfs_block_compact_device(tfs_crc_ctx* ctx, const void* d_src, uint64_t src_len, const tfs_raw_meta* d_live_metas,
                             const int32_t* d_flags, const int64_t* d_dest_off, uint32_t n, void* d_dest,
                             uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad, void* stream);

/* The same data pass over many device-resident blocks in one launch (64-bit
 * offsets; one entry per live record, any order).  Writes FileInfo{offset_ =
 * new_offset, size_ = usize_ = size, flag_ = flag} | payload at d_dest +
 * dest_offset after checking id/size/crc as above.  `reserved`: 0, or
 * TFS_COMPACT_JOB_EDGE when fewer than 128 readable bytes follow the record (the
 * kernel then reads no byte past it; with 0 it may read up to 112 bytes past a
 * record that ends at least 128 bytes before src_len, to write whole lines). */
#define TFS_COMPACT_JOB_EDGE 1
typedef struct tfs_compact_job {
  uint64_t src_offset;
  uint64_t dest_offset;
  uint64_t file_id;
  int32_t size;
  int32_t flag;
  int32_t new_offset;
  int32_t reserved;
} tfs_compact_job;
int tfs_compact_jobs_device(tfs_crc_ctx* ctx, const void* d_src, uint64_t src_len, const tfs_compact_job* d_jobs,
                            uint32_t n, void* d_dest, uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad,
                            void* stream);

/* Verify-on-read of the records of many device-resident blocks in one launch
 * (64-bit offsets): per job, the FileInfo at d_src + src_offset is checked
 * against file_id and size and the payload CRC against its crc_, statuses as
 * tfs_block_verify.  The dest_offset / flag / new_offset fields of the jobs are
 * not used.  Asynchronous on `stream`; d_n_bad accumulated into. */
int tfs_blocks_verify_device(tfs_crc_ctx* ctx, const void* d_src, uint64_t src_len, const tfs_compact_job* d_jobs,
                             uint32_t n, uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad, void* stream);

/* Many blocks in one call (the compaction task thread's queue): each job is
 * tfs_block_compact's arguments plus its outputs.  Jobs are pipelined over
 * several streams so the H2D copy of one block, the verify/repack kernels of
 * the next and the D2H copy of another overlap.  When both source and dest
 * images are page-locked (tfs_crc32_host_malloc_pinned / hipHostRegister), the
 * kernel reads the live records from, and writes the new block to, host memory
 * directly (zero-copy: only live bytes cross PCIe, no whole-block copies).
 * Otherwise page-locked
 * images are copied directly (whole block H2D, new block D2H); pageable ones are
 * staged.  Returns the worst job status (TFS_EXIT_CHECK_CRC_ERROR if only CRC
 * mismatches were found). */
typedef struct tfs_block_job {
  const void* src_image;
  uint64_t src_len;
  const tfs_raw_meta* metas;
  const int32_t* flags;
  uint32_t n;
  void* dest_image;
  uint64_t dest_cap;
  tfs_raw_meta* dest_metas; /* out, n_live entries (may be NULL) */
  uint8_t* crc_ok;          /* out, n entries (may be NULL) */
  uint64_t dest_len;        /* out */
  uint32_t n_live;          /* out */
  int status;               /* out */
} tfs_block_job;
int tfs_blocks_compact(tfs_crc_ctx* ctx, tfs_block_job* jobs, uint32_t njobs);

/* ---- packet CRC (BasePacket, src/common/base_packet.{h,cpp}) ------------ */

/* Every V1 RPC frame carries Func::crc(TFS_PACKET_FLAG_V1, body, length) in its
 * header: the send side computes it (BasePacket::copy / reply,
 * base_packet.cpp:74,208; serialized by BasePacketStreamer::encode,
 * base_packet_streamer.cpp:159-200), the receive side checks it
 * (BasePacket::decode, base_packet.cpp:117-148) -- for every 64 KiB write and
 * each of its forwarded replica copies.  A frame is the serialized header
 * (TfsPacketNewHeaderV1, base_packet.h:92-162, little-endian: flag u32,
 * length i32, type i16, version i16, id u64, crc u32 = 24 bytes; a V0 frame
 * has only flag/length/type/check = 12 bytes) followed by `length` body bytes. */
#define TFS_PACKET_FLAG_V0 0x4d534654u /* "TFSM", base_packet.h:347 */
#define TFS_PACKET_FLAG_V1 0x4e534654u /* "TFSN", base_packet.h:348; also the CRC seed */
#define TFS_PACKET_HEADER_V0_SIZE 12
#define TFS_PACKET_HEADER_V1_SIZE 24
#define TFS_ERROR (-1)            /* cdefine.h: broken stream */
#define TFS_PACKET_INCOMPLETE 1   /* frame shorter than its header/body: the streamer waits */

/* One frame: `len` bytes available at base + offset, starting at its header. 16 bytes. */
typedef struct tfs_packet_desc {
  uint64_t offset;
  uint32_t len;
  uint32_t reserved;
} tfs_packet_desc;

/* Receive side, batched.  Per frame, in the reference's order
 * (getPacketInfo, base_packet_streamer.cpp:43-124; decode, base_packet.cpp:100-170):
 *   TFS_PACKET_INCOMPLETE   fewer than 12 bytes, a V1 flag with fewer than 24, or
 *                           the body not all there;
 *   TFS_ERROR               flag neither V0 nor V1, or length <= 0 or > 64 MiB (:78-87);
 *   TFS_EXIT_CHECK_CRC_ERROR  decode's CRC check failed (:141-148);
 *   TFS_SUCCESS             decoded: CRC matched, or the frame carries none
 *                           (V0 flag / version 0; decode checks when
 *                           ((pcode >> 16) & 0xFFFF) >= 1, pcode = type | check << 16).
 * out_crc[i] = the computed body CRC for checked frames, else 0.  out_status /
 * out_crc / n_bad may be NULL.  Returns TFS_SUCCESS when every frame decoded,
 * TFS_EXIT_CHECK_CRC_ERROR otherwise (see out_status), other negatives on error. */
int tfs_packet_verify(tfs_crc_ctx* ctx, const tfs_packet_desc* d, uint32_t n, const void* base, uint64_t base_len,
                      uint32_t* out_crc, int32_t* out_status, uint32_t* n_bad);
/* Device-resident form (asynchronous on `stream`; d_n_bad accumulated into). */
int tfs_packet_verify_device(tfs_crc_ctx* ctx, const tfs_packet_desc* d_desc, uint32_t n, const void* d_base,
                             uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad, void* stream);
/* Send side, batched: for every V1 frame whose version is >= 1, compute the body
 * CRC and store it in the header's crc field (bytes 20..23) -- what
 * BasePacket::copy/reply + BasePacketStreamer::encode produce.  Other frames are
 * left as they are.  out_status as tfs_packet_verify (never a CRC error);
 * out_crc[i] = the stored CRC or 0.  Host form writes into `base`. */
int tfs_packet_seal(tfs_crc_ctx* ctx, const tfs_packet_desc* d, uint32_t n, void* base, uint64_t base_len,
                    uint32_t* out_crc, int32_t* out_status);
int tfs_packet_seal_device(tfs_crc_ctx* ctx, const tfs_packet_desc* d_desc, uint32_t n, void* d_base,
                           uint32_t* d_out_crc, int32_t* d_out_status, void* stream);

/* ---- device group: one context per local GPU --------------- */

/* The dataserver is one process (DataService::initialize, dataservice.cpp:151-377;
 * PacketQueueThread workers, base_service.cpp:187-192).  A group holds one
 * context per GPU, each with a host worker thread bound to the GPU's NUMA node
 * and page-locked memory from that node.  Blocks are routed by block id
 * (member = block_id % size): a block's files never straddle GPUs and nothing
 * is exchanged between members -- no collective.  `devices` lists the member
 * devices (repeats allowed: several contexts on one GPU); NULL = every visible
 * device.  On failure *out is still set (read tfs_crc_group_last_error, then
 * destroy it). */
typedef struct tfs_crc_group tfs_crc_group;
int tfs_crc_group_create(const int* devices, uint32_t n, tfs_crc_group** out);
int tfs_crc_group_destroy(tfs_crc_group* g);
const char* tfs_crc_group_last_error(const tfs_crc_group* g);
uint32_t tfs_crc_group_size(const tfs_crc_group* g);
/* Member i's context (for the per-file calls above), and the routing rule. */
tfs_crc_ctx* tfs_crc_group_ctx(tfs_crc_group* g, uint32_t i);
uint32_t tfs_crc_group_member_of(const tfs_crc_group* g, uint32_t block_id);
tfs_crc_ctx* tfs_crc_group_ctx_for_block(tfs_crc_group* g, uint32_t block_id);
/* NUMA node of member i's GPU (-1 unknown); 1 when its worker thread runs on it. */
int tfs_crc_group_numa_node(const tfs_crc_group* g, uint32_t i);
int tfs_crc_group_member_bound(const tfs_crc_group* g, uint32_t i);
/* Page-locked host memory allocated on member i's NUMA node (block images,
 * receive buffers of that GPU's blocks).  Free it only with
 * tfs_crc_group_host_free: the library keeps its own registry of the page-locked
 * memory it allocated (no runtime query per call), which hipHostFree would leave
 * stale. */
int tfs_crc_group_host_malloc(tfs_crc_group* g, uint32_t i, uint64_t bytes, void** p);
int tfs_crc_group_host_free(tfs_crc_group* g, uint32_t i, void* p);

/* Verify-on-read of many block images (tfs_block_verify's arguments per job),
 * each on its block's GPU; members run concurrently.  Returns the worst job
 * status (TFS_EXIT_CHECK_CRC_ERROR if only CRC mismatches were found). */
typedef struct tfs_block_verify_job {
  uint32_t block_id;
  const void* image;
  uint64_t image_len;
  const tfs_raw_meta* metas;
  uint32_t n;
  uint32_t* out_crc;    /* n entries or NULL */
  int32_t* out_status;  /* n entries or NULL */
  uint32_t n_bad;       /* out */
  int status;           /* out */
} tfs_block_verify_job;
int tfs_crc_group_blocks_verify(tfs_crc_group* g, tfs_block_verify_job* jobs, uint32_t njobs);
/* Compaction of many blocks (tfs_blocks_compact per member), block_ids[j] routes jobs[j]. */
int tfs_crc_group_blocks_compact(tfs_crc_group* g, const uint32_t* block_ids, tfs_block_job* jobs, uint32_t njobs);

/* ---- memory, stream and event helpers ---------------------------------- */

/* Device / pinned memory and event plumbing for callers that hold no HIP
 * runtime of their own (tests, bench, a dataserver without HIP code).
 * tfs_crc32_memcpy: hipMemcpyDefault direction; stream NULL = ctx stream and
 * synchronous, otherwise asynchronous on `stream`. */
int tfs_crc32_dev_malloc(tfs_crc_ctx* ctx, uint64_t bytes, void** d_ptr);
int tfs_crc32_dev_free(tfs_crc_ctx* ctx, void* d_ptr);
/* Page-locked memory from tfs_crc32_host_malloc_pinned is freed only with
 * tfs_crc32_host_free_pinned (see tfs_crc_group_host_malloc: the library's
 * registry of its page-locked allocations). */
int tfs_crc32_host_malloc_pinned(tfs_crc_ctx* ctx, uint64_t bytes, void** h_ptr);
int tfs_crc32_host_free_pinned(tfs_crc_ctx* ctx, void* h_ptr);
/* Device address of page-locked host memory (hipHostGetDevicePointer), for
 * passing host buffers to the *_device calls (zero-copy over PCIe). */
int tfs_crc32_host_device_ptr(tfs_crc_ctx* ctx, const void* h_ptr, void** d_ptr);
int tfs_crc32_memcpy(tfs_crc_ctx* ctx, void* dst, const void* src, uint64_t bytes, void* stream);
int tfs_crc32_memset_device(tfs_crc_ctx* ctx, void* d_ptr, int value, uint64_t bytes, void* stream);
int tfs_crc32_event_create(tfs_crc_ctx* ctx, void** ev);
int tfs_crc32_event_record(tfs_crc_ctx* ctx, void* ev, void* stream);
int tfs_crc32_event_elapsed_ms(tfs_crc_ctx* ctx, void* ev_start, void* ev_end, float* ms);
int tfs_crc32_event_destroy(tfs_crc_ctx* ctx, void* ev);
/* The ctx's HIP stream (as void*); tfs_crc32_sync drains it and the ctx's
 * latency stream (the zero-copy small batches and async submissions launched
 * there), i.e. every launch the ctx queued on its own streams. */
void* tfs_crc32_stream(tfs_crc_ctx* ctx);
int tfs_crc32_sync(tfs_crc_ctx* ctx);
/* Extra non-blocking streams on ctx's device for the *_device calls (each
 * stream gets its own self-resetting scheduler slot; at most 192 live per ctx
 * incl. its own and the compaction streams), a synchronize on one, and its
 * release.  The *_device calls also take any other hipStream_t of the caller's
 * (each launch then leases a pooled slot and zeroes it on that stream first: one
 * memset more per launch); hipStreamPerThread is refused
 * (TFS_EXIT_PARAMETER_ERROR): it names a different queue on every thread. */
int tfs_crc32_stream_create(tfs_crc_ctx* ctx, void** stream);
int tfs_crc32_stream_sync(tfs_crc_ctx* ctx, void* stream);
int tfs_crc32_stream_destroy(tfs_crc_ctx* ctx, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TFS_CRC_H_ */
