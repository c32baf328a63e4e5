// tfs_crc_device.h -- layouts and constants shared by the gfx950 kernels and
// the host ABI (tfs_crc_abi.cpp).  Plain structs; no HIP types.
#pragma once
#include <stdint.h>

namespace tfscrc {

constexpr int kWave = 64;            // CDNA wavefront
constexpr int kBlock = 1024;         // 16 waves per workgroup, one file per wave, 1 workgroup per CU
constexpr unsigned kMaxGrid = 256;   // persistent: one workgroup per CU (LDS-bound)
constexpr uint32_t kMinParallelLen = 32;  // shorter payloads: byte loop in every lane
// Lane runs: each lane owns RUN contiguous bytes of every 64*RUN-byte stripe.
constexpr int kNumRuns = 4;               // RUN = 16 << ri, ri = 0..3 -> 16, 32, 64, 128 bytes
constexpr int kLevels = 6;                // shift tables for RUN*2^j, j = 0..5 (final lane combine)
// LDS layout (bytes): 4 slice tables replicated 32x (lane & 31 owns bank lane & 31),
// then the stripe-shift byte tables and the six level-shift byte tables (not replicated).
constexpr uint32_t kRepTableBytes = 256u * 32u * 4u;      // 32 KiB per slice table
constexpr uint32_t kLdsStripeOff = 4u * kRepTableBytes;   // 128 KiB
// Shift tables are indexed by 5-bit chunks of the CRC register (7 chunks, 32
// entries each): 32 entries sit in 32 distinct banks, so a random-index lookup
// never conflicts -- unlike a 256-entry byte table (~3.5x conflict cost).
// Alternatively (S8 kernels) 4x256 byte tables: 4 lookups instead of 7, but
// random indices conflict.  Both layouts are kept; DESIGN.md §4 has the numbers.
constexpr int kShiftChunks = 7;
constexpr uint32_t kShift5Stride = 1024u;                          // 896 B table, padded
constexpr uint32_t kShift8Stride = 4096u;                          // 4 x 256 x 4 B
// Table layouts (LY): 0 slice tables 32x + 5-bit shift tables (135 KiB); 1 slice
// tables 32x + byte shift tables (156 KiB, the product's one workgroup per CU);
// 2 slice tables 16x (64 KiB, four tables in one 256-byte bank row per byte value),
// the per-stripe shift as byte tables and the once-per-file level shifts 5-bit:
// 74 KiB, so two workgroups fit a CU's 160 KiB (round 5, the record kernel).
template <int LY> struct LdsLayout {
  static constexpr bool rep16 = LY == 2;
  static constexpr bool stripe_s8 = LY >= 1;
  static constexpr bool level_s8 = LY == 1;
  static constexpr uint32_t stripe_off = rep16 ? 65536u : kLdsStripeOff;
  static constexpr uint32_t stride = level_s8 ? kShift8Stride : kShift5Stride;  // level tables
  static constexpr uint32_t level_off = stripe_off + (stripe_s8 ? kShift8Stride : kShift5Stride);
  static constexpr uint32_t bytes = level_off + 6u * stride;  // 135 / 156 / 74 KiB
};

constexpr int kFileInfoSize = 36;  // sizeof(FileInfo), internal.h:432-446

// Dynamic work distribution: 8 ticket counters per launch, each on its own
// 256-byte line (atomics to one line serialise: ~88 per us for the whole line),
// and a ninth line counting finished waves (or workgroups).  A slot is bound to
// one stream, so its launches are ordered; the last wave (workgroup) to finish
// zeroes the slot, so the next launch on that stream finds it clean without a
// memset launch in between.
constexpr uint32_t kSchedStride = 64;                    // u32 between counters
constexpr uint32_t kSchedDone = 8u * kSchedStride;       // index of the finished-waves counter
constexpr uint32_t kSchedSlotBytes = 9u * kSchedStride * 4u;  // 2.25 KiB per stream
constexpr uint32_t kDynMinPerWave = 16;  // dynamic tickets only for launches of >= 16 files per wave

// Latency form (small batches): one workgroup of kWgWaves waves per file; wave w
// takes stripes w, w+16, ... of the file, so a 64 KiB file is 4-5 stripes per
// wave instead of 65 in one wave.  Lane chains jump over the 1023 foreign runs
// between two of their stripes (shift(c, 16*1023)), are moved into place with
// shift(c, 16*d) for d < 2^kWgLevels runs, XOR-reduced in the wave, then across
// waves through LDS.  Shift tables in 5-bit form (conflict-free, 1 KiB each).
constexpr int kWgWaves = kBlock / kWave;  // 16
constexpr int kWgLevels = 11;             // 16 B * 2^0 .. 2^10
constexpr uint32_t kWgMaxFiles = 256;     // batches up to this many files take the latency form
constexpr uint32_t kWgJumpOff = 4u * 256u * 32u * 4u;             // after the replicated slice tables (128 KiB)
constexpr uint32_t kWgLevelOff = kWgJumpOff + 1024u;
constexpr uint32_t kWgLdsBytes = kWgLevelOff + uint32_t(kWgLevels) * 1024u;  // 140 KiB

// Resident form (small synchronous host batches without a launch per batch):
// the host appends one ResUnit per file to ResHost, in page-locked fine-grained
// memory the kernel reads over PCIe, and bumps `published`.  Unit u belongs to
// workgroup u % grid (no claiming); each workgroup keeps the count of units it
// has done on its own device line across launches.  A file's result is one
// 8-byte store {crc, seq << 32} into the batch's page-locked result words, which
// the host spins on -- no counters, no flag.  A unit is never rewritten before
// its file is done: the host posts units [P, P + n) only while
// P + n - kResUnits <= the first unit of every batch still outstanding
// (tfs_crc_abi.cpp resident_post), otherwise it launches instead.
constexpr uint32_t kResUnits = 4096;            // ring of units
constexpr uint32_t kResMaxGrid = 256;           // workgroups of the resident kernel, at most
constexpr uint32_t kResExitLine = kResMaxGrid * kSchedStride;  // dstate: generation of the launch that is leaving
constexpr uint32_t kResLeftLine = kResExitLine + kSchedStride;  // dstate: workgroups of this launch that have left
constexpr uint32_t kResStateBytes = (kResMaxGrid + 2u) * kSchedStride * 4u;  // a line per workgroup + 2
constexpr uint32_t kResMaxPolls = 1u << 22;     // hard bound on one workgroup's idle polls
// A unit is one 128-byte line of eight 16-byte parts, each read by the kernel with
// one 16-byte load (lane p of the polling wave takes part p) and written by the
// host with one 16-byte store (an aligned 16-byte access is one PCIe read and
// never torn), and every part in use carries the unit's tag -- its index + 1,
// wrapping (0 never matches the zeroed ring).  A workgroup polls its next unit
// itself and takes it when the parts show the tag it expects: the unit comes back
// with the poll that finds it, with no second round trip (round 6).  Its result
// word is {crc, tag}.
// A body of at most kResInline bytes travels in the unit itself: its first 8
// bytes in `addr`, the rest 12 to a part in body[] -- no payload read over PCIe
// and no acquire fence for it.
constexpr uint32_t kResInline = 8u + 6u * 12u;  // 80 bytes
// The ring's workgroups read bodies with system-coherent loads and no fence:
// 0.6-1.2 us less per lone call, but ~10 % less rate than non-temporal loads once
// 16 workgroups stream together (64 files of 64 KiB: 92.8 against 84.4 us fenced,
// DESIGN.md section 5.5).  The units of a batch that reads more than
// kResBulkBytes over PCIe carry kResBulk in their length word: fence, then
// non-temporal stripes.
constexpr uint32_t kResBulk = 0x80000000u;
// With the ring in device memory (large BAR), a body of kResInline..kResLandMax
// bytes is copied by the host through the BAR into unit i's landing slot (slot
// i % kResUnits, kResLandMax bytes each) before the unit is written: the workgroup
// reads it from HBM instead of over PCIe.  PCIe keeps the host's posted writes in
// order, so the body lands before the unit that names it.
constexpr uint32_t kResLandMax = 16384;
// At most this many bytes are landed per batch: the host's copies through the BAR
// cost the calling thread ~0.1 us per KiB, while 16 workgroups pull a larger
// batch over PCIe in parallel (64 frames of 4 KiB: 0.61 us a frame landed, 0.44
// read over PCIe; of 1 KiB: 0.29 landed, 0.40 over PCIe).
constexpr uint64_t kResLandBatch = 64u << 10;
constexpr uint64_t kResBulkBytes = 1u << 20;
struct ResUnit {         // one file
  uint64_t addr;         // device-visible address of its first byte (inline: bytes 0..7)
  uint32_t len, tag_a;
  uint64_t out;          // device-visible address of its result word
  uint32_t seed, tag_b;  // seed 0 for a verify (the host compares)
  uint32_t body[6][4];   // inline: bytes 8 + 12 k .. 19 + 12 k in [k][0..2], the tag in [k][3]
};
struct ResHost {
  uint64_t published;    // low 32 bits: units published (wrapping); high 32 bits: stop
  uint64_t pad0[15];
  uint32_t left;         // generation of the last launch whose every workgroup has left (GPU-written)
  uint32_t pad1[31];
  ResUnit units[kResUnits];
};
static_assert(sizeof(ResHost) == 256 + sizeof(ResUnit) * kResUnits, "resident ring header");
static_assert(sizeof(ResUnit) == 128, "resident ring layout: one line per unit");

// TFS status codes (src/common/error_msg.h)
constexpr int32_t kSuccess = 0;
constexpr int32_t kExitCheckCrcError = -1010;
constexpr int32_t kExitParameterError = -1016;
constexpr int32_t kExitFileInfoError = -8016;
constexpr int32_t kExitReadFileSizeError = -8034;
constexpr int32_t kExitSyncFileError = -8038;

// 16-byte descriptor: {offset, len, seed | expected}.  Same bytes as
// tfs_crc_desc / tfs_crc_vdesc in include/tfs_crc.h.
struct Desc {
  uint64_t offset;
  uint32_t len;
  uint32_t aux;
};

// RawMeta (internal.h:535-645): file id, logical offset of the FileInfo, size incl. header.
struct RawMeta {
  uint64_t file_id;
  int32_t offset;
  int32_t size;
};

// One live record of a multi-block device compaction (same bytes as
// tfs_compact_job in include/tfs_crc.h).
struct CompactJob {
  uint64_t src_offset;   // FileInfo of the record in the source images
  uint64_t dest_offset;  // where the repacked record goes
  uint64_t file_id;      // expected FileInfo.id_
  int32_t size;          // record size incl. the 36-byte FileInfo
  int32_t flag;          // FileInfo.flag_ to write
  int32_t new_offset;    // FileInfo.offset_ to write (offset inside the new block)
  int32_t reserved;      // bit 0 (TFS_COMPACT_JOB_EDGE): read no byte past the record
};

// Packet frames (BasePacket / BasePacketStreamer, src/common/base_packet*.{h,cpp}).
// Same bytes as tfs_packet_desc in include/tfs_crc.h.
struct PacketDesc {
  uint64_t offset;  // frame start (the TfsPacketNewHeaderV0/V1 header)
  uint32_t len;     // bytes of the frame available at offset
  uint32_t reserved;
};
constexpr uint32_t kPacketFlagV0 = 0x4d534654u;  // "TFSM", base_packet.h:347
constexpr uint32_t kPacketFlagV1 = 0x4e534654u;  // "TFSN", base_packet.h:348 (also the CRC seed)
constexpr int32_t kPacketHeaderV0Size = 12;      // sizeof(TfsPacketNewHeaderV0), pack(4)
constexpr int32_t kPacketHeaderDiffSize = 12;    // V1 - V0: id_ (8) + crc_ (4)
constexpr int32_t kPacketMaxDataLen = 0x4000000; // base_packet_streamer.cpp:81 (64 MiB)
constexpr int32_t kTfsError = -1;                // cdefine.h TFS_ERROR: broken stream
constexpr int32_t kPacketIncomplete = 1;         // streamer waits for more bytes
constexpr int32_t kPacketPending = 0x7fffffff;   // internal: CRC check outstanding

#pragma pack(push, 4)
struct FileInfoHdr {  // FileInfo, internal.h:432-446
  uint64_t id;
  int32_t offset;
  int32_t size;
  int32_t usize;
  int32_t mtime;
  int32_t ctime;
  int32_t flag;
  uint32_t crc;
};
#pragma pack(pop)
static_assert(sizeof(FileInfoHdr) == kFileInfoSize, "FileInfo must be 36 bytes");

// Split files.  A throughput launch of crc_files_kernel cuts
// every file longer than kSplitMin into a ragged head and kSegBytes segments, so
// no wave streams more than kSegBytes of one file alone (a wave that walks a
// 1 MiB file alone reads slower than the moving window of the rest: Zipf +4-5 %).
// The plan lists every unit of the launch -- whole files, heads and segments --
// in address order (split_ao_count / _scan / _write); the main kernel checksums a
// head with its file's seed and each segment with seed 0, and the fold
// (split_ao_fold_kernel) joins them: crc = shift(...shift(crc_head, S) ^ crc_1
// ..., S) ^ crc_K, shift by S bytes from one table.
#ifndef TFS_SEG_KIB
#define TFS_SEG_KIB 128  // measurement builds may set another segment size
#endif
constexpr uint32_t kSegBytes = uint32_t(TFS_SEG_KIB) << 10;
constexpr uint32_t kSplitMin = kSegBytes;
constexpr uint32_t kNoSplit = 0xffffffffu;
constexpr uint32_t kSplitMaxUnits = 4u << 20;  // segments per launch at most (files past the cut stay whole)
struct SplitArgs {
  uint8_t* plan;  // nullptr: no split plan
  uint32_t cap;   // units (files + segments) at most
};

// The plan (one allocation per scheduler slot):
// [units u32 | nosplit u32 | ext u32 | cut u32][blk u32 x nblk][ubase u32 x n]
// [ucrc u32 x ucap][pad to 16][SplitUnit x ucap], nblk = ceil(n / 256).  When the
// segments of every file would pass the room (cap - n), only files [0, cut) are
// split (the longest prefix whose segments fit); the rest stay whole.
struct SplitUnit {
  uint64_t offset;
  uint32_t len, aux;   // aux: the file's seed / expected CRC on a whole file or head, 0 on a segment
  uint32_t file, kind; // kind 0 a whole file, 1 a segment, 2 a split file's head
  uint64_t pad;
};
static_assert(sizeof(SplitUnit) == 32, "split unit layout");
constexpr uint32_t kAoBlock = 256;
constexpr uint32_t ao_nblk(uint32_t n) { return (n + kAoBlock - 1u) / kAoBlock; }
constexpr uint64_t ao_off_blk() { return 16u; }
constexpr uint64_t ao_off_ubase(uint32_t n) { return 16u + 4ull * ao_nblk(n); }
constexpr uint64_t ao_off_ucrc(uint32_t n) { return ao_off_ubase(n) + 4ull * n; }
constexpr uint64_t ao_off_units(uint32_t n, uint32_t ucap) { return (ao_off_ucrc(n) + 4ull * ucap + 15u) & ~15ull; }
constexpr uint64_t ao_bytes(uint32_t n, uint32_t ucap) { return ao_off_units(n, ucap) + 32ull * ucap; }

// Segmented compaction (round 4): a throughput compaction launch
// cuts every live record whose payload is longer than one segment into a ragged
// head (the FileInfo and the first len - K*seg payload bytes, in the record's own
// ticket slot) and K whole `seg`-byte payload segments appended after the jobs as
// extra units, so the waves of a launch copy and checksum segment-sized pieces
// (a tighter window of addresses in flight than one wave per record);
// compact_seg_fold_kernel joins each record's CRCs and writes its CRC / status.
// Plan (one allocation per scheduler slot, like SplitArgs):
// [used u64 | pad][base u32 x n][head_crc u32 x n][hdr_crc u32 x n][pre i32 x n]
// [ext_crc u32 x cap][pad to 16][CSegUnit x cap]
struct CSegArgs {
  uint8_t* plan;  // nullptr: records stay whole
  uint32_t cap;   // ext units at most (records past it stay whole)
  uint32_t lg;    // seg = 1 KiB << lg (lg 3..5: 8, 16, 32 KiB)
};
struct CSegUnit {  // one whole payload segment of a split record
  uint64_t src, dst;  // payload byte offsets in the source / destination images
  uint32_t len, job;
  uint64_t pad;  // bit 0: the record's TFS_COMPACT_JOB_EDGE, on its last segment only
};
static_assert(sizeof(CSegUnit) == 32, "segment unit layout");
constexpr uint32_t kCSegLgMin = 3, kCSegLgMax = 5;
constexpr uint64_t cseg_off_base() { return 16u; }
constexpr uint64_t cseg_off_head(uint32_t n) { return 16u + 4ull * n; }
constexpr uint64_t cseg_off_hdr(uint32_t n) { return 16u + 8ull * n; }
constexpr uint64_t cseg_off_pre(uint32_t n) { return 16u + 12ull * n; }
constexpr uint64_t cseg_off_ext_crc(uint32_t n) { return 16u + 16ull * n; }
constexpr uint64_t cseg_off_ext(uint32_t n, uint32_t cap) { return (16u + 16ull * n + 4ull * cap + 15u) & ~15ull; }
constexpr uint64_t cseg_bytes(uint32_t n, uint32_t cap) { return cseg_off_ext(n, cap) + 32ull * cap; }

// Device-resident constant tables (built on the host by crc_math.h).
struct Tables {
  uint32_t slice[4][256];                          // slice-by-4 (slice k: byte then k zero bytes)
  uint32_t stripe[kNumRuns][kShiftChunks][32];          // 5-bit-chunk tables of shift(c, 63*RUN)
  uint32_t stripe64[kNumRuns][kShiftChunks][32];        // shift(c, 64*RUN) (parallel-shift form)
  uint32_t level[kNumRuns][kLevels][kShiftChunks][32];  // shift(c, RUN*2^j), final lane combine
  uint32_t stripe8[kNumRuns][4][256];                   // byte-table forms of the same shifts
  uint32_t stripe64_8[kNumRuns][4][256];
  uint32_t level8[kNumRuns][kLevels][4][256];
  uint32_t wg_jump[kShiftChunks][32];              // latency form: shift(c, 16 * (64 * kWgWaves - 1))
  uint32_t wg_level[kWgLevels][kShiftChunks][32];  // latency form: shift(c, 16 * 2^j)
  uint32_t seg_shift[kShiftChunks][32];            // split files: shift(c, kSegBytes)
  uint32_t cseg_shift[kCSegLgMax - kCSegLgMin + 1][kShiftChunks][32];  // segmented compaction: shift(c, 1 KiB << lg)
};

constexpr int run_index(int run) { return run == 16 ? 0 : run == 32 ? 1 : run == 64 ? 2 : 3; }

}  // namespace tfscrc
