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
constexpr uint32_t kLdsLevelOff = kLdsStripeOff + 4096u;          // + 4 KiB stripe-shift tables
constexpr uint32_t kLdsBytes = kLdsLevelOff + 6u * 4096u;          // + 24 KiB level tables = 156 KiB

constexpr int kFileInfoSize = 36;  // sizeof(FileInfo), internal.h:432-446

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

// Device-resident constant tables (built on the host by crc_math.h).
struct Tables {
  uint32_t slice[4][256];                          // slice-by-4 (slice k: byte then k zero bytes)
  uint32_t stripe[kNumRuns][4][256];               // byte tables of shift(c, 63*RUN)
  uint32_t level[kNumRuns][kLevels][4][256];       // byte tables of shift(c, RUN*2^j)
};

constexpr int run_index(int run) { return run == 16 ? 0 : run == 32 ? 1 : run == 64 ? 2 : 3; }

}  // namespace tfscrc
