// tfs_crc_device.h -- layouts and constants shared by the gfx950 kernels and
// the host ABI (tfs_crc_abi.cpp).  Plain structs; no HIP types.
#pragma once
#include <stdint.h>

namespace tfscrc {

constexpr int kWave = 64;           // CDNA wavefront
constexpr int kBlock = 256;         // 4 waves per workgroup, one file per wave
constexpr unsigned kMaxGrid = 8192; // grid-stride beyond 32 workgroups/CU
constexpr uint32_t kMinParallelLen = 32;  // shorter payloads: byte loop in every lane
constexpr uint32_t kMinSeg = 64;          // lane segment L = kMinSeg << li
constexpr int kNumSegLog = 5;             // li = 0..4 -> L = 64..1024 bytes
constexpr int kLevels = 6;                // shift tables for L*2^j, j = 0..5
constexpr int kStripeShift = 6;           // shift table for 63*L (between stripes)
constexpr int kShiftTabs = 7;

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
  uint32_t slice[4][256];                                // slice-by-4, LDS-staged per workgroup
  uint32_t shift[kNumSegLog][kShiftTabs][4][256];        // byte tables of shift(c, L*2^j) and shift(c, 63*L)
};

// Segment size for a body of `body` bytes: the largest L in 64..1024 with
// 64 * L <= body (so a wave's 64 lanes are busy), at least 64.
__host__ __device__ inline uint32_t pick_segment_log(uint32_t body) {
  const uint32_t q = body >> 6;
  return q >= 1024u ? 4u : q >= 512u ? 3u : q >= 256u ? 2u : q >= 128u ? 1u : 0u;
}

}  // namespace tfscrc
