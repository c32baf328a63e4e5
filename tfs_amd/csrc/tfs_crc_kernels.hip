// tfs_crc_kernels.hip -- gfx950 kernels for TFS's per-file CRC32 path.
//
// Replaces the byte loop of tfs::common::Func::crc (src/common/func.cpp:426-435)
// at the dataserver's per-file call sites (write: data_file.cpp:190; verify:
// sync_backup.cpp:383/412, block_console.cpp:570; compact: task.cpp:795-798).
// Bit-identical arithmetic: reflected CRC-32 (0xEDB88320), caller seed, no
// inversion.
//
// Execution model: one wavefront per file.  The file's aligned
// body is cut into lane segments of L bytes (L = 64..1024, chosen per file),
// laid out so the LAST segment ends at the last 16-byte boundary of the file
// (leading bytes of a seed-0 CRC that are zero do not change it, so the body is
// zero-extended at the front).  Each lane runs the slice-by-4 table recurrence
// (LDS tables) over its segments; segments of later 64-segment stripes continue
// the same lane chain after a shift over the 63 foreign segments in between.
// Lane results are moved to their position by shift(c, (63-lane)*L) -- a
// product of level shifts looked up in byte tables -- and XOR-reduced across
// the wave with __shfl_xor (the CRC is linear over GF(2)).  The <=15 tail bytes
// after the last 16-byte boundary are folded in by every lane redundantly.
// The seed is injected by XOR into the first four message bytes, which is
// exactly what Func::crc does with its initial register.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tfs_crc_device.h"

namespace tfscrc {

// ---------------------------------------------------------------------------
// Table helpers.  T points at 4x256 slice tables in LDS (slice k = byte followed
// by k zero bytes); shift tables live in global memory (L2-resident, touched a
// few times per file).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t step4(const uint32_t* T, uint32_t c, uint32_t w) {
  const uint32_t x = c ^ w;
  return T[768 + (x & 0xffu)] ^ T[512 + ((x >> 8) & 0xffu)] ^ T[256 + ((x >> 16) & 0xffu)] ^ T[x >> 24];
}

__device__ __forceinline__ uint32_t step1(const uint32_t* T, uint32_t c, uint32_t b) {
  return (c >> 8) ^ T[(c ^ b) & 0xffu];
}

__device__ __forceinline__ uint32_t shift_tab(const uint32_t* __restrict__ S, uint32_t c) {
  return S[c & 0xffu] ^ S[256 + ((c >> 8) & 0xffu)] ^ S[512 + ((c >> 16) & 0xffu)] ^ S[768 + (c >> 24)];
}

__device__ __forceinline__ uint32_t ld32(uintptr_t a) { return *reinterpret_cast<const uint32_t*>(a); }
__device__ __forceinline__ uint4 ld128(uintptr_t a) { return *reinterpret_cast<const uint4*>(a); }

// CRC of `len` bytes at p with initial register `seed`, computed by the whole
// wave; the result is returned in every lane.  `lane` = threadIdx.x & 63.
__device__ uint32_t wave_crc(const uint8_t* p, uint32_t len, uint32_t seed, const uint32_t* T,
                             const Tables* __restrict__ tg, int lane) {
  if (len < kMinParallelLen) {  // tiny: every lane runs the byte loop of func.cpp:429-433
    uint32_t c = seed;
    for (uint32_t i = 0; i < len; ++i) c = step1(T, c, p[i]);
    return c;
  }
  const uintptr_t start = reinterpret_cast<uintptr_t>(p);
  const uintptr_t end = start + len;
  const uintptr_t A = start & ~uintptr_t(3);
  const uintptr_t B16 = end & ~uintptr_t(15);
  const uint32_t s = uint32_t(start - A);
  const uint32_t body = uint32_t(B16 - A);  // >= 20 because len >= kMinParallelLen

  const uint32_t li = pick_segment_log(body);
  const uint32_t L = kMinSeg << li;
  const uint32_t nseg = (body + L - 1) / L;
  const uint32_t nstripes = (nseg + kWave - 1) / kWave;
  const uint32_t vsegs = nstripes * kWave;

  const uint32_t* __restrict__ Sstripe = tg->shift[li][kStripeShift][0];
  const uint32_t headmask = 0xffffffffu << (8 * s);
  const uint32_t seed_lo = seed << (8 * s);
  const uint32_t seed_hi = s ? (seed >> (32 - 8 * s)) : 0u;

  uint32_t c = 0;
  for (uint32_t r = 0; r < nstripes; ++r) {
    if (r) c = shift_tab(Sstripe, c);
    const uint32_t v = r * kWave + lane;
    const uint64_t dist_hi = uint64_t(vsegs - 1 - v) * L;  // bytes between segment end and B16
    if (dist_hi >= body) continue;                          // segment wholly in the zero extension
    const uintptr_t hi = B16 - dist_hi;
    uintptr_t q = (dist_hi + L >= body) ? A : hi - L;
    if (q == A) {
      c = step4(T, c, (ld32(q) & headmask) ^ seed_lo);
      q += 4;
    }
    if (q == A + 4 && q < hi) {
      c = step4(T, c, ld32(q) ^ seed_hi);
      q += 4;
    }
    while ((q & 15) && q < hi) {
      c = step4(T, c, ld32(q));
      q += 4;
    }
    for (; q + 64 <= hi; q += 64) {
      const uint4 a = ld128(q), b = ld128(q + 16), d = ld128(q + 32), e = ld128(q + 48);
      c = step4(T, c, a.x); c = step4(T, c, a.y); c = step4(T, c, a.z); c = step4(T, c, a.w);
      c = step4(T, c, b.x); c = step4(T, c, b.y); c = step4(T, c, b.z); c = step4(T, c, b.w);
      c = step4(T, c, d.x); c = step4(T, c, d.y); c = step4(T, c, d.z); c = step4(T, c, d.w);
      c = step4(T, c, e.x); c = step4(T, c, e.y); c = step4(T, c, e.z); c = step4(T, c, e.w);
    }
    for (; q < hi; q += 16) {
      const uint4 a = ld128(q);
      c = step4(T, c, a.x); c = step4(T, c, a.y); c = step4(T, c, a.z); c = step4(T, c, a.w);
    }
  }
  // Move the lane's chain to its place in the body: shift by (63-lane)*L.
  const uint32_t k = uint32_t(kWave - 1 - lane);
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const uint32_t sh = shift_tab(tg->shift[li][j][0], c);
    c = ((k >> j) & 1u) ? sh : c;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c ^= __shfl_xor(c, m, kWave);
  // Tail after the last 16-byte boundary (same in every lane).
  uintptr_t q = B16;
  for (; q + 4 <= end; q += 4) c = step4(T, c, ld32(q));
  for (; q < end; ++q) c = step1(T, c, *reinterpret_cast<const uint8_t*>(q));
  return c;
}

__device__ __forceinline__ void load_slice_tables(uint32_t* T, const Tables* __restrict__ tg) {
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) T[i] = tg->slice[0][i];
  __syncthreads();
}

// MODE 0: compute (aux = seed) -> out_crc.  MODE 1: verify (aux = expected, seed 0).
template <int MODE>
__global__ void __launch_bounds__(kBlock) crc_files_kernel(const uint8_t* __restrict__ base,
                                                           const Desc* __restrict__ desc, uint32_t n,
                                                           const Tables* __restrict__ tg, uint32_t* out_crc,
                                                           uint8_t* out_ok, uint32_t* n_bad) {
  __shared__ uint32_t T[1024];
  load_slice_tables(T, tg);
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t wpb = kBlock / kWave;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  uint32_t bad = 0;
  for (uint32_t f = blockIdx.x * wpb + wave; f < n; f += gridDim.x * wpb) {
    const Desc d = desc[f];
    const uint32_t seed = MODE == 0 ? d.aux : 0u;
    const uint32_t c = wave_crc(base + d.offset, d.len, seed, T, tg, lane);
    if (lane == 0) {
      if (out_crc) out_crc[f] = c;
      if (MODE == 1) {
        const bool ok = c == d.aux;
        if (out_ok) out_ok[f] = ok ? 1 : 0;
        bad += ok ? 0u : 1u;
      }
    }
  }
  if (MODE == 1 && lane == 0 && bad && n_bad) atomicAdd(n_bad, bad);
}

// Verify files stored in a block image (FileInfo header + payload per RawMeta):
// the checks of sync_backup.cpp:345-435 / block_console.cpp:543-577.
__global__ void __launch_bounds__(kBlock) block_verify_kernel(const uint8_t* __restrict__ image, uint64_t image_len,
                                                              const RawMeta* __restrict__ metas, uint32_t n,
                                                              const Tables* __restrict__ tg, uint32_t* out_crc,
                                                              int32_t* out_status, uint32_t* n_bad) {
  __shared__ uint32_t T[1024];
  load_slice_tables(T, tg);
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t wpb = kBlock / kWave;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  uint32_t bad = 0;
  for (uint32_t f = blockIdx.x * wpb + wave; f < n; f += gridDim.x * wpb) {
    const RawMeta m = metas[f];
    int32_t status = kSuccess;
    uint32_t c = 0;
    if (m.size <= kFileInfoSize) {
      status = kExitReadFileSizeError;
    } else if (m.offset < 0 || uint64_t(m.offset) + uint64_t(m.size) > image_len) {
      status = kExitParameterError;
    } else {
      const uint8_t* rec = image + m.offset;
      FileInfoHdr h;
      // 36-byte header at an arbitrary byte offset: byte-wise read, same in all lanes.
      uint8_t* hb = reinterpret_cast<uint8_t*>(&h);
      for (int i = 0; i < kFileInfoSize; ++i) hb[i] = rec[i];
      c = wave_crc(rec + kFileInfoSize, uint32_t(m.size - kFileInfoSize), 0u, T, tg, lane);
      if (h.id != m.file_id) status = kExitFileInfoError;
      else if (h.size != m.size) status = kExitSyncFileError;
      else if (c != h.crc) status = kExitCheckCrcError;
    }
    if (lane == 0) {
      if (out_crc) out_crc[f] = c;
      if (out_status) out_status[f] = status;
      bad += status != kSuccess ? 1u : 0u;
    }
  }
  if (lane == 0 && bad && n_bad) atomicAdd(n_bad, bad);
}

// Compaction repack (task.cpp:753-798): copy each live record (FileInfo|payload)
// to its new offset and rewrite offset_/size_/usize_/flag_.  One wave per record.
__global__ void __launch_bounds__(kBlock) compact_copy_kernel(const uint8_t* __restrict__ src,
                                                              const RawMeta* __restrict__ metas,
                                                              const int32_t* __restrict__ flags,
                                                              const int64_t* __restrict__ dest_off, uint32_t n,
                                                              uint8_t* __restrict__ dst) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t wpb = kBlock / kWave;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  for (uint32_t f = blockIdx.x * wpb + wave; f < n; f += gridDim.x * wpb) {
    const int64_t doff = dest_off[f];
    if (doff < 0) continue;
    const RawMeta m = metas[f];
    const uint8_t* s = src + m.offset;
    uint8_t* d = dst + doff;
    // Header: FileInfo with offset_(8) size_(12) usize_(16) flag_(28) rewritten,
    // id_, times and crc_ copied (task.cpp:753-759).  Lanes 0..35 write one byte each.
    if (lane < kFileInfoSize) {
      uint8_t b = s[lane];
      const int fld = lane >> 2, sh = 8 * (lane & 3);
      if (fld == 2) b = uint8_t(uint32_t(int32_t(doff)) >> sh);
      else if (fld == 3 || fld == 4) b = uint8_t(uint32_t(m.size) >> sh);
      else if (fld == 7) b = uint8_t(uint32_t(flags[f]) >> sh);
      d[lane] = b;
    }
    // Payload.
    const uint8_t* sp = s + kFileInfoSize;
    uint8_t* dp = d + kFileInfoSize;
    const uint32_t size = uint32_t(m.size - kFileInfoSize);
    const uintptr_t sa = reinterpret_cast<uintptr_t>(sp), da = reinterpret_cast<uintptr_t>(dp);
    if (((sa ^ da) & 3u) == 0) {
      // Same alignment mod 4: byte head, dword body, byte tail.
      uint32_t head = uint32_t((4u - (da & 3u)) & 3u);
      if (head > size) head = size;
      for (uint32_t i = lane; i < head; i += kWave) dp[i] = sp[i];
      const uint32_t nw = (size - head) / 4;
      const uint32_t* s4 = reinterpret_cast<const uint32_t*>(sp + head);
      uint32_t* d4 = reinterpret_cast<uint32_t*>(dp + head);
      for (uint32_t i = lane; i < nw; i += kWave) d4[i] = s4[i];
      for (uint32_t i = head + nw * 4 + lane; i < size; i += kWave) dp[i] = sp[i];
    } else {
      for (uint32_t i = lane; i < size; i += kWave) dp[i] = sp[i];
    }
  }
}

// Synthetic payload bytes: word i = splitmix64(seed + (first_word + i + 1) * GOLDEN)
// (same stream as tfs_amd/synth.py).
__global__ void synth_fill_kernel(uint64_t* __restrict__ dst, uint64_t nwords, uint64_t seed, uint64_t first_word) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nwords; i += stride) {
    uint64_t z = seed + (first_word + i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    dst[i] = z ^ (z >> 31);
  }
}

// Write FileInfo headers for a packed block layout (bench / test helper):
// record f at rec_off[f], payload len[f], crc[f].
__global__ void write_headers_kernel(uint8_t* __restrict__ image, const uint64_t* __restrict__ rec_off,
                                     const uint32_t* __restrict__ len, const uint32_t* __restrict__ crc,
                                     uint64_t first_id, uint32_t n) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  FileInfoHdr h;
  h.id = first_id + f;
  h.offset = int32_t(rec_off[f]);
  h.size = int32_t(len[f] + kFileInfoSize);
  h.usize = h.size;
  h.mtime = 0;
  h.ctime = 0;
  h.flag = 0;
  h.crc = crc[f];
  const uint8_t* hb = reinterpret_cast<const uint8_t*>(&h);
  uint8_t* d = image + rec_off[f];
  for (int i = 0; i < kFileInfoSize; ++i) d[i] = hb[i];
}

// Calibration kernels (not on the product path): how fast can this GPU stream
// the same bytes without the CRC arithmetic?  PATTERN 0: fully coalesced
// grid-stride 16 B/lane.  PATTERN 1: the CRC kernel's access pattern (one
// wave per file, lane segments of L bytes, 4 x 16 B loads in flight per lane).
template <int PATTERN>
__global__ void __launch_bounds__(kBlock) membench_kernel(const uint8_t* __restrict__ base, const Desc* __restrict__ desc,
                                                          uint32_t n, uint64_t nbytes, uint32_t* out) {
  uint32_t acc = 0;
  if (PATTERN == 0) {
    const uint4* p = reinterpret_cast<const uint4*>(base);
    const uint64_t nv = nbytes / 16;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nv; i += stride) {
      const uint4 v = p[i];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  } else {
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wpb = kBlock / kWave;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    for (uint32_t f = blockIdx.x * wpb + wave; f < n; f += gridDim.x * wpb) {
      const Desc d = desc[f];
      const uintptr_t start = reinterpret_cast<uintptr_t>(base + d.offset);
      const uint32_t L = d.len / kWave;  // assumes len multiple of 1 KiB, 16-aligned start
      uintptr_t q = (start + 15) & ~uintptr_t(15);
      q += uint64_t(lane) * L;
      const uintptr_t hi = q + L;
      for (; q + 64 <= hi; q += 64) {
        const uint4 a = ld128(q), b = ld128(q + 16), c = ld128(q + 32), e = ld128(q + 48);
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ e.x ^ e.y ^ e.z ^ e.w;
      }
    }
  }
  if (acc == 0x9E3779B9u) out[0] = acc;  // keep the loads alive
}

}  // namespace tfscrc

// ---------------------------------------------------------------------------
// Launch wrappers (called from tfs_crc_abi.cpp; no HIP types leak past this TU
// except through that file).
// ---------------------------------------------------------------------------
namespace tfscrc {

static unsigned grid_for(uint32_t nwork) {
  const uint32_t wpb = kBlock / kWave;
  uint64_t g = (uint64_t(nwork) + wpb - 1) / wpb;
  if (g > kMaxGrid) g = kMaxGrid;
  if (g == 0) g = 1;
  return unsigned(g);
}

hipError_t launch_crc_files(int mode, const uint8_t* base, const Desc* desc, uint32_t n, const Tables* tg,
                            uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const dim3 grid(grid_for(n)), block(kBlock);
  if (mode == 0)
    hipLaunchKernelGGL(crc_files_kernel<0>, grid, block, 0, stream, base, desc, n, tg, out_crc, out_ok, n_bad);
  else
    hipLaunchKernelGGL(crc_files_kernel<1>, grid, block, 0, stream, base, desc, n, tg, out_crc, out_ok, n_bad);
  return hipGetLastError();
}

hipError_t launch_block_verify(const uint8_t* image, uint64_t image_len, const RawMeta* metas, uint32_t n,
                               const Tables* tg, uint32_t* out_crc, int32_t* out_status, uint32_t* n_bad,
                               hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(block_verify_kernel, dim3(grid_for(n)), dim3(kBlock), 0, stream, image, image_len, metas, n, tg,
                     out_crc, out_status, n_bad);
  return hipGetLastError();
}

hipError_t launch_compact_copy(const uint8_t* src, const RawMeta* metas, const int32_t* flags, const int64_t* dest_off,
                               uint32_t n, uint8_t* dst, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(compact_copy_kernel, dim3(grid_for(n)), dim3(kBlock), 0, stream, src, metas, flags, dest_off, n,
                     dst);
  return hipGetLastError();
}

hipError_t launch_synth_fill(uint64_t* dst, uint64_t nwords, uint64_t seed, uint64_t first_word, hipStream_t stream) {
  if (nwords == 0) return hipSuccess;
  uint64_t g = (nwords + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(synth_fill_kernel, dim3(unsigned(g)), dim3(256), 0, stream, dst, nwords, seed, first_word);
  return hipGetLastError();
}

hipError_t launch_membench(int pattern, const uint8_t* base, const Desc* desc, uint32_t n, uint64_t nbytes,
                           uint32_t* out, unsigned grid, hipStream_t stream) {
  if (pattern == 0)
    hipLaunchKernelGGL(membench_kernel<0>, dim3(grid ? grid : 4096), dim3(kBlock), 0, stream, base, desc, n, nbytes, out);
  else
    hipLaunchKernelGGL(membench_kernel<1>, dim3(grid ? grid : grid_for(n)), dim3(kBlock), 0, stream, base, desc, n,
                       nbytes, out);
  return hipGetLastError();
}

hipError_t launch_write_headers(uint8_t* image, const uint64_t* rec_off, const uint32_t* len, const uint32_t* crc,
                                uint64_t first_id, uint32_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(write_headers_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, image, rec_off, len, crc,
                     first_id, n);
  return hipGetLastError();
}

}  // namespace tfscrc
