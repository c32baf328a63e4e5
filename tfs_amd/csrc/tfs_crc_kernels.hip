// tfs_crc_kernels.hip -- gfx950 kernels for TFS's per-file CRC32 path.
//
// Replaces the byte loop of tfs::common::Func::crc (src/common/func.cpp:426-435)
// at the dataserver's per-file call sites (write: data_file.cpp:190; verify:
// sync_backup.cpp:383/412, block_console.cpp:570; compact: task.cpp:795-798).
// Bit-identical arithmetic: reflected CRC-32 (0xEDB88320), caller seed, no
// inversion.
//
// Execution model: one wavefront per file, 16 waves per
// workgroup, one workgroup per CU (persistent grid-stride over files).
//
// Byte -> lane mapping ("stripes"): the file's aligned body is cut, from its
// last 16-byte boundary backwards, into stripes of 64*RUN bytes; lane l owns
// bytes [l*RUN, (l+1)*RUN) of every stripe.  A stripe is therefore one
// coalesced sweep of the wave (RUN/16 dwordx4 loads per lane, contiguous across
// lanes), so the HBM stream is read in whole cache lines straight into VGPRs.
// Each lane runs one CRC chain over its runs: slice-by-4 steps whose four
// 1 KiB tables are replicated 32x in LDS so that lane (l & 31) always hits
// bank (l & 31) -- a random-byte table lookup never bank-conflicts -- and, at
// every stripe boundary, a jump over the 63 foreign runs (shift(c, 63*RUN), one
// byte-table lookup per state byte).  Finally lane chains are moved to their
// place with shift(c, (63-lane)*RUN) (level tables) and XOR-reduced across the
// wave with __shfl_xor -- the CRC is linear over GF(2).  The body starts zero-
// extended in front (leading zero bytes do not change a seed-0 CRC register);
// the seed is injected by XOR into the first four message bytes, which is
// exactly Func::crc's initial register; the <=15 tail bytes after the last
// 16-byte boundary are folded in by every lane redundantly.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "tfs_crc_device.h"

namespace tfscrc {

// ---------------------------------------------------------------------------
// LDS table access.  Replicated slice table k (k zero bytes follow the byte)
// lives at k*32 KiB; entry b of copy j at b*128 + j*4.  `lb` = this lane's
// copy offset ((lane & 31) * 4); it has no bits in 7..14, so OR == ADD.
// ---------------------------------------------------------------------------
// Payload loads through explicit global (addrspace 1) pointers: flat loads would
// also count on lgkmcnt and serialise against the LDS table lookups.
typedef const __attribute__((address_space(1))) uint32_t* gu32p;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gu128p;
typedef const __attribute__((address_space(1))) uint8_t* gu8p;
__device__ __forceinline__ uint32_t ld32(uintptr_t a) { return *reinterpret_cast<gu32p>(a); }
__device__ __forceinline__ uint4 ld128(uintptr_t a) {
  const u32x4 v = *reinterpret_cast<gu128p>(a);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// Streaming payload load: read once, never re-used -> non-temporal (nt) policy.
template <bool NT>
__device__ __forceinline__ uint4 ld128s(uintptr_t a) {
  if (NT) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<gu128p>(a));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return ld128(a);
}
__device__ __forceinline__ uint32_t ld8(uintptr_t a) { return *reinterpret_cast<gu8p>(a); }

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// `T` is the workgroup's __shared__ table array (LDS address 0 in practice).
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* T, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(T) + byte_addr);
}

// Replicated slice tables, laid out for one-instruction addressing: the byte
// address of (table t, entry b, copy j) is
//   region(t) << 16 | b << 8 | half(t) << 7 | j << 2
// with T3 = (region 0, half 0), T2 = (0, 1), T1 = (1, 0), T0 = (1, 1).  Bits 2..6
// are the lane's copy, so lane (l & 31) always reads bank (l & 31): no bank
// conflicts for any data.  The address is a byte permutation of {x, Lk}:
// v_perm_b32 places byte k of x in bits 8..15 and keeps Lk's bytes 0 and 2.
__device__ __forceinline__ uint32_t perm_addr(uint32_t x, uint32_t L, uint32_t sel) {
  return __builtin_amdgcn_perm(x, L, sel);
}
constexpr uint32_t kSelByte0 = 0x0C020400u, kSelByte1 = 0x0C020500u, kSelByte2 = 0x0C020600u, kSelByte3 = 0x0C020700u;
// Lane bases for the four slice tables.
struct LaneBase {
  uint32_t t3, t2, t1, t0;
};
__device__ __forceinline__ LaneBase lane_base_of(int lane) {
  const uint32_t l4 = uint32_t(lane & 31) * 4u;
  return LaneBase{l4, l4 | 0x80u, l4 | 0x10000u, l4 | 0x10080u};
}
// Layout 2 (16 copies, LdsLayout<2>): entry (table t, byte b, copy j < 16) at
// b << 8 | tsel(t) << 6 | j << 2 with T3..T0 = tsel 0..3 -- the same v_perm
// addressing (bits 16.. zero); lanes l, l+16, l+32, l+48 share a bank.
template <int LY>
__device__ __forceinline__ LaneBase lane_base_for(int lane) {
  if constexpr (LdsLayout<LY>::rep16) {
    const uint32_t l4 = uint32_t(lane & 15) * 4u;
    return LaneBase{l4, l4 | 0x40u, l4 | 0x80u, l4 | 0xC0u};
  }
  return lane_base_of(lane);
}

// One dword of the slice-by-4 recurrence on x = c ^ w, fused with the XOR of the
// next payload dword: returns M(x) ^ w_next.
__device__ __forceinline__ uint32_t step4x(const uint32_t* T, const LaneBase& lb, uint32_t x, uint32_t w_next) {
  const uint32_t a = xor3(lds_ld(T, perm_addr(x, lb.t3, kSelByte0)), lds_ld(T, perm_addr(x, lb.t2, kSelByte1)),
                          lds_ld(T, perm_addr(x, lb.t1, kSelByte2)));
  return xor3(a, lds_ld(T, perm_addr(x, lb.t0, kSelByte3)), w_next);
}
__device__ __forceinline__ uint32_t step4(const uint32_t* T, const LaneBase& lb, uint32_t c, uint32_t w) {
  return step4x(T, lb, c ^ w, 0u);
}

__device__ __forceinline__ uint32_t step1(const uint32_t* T, const LaneBase& lb, uint32_t c, uint32_t b) {
  return (c >> 8) ^ lds_ld(T, perm_addr(c ^ b, lb.t0, kSelByte0));
}

// shift(c, d) from a 7x32 chunk table at LDS offset `off`: conflict-free lookups.
__device__ __forceinline__ uint32_t shift5(const uint32_t* T, uint32_t off, uint32_t c) {
  const uint32_t a = xor3(lds_ld(T, off + ((c << 2) & 0x7Cu)), lds_ld(T, off + 128u + ((c >> 3) & 0x7Cu)),
                          lds_ld(T, off + 256u + ((c >> 8) & 0x7Cu)));
  const uint32_t b = xor3(lds_ld(T, off + 384u + ((c >> 13) & 0x7Cu)), lds_ld(T, off + 512u + ((c >> 18) & 0x7Cu)),
                          lds_ld(T, off + 640u + ((c >> 23) & 0x7Cu)));
  return xor3(a, b, lds_ld(T, off + 768u + ((c >> 28) & 0x0Cu)));
}
// shift(c, d) from 4x256 byte tables at `off` (fewer lookups, random bank conflicts).
__device__ __forceinline__ uint32_t shift8(const uint32_t* T, uint32_t off, uint32_t c) {
  const uint32_t a = xor3(lds_ld(T, off + ((c << 2) & 0x3FCu)), lds_ld(T, off + 1024u + ((c >> 6) & 0x3FCu)),
                          lds_ld(T, off + 2048u + ((c >> 14) & 0x3FCu)));
  return a ^ lds_ld(T, off + 3072u + ((c >> 22) & 0x3FCu));
}
template <bool S8>
__device__ __forceinline__ uint32_t shift_lds(const uint32_t* T, uint32_t off, uint32_t c) {
  return S8 ? shift8(T, off, c) : shift5(T, off, c);
}
// shift(c, 63*RUN) (or 64*RUN in PAR form): the jump between two stripes of a lane.
template <int LY>
__device__ __forceinline__ uint32_t shift_stripe(const uint32_t* T, uint32_t c) {
  return shift_lds<LdsLayout<LY>::stripe_s8>(T, LdsLayout<LY>::stripe_off, c);
}

__device__ __forceinline__ uint32_t steps16(const uint32_t* T, const LaneBase& lb, uint32_t c, const uint4& v) {
  uint32_t x = c ^ v.x;
  x = step4x(T, lb, x, v.y);
  x = step4x(T, lb, x, v.z);
  x = step4x(T, lb, x, v.w);
  return step4x(T, lb, x, 0u);
}

// The 32 copies of the four slice tables (conflict-free lookups).  Dword index
// i = region<<14 | b<<6 | half<<5 | j (see the address layout above): copies
// j..j+3 of one entry are adjacent, so each thread writes four copies with one
// 16-byte LDS store (8 per thread for 128 KiB).
__device__ __forceinline__ void load_slice_tables(uint32_t* T, const Tables* __restrict__ tg) {
  for (uint32_t q = threadIdx.x; q < 4u * 256u * 8u; q += blockDim.x) {
    const uint32_t region = q >> 12, b = (q >> 4) & 255u, half = (q >> 3) & 1u;
    const uint32_t t = 3u - (region * 2u + half);  // T3, T2, T1, T0
    const uint32_t v = tg->slice[t][b];
    *reinterpret_cast<uint4*>(T + 4u * q) = make_uint4(v, v, v, v);
  }
}

// Layout 2: 16 copies, dword index b<<6 | tsel<<4 | j; four copies per 16-byte store.
__device__ __forceinline__ void load_slice_tables16(uint32_t* T, const Tables* __restrict__ tg) {
  for (uint32_t q = threadIdx.x; q < 4u * 256u * 4u; q += blockDim.x) {
    const uint32_t b = q >> 4, tsel = (q >> 2) & 3u;
    const uint32_t v = tg->slice[3u - tsel][b];  // T3, T2, T1, T0
    *reinterpret_cast<uint4*>(T + 4u * q) = make_uint4(v, v, v, v);
  }
}

// Stage the tables: the copies of the slice tables (conflict-free lookups, or
// 4-way with layout 2) and the stripe- and level-shift tables for RUN.  Every
// thread of the workgroup takes part.
template <int RUN, bool PAR, int LY>
__device__ __forceinline__ void load_tables(uint32_t* T, const Tables* __restrict__ tg) {
  using LL = LdsLayout<LY>;
  if constexpr (LL::rep16) load_slice_tables16(T, tg);
  else load_slice_tables(T, tg);
  const uint32_t ri = run_index(RUN);
  const uint32_t sent = LL::stripe_s8 ? 1024u : kShiftChunks * 32u;
  const uint32_t* st = LL::stripe_s8 ? (PAR ? tg->stripe64_8[ri][0] : tg->stripe8[ri][0])
                                     : (PAR ? tg->stripe64[ri][0] : tg->stripe[ri][0]);
  for (uint32_t i = threadIdx.x; i < sent; i += blockDim.x) T[LL::stripe_off / 4 + i] = st[i];
  const uint32_t lent = LL::level_s8 ? 1024u : kShiftChunks * 32u;
  const uint32_t* lv = LL::level_s8 ? tg->level8[ri][0][0] : tg->level[ri][0][0];
  for (uint32_t i = threadIdx.x; i < 6u * lent; i += blockDim.x) {
    const uint32_t j = i / lent, r = i % lent;
    T[(LL::level_off + LL::stride * j) / 4 + r] = lv[i];
  }
  __syncthreads();
}

// CRC of `len` bytes at p with initial register `seed`, computed by the whole
// wave; the result is returned in every lane.
// ---------------------------------------------------------------------------
// One file as the wave sees it.  All of this is wave-uniform (scalar) state.
// ---------------------------------------------------------------------------
template <int RUN>
struct FileGeo {
  uintptr_t start, end, A, B16, E, sb0;
  uint32_t len, s, nstripes, seed;
  uint32_t nvalid;  // lanes whose run in the last stripe holds payload (the rest lie past B16)
};

template <int RUN>
__device__ __forceinline__ FileGeo<RUN> make_geo(const uint8_t* p, uint32_t len, uint32_t seed, uint32_t aoff = 0u) {
  constexpr uint32_t kStripe = 64u * RUN;
  FileGeo<RUN> g;
  g.start = reinterpret_cast<uintptr_t>(p);
  g.len = len;
  g.seed = seed;
  g.end = g.start + len;
  g.A = g.start & ~uintptr_t(3);
  g.B16 = g.end & ~uintptr_t(15);
  g.s = uint32_t(g.start - g.A);
  // Stripe grid anchor E: B16 rounded up to a 128-byte line (RUN = 16), so every
  // stripe is exactly eight whole lines -- with non-temporal loads a line split
  // between two stripes was fetched twice (+2 % HBM traffic).  Runs in
  // [B16, E) lie in the same line as payload bytes (safe to read) and are
  // excluded from their lanes' chains (`nvalid`).  `aoff` (16-byte multiple,
  // record kernel only): anchor the grid at 128k + aoff instead, so that the
  // copy-through writes whole destination lines; the caller checks that the
  // last stripe's up to 112 bytes past B16 stay inside the source.
  g.E = RUN == 16 ? (((g.B16 - aoff + 127) & ~uintptr_t(127)) + aoff) : g.B16;
  g.nvalid = 64u - uint32_t(g.E - g.B16) / RUN;
  const uint32_t body = len >= kMinParallelLen ? uint32_t(g.E - g.A) : 0u;
  g.nstripes = (body + kStripe - 1) / kStripe;
  g.sb0 = g.E - uintptr_t(g.nstripes) * kStripe;
  return g;
}

// Per-lane registers loaded ahead of a file's compute: the lane's run of
// stripe 0 (zero in front of the payload, masked and seed-injected at A) and
// the <= 15 tail bytes after the last 16-byte boundary (same in every lane).
template <int RUN>
struct Head {
  uint32_t w[RUN / 4];
  uint32_t tw[3];
  uint32_t tb[3];
};

template <int RUN>
__device__ __forceinline__ Head<RUN> load_head(const FileGeo<RUN>& g, int lane) {
  Head<RUN> h;
  const uintptr_t lo = g.sb0 + uintptr_t(lane) * RUN;
#pragma unroll
  for (int i = 0; i < RUN / 4; ++i) {
    const uintptr_t q = lo + 4u * i;
    h.w[i] = (g.nstripes && q >= g.A && q < g.B16) ? ld32(q) : 0u;  // zero chain stays zero
  }
  const uintptr_t tq = g.nstripes ? g.B16 : g.start;  // tiny files: everything is "tail"
#pragma unroll
  for (int i = 0; i < 3; ++i) h.tw[i] = (g.nstripes && g.B16 + 4u * i + 4u <= g.end) ? ld32(g.B16 + 4u * i) : 0u;
  const uintptr_t B = g.nstripes ? (g.end & ~uintptr_t(3)) : tq;
#pragma unroll
  for (int i = 0; i < 3; ++i) h.tb[i] = (g.nstripes && B + i < g.end) ? ld8(B + i) : 0u;
  return h;
}

// Stripes 1.. of a file: PF stripes in flight per lane.  Ring slots past the
// file's last stripe load a fixed, always L2-resident 64*RUN-byte region
// (`junk`, the global copy of the slice tables) instead: the steady state stays
// branch-free (so the compiler's vmcnt waits stay counted) without fetching
// anything from HBM twice.  The wave-uniform part of the address is a scalar
// select.
template <int RUN>
__device__ __forceinline__ uintptr_t stripe_base(const FileGeo<RUN>& g, uint32_t st, uintptr_t junk) {
  return (st >= 1u && st < g.nstripes) ? g.sb0 + uintptr_t(st) * (64u * RUN) : junk;
}

template <int RUN, int PF, bool NT>
__device__ __forceinline__ void load_ring(const FileGeo<RUN>& g, int lane, uint4 (&buf)[PF][RUN / 16],
                                          uintptr_t junk) {
#pragma unroll
  for (int f = 0; f < PF; ++f) {
    const uintptr_t sb = stripe_base<RUN>(g, 1u + f, junk) + uintptr_t(lane) * RUN;
#pragma unroll
    for (int v = 0; v < RUN / 16; ++v) buf[f][v] = ld128s<NT>(sb + 16u * v);
  }
}

// LDS-DMA ring (measurement build; TFS_CRC_VARIANT 120-121):
// the PF stripes in flight live in LDS instead of VGPRs.  Each refill is one
// global_load_lds_dwordx4 (lane l's 16 bytes land at the wave's slot base + 16 l,
// exactly the stripe's lane order); a stripe is read back with ds_read_b128 in
// inline asm behind an explicit s_waitcnt vmcnt(N): hipcc does not order its own
// ds_reads after a pending LDS-DMA to the same array (it waits vmcnt(0) or moves
// the read past the next refill), so the waits are counted here.  N counts only
// the younger LDS-DMAs (PF - 1 in the steady state): loads, stores and LDS-DMAs
// retire in issue order (MI355X_MICROARCH.md), so ignoring the younger stores
// only waits longer, never too little.
typedef __attribute__((address_space(3))) void* lds_vp;
typedef const __attribute__((address_space(1))) void* glb_vp;
__device__ __forceinline__ void glds16(uintptr_t gsrc, uint4* lds_slot) {
  __builtin_amdgcn_global_load_lds(reinterpret_cast<glb_vp>(gsrc), (lds_vp)(lds_slot), 16, 0, 0);
}
template <int N>
__device__ __forceinline__ uint4 ring_rd(uint32_t lds_addr) {
  u32x4 v;
  asm volatile("s_waitcnt vmcnt(%1)\n\tds_read_b128 %0, %2\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(v) : "i"(N), "v"(lds_addr) : "memory");
  return make_uint4(v.x, v.y, v.z, v.w);
}
// Slot f of the wave's ring: `base` (generic) / `addr` (LDS byte address) of slot 0,
// slots `stride` uint4 apart.
struct LdsRing {
  uint4* base;
  uint32_t addr;
  uint32_t stride;
};
template <int RUN, int PF>
__device__ __forceinline__ void load_ring_lds(const FileGeo<RUN>& g, int lane, const LdsRing& rg, uintptr_t junk) {
  static_assert(RUN == 16, "one 16-byte run per lane");
#pragma unroll
  for (int f = 0; f < PF; ++f) glds16(stripe_base<RUN>(g, 1u + f, junk) + uintptr_t(lane) * RUN, rg.base + f * rg.stride);
}
template <int PF>
__device__ __forceinline__ uint4 ring_slot(const LdsRing& rg, int lane, int f, int younger) {
  const uint32_t a = rg.addr + uint32_t(f) * rg.stride * 16u + uint32_t(lane) * 16u;
  switch (younger) {  // folded: f and younger are compile-time after unrolling
    case 0: return ring_rd<0>(a);
    case 1: return ring_rd<1>(a);
    case 2: return ring_rd<2>(a);
    case 3: return ring_rd<3>(a);
    case 4: return ring_rd<4>(a);
    case 5: return ring_rd<5>(a);
    case 6: return ring_rd<6>(a);
    case 7: return ring_rd<7>(a);
    case 8: return ring_rd<8>(a);
    case 9: return ring_rd<9>(a);
    case 10: return ring_rd<10>(a);
    case 11: return ring_rd<11>(a);
    case 12: return ring_rd<12>(a);
    case 13: return ring_rd<13>(a);
    default: return ring_rd<14>(a);
  }
}

// Copy-through stores of the fused compaction kernel: the payload bytes a lane
// holds in registers go to the same position of the destination record
// (dst = src + delta, delta a multiple of 4).  Written once, never re-read here.
typedef __attribute__((address_space(1))) uint32_t* gu32wp;
typedef __attribute__((address_space(1))) u32x4* gu128wp;
__device__ __forceinline__ void st32(uintptr_t a, uint32_t v) { *reinterpret_cast<gu32wp>(a) = v; }
// Stores at any byte address (HSA unaligned access mode: one global_store_dword
// / _dwordx4 whatever the alignment), for destinations not congruent to the
// source mod 4.
typedef uint32_t __attribute__((aligned(1))) u32u;
typedef u32x4 __attribute__((aligned(1))) u32x4u;
typedef __attribute__((address_space(1))) u32u* gu32up;
typedef __attribute__((address_space(1))) u32x4u* gu128up;
__device__ __forceinline__ void st32u(uintptr_t a, uint32_t v) { *reinterpret_cast<gu32up>(a) = v; }
// Copy-through store kinds (NTS): 1 non-temporal (product); measurement only:
// 0 plain (TFS_CRC_VARIANT=25: partial lines at record and stripe edges can merge
// in L2 before they are written back), 2 sc1 (variant 36: the line is dropped
// from L2 as the store passes, MI355X_MICROARCH.md store flavours).
template <int NTS>
__device__ __forceinline__ void st128_kind(uintptr_t a, const u32x4& w) {
  if (NTS == 1) {
    __builtin_nontemporal_store(w, reinterpret_cast<gu128wp>(a));
  } else if (NTS == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(a), "v"(w) : "memory");
  } else {
    *reinterpret_cast<gu128wp>(a) = w;
  }
}
template <int NTS = 1>
__device__ __forceinline__ void st128u(uintptr_t a, const uint4& v) {
  const u32x4 w = {v.x, v.y, v.z, v.w};
  if (NTS == 1) __builtin_nontemporal_store(w, reinterpret_cast<gu128up>(a));
  else if (NTS == 2) st128_kind<2>(a, w);  // the hardware takes any byte address (unaligned access mode)
  else *reinterpret_cast<gu128up>(a) = w;
}

template <int NTS = 1>
__device__ __forceinline__ void st128_nt(uintptr_t a, const uint4& v) {
  u32x4 w = {v.x, v.y, v.z, v.w};
  if ((a & 15u) == 0) {
    st128_kind<NTS>(a, w);
  } else {  // 4-aligned: four dword stores
    st32(a, v.x); st32(a + 4, v.y); st32(a + 8, v.z); st32(a + 12, v.w);
  }
}

// Copy-through of one stripe (RUN = 16) to dst = src + delta, delta = 16m + 4k
// with k in 1..3: the aligned 16-byte destination chunk under lane l holds the
// last k dwords of lane l-1 and the first 4-k of lane l, so every lane stores
// one whole dwordx4 instead of four dword stores (over PCIe -- zero-copy host
// compaction -- four partial writes per 16 bytes cost 6 %).  Lane 0 takes the
// previous stripe's lane-63 dwords (`cy/cz/cw`); right after stripe 0 (stored
// dword by dword) it stores only its own dwords.  `flush`: this lane ends the
// record's last stripe, so its own last k dwords go out as dword stores.
struct ShiftCarry {
  uint32_t y, z, w;
  bool valid;
  uint32_t x;  // byte shifts only (store_bshift)
};
// DPP: lane l-1's dwords by a wave_shr:1 DPP move (VALU) instead of ds_bpermute
// (__shfl_up), which goes through the LDS crossbar beside the table lookups.
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v) {
  return __builtin_amdgcn_update_dpp(0u, v, 0x138 /* wave_shr:1 */, 0xf, 0xf, false);
}
template <bool DPP = true, int NTS = 1>
__device__ __forceinline__ void store_shifted(uintptr_t chunk, const uint4& v, uint32_t k, int lane, ShiftCarry& cr,
                                              bool store, bool flush) {
  uint32_t p1, p2, p3;
  if (DPP) {
    p1 = from_prev_lane(v.w), p2 = from_prev_lane(v.z), p3 = from_prev_lane(v.y);
  } else {
    p1 = __shfl_up(v.w, 1, kWave), p2 = __shfl_up(v.z, 1, kWave), p3 = __shfl_up(v.y, 1, kWave);
  }
  if (lane == 0) {
    p1 = cr.w;
    p2 = cr.z;
    p3 = cr.y;
  }
  if (store) {
    if (lane == 0 && !cr.valid) {
      if (k == 1) {
        st32(chunk + 4, v.x); st32(chunk + 8, v.y); st32(chunk + 12, v.z);
      } else if (k == 2) {
        st32(chunk + 8, v.x); st32(chunk + 12, v.y);
      } else {
        st32(chunk + 12, v.x);
      }
    } else {
      const uint4 o = k == 1 ? make_uint4(p1, v.x, v.y, v.z)
                             : (k == 2 ? make_uint4(p2, p1, v.x, v.y) : make_uint4(p3, p2, p1, v.x));
      st128_nt<NTS>(chunk, o);
    }
    if (flush) {
      if (k == 1) {
        st32(chunk + 16, v.w);
      } else if (k == 2) {
        st32(chunk + 16, v.z); st32(chunk + 20, v.w);
      } else {
        st32(chunk + 16, v.y); st32(chunk + 20, v.z); st32(chunk + 24, v.w);
      }
    }
  }
  cr.y = __builtin_amdgcn_readlane(v.y, kWave - 1);
  cr.z = __builtin_amdgcn_readlane(v.z, kWave - 1);
  cr.w = __builtin_amdgcn_readlane(v.w, kWave - 1);
  cr.valid = true;
}

// Copy-through of one stripe to dst = src + delta with a byte shift
// (delta = 16m + 4K + b, b in 1..3): the aligned 16-byte destination chunk under
// lane l (`chunk` = q + delta - 4K - b, the stripe grid anchored so that lane 0's
// chunk starts a 128-byte line) holds the last 4K + b bytes of lane l-1's run and
// the first 16 - 4K - b of lane l's: with S = lane l-1's four dwords followed by
// lane l's, dword i of the chunk is alignbyte(S[4-K+i], S[3-K+i], 4-b).  Lane 0
// takes the previous stripe's lane-63 dwords; right after stripe 0 (stored dword
// by dword) it stores only its own 16 bytes, unaligned (`own`), and so does the
// record's last valid lane (`flush`) for the bytes past its chunk.  The byte
// ranges those extra stores share with a neighbouring chunk hold the same values.
template <int K, int NTS>
__device__ __forceinline__ void store_bshift(uintptr_t chunk, uintptr_t own, const uint4& v, uint32_t sh, int lane,
                                             ShiftCarry& cr, bool store, bool flush) {
  uint32_t p0 = 0u, p1 = 0u, p2 = 0u, p3 = from_prev_lane(v.w);
  if (K >= 1) p2 = from_prev_lane(v.z);
  if (K >= 2) p1 = from_prev_lane(v.y);
  if (K >= 3) p0 = from_prev_lane(v.x);
  if (lane == 0) {
    p0 = cr.x;
    p1 = cr.y;
    p2 = cr.z;
    p3 = cr.w;
  }
  if (store) {
    if (lane == 0 && !cr.valid) {
      st128u<NTS>(own, v);
    } else {
      const uint32_t S[8] = {p0, p1, p2, p3, v.x, v.y, v.z, v.w};
      const uint4 o = make_uint4(__builtin_amdgcn_alignbyte(S[4 - K], S[3 - K], sh),
                                 __builtin_amdgcn_alignbyte(S[5 - K], S[4 - K], sh),
                                 __builtin_amdgcn_alignbyte(S[6 - K], S[5 - K], sh),
                                 __builtin_amdgcn_alignbyte(S[7 - K], S[6 - K], sh));
      st128_nt<NTS>(chunk, o);
    }
    if (flush) st128u<NTS>(own, v);
  }
  cr.x = __builtin_amdgcn_readlane(v.x, kWave - 1);
  cr.y = __builtin_amdgcn_readlane(v.y, kWave - 1);
  cr.z = __builtin_amdgcn_readlane(v.z, kWave - 1);
  cr.w = __builtin_amdgcn_readlane(v.w, kWave - 1);
  cr.valid = true;
}

// The lane's chain over stripes 0..nstripes-1 (before the final combine).
// COPY: also store every payload byte of [start, B16) to dst = src + delta.
// NTS: non-temporal copy-through stores (product).  NOCRC (measurement only,
// TFS_CRC_VARIANT=26: wrong CRCs): skip the payload steps, so the record kernel
// runs its own load/store schedule without the table lookups.
template <int RUN, int PF, bool NT, int LY, bool COPY = false, bool DPPSH = false, int NTS = 1, bool NOCRC = false,
          bool LR = false>
__device__ __forceinline__ uint32_t lane_chain(const uint32_t* T, const LaneBase& lb, const FileGeo<RUN>& g,
                                               const Head<RUN>& h, uint4 (&buf)[PF][RUN / 16], int lane,
                                               uintptr_t junk, intptr_t delta = 0, bool copy_on = false,
                                               const LdsRing* ring = nullptr) {
  static_assert(!LR || (RUN == 16 && PF <= 8), "LDS ring: one run per lane, counted waits up to 14");
  constexpr uint32_t kStripe = 64u * RUN;
  constexpr int kVec = RUN / 16;
  // Stripe 0: mask the bytes before `start` in the dword at A and inject the
  // seed into the first four message bytes (that is Func::crc's initial
  // register).  When A is the last dword of stripe 0, the high seed bytes
  // belong to lane 0's first dword of stripe 1: `inj` carries them there.
  const uint32_t headmask = 0xffffffffu << (8 * g.s);
  const uint32_t seed_lo = g.seed << (8 * g.s);
  const uint32_t seed_hi = g.s ? (g.seed >> (32 - 8 * g.s)) : 0u;
  uint32_t inj = (lane == 0 && g.A + 4 == g.sb0 + kStripe) ? seed_hi : 0u;
  uint32_t c = 0;
  {
    const uintptr_t lo = g.sb0 + uintptr_t(lane) * RUN;
#pragma unroll
    for (int i = 0; i < RUN / 4; ++i) {
      const uintptr_t q = lo + 4u * i;
      uint32_t w = h.w[i];
      if (COPY && copy_on) {
        if (q >= g.start && q < g.B16) {
          st32u(q + delta, w);
        } else if (q == g.A && g.s) {  // the dword holding `start`: its payload bytes only
          for (uint32_t k = g.s; k < 4u; ++k) *reinterpret_cast<uint8_t*>(q + k + delta) = uint8_t(w >> (8 * k));
        }
      }
      w = q == g.A ? ((w & headmask) ^ seed_lo) : w;
      w = q == g.A + 4 ? (w ^ seed_hi) : w;
      c = step4(T, lb, c, w);
    }
  }
  if (g.nstripes > 1) {
    // Full groups of PF stripes: straight-line, every buffer consumed then
    // refilled (past the last stripe: the L2-resident `junk` region).
    const uint32_t last = g.nstripes - 1;
    const bool lane_in_last = uint32_t(lane) < g.nvalid;
    // Copy-through of stripe st (COPY only): whole dwordx4 stores at any
    // destination shift (store_shifted, store_bshift).
    const uint32_t kshift = uint32_t(delta >> 2) & 3u;
    const bool bshift = (delta & 3) != 0;  // wave-uniform
    ShiftCarry carry{0u, 0u, 0u, false, 0u};
    static_assert(!COPY || RUN == 16, "copy-through assumes one 16-byte run per lane");
    auto copy_stripe = [&](uint32_t st, const uint4& v) {
      const bool valid = !(st == last && !lane_in_last);
      const uintptr_t q = g.sb0 + uintptr_t(st) * kStripe + uintptr_t(lane) * RUN;
      if (bshift) {  // byte shift: line-aligned chunks built by alignbyte
        const uintptr_t chunk = q + uintptr_t(delta & ~intptr_t(15));
        const uint32_t sh = 4u - uint32_t(delta & 3);
        const bool fl = st == last && uint32_t(lane) + 1u == g.nvalid;
        if (kshift == 0u) store_bshift<0, NTS>(chunk, q + delta, v, sh, lane, carry, valid, fl);
        else if (kshift == 1u) store_bshift<1, NTS>(chunk, q + delta, v, sh, lane, carry, valid, fl);
        else if (kshift == 2u) store_bshift<2, NTS>(chunk, q + delta, v, sh, lane, carry, valid, fl);
        else store_bshift<3, NTS>(chunk, q + delta, v, sh, lane, carry, valid, fl);
      } else if (kshift == 0u) {
        if (valid) st128_nt<NTS>(q + delta, v);
      } else {
        store_shifted<DPPSH, NTS>(q + uintptr_t(delta) - 4u * kshift, v, kshift, lane, carry, valid,
                                  st == last && uint32_t(lane) + 1u == g.nvalid);
      }
    };
    uint32_t r = 1;
    // One full group of PF stripes.  LR (YC: 0 the first group, 1 later ones): slot
    // f's refill has at least this many younger vector-memory ops when slot f is
    // read -- first group: the PF - 1 other first loads and refills (PF - 1) and
    // the f stripes' stores before it; later groups: the PF - 1 younger refills
    // and the PF - 1 stripes' copy-through stores between them (every stripe of a
    // full group issues at least one store instruction): 2 (PF - 1).
    auto group = [&](auto yc) {  // (LR only)
#pragma unroll
      for (int f = 0; f < PF; ++f) {
        buf[f][0] = ring_slot<PF>(*ring, lane, f, decltype(yc)::value == 0 ? PF - 1 + f : 2 * (PF - 1));
        const uint32_t c_old = c;
        c = shift_stripe<LY>(T, c);
        if (f == 0) {
          c ^= inj;  // XOR into the stripe's first dword == XOR into the register before its step
          inj = 0;
        }
#pragma unroll
        for (int v = 0; v < kVec; ++v) c = NOCRC ? c ^ buf[f][v].x : steps16(T, lb, c, buf[f][v]);
        c = (r + f == last && !lane_in_last) ? c_old : c;  // run past B16: not part of the chain
        if (COPY && copy_on) copy_stripe(r + f, buf[f][0]);
        const uintptr_t sb = stripe_base<RUN>(g, r + uint32_t(f) + uint32_t(PF), junk) + uintptr_t(lane) * RUN;
        glds16(sb, ring->base + f * ring->stride);
      }
    };
    if constexpr (LR) {
      if (r + PF <= g.nstripes) {
        group(std::integral_constant<int, 0>{});
        r += PF;
      }
      for (; r + PF <= g.nstripes; r += PF) group(std::integral_constant<int, 1>{});
    } else {
      for (; r + PF <= g.nstripes; r += PF) {
#pragma unroll
        for (int f = 0; f < PF; ++f) {
          const uint32_t c_old = c;
          c = shift_stripe<LY>(T, c);
          if (f == 0) {
            c ^= inj;  // XOR into the stripe's first dword == XOR into the register before its step
            inj = 0;
          }
#pragma unroll
          for (int v = 0; v < kVec; ++v) c = NOCRC ? c ^ buf[f][v].x : steps16(T, lb, c, buf[f][v]);
          c = (r + f == last && !lane_in_last) ? c_old : c;  // run past B16: not part of the chain
          if (COPY && copy_on) copy_stripe(r + f, buf[f][0]);
          const uintptr_t sb = stripe_base<RUN>(g, r + uint32_t(f) + uint32_t(PF), junk) + uintptr_t(lane) * RUN;
#pragma unroll
          for (int v = 0; v < kVec; ++v) buf[f][v] = ld128s<NT>(sb + 16u * v);
        }
      }
    }
    // Remaining 0..PF-1 stripes are already in buf[0..] (LR: in ring slots 0.., the
    // refills of slots f+1..PF-1 younger than slot f's).
#pragma unroll
    for (int f = 0; f < PF - 1; ++f) {
      if (r + f < g.nstripes) {
        // at least PF - 1 younger: the refills of slots f+1.. and the stores of the
        // remaining stripes before it (or, with no full group, the first loads)
        if constexpr (LR) buf[f][0] = ring_slot<PF>(*ring, lane, f, PF - 1);
        const uint32_t c_old = c;
        c = shift_stripe<LY>(T, c);
        if (f == 0) c ^= inj;
#pragma unroll
        for (int v = 0; v < kVec; ++v) c = NOCRC ? c ^ buf[f][v].x : steps16(T, lb, c, buf[f][v]);
        c = (r + f == last && !lane_in_last) ? c_old : c;
        if (COPY && copy_on) copy_stripe(r + f, buf[f][0]);
      }
    }
  }
  return c;
}

// Combine the lane chains into the file CRC and fold in the tail.
template <int RUN, int LY>
__device__ __forceinline__ uint32_t finish_file(const uint32_t* T, const LaneBase& lb, const FileGeo<RUN>& g,
                                                const Head<RUN>& h, uint32_t c, int lane) {
  if (g.nstripes == 0) {  // tiny (< kMinParallelLen): the byte loop of func.cpp:429-433 in every lane
    uint32_t t = g.seed;
    for (uint32_t i = 0; i < g.len; ++i) t = step1(T, lb, t, ld8(g.start + i));
    return t;
  }
#ifdef TFS_DIAG_SKIP_COMBINE
  return c;  // diagnostic build only (tools/combine_probe.sh): wrong CRCs, times the kernel without the combine
#endif
  // Move each lane's chain to its place: the distance from the end of its last
  // run to B16, in runs: (63-lane) - (E-B16)/RUN, plus a whole stripe for lanes
  // whose run in the last stripe lies past B16 (their chain ended a stripe earlier).
  const uint32_t e_runs = 64u - g.nvalid;
  const uint32_t k = uint32_t(kWave - 1 - lane) - e_runs + (uint32_t(lane) < g.nvalid ? 0u : 64u);
#pragma unroll
  for (int j = 0; j < kLevels; ++j) {
    const uint32_t sh = shift_lds<LdsLayout<LY>::level_s8>(T, LdsLayout<LY>::level_off + LdsLayout<LY>::stride * j, c);
    c = ((k >> j) & 1u) ? sh : c;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c ^= __shfl_xor(c, m, kWave);
  // Tail after the last 16-byte boundary (same in every lane).
  const uint32_t ntw = uint32_t((g.end & ~uintptr_t(3)) - g.B16) / 4u;
  const uint32_t ntb = uint32_t(g.end & 3u);
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (uint32_t(i) < ntw) c = step4(T, lb, c, h.tw[i]);
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (uint32_t(i) < ntb) c = step1(T, lb, c, h.tb[i]);
  return c;
}

// Single-file form (used by the block-verify kernel).
template <int RUN, int PF, bool NT, int LY>
__device__ __forceinline__ uint32_t wave_crc(const uint32_t* T, const uint8_t* p, uint32_t len, uint32_t seed,
                                             int lane, uintptr_t junk) {
  const LaneBase lb = lane_base_of(lane);
  const FileGeo<RUN> g = make_geo<RUN>(p, len, seed);
  const Head<RUN> h = load_head<RUN>(g, lane);
  uint4 buf[PF][RUN / 16];
  load_ring<RUN, PF, NT>(g, lane, buf, junk);
  const uint32_t c = g.nstripes ? lane_chain<RUN, PF, NT, LY>(T, lb, g, h, buf, lane, junk) : 0u;
  return finish_file<RUN, LY>(T, lb, g, h, c, lane);
}

constexpr int kRun = 16;  // product configuration (see DESIGN.md §4 for the sweep)
constexpr int kPF = 5;
constexpr bool kNT = true;
constexpr bool kPAR = false;
constexpr int kLY = 1;  // LDS table layout (LdsLayout): 32 slice-table copies, byte shift tables
constexpr bool kIL = true;  // interleaved ticket groups (Tickets<IL>): +3 % Zipf, box-dependent +-3 % verify
// Chunked tickets (FileCursor): 4 consecutive files per ticket, the last n/8 one
// by one -- verify -2.8 to -3.8 %, Zipf -2.5 to -3.9 %, device block verify
// -3.6 % against one file per ticket, in-process A/B on three boxes.
constexpr int kCF = 4;
constexpr int kTS = 3;

// Work distribution.  Static: wave w takes files w, w+W, w+2W, ... (W = all
// waves) -- ideal when every file has the same size.  Dynamic: eight ticket
// counters (one per group of workgroups, blockIdx % 8, i.e. one per XCD under
// round-robin placement) each own 1/8 of the files; a wave takes the
// next ticket of its group and steals from the other groups once its own is
// exhausted, so waves finish together for any size distribution (the kernel
// ends with its slowest wave).  The ticket for the next-but-one file is taken
// one file ahead, so the atomic's latency hides under a file's work.
// IL (product default, kIL): group g owns files g, g+8, g+16, ..., so the eight
// XCDs read one moving address window together; IL = false gives group g the
// contiguous eighth [n*g/8, n*(g+1)/8) (eight windows 1/8 of the batch apart;
// 2.5-3.7 % slower on Zipf, +-3 % box-dependent on uniform files; TFS_CRC_VARIANT=14).
template <bool IL = false>
struct Tickets {
  uint32_t* ctr;  // 8 zeroed counters for this launch, kSchedStride u32 apart (one per 256-byte line)
  uint32_t n, group;
  // Short launches (fewer than kDynMinPerWave files per wave) take files
  // round-robin instead: atomics to one line serialise (~88 per us), which a
  // launch of a few files per wave does not amortise (a 31-block window: ~40 us).
  bool dyn = true;
  uint32_t snext = 0, sstride = 0;
  __device__ __forceinline__ void init_static(uint32_t waves_total, uint32_t global_wave) {
    dyn = n >= kDynMinPerWave * waves_total;
    snext = global_wave;
    sstride = waves_total;
  }
  __device__ __forceinline__ uint32_t gbegin(uint32_t g) const { return uint32_t((uint64_t(n) * g) >> 3); }
  __device__ __forceinline__ uint32_t gcount(uint32_t g) const {
    return IL ? (n > g ? (n - g + 7u) >> 3 : 0u) : gbegin(g + 1) - gbegin(g);
  }
  __device__ __forceinline__ uint32_t file_of(uint32_t g, uint32_t j) const { return IL ? j * 8u + g : gbegin(g) + j; }
  // Issue the atomic of the home group in lane 0; the result stays in lane 0's register.
  __device__ __forceinline__ uint32_t issue(int lane) {
    if (!dyn) {
      const uint32_t j = snext;
      snext += sstride;
      return j;
    }
    uint32_t j = 0;
    if (lane == 0) j = atomicAdd(&ctr[group * kSchedStride], 1u);
    return j;
  }
  // Turn an issued ticket into a file index (n = no work left).  (Skipping an
  // exhausted group after a plain load of its counter, instead of an atomic,
  // measured 4-7 % slower on the headline: DESIGN.md §4.)
  __device__ __forceinline__ uint32_t resolve(uint32_t jv, int lane) {
    // readlane keeps the file index wave-uniform (SGPR) in both modes, so the
    // descriptor loads stay scalar loads and the geometry stays in SGPRs.
    uint32_t j = __builtin_amdgcn_readlane(jv, 0);
    if (!dyn) return j < n ? j : n;
    for (uint32_t tries = 0;; ++tries) {
      if (j < gcount(group)) return file_of(group, j);
      if (tries == 7) return n;
      group = (group + 1) & 7u;  // steal
      uint32_t k = 0;
      if (lane == 0) k = atomicAdd(&ctr[group * kSchedStride], 1u);
      j = __builtin_amdgcn_readlane(k, 0);
    }
  }
};

// A wave's walk over the files of a launch by tickets of CF consecutive files
// (a wave that stays in one address range for several files reads
// faster; all waves still take their chunks from one moving window).  Tickets
// [0, nA) are chunks of CF files from file 0 on; with TS > 0 the last n >> TS
// files come one per ticket (tickets [nA, nt)), so a chunk of large files
// cannot become the launch's tail.  The ticket of the wave's next chunk is in
// flight while it works through this one; every issued ticket is resolved
// before take() returns n (launch_exit relies on that).  A launch too short
// for dynamic tickets over chunks (fewer than kDynMinPerWave chunks per wave:
// a block of 1,024 files, a small batch) takes single files as before, so its
// files stay spread over all waves.
// HS (measurement, compaction): a long launch hands its first n - (n >> HS) files
// out statically (wave w takes w, w+W, ...: one contiguous window, 16 consecutive
// files per workgroup) and only the rest by single-file tickets, which even out the
// waves' ends.
template <bool IL, int CF, int TS, int HS = 0>
struct FileCursor {
  Tickets<IL> tk;
  uint32_t n = 0, cf = 1, nA = 0, nt = 0, jv = 0, next = 0, end = 0;
  uint32_t hbase = 0, hnext = 0, hstride = 0;  // HS: the static phase covers files [0, hbase)
  bool done = false;
  __device__ __forceinline__ void init(uint32_t* sched, uint32_t n_, uint32_t group, uint32_t waves_total,
                                       uint32_t global_wave) {
    n = n_;
    cf = uint32_t(CF);
    nA = CF > 1 ? (TS > 0 ? (n - (n >> TS)) / uint32_t(CF) : (n + uint32_t(CF) - 1u) / uint32_t(CF)) : n;
    nt = CF > 1 && TS > 0 ? nA + (n - nA * uint32_t(CF)) : nA;
    if (CF > 1 && uint64_t(nt) < uint64_t(kDynMinPerWave) * waves_total) {
      cf = 1u;
      nA = nt = n;
    }
    if (HS > 0 && uint64_t(n) >= uint64_t(kDynMinPerWave) * waves_total) {
      // static chunks [0, hbase) of CF files, the rest by chunk tickets (no TS tail)
      const uint32_t nc = (n + uint32_t(CF) - 1u) / uint32_t(CF);
      hbase = (nc - (nc >> HS)) / waves_total * waves_total;
      hnext = global_wave;
      hstride = waves_total;
      cf = uint32_t(CF);
      nA = nt = nc - hbase;
    }
    tk.ctr = sched;
    tk.n = nt;
    tk.group = group;
    tk.init_static(waves_total, global_wave);
    if (hbase) tk.dyn = true;  // the tail goes by tickets however short it is
  }
  __device__ __forceinline__ void start(int lane) { jv = tk.issue(lane); }
  __device__ __forceinline__ uint32_t take(int lane) {  // next file of this wave, n = none left
    if (next < end) return next++;
    if (HS > 0 && hnext < hbase) {
      next = hnext * cf;
      end = min(next + cf, n);
      hnext += hstride;
      return next++;
    }
    if (done) return n;
    const uint32_t c = tk.resolve(jv, lane);
    if (c >= nt) {
      done = true;
      return n;
    }
    if (c < nA) {
      next = (hbase + c) * cf;
      end = min(next + cf, n);
    } else {
      next = nA * cf + (c - nA);
      end = next + 1u;
    }
    jv = tk.issue(lane);
    return next++;
  }
};

// End of a launch (every wave, or every workgroup, calls this once, after its
// last ticket atomic has returned): count it on the slot's finished line; the
// last one zeroes the slot for the next launch on the same stream and, for a
// zero-copy host batch, stores `seq` into the page-locked completion word the
// host spins on.  The system-scope fences make each unit's verdicts in host
// memory visible before it is counted, and all of them before the flag.
__device__ __forceinline__ void launch_exit(uint32_t* sched, uint32_t units, uint32_t* done_flag, uint32_t seq) {
  if (done_flag) __threadfence_system();
  if (!sched) return;
  const uint32_t old = atomicAdd(&sched[kSchedDone], 1u);
  if (old + 1u == units) {
#pragma unroll
    for (uint32_t gi = 0; gi < 8u; ++gi) atomicExch(&sched[gi * kSchedStride], 0u);
    atomicExch(&sched[kSchedDone], 0u);
    if (done_flag) {
      __threadfence_system();
      __hip_atomic_store(done_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// MODE 0: compute (aux = seed) -> out_crc.  MODE 1: verify (aux = expected, seed
// `vseed`: 0 for files, TFS_PACKET_FLAG_V1 for packet bodies).
// Files are software-pipelined per wave: the next file's stripe-0/tail words
// and its first PF stripes are in flight while this file's lane chains are
// combined, so HBM never waits on a file boundary.  Work goes by interleaved
// dynamic tickets (Tickets, FileCursor): a ticket hands its wave CF consecutive
// files (the product: kCF, the last n >> kTS files one by one, DESIGN §3.1;
// measurement variant 50: one file per ticket).  With a split plan (SplitArgs)
// the launch's units are its address-ordered SplitUnit list instead of desc.
template <int MODE, int CF = kCF, int TS = kTS>
__global__ void __launch_bounds__(kBlock) crc_files_kernel(const uint8_t* __restrict__ base,
                                                           const Desc* __restrict__ desc, uint32_t n,
                                                           const Tables* __restrict__ tg, uint32_t* out_crc,
                                                           uint8_t* out_ok, uint32_t* n_bad, uint32_t* sched,
                                                           uint32_t vseed, uint32_t* done_flag, uint32_t seq,
                                                           SplitArgs sa) {
  constexpr int RUN = kRun, PF = kPF;
  __shared__ uint32_t lds_tables[LdsLayout<kLY>::bytes / 4];
  load_tables<RUN, false, kLY>(lds_tables, tg);
  // Work units: the launch's files, or -- when the plan split some -- its unit
  // list (whole files, heads and segments in address order).
  const uint32_t nfiles = n;
  const SplitUnit* aou = nullptr;  // null: nothing split, the units are desc
  uint32_t* ucrc = nullptr;
  if (sa.plan) {
    const uint32_t* hdr = reinterpret_cast<const uint32_t*>(sa.plan);
    if (hdr[1] == 0u) {
      n = hdr[0];
      aou = reinterpret_cast<const SplitUnit*>(sa.plan + ao_off_units(nfiles, sa.cap));
      ucrc = reinterpret_cast<uint32_t*>(sa.plan + ao_off_ucrc(nfiles));
    }
  }
  // kind: 0 a whole file, 1 a segment, 2 a split file's ragged head; fi: the file
  // whose output a kind-0 unit writes
  auto unit = [&](uint32_t u, uint32_t& kind, uint32_t& fi) -> Desc {
    fi = u;
    kind = 0u;
    if (!aou) return desc[u];
    const SplitUnit U = aou[u];
    kind = U.kind;
    fi = U.file;
    return Desc{U.offset, U.len, U.aux};
  };
  // segments carry seed 0; a head keeps its file's seed (compute) or vseed (verify)
  auto seed_of = [&](const Desc& d, uint32_t kind) -> uint32_t { return (MODE == 0 || kind == 1u) ? d.aux : vseed; };
  const int lane = threadIdx.x & (kWave - 1);
  const LaneBase lb = lane_base_of(lane);
  const uint32_t wpb = kBlock / kWave;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t stride = gridDim.x * wpb;
  FileCursor<kIL, CF, TS> cur_files;
  Tickets<kIL>& tk = cur_files.tk;
  cur_files.init(sched, n, blockIdx.x & 7u, stride, blockIdx.x * wpb + wave);
  if (CF > 1) cur_files.start(lane);
  auto take = [&]() -> uint32_t { return CF > 1 ? cur_files.take(lane) : tk.resolve(tk.issue(lane), lane); };
  uint32_t bad = 0;
  do {  // `break` = this wave has no (more) files; every wave reaches launch_exit
  uint32_t f = take();
  if (f >= n) break;
  uint32_t fn = take();
  uint32_t kcur = 0, knxt = 0, ocur = 0, onxt = 0;
  Desc cur = unit(f, kcur, ocur);
  FileGeo<RUN> g = make_geo<RUN>(base + cur.offset, cur.len, seed_of(cur, kcur));
  Head<RUN> h = load_head<RUN>(g, lane);
  const uintptr_t junk = reinterpret_cast<uintptr_t>(tg->slice);
  uint4 buf[PF][RUN / 16];
  load_ring<RUN, PF, kNT>(g, lane, buf, junk);
  Desc nxt = fn < n ? unit(fn, knxt, onxt) : Desc{0, 0, 0};
  uint32_t jv = CF == 1 && fn < n ? tk.issue(lane) : 0u;  // ticket of the file after next, in flight
  for (;;) {
    const bool more = fn < n;
    const Desc ncur = nxt;
    const uint32_t kn = knxt, on = onxt;
    const uint32_t c = g.nstripes ? lane_chain<RUN, PF, kNT, kLY>(lds_tables, lb, g, h, buf, lane, junk) : 0u;
    // Start the next file's loads before combining this one.
    FileGeo<RUN> ng = g;
    Head<RUN> nh = h;
    uint32_t fnn = n;
    if (more) {
      ng = make_geo<RUN>(base + ncur.offset, ncur.len, seed_of(ncur, kn));
      nh = load_head<RUN>(ng, lane);
      load_ring<RUN, PF, kNT>(ng, lane, buf, junk);
      fnn = CF > 1 ? cur_files.take(lane) : tk.resolve(jv, lane);
      if (fnn < n) nxt = unit(fnn, knxt, onxt);
      if (CF == 1 && fnn < n) jv = tk.issue(lane);
    }
    const uint32_t crc = finish_file<RUN, kLY>(lds_tables, lb, g, h, c, lane);
    if (lane == 0) {
      if (kcur != 0u) {
        ucrc[f] = crc;  // a head or a segment: the fold joins them
      } else {
        if (out_crc) out_crc[ocur] = crc;
        if (MODE == 1) {
          const bool ok = crc == cur.aux;
          if (out_ok) out_ok[ocur] = ok ? 1 : 0;
          bad += ok ? 0u : 1u;
        }
      }
    }
    if (!more) break;
    f = fn;
    fn = fnn;
    cur = ncur;
    kcur = kn;
    ocur = on;
    g = ng;
    h = nh;
  }
  } while (false);
  if (MODE == 1 && lane == 0 && bad && n_bad) atomicAdd(n_bad, bad);
  if (lane == 0) launch_exit(sched, gridDim.x * wpb, done_flag, seq);
}

// Address-ordered split plan (SplitUnit list, tfs_crc_device.h), step 1 of 3: the
// number of whole segments of each block of kAoBlock files.
__device__ __forceinline__ uint32_t ao_segments(const Desc& d) {
  return d.len > kSplitMin ? (d.len - 1u) / kSegBytes : 0u;
}

__global__ void __launch_bounds__(kAoBlock) split_ao_count_kernel(const Desc* __restrict__ desc, uint32_t n,
                                                                  SplitArgs sa) {
  __shared__ uint32_t wsum[kAoBlock / kWave];
  const uint32_t i = blockIdx.x * kAoBlock + threadIdx.x;
  uint32_t K = i < n ? ao_segments(desc[i]) : 0u;
#pragma unroll
  for (int m = kWave / 2; m >= 1; m >>= 1) K += __shfl_xor(K, m, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) wsum[threadIdx.x / kWave] = K;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < kAoBlock / kWave; ++w) t += wsum[w];
    reinterpret_cast<uint32_t*>(sa.plan + ao_off_blk())[blockIdx.x] = t;
  }
}

// Step 2 (one workgroup): exclusive scan of the block counts in place, and the
// cut: when the segments of all files would pass the plan's room (cap - n ext
// units), only the longest prefix of files whose segments fit is split (ADVICE
// r4: one workgroup of the scan reads the 256 descriptors of the block the cut
// falls in); the files from the cut on stay whole.  Header {units, nosplit,
// ext, cut}: units = n + ext, ext = the segments of the files before `cut`.
__global__ void __launch_bounds__(1024) split_ao_scan_kernel(const Desc* __restrict__ desc, uint32_t n, SplitArgs sa) {
  __shared__ uint32_t part[1024];
  __shared__ uint32_t cut_blk, wsum[kAoBlock / kWave];
  uint32_t* blk = reinterpret_cast<uint32_t*>(sa.plan + ao_off_blk());
  const uint32_t nb = ao_nblk(n);
  const uint32_t per = (nb + 1023u) / 1024u;
  const uint32_t b0 = threadIdx.x * per, b1 = min(b0 + per, nb);
  const uint64_t room = sa.cap > n ? uint64_t(sa.cap - n) : 0u;
  if (threadIdx.x == 0) cut_blk = nb;
  uint32_t t = 0;
  for (uint32_t b = b0; b < b1; ++b) t += blk[b];
  part[threadIdx.x] = t;
  __syncthreads();
  for (uint32_t o = 1; o < 1024u; o <<= 1) {  // inclusive scan of the per-thread sums
    const uint32_t v = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - t;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t v = blk[b];
    blk[b] = run;
    if (uint64_t(run) + v > room) atomicMin(&cut_blk, b);  // the first block that does not fit
    run += v;
  }
  __syncthreads();
  const uint32_t cb = cut_blk;
  uint32_t ext = part[1023], cut = n;
  if (cb < nb) {  // split the files of block cb up to the last one whose segments still fit
    const uint32_t base = blk[cb];
    const uint32_t i = cb * kAoBlock + threadIdx.x;
    const int lane = threadIdx.x & (kWave - 1);
    uint32_t K = threadIdx.x < kAoBlock && i < n ? ao_segments(desc[i]) : 0u;
    uint32_t x = K;  // inclusive scan over the wave, then over the block's waves
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, kWave);
      if (lane >= o) x += y;
    }
    if (threadIdx.x < kAoBlock && lane == kWave - 1) wsum[threadIdx.x / kWave] = x;
    __syncthreads();
    if (threadIdx.x < kAoBlock)
      for (uint32_t w = 0; w < threadIdx.x / kWave; ++w) x += wsum[w];
    const bool fits = threadIdx.x < kAoBlock && i < n && uint64_t(base) + x <= room;
    part[threadIdx.x] = fits ? 1u : 0u;  // the fitting files are a prefix of the block
    __syncthreads();
    if (fits && (threadIdx.x + 1u == kAoBlock || !part[threadIdx.x + 1u])) {  // the last fitting file
      part[1023] = base + x;
      part[1022] = i + 1u;
    }
    if (threadIdx.x == 0 && !fits) {  // not even the block's first file fits
      part[1023] = base;
      part[1022] = i;
    }
    __syncthreads();
    ext = part[1023];
    cut = part[1022];
  }
  if (threadIdx.x == 1023u) {
    uint32_t* hdr = reinterpret_cast<uint32_t*>(sa.plan);
    hdr[0] = n + ext;
    hdr[1] = ext ? 0u : 1u;
    hdr[2] = ext;
    hdr[3] = ext ? cut : 0u;
  }
}

// Step 3: every file's units at its place in address order: file i < cut starts
// at unit i + (segments of the files before it), file i >= cut (whole) at i + ext.
__global__ void __launch_bounds__(kAoBlock) split_ao_write_kernel(const Desc* __restrict__ desc, uint32_t n,
                                                                  SplitArgs sa) {
  __shared__ uint32_t wsum[kAoBlock / kWave];
  const uint32_t* hdr = reinterpret_cast<const uint32_t*>(sa.plan);
  if (hdr[1] != 0u) return;  // nothing split: the kernel reads desc
  const uint32_t ext = hdr[2], cut = hdr[3];
  const uint32_t i = blockIdx.x * kAoBlock + threadIdx.x;
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t w = threadIdx.x / kWave;
  Desc d{0, 0, 0};
  if (i < n) d = desc[i];
  const uint32_t K = i < cut ? ao_segments(d) : 0u;
  uint32_t x = K;  // inclusive scan over the wave
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == kWave - 1) wsum[w] = x;
  __syncthreads();
  if (i >= n) return;
  uint32_t before = reinterpret_cast<const uint32_t*>(sa.plan + ao_off_blk())[blockIdx.x] + (x - K);
  for (uint32_t k = 0; k < w; ++k) before += wsum[k];
  const uint32_t base = i + (i < cut ? before : ext);
  reinterpret_cast<uint32_t*>(sa.plan + ao_off_ubase(n))[i] = base;
  SplitUnit* U = reinterpret_cast<SplitUnit*>(sa.plan + ao_off_units(n, sa.cap));
  const uint32_t head = d.len - K * kSegBytes;
  U[base] = SplitUnit{d.offset, head, d.aux, i, K ? 2u : 0u, 0u};
  for (uint32_t k = 0; k < K; ++k)
    U[base + 1u + k] = SplitUnit{d.offset + head + uint64_t(k) * kSegBytes, kSegBytes, 0u, i, 1u, 0u};
}

// Fold of the address-ordered form: a split file's CRC from its head (unit
// ubase[i]) and segments (the K units after it).
template <int MODE>
__global__ void __launch_bounds__(256) split_ao_fold_kernel(const Desc* __restrict__ desc, uint32_t n,
                                                            const Tables* __restrict__ tg, SplitArgs sa,
                                                            uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad) {
  __shared__ uint32_t T[uint32_t(kShiftChunks) * 32u];
  if (reinterpret_cast<const uint32_t*>(sa.plan)[1] != 0u) return;  // nothing was split
  const uint32_t* ubase = reinterpret_cast<const uint32_t*>(sa.plan + ao_off_ubase(n));
  const uint32_t* ucrc = reinterpret_cast<const uint32_t*>(sa.plan + ao_off_ucrc(n));
  const uint32_t cut = reinterpret_cast<const uint32_t*>(sa.plan)[3];  // files from here on stayed whole
  for (uint32_t k = threadIdx.x; k < uint32_t(kShiftChunks) * 32u; k += blockDim.x) T[k] = (&tg->seg_shift[0][0])[k];
  __syncthreads();
  uint32_t bad = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cut; i += gridDim.x * blockDim.x) {
    const Desc d = desc[i];
    const uint32_t K = ao_segments(d);
    if (K == 0u) continue;
    const uint32_t b = ubase[i];
    uint32_t c = ucrc[b];
    for (uint32_t j = 1; j <= K; ++j) c = shift5(T, 0u, c) ^ ucrc[b + j];
    if (out_crc) out_crc[i] = c;
    if (MODE == 1) {
      const bool ok = c == d.aux;
      if (out_ok) out_ok[i] = ok ? 1 : 0;
      bad += ok ? 0u : 1u;
    }
  }
  if (MODE == 1 && n_bad) {  // one atomic per wave
#pragma unroll
    for (int m = kWave / 2; m >= 1; m >>= 1) bad += __shfl_xor(bad, m, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0 && bad) atomicAdd(n_bad, bad);
  }
}

// ---------------------------------------------------------------------------
// Latency form: one workgroup of 16 waves per file, for batches
// of at most kWgMaxFiles files -- a CloseBatcher batch, one scalar Func::crc
// call, one file read back.  Such calls are bound by latency, not bandwidth:
// with one wave per file a 64 KiB file is a chain of 65 dependent stripes; here
// wave w takes stripes w, w+16, ... (4-5 for 64 KiB), all loads in flight at
// once.  Same stripe geometry and slice tables as crc_files_kernel; lane chains
// jump over the 1023 foreign runs between two of their stripes, are moved to
// the end of the body with shift(c, 16*d), XOR-reduced in the wave and then
// across the 16 waves through LDS.  Wave 0 folds in the tail and writes the
// verdict.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_wg_tables(uint32_t* T, const Tables* __restrict__ tg) {
  load_slice_tables(T, tg);
  constexpr uint32_t kEnt = uint32_t(kShiftChunks) * 32u;
  const uint32_t* jt = tg->wg_jump[0];
  for (uint32_t i = threadIdx.x; i < kEnt; i += blockDim.x) T[kWgJumpOff / 4u + i] = jt[i];
  const uint32_t* lv = tg->wg_level[0][0];
  for (uint32_t i = threadIdx.x; i < uint32_t(kWgLevels) * kEnt; i += blockDim.x)
    T[(kWgLevelOff + 1024u * (i / kEnt)) / 4u + i % kEnt] = lv[i];
}

// shift(c, 16 * d) for d < 2^kWgLevels.
// dmax: a wave-uniform bound on d (the wave's lane 0 distance): the levels above
// its highest bit are skipped -- a body of a few stripes needs 6-8 of the 11
// (round 6: 5 dependent 7-lookup levels less per lone small call).
__device__ __forceinline__ uint32_t wg_shift_runs(const uint32_t* T, uint32_t c, uint32_t d, uint32_t dmax) {
  const uint32_t nlev = 32u - uint32_t(__builtin_clz(dmax | 1u));
#pragma unroll
  for (int j = 0; j < kWgLevels; ++j) {
    if (uint32_t(j) < nlev) {
      const uint32_t sh = shift5(T, kWgLevelOff + 1024u * uint32_t(j), c);
      c = ((d >> j) & 1u) ? sh : c;
    }
  }
  return c;
}

constexpr int kWgPF = 4;  // stripes in flight per wave

// Address of this lane's run of stripe s (junk past the file / for the head stripe).
__device__ __forceinline__ uintptr_t wg_run_addr(const FileGeo<16>& g, uint32_t s, int lane, uintptr_t junk) {
  return (s >= 1u && s < g.nstripes ? g.sb0 + uintptr_t(s) * 1024u : junk) + uintptr_t(lane) * 16u;
}

// Where the latency form reads a file from.  SYS = false (crc_wg_kernel): global
// loads, payload stripes non-temporal, ring refills past the file from `junk`.
// SYS = true (crc_resident_kernel): buffer loads with the system-coherent policy
// (sc0 sc1) off a wave-uniform resource at the file's stripe base -- a payload
// the host rewrote since the workgroup last looked is never served from a stale
// cached line, so no acquire fence per file -- and every load the file does not
// need (ring refills past its end, masked head lanes) is out of the resource's
// range: it returns 0 and moves no bytes.
struct WgSrc {
  __amdgpu_buffer_rsrc_t r;
  uintptr_t base;
  bool bulk;  // stripes by non-temporal loads (the caller fenced): a bulk batch, kResBulk
};
constexpr uint32_t kWgOOR = 0xFFFFFFF0u;           // an offset past every resource's range
constexpr int kSysPolicy = 1 | 16;                 // sc0 | sc1 (system scope)
constexpr int kNtPolicy = 2;                       // nt (streaming)
__device__ __forceinline__ WgSrc wg_src(const FileGeo<16>& g, bool bulk) {
  const uintptr_t base = g.nstripes ? g.sb0 : g.start;
  return WgSrc{__builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, 0x7fffffff, 0x00020000), base,
               bulk};
}
__device__ __forceinline__ int wg_off(const WgSrc& src, bool ok, uintptr_t a) {
  return int(ok ? uint32_t(a - src.base) : kWgOOR);
}
// A payload stripe: system-coherent, or (bulk) non-temporal -- one load either way
// (a wave-uniform branch).
__device__ __forceinline__ uint4 sys128(const WgSrc& src, bool ok, uintptr_t a) {
  const int off = wg_off(src, ok, a);
  u32x4 v;
  if (src.bulk) v = __builtin_amdgcn_raw_buffer_load_b128(src.r, off, 0, kNtPolicy);
  else v = __builtin_amdgcn_raw_buffer_load_b128(src.r, off, 0, kSysPolicy);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t sys32(const WgSrc& src, bool ok, uintptr_t a) {
  return __builtin_amdgcn_raw_buffer_load_b32(src.r, wg_off(src, ok, a), 0, kSysPolicy);
}
__device__ __forceinline__ uint32_t sys8(const WgSrc& src, bool ok, uintptr_t a) {
  return __builtin_amdgcn_raw_buffer_load_b8(src.r, wg_off(src, ok, a), 0, kSysPolicy);
}
// load_head<16> through the resource (same words, same zeros).
__device__ __forceinline__ Head<16> load_head_sys(const FileGeo<16>& g, const WgSrc& src, int lane) {
  Head<16> h;
  const uintptr_t lo = g.sb0 + uintptr_t(lane) * 16u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uintptr_t q = lo + 4u * i;
    h.w[i] = sys32(src, g.nstripes && q >= g.A && q < g.B16, q);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) h.tw[i] = sys32(src, g.nstripes && g.B16 + 4u * i + 4u <= g.end, g.B16 + 4u * i);
  const uintptr_t B = g.nstripes ? (g.end & ~uintptr_t(3)) : g.start;
#pragma unroll
  for (int i = 0; i < 3; ++i) h.tb[i] = sys8(src, g.nstripes && B + i < g.end, B + i);
  return h;
}
// Stripe st's run of this lane (junk / out of range past the file).
template <bool SYS>
__device__ __forceinline__ uint4 wg_run_load(const FileGeo<16>& g, const WgSrc& src, uint32_t st, int lane,
                                             uintptr_t junk) {
  if constexpr (SYS) return sys128(src, st >= 1u && st < g.nstripes, g.sb0 + uintptr_t(st) * 1024u + uintptr_t(lane) * 16u);
  return ld128s<true>(wg_run_addr(g, st, lane, junk));
}

// Issue one file's loads for the latency form: (wave 0) the head stripe and tail
// words, and this wave's first kWgPF stripes.
template <bool SYS>
__device__ __forceinline__ void wg_issue(const FileGeo<16>& g, const WgSrc& src, Head<16>& h, uint4 (&buf)[kWgPF],
                                         uint32_t wave, int lane, uintptr_t junk) {
  if (wave == 0) {
    if constexpr (SYS) h = load_head_sys(g, src, lane);
    else h = load_head<16>(g, lane);
    // a tiny body (< kMinParallelLen bytes, no stripes): lane i loads byte i, all
    // in one instruction (one PCIe round trip from host memory instead of one per
    // byte); wg_file_crc takes them in order with readlane
    if constexpr (SYS) {
      if (g.nstripes == 0) h.tb[0] = sys8(src, uint32_t(lane) < g.len, g.start + uint32_t(lane));
    } else {
      if (g.nstripes == 0 && uint32_t(lane) < g.len) h.tb[0] = ld8(g.start + uint32_t(lane));
    }
  }
  // Only the stripes the file has: a short body's waves issue nothing (no `junk`
  // loads either -- right after a fence those miss to HBM).
#pragma unroll
  for (int k = 0; k < kWgPF; ++k) {
    const uint32_t st = wave + 16u * uint32_t(k);  // (stripe 0 is the head: load_head)
    if (st >= 1u && st < g.nstripes) buf[k] = wg_run_load<SYS>(g, src, st, lane, junk);
  }
}

// One file by the whole workgroup (its loads issued by wg_issue): wave w's lane
// chains over stripes w, w+16, ..., moved to the end of the body, reduced in
// the wave and across waves through `part`.  The CRC is returned in wave 0
// (undefined in the other waves); `part` must not be rewritten before the
// caller's next __syncthreads.
template <bool SYS>
__device__ __forceinline__ uint32_t wg_file_crc(const uint32_t* lds_tables, uint32_t* part, const LaneBase& lb,
                                                const FileGeo<16>& g, const WgSrc& src, const Head<16>& h,
                                                uint4 (&buf)[kWgPF], uint32_t wave, int lane, uintptr_t junk) {
  uint32_t crc = 0;
  {
    // ---- this wave's lane chains over stripes wave, wave+16, ...
    const uint32_t K = g.nstripes > wave ? (g.nstripes - 1u - wave) / 16u + 1u : 0u;
    const uint32_t last = g.nstripes - 1u;
    const bool lane_in_last = uint32_t(lane) < g.nvalid;
    const uint32_t headmask = 0xffffffffu << (8 * g.s);
    const uint32_t seed_lo = g.seed << (8 * g.s);
    const uint32_t seed_hi = g.s ? (g.seed >> (32 - 8 * g.s)) : 0u;
    // seed bytes owed to lane 0's first dword of stripe 1 (A is the last dword of stripe 0)
    const uint32_t inj = (wave == 1 && lane == 0 && g.A + 4 == g.sb0 + 1024u) ? seed_hi : 0u;
    uint32_t c = 0;
    for (uint32_t k0 = 0; k0 < K; k0 += kWgPF) {
#pragma unroll
      for (int fi = 0; fi < kWgPF; ++fi) {
        const uint32_t k = k0 + uint32_t(fi);
        if (k < K) {
          const uint32_t st = wave + 16u * k;
          const uint32_t c_old = c;
          if (k) c = shift5(lds_tables, kWgJumpOff, c);
          if (st == 0) {  // head stripe: bytes before `start` masked, seed injected at A
            const uintptr_t lo = g.sb0 + uintptr_t(lane) * 16u;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const uintptr_t q = lo + 4u * i;
              uint32_t w = h.w[i];
              w = q == g.A ? ((w & headmask) ^ seed_lo) : w;
              w = q == g.A + 4 ? (w ^ seed_hi) : w;
              c = step4(lds_tables, lb, c, w);
            }
          } else {
            c = steps16(lds_tables, lb, c ^ (st == 1u ? inj : 0u), buf[fi]);
          }
          c = (st == last && !lane_in_last) ? c_old : c;  // run past B16: not part of the chain
          buf[fi] = wg_run_load<SYS>(g, src, st + 16u * kWgPF, lane, junk);
        }
      }
    }
    // ---- move the chain to the end of the body: its last valid run is
    // r = slast*64 + lane of R = (nstripes-1)*64 + nvalid runs
    uint32_t slast = wave + 16u * (K - 1u);
    bool has = K > 0u;
    if (has && slast == last && !lane_in_last) {
      has = K >= 2u;
      slast -= 16u;
    }
    const uint32_t R = last * 64u + g.nvalid;
    c = has ? wg_shift_runs(lds_tables, c, R - 1u - (slast * 64u + uint32_t(lane)), R - 1u - slast * 64u) : 0u;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) c ^= __shfl_xor(c, m, kWave);
    if (lane == 0) part[wave] = c;
    __syncthreads();
    if (wave == 0) {
      if (g.nstripes == 0) {  // tiny (< kMinParallelLen): the byte loop of func.cpp:429-433
        crc = g.seed;         // over the bytes wg_issue loaded, byte i in lane i
        for (uint32_t i = 0; i < g.len; ++i) crc = step1(lds_tables, lb, crc, __builtin_amdgcn_readlane(h.tb[0], i));
      } else {
        crc = 0;
#pragma unroll
        for (int w = 0; w < kWgWaves; ++w) crc ^= part[w];
        const uint32_t ntw = uint32_t((g.end & ~uintptr_t(3)) - g.B16) / 4u;
        const uint32_t ntb = uint32_t(g.end & 3u);
#pragma unroll
        for (int i = 0; i < 3; ++i)
          if (uint32_t(i) < ntw) crc = step4(lds_tables, lb, crc, h.tw[i]);
#pragma unroll
        for (int i = 0; i < 3; ++i)
          if (uint32_t(i) < ntb) crc = step1(lds_tables, lb, crc, h.tb[i]);
      }
    }
  }
  return crc;
}

template <int MODE>
__global__ void __launch_bounds__(kBlock) crc_wg_kernel(const uint8_t* __restrict__ base,
                                                        const Desc* __restrict__ desc, uint32_t n,
                                                        const Tables* __restrict__ tg, uint32_t* out_crc,
                                                        uint8_t* out_ok, uint32_t* n_bad, uint32_t* sched,
                                                        uint32_t vseed, uint32_t* done_flag, uint32_t seq) {
  __shared__ uint32_t lds_tables[kWgLdsBytes / 4];
  __shared__ uint32_t part[kWgWaves];
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const LaneBase lb = lane_base_of(lane);
  const uintptr_t junk = reinterpret_cast<uintptr_t>(tg->slice);
  uint32_t f = blockIdx.x;
  Desc cur{0, 0, 0};
  FileGeo<16> g{};
  Head<16> h{};
  uint4 buf[kWgPF];
  auto issue = [&](uint32_t ff) {
    cur = desc[ff];
    g = make_geo<16>(base + cur.offset, cur.len, MODE == 0 ? cur.aux : vseed);
    wg_issue<false>(g, WgSrc{}, h, buf, wave, lane, junk);
  };
  // The first file's loads are in flight while the tables are staged.
  if (f < n) issue(f);
  load_wg_tables(lds_tables, tg);
  __syncthreads();
  uint32_t bad = 0;
  while (f < n) {
    const uint32_t crc = wg_file_crc<false>(lds_tables, part, lb, g, WgSrc{}, h, buf, wave, lane, junk);
    if (wave == 0 && lane == 0) {
      if (out_crc) out_crc[f] = crc;
      if (MODE == 1) {
        const bool ok = crc == cur.aux;
        if (out_ok) out_ok[f] = ok ? 1 : 0;
        bad += ok ? 0u : 1u;
      }
    }
    f += gridDim.x;
    if (f < n) issue(f);
    __syncthreads();  // part[] is rewritten for the next file
  }
  if (threadIdx.x == 0) {
    if (MODE == 1 && bad && n_bad) atomicAdd(n_bad, bad);
    launch_exit(sched, gridDim.x, done_flag, seq);
  }
}

// ---------------------------------------------------------------------------
// Resident form: the latency form's workgroup-per-file body in
// a kernel that stays on the GPU and takes files from a page-locked ring that
// the host appends to (ResHost), so a close batch costs no launch.  Unit u is
// workgroup (u % grid)'s: wave 0 polls its next unit itself (the unit's 128-byte
// line, a 16-byte part per lane, read together with `published`: one PCIe round
// trip per poll) until the unit's tag shows it posted, and the workgroup CRCs the
// file -- wave 0 alone, from the unit's own words, for a body of at most
// kResInline bytes; thread 0 stores {crc, tag} as one 8-byte system-scope store
// into the file's result word, which the host spins on.  (Until round 5 the poll
// read `published` and a second round trip read the unit: 1.6-1.9 us more per
// batch; until the inline bodies every body was a third round trip after an
// acquire fence)  The kernel leaves when `published` has not moved for `idle_ticks` of the
// 100 MHz wall clock, after `life_ticks` in all, when the host sets `stop`, or
// after kResMaxPolls polls: the first workgroup to decide so stores the launch's
// generation into the exit line, and the others, which poll it, follow at once
// (so a unit posted to a workgroup that has left waits for a relaunch, not for
// the others' timers).  Each workgroup saves its count of units done for the
// next launch; the host relaunches the kernel when it finds it gone with work
// pending.
// ---------------------------------------------------------------------------
// Dword j of an inline body as the polling wave holds it (tfs_crc_device.h
// ResUnit): bytes 0..7 in part 0's first two words, then 12 bytes per part from
// part 2 on.  j is wave-uniform.
__device__ __forceinline__ uint32_t inline_word(const u32x4& u, uint32_t j) {
  const uint32_t p = j < 2u ? 0u : 2u + (j - 2u) / 3u;
  const uint32_t k = j < 2u ? j : (j - 2u) % 3u;
  return uint32_t(__builtin_amdgcn_readlane(k == 0u ? u.x : (k == 1u ? u.y : u.z), p));
}
// Func::crc(seed, body) over an inline body (len <= kResInline), the byte loop of
// func.cpp:429-433 restated by linearity, in wave 0: lane j < len / 4 takes dword j
// (the seed folded into dword 0), its CRC from register 0 (one slice-by-4 step),
// moved past the dwords after it -- 4 * m bytes, m = len / 4 - 1 - j, one table
// step per bit of m (4 and 8 bytes by zero-dword steps, 16, 32 and 64 by the
// level tables) -- and the lanes' values XOR-reduced; the last len % 4 bytes
// then go one at a time.  Every lane of the wave returns the CRC.
__device__ __forceinline__ uint32_t inline_crc(const uint32_t* T, const LaneBase& lb, const u32x4& u, uint32_t len,
                                               uint32_t seed, int lane) {
  const uint32_t nd = len / 4u;  // wave-uniform
  uint32_t c = seed;
  if (nd) {
    const uint32_t j = uint32_t(lane);
    const int src = j < 2u ? 0 : int(2u + (j - 2u) / 3u);
    const uint32_t k = j < 2u ? j : (j - 2u) % 3u;
    const uint32_t vx = uint32_t(__shfl(int(u.x), src, kWave)), vy = uint32_t(__shfl(int(u.y), src, kWave)),
                   vz = uint32_t(__shfl(int(u.z), src, kWave));
    uint32_t w = k == 0u ? vx : (k == 1u ? vy : vz);
    w = j == 0u ? (w ^ seed) : w;
    uint32_t x = step4(T, lb, 0u, w);
    const uint32_t m = j < nd ? nd - 1u - j : 0u;
    const uint32_t mmax = nd - 1u;
    if (mmax >= 1u) {
      const uint32_t t = step4(T, lb, x, 0u);
      x = (m & 1u) ? t : x;
    }
    if (mmax >= 2u) {
      const uint32_t t = step4(T, lb, step4(T, lb, x, 0u), 0u);
      x = (m & 2u) ? t : x;
    }
#pragma unroll
    for (uint32_t bit = 2; bit < 5; ++bit) {
      if ((mmax >> bit) != 0u) {
        const uint32_t t = shift5(T, kWgLevelOff + 1024u * (bit - 2u), x);  // 16 << (bit - 2) bytes
        x = ((m >> bit) & 1u) ? t : x;
      }
    }
    x = j < nd ? x : 0u;
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) x ^= uint32_t(__shfl_xor(int(x), o, kWave));  // nd <= 20 < 32 lanes
    c = uint32_t(__builtin_amdgcn_readfirstlane(x));
  }
  const uint32_t nb = len & 3u;
  if (nb) {
    const uint32_t w = inline_word(u, nd);
    for (uint32_t i = 0; i < nb; ++i) c = step1(T, lb, c, w >> (8u * i));
  }
  return c;
}

__device__ __forceinline__ uint64_t ld_sys64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

#ifdef TFS_CRC_MEASURE
__device__ uint32_t g_res_fence = 0;  // measurement: resident kernels fence before each payload (the pre-round-6 form)
hipError_t set_res_fence(uint32_t v) { return hipMemcpyToSymbol(HIP_SYMBOL(g_res_fence), &v, 4); }
#endif
// trace (measurement build only, tfs_crc32_res_trace; always null in the product):
// per ring unit, eight words of 100 MHz wall-clock stamps of the workgroup that
// took it -- the issue of the poll that found it published, that poll's return,
// the unit's words back, the acquire fence done, wave 0's payload loads back, its
// CRC done (just before the result store).
__global__ void __launch_bounds__(kBlock) crc_resident_kernel(const Tables* __restrict__ tg, const ResHost* hs,
                                                              uint32_t* left, uint32_t* dstate, uint32_t idle_ticks,
                                                              uint32_t life_ticks, uint32_t gen, uint64_t* trace) {
  __shared__ uint32_t lds_tables[kWgLdsBytes / 4];
  __shared__ uint32_t part[kWgWaves];
  __shared__ uint64_t claim[4];  // go, then the unit's addr, out, len | seed << 32 (seq kept by thread 0)
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const LaneBase lb = lane_base_of(lane);
  const uintptr_t junk = reinterpret_cast<uintptr_t>(tg->slice);
  uint32_t* mine = &dstate[blockIdx.x * kSchedStride];
  // wave 0 (every lane the same): units this workgroup has done (all launches),
  // the unit's tag, `published` when last looked
  uint32_t done = 0, tag = 0, seen = 0;
  if (wave == 0) done = __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  load_wg_tables(lds_tables, tg);
  const uint64_t t0 = wall_clock64();
  uint64_t last = t0;
  if (wave == 0) seen = uint32_t(ld_sys64(&hs->published));
#ifdef TFS_CRC_MEASURE
  uint64_t t_issue = 0, t_go = 0, t_unit = 0, t_fence = 0, t_loaded = 0;
  uint32_t t_want = 0;
  const uint32_t fence_ab = g_res_fence;
#else
  (void)trace;
#endif
  for (;;) {
    u32x4 u = {0u, 0u, 0u, 0u};  // wave 0, lane p < 8: part p of the unit (tfs_crc_device.h ResUnit)
    if (wave == 0) {
      const uint32_t want = blockIdx.x + done * gridDim.x;  // this workgroup's next unit
      const uint32_t wtag = want + 1u;                       // its tag
      const ResUnit* up = &hs->units[want % kResUnits];
      const u32x4* part_p = reinterpret_cast<const u32x4*>(up) + (lane & 7);
      uint32_t go = 0;
      for (uint32_t it = 0;; ++it) {
#ifdef TFS_CRC_MEASURE
        const uint64_t ti = trace ? wall_clock64() : 0u;
#endif
        // One PCIe round trip per poll: `published` (idle / stop) and the unit's
        // line, a 16-byte part per lane, all in flight together (system-coherent
        // loads), beside the exit line in device memory.
        const uint32_t ex = __hip_atomic_load(&dstate[kResExitLine], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint64_t ps = 0;
        if (lane < 8) {
          asm volatile(
              "global_load_dwordx2 %0, %2, off sc0 sc1\n\t"
              "global_load_dwordx4 %1, %3, off sc0 sc1\n\t"
              "s_waitcnt vmcnt(0)"
              : "=&v"(ps), "=&v"(u)
              : "v"(&hs->published), "v"(part_p)
              : "memory");
        }
        // the parts in use: the two halves, and an inline body's parts
        const uint32_t len0 = __builtin_amdgcn_readlane(u.z, 0);
        const uint32_t nparts = 2u + (len0 <= kResInline && len0 > 8u ? (len0 - 8u + 11u) / 12u : 0u);
        const bool stale = uint32_t(lane) < nparts && u.w != wtag;
        if (__builtin_amdgcn_ballot_w64(stale) == 0) {  // the unit, whole, came back with this poll
          go = 1;
          if (lane == 0) {
            claim[1] = uint64_t(u.x) | uint64_t(u.y) << 32;  // addr
            claim[2] = uint64_t(uint32_t(__builtin_amdgcn_readlane(u.x, 1))) |
                       uint64_t(uint32_t(__builtin_amdgcn_readlane(u.y, 1))) << 32;  // out
            claim[3] = uint64_t(len0) | uint64_t(uint32_t(__builtin_amdgcn_readlane(u.z, 1))) << 32;  // len | seed << 32
          }
          tag = wtag;
          ++done;
#ifdef TFS_CRC_MEASURE
          if (trace) {
            t_issue = ti;
            t_go = wall_clock64();
            t_unit = t_go;  // the unit arrives with the poll (no separate read)
            t_want = want;
          }
#endif
          break;
        }
        if (ex == gen) break;
        const uint64_t now = wall_clock64();
        const uint64_t ps0 = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(ps)))) |
                             uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(ps >> 32)))) << 32;
        if (uint32_t(ps0) != seen) {  // units posted (to any workgroup): not idle
          seen = uint32_t(ps0);
          last = now;
        }
        if (uint32_t(ps0 >> 32) || now - last > idle_ticks || now - t0 > life_ticks || it >= kResMaxPolls) {
          if (lane == 0) __hip_atomic_store(&dstate[kResExitLine], gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) claim[0] = go;
    }
    __syncthreads();
    if (!claim[0]) break;
    const uint32_t lw = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(claim[3])));  // wave-uniform
    const uint32_t len = lw & ~kResBulk, seed = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(claim[3] >> 32)));
    const bool bulk = (lw & kResBulk) != 0u;
    uint32_t crc = 0;
    if (len <= kResInline) {
      // The body came with the unit: wave 0 computes its CRC from the unit's
      // words (no payload read, so no fence).
#ifdef TFS_CRC_MEASURE
      if (trace && threadIdx.x == 0) t_fence = t_loaded = wall_clock64();
#endif
      if (wave == 0) crc = inline_crc(lds_tables, lb, u, len, seed, lane);
    } else {
      // The payload sits in page-locked memory the host rewrote since this
      // workgroup last looked.  A lone or small batch's body is read with
      // system-coherent loads (wg_src), never from a stale cached line, so no
      // acquire fence (round 6; before, a fence per file as a launch has: 0.6 us);
      // a bulk batch's (kResBulk) stripes stream with non-temporal loads (the
      // link's full rate) after the fence drops stale lines.
#ifdef TFS_CRC_MEASURE
      if (bulk || fence_ab)  // fence_ab: measurement only, the fenced form for A/B
#else
      if (bulk)
#endif
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#ifdef TFS_CRC_MEASURE
      if (trace && threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        t_fence = wall_clock64();
      }
#endif
      const uint64_t addr = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(claim[1])))) |
                            uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(claim[1] >> 32)))) << 32;
      const FileGeo<16> g = make_geo<16>(reinterpret_cast<const uint8_t*>(uintptr_t(addr)), len, seed);
      const WgSrc src = wg_src(g, bulk);  // wave-uniform: the resource in SGPRs
      Head<16> h{};
      uint4 buf[kWgPF];
      wg_issue<true>(g, src, h, buf, wave, lane, junk);
#ifdef TFS_CRC_MEASURE
      if (trace && threadIdx.x == 0) {  // wave 0's head and first stripe loads back
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        t_loaded = wall_clock64();
      }
#endif
      crc = wg_file_crc<true>(lds_tables, part, lb, g, src, h, buf, wave, lane, junk);
    }
#ifdef TFS_CRC_MEASURE
    if (trace && threadIdx.x == 0) {  // vector stores to page-locked host memory
      uint64_t* tr = trace + 8u * (t_want % kResUnits);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const uint64_t t_crc = wall_clock64();
      __hip_atomic_store(tr + 0, t_issue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(tr + 1, t_go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(tr + 2, t_unit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(tr + 3, t_fence, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(tr + 4, t_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(tr + 5, t_crc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#endif
    if (threadIdx.x == 0)
      __hip_atomic_store(reinterpret_cast<uint64_t*>(uintptr_t(claim[2])), uint64_t(crc) | uint64_t(tag) << 32,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();  // claim[] and part[] are rewritten for the next file
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(mine, done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // The last workgroup out tells the host (which may be exiting and waits on it
    // without HIP calls, tfs_crc_abi.cpp resident_atexit).
    if (atomicAdd(&dstate[kResLeftLine], 1u) + 1u == gridDim.x) {
      atomicExch(&dstate[kResLeftLine], 0u);
      __hip_atomic_store(left, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// The FileInfo fields the checks need (id_ +0, size_ +12, crc_ +32), read from a
// header at an arbitrary byte offset (records are packed) -- same in all lanes.
struct HdrFields {
  uint64_t id;
  int32_t size;
  uint32_t crc;
};
__device__ __forceinline__ uint32_t ldu32(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}
__device__ __forceinline__ HdrFields read_hdr(const uint8_t* rec) {
  HdrFields h;
  h.id = uint64_t(ldu32(rec)) | uint64_t(ldu32(rec + 4)) << 32;
  h.size = int32_t(ldu32(rec + 12));
  h.crc = ldu32(rec + 32);
  return h;
}


// ---------------------------------------------------------------------------
// Packet CRC (BasePacket, src/common/base_packet.cpp).  A wire frame is the
// serialized TfsPacketNewHeaderV1 (base_packet.h:92-162, little-endian:
// flag u32, length i32, type i16, version i16, id u64, crc u32 = 24 B) and
// `length` body bytes; a V0 frame has only the first 12 header bytes.  The
// receive side (BasePacketStreamer::getPacketInfo, base_packet_streamer.cpp:
// 43-124, then BasePacket::decode, base_packet.cpp:100-170) checks
// Func::crc(TFS_PACKET_FLAG_V1, body) == header crc; the send side
// (BasePacket::copy/reply, base_packet.cpp:74,208) computes it.
//
// Throughput launches (more than kWgMaxFiles frames) run packet_files_kernel
// below: one pass, the header parsed by the wave that checksums the body.  Small
// launches keep three steps: packet_parse_kernel turns frames into CRC
// descriptors (one thread per frame), the latency form computes the bodies, and
// packet_finish_kernel folds in the verdicts (verify) or writes the CRC into the
// header (seal).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}
__device__ __forceinline__ int32_t ld_le16s(const uint8_t* p) { return int16_t(uint16_t(p[0] | p[1] << 8)); }
// Header words at any byte address (HSA unaligned access mode: one global_load_dwordx4 /
// _dword whatever the alignment) -- two loads per frame instead of sixteen byte loads.
typedef const __attribute__((address_space(1))) u32x4u* gu128ucp;
typedef const __attribute__((address_space(1))) u32u* gu32ucp;
__device__ __forceinline__ u32x4 ld128u(const uint8_t* p) {
  return *reinterpret_cast<gu128ucp>(reinterpret_cast<uintptr_t>(p));
}
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) {
  return *reinterpret_cast<gu32ucp>(reinterpret_cast<uintptr_t>(p));
}

// One frame's header by the rules of getPacketInfo (base_packet_streamer.cpp:
// 43-124) and the version decode() sees (base_packet.cpp:100-141): h = the first
// 24 header bytes as little-endian dwords (only bytes inside `avail` are ever
// used); d = the body to checksum (len 0 when there is none).  Returns the
// frame's status, or kPacketPending when its body CRC decides it.
// mode 1 = verify (d.aux = stored crc), 0 = seal (d.aux = seed).
__device__ __forceinline__ int32_t parse_frame(const uint32_t (&h)[6], uint32_t avail, uint64_t off, int mode,
                                               Desc& d) {
  d = Desc{off, 0u, kPacketFlagV1};  // len 0: Func::crc returns the seed
  if (avail < uint32_t(kPacketHeaderV0Size)) return kPacketIncomplete;  // getPacketInfo:49
  const uint32_t flag = h[0];
  const int32_t length = int32_t(h[1]);
  const int32_t type = int16_t(uint16_t(h[2])), check = int16_t(uint16_t(h[2] >> 16));
  const bool v1 = flag == kPacketFlagV1;
  if (v1 && avail < uint32_t(kPacketHeaderV0Size + kPacketHeaderDiffSize))
    return kPacketIncomplete;  // :65-69, the V1 header's last 12 bytes are not there yet
  if ((flag != kPacketFlagV0 && !v1) || length <= 0 || length > kPacketMaxDataLen)
    return kTfsError;  // :78-87 "stream error": broken
  // _dataLen (:73,93) and the version decode() sees: _pcode = type (sign-extended)
  // | check << 16 for V1 (:89), version = (_pcode >> 16) & 0xFFFF (base_packet.cpp:104).
  const int64_t data_len = int64_t(length) + (v1 ? kPacketHeaderDiffSize : 0);
  const uint32_t version = ((type < 0) ? 0xFFFFu : 0u) | (v1 ? uint32_t(uint16_t(check)) : 0u);
  if (uint64_t(kPacketHeaderV0Size) + uint64_t(data_len) > avail) return kPacketIncomplete;
  if (version < 1u) return kSuccess;  // decoded without a CRC check
  if (data_len < kPacketHeaderDiffSize) return kTfsError;  // id/crc would be read past the packet
  // decode: id (8) and crc (4) follow the V0 header, the body after them (:117-141).
  d.offset = off + kPacketHeaderV0Size + kPacketHeaderDiffSize;
  d.len = uint32_t(data_len - kPacketHeaderDiffSize);
  d.aux = mode == 1 ? h[5] : kPacketFlagV1;  // avail >= 24 here
  return kPacketPending;
}

// Small launches (<= kWgMaxFiles frames, the latency form) and the measurement
// build's three-launch form: one thread per frame turns frames into CRC
// descriptors and pre-statuses.
__global__ void packet_parse_kernel(const uint8_t* __restrict__ base, const PacketDesc* __restrict__ pd, uint32_t n,
                                    int mode, Desc* __restrict__ desc, int32_t* __restrict__ pre) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const PacketDesc f = pd[i];
  const uint8_t* p = base + f.offset;
  // A frame of at least 24 bytes takes its header as one 16-byte and two 4-byte
  // loads; shorter ones byte by byte (never a byte past `avail`).
  uint32_t h[6] = {0u, 0u, 0u, 0u, 0u, 0u};
  if (f.len >= uint32_t(kPacketHeaderV0Size + kPacketHeaderDiffSize)) {
    const u32x4 v = ld128u(p);
    h[0] = v.x, h[1] = v.y, h[2] = v.z, h[3] = v.w, h[4] = ld32u(p + 16), h[5] = ld32u(p + 20);
  } else if (f.len >= uint32_t(kPacketHeaderV0Size)) {
    h[0] = ld_le32(p), h[1] = ld_le32(p + 4), h[2] = ld_le32(p + 8);
  }
  Desc d;
  pre[i] = parse_frame(h, f.len, f.offset, mode, d);
  desc[i] = d;
}

__global__ void packet_finish_kernel(uint8_t* __restrict__ base, const PacketDesc* __restrict__ pd,
                                     const Desc* __restrict__ desc, uint32_t n, int mode,
                                     const int32_t* __restrict__ pre, const uint8_t* __restrict__ ok,
                                     uint32_t* __restrict__ crc, int32_t* __restrict__ status,
                                     uint32_t* __restrict__ n_bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t bad = 0;
  if (i < n) {
    int32_t st = pre[i];
    const bool checked = st == kPacketPending;
    if (checked) {
      if (mode == 1) {
        st = ok[i] ? kSuccess : kExitCheckCrcError;  // decode returns false on mismatch (:142-148)
      } else {
        st = kSuccess;
        // Seal: store the body CRC into the V1 header's crc_ (serialized at +20).
        // (base_packet_streamer.cpp:166-175 writes only V1 headers; a V0-flag
        // frame keeps its bytes.)
        uint8_t* p = base + pd[i].offset;
        if (ld_le32(p) == kPacketFlagV1) {
          const uint32_t c = crc[i];
          for (int b = 0; b < 4; ++b) p[kPacketHeaderV0Size + 8 + b] = uint8_t(c >> (8 * b));
        }
      }
    } else if (crc) {
      crc[i] = 0u;  // not checked
    }
    status[i] = st;
    bad = st != kSuccess ? 1u : 0u;
  }
  // One atomic per wave.
  const uint64_t m = __ballot(bad != 0);
  if (n_bad && m && (threadIdx.x & (kWave - 1)) == 0) atomicAdd(n_bad, uint32_t(__popcll(m)));
  (void)desc;
}

#ifdef TFS_CRC_MEASURE
// Calibration (variants 65/66, measurement only): the record list of a device
// compaction copied by the chunk copy's loop -- per job, bursts of 8 stripes of
// 1 KiB (16 B per lane, nt loads and stores) over the 16-aligned body, the ragged
// ends byte by byte; no CRC, no header rewrite, no statuses.  Needs destinations
// congruent to their sources mod AL, bodies from AL-aligned addresses (67/68: AL
// 128, whole lines like the kernel's anchored grid).  DYN: the product's interleaved tickets;
// else job j -> wave j mod W (53104's order).  Where the record kernel trails the
// chunk copy of the same bytes, this says whether the record list or the kernel's
// own schedule costs it.
template <bool DYN, uint32_t AL = 16>
__global__ void __launch_bounds__(kBlock) compact_probe_copy_kernel(const uint8_t* __restrict__ src,
                                                                    const CompactJob* __restrict__ jobs, uint32_t n,
                                                                    uint8_t* __restrict__ dst, uint32_t* sched) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t wpb = kBlock / kWave;
  Tickets<kIL> tk;
  tk.ctr = sched;
  tk.n = n;
  tk.group = blockIdx.x & 7u;
  tk.init_static(gridDim.x * wpb, blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave));
  if (!DYN) tk.dyn = false;
  for (;;) {
    const uint32_t f = tk.resolve(tk.issue(lane), lane);
    if (f >= n) break;
    const CompactJob j = jobs[f];
    const uintptr_t s0 = reinterpret_cast<uintptr_t>(src) + j.src_offset;
    const intptr_t delta = intptr_t(reinterpret_cast<uintptr_t>(dst) + j.dest_offset) - intptr_t(s0);
    const uintptr_t s1 = s0 + uint32_t(j.size);
    const uintptr_t a0 = (s0 + AL - 1u) & ~uintptr_t(AL - 1u), a1 = s1 & ~uintptr_t(AL - 1u);
    for (uintptr_t i = uintptr_t(lane); i < a0 - s0; i += kWave)
      *reinterpret_cast<uint8_t*>(s0 + i + delta) = *reinterpret_cast<const uint8_t*>(s0 + i);
    for (uintptr_t i = uintptr_t(lane); i < s1 - a1; i += kWave)
      *reinterpret_cast<uint8_t*>(a1 + i + delta) = *reinterpret_cast<const uint8_t*>(a1 + i);
    for (uintptr_t o = a0; o < a1; o += 8u * 1024u) {
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uintptr_t q = o + 1024u * k + 16u * uint32_t(lane);
        if (q < a1) v[k] = ld128s<true>(q);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uintptr_t q = o + 1024u * k + 16u * uint32_t(lane);
        if (q < a1) st128_kind<1>(q + delta, u32x4{v[k].x, v[k].y, v[k].z, v[k].w});
      }
    }
  }
  if (lane == 0) launch_exit(sched, gridDim.x * wpb, nullptr, 0u);
}

#endif  // TFS_CRC_MEASURE

// ---------------------------------------------------------------------------
// Pipelined compaction (task.cpp:713-836): the crc_files_kernel
// schedule applied to the fused re-CRC + repack.  Records are taken by dynamic
// tickets (Tickets<kIL>, stream-bound slot, launch_exit), and the next record's
// descriptor, FileInfo, head and first PF stripes are in flight while the current
// one is finished (tail and header stores, combine, checks).  The 36-byte
// FileInfo is read with one byte load per lane (lanes 0..35) and written with one
// byte store per lane (offset_/size_/usize_/flag_ rewritten); the fields the
// checks need come out of those registers by readlane.  Payload bytes take the
// copy-through of lane_chain at every shift: whole aligned dwordx4 stores for a
// destination congruent mod 4, one unaligned dwordx4 per lane otherwise;
// payloads too short for stripes take copy_unaligned.
// ---------------------------------------------------------------------------
struct CRec {
  uint64_t soff, doff, fid;
  int32_t size, flag, new_off;
  int32_t pre;  // kSuccess, or the status decided before reading (size / range)
  uint32_t plen;  // payload bytes this unit covers (size - 36 for a whole record)
  uint32_t kind;  // 0 a whole record, 1 a payload segment of a split record, 2 a split record's head
  uint32_t edge;  // 1: no byte past the record may be read (CompactJob.reserved bit 0)
};

template <bool WIDE, bool VERIFY = false>
__device__ __forceinline__ CRec load_crec(uint32_t f, uint64_t src_len, const RawMeta* __restrict__ metas,
                                          const int32_t* __restrict__ flags, const int64_t* __restrict__ dest_off,
                                          const CompactJob* __restrict__ jobs) {
  CRec r;
  r.edge = 0u;
  bool range_ok;
  if (VERIFY && !WIDE) {
    const RawMeta m = metas[f];
    r.soff = uint64_t(int64_t(m.offset)), r.doff = 0, r.fid = m.file_id;
    r.size = m.size, r.flag = 0, r.new_off = 0;
    range_ok = m.offset >= 0 && uint64_t(m.offset) + uint64_t(uint32_t(m.size)) <= src_len;
  } else if (WIDE) {
    const CompactJob j = jobs[f];
    r.soff = j.src_offset, r.doff = j.dest_offset, r.fid = j.file_id;
    r.size = j.size, r.flag = j.flag, r.new_off = j.new_offset;
    r.edge = uint32_t(j.reserved) & 1u;
    range_ok = r.soff + uint64_t(uint32_t(r.size)) <= src_len;
  } else {
    const RawMeta m = metas[f];
    const int64_t d = dest_off[f];
    r.soff = uint64_t(int64_t(m.offset)), r.doff = uint64_t(d), r.fid = m.file_id;
    r.size = m.size, r.flag = flags[f], r.new_off = int32_t(d);
    range_ok = m.offset >= 0 && d >= 0 && uint64_t(m.offset) + uint64_t(uint32_t(m.size)) <= src_len;
  }
  // Verify rejects a record with no payload byte (sync_backup.cpp:348-351); the
  // compaction copies an empty file like any other (task.cpp:753-798).
  const bool short_rec = VERIFY ? r.size <= kFileInfoSize : r.size < kFileInfoSize;
  r.pre = short_rec ? kExitReadFileSizeError : (range_ok ? kSuccess : kExitParameterError);
  r.plen = r.pre == kSuccess ? uint32_t(r.size - kFileInfoSize) : 0u;
  r.kind = 0u;
  return r;
}

// Unit f of a segmented compaction launch (CSegArgs): jobs [0, njobs) -- a split
// record's job is its head (FileInfo + the ragged first payload bytes) -- then
// the ext units, whole payload segments with no FileInfo.
__device__ __forceinline__ CRec load_cunit(uint32_t f, uint32_t njobs, uint64_t src_len,
                                           const CompactJob* __restrict__ jobs, const uint8_t* plan, uint32_t cap,
                                           uint32_t lg) {
  if (f < njobs) {
    CRec r = load_crec<true>(f, src_len, nullptr, nullptr, nullptr, jobs);
    if (plan && reinterpret_cast<const uint32_t*>(plan + cseg_off_base())[f] != kNoSplit) {
      const uint32_t seg = 1024u << lg;
      r.kind = 2u;
      r.plen -= ((r.plen - 1u) >> (10u + lg)) * seg;
    }
    return r;
  }
  const CSegUnit u = reinterpret_cast<const CSegUnit*>(plan + cseg_off_ext(njobs, cap))[f - njobs];
  CRec r;
  r.soff = u.src - kFileInfoSize;  // a pseudo-record whose payload is the segment
  r.doff = u.dst - kFileInfoSize;
  r.fid = 0;
  r.size = int32_t(u.len) + kFileInfoSize;
  r.flag = r.new_off = 0;
  r.pre = kSuccess;
  r.plen = u.len;
  r.kind = 1u;
  r.edge = uint32_t(u.pad) & 1u;
  return r;
}

// A record's registers issued ahead of its compute.
struct CState {
  FileGeo<kRun> g;
  Head<kRun> h;
  uint32_t hb;  // this lane's FileInfo byte (lanes 0..35)
  intptr_t delta;
};

// DA: anchor the record's stripe grid on destination lines (make_geo's `aoff`):
// every stripe's copy-through store then covers eight whole 128-byte lines of the
// new block instead of splitting two lines with its neighbours (a split line
// leaves the chip as two partial writes).  Needs a destination congruent to the
// source mod 4 and 128 readable bytes past the record inside the source.
// The payload geometry of a record (and its copy distance): wave-uniform, no loads.
template <bool DA>
__device__ __forceinline__ FileGeo<kRun> crec_geo(const CRec& r, const uint8_t* src, uint64_t src_len, uint8_t* dst,
                                                  uintptr_t junk, intptr_t& delta) {
  if (r.pre != kSuccess) {  // nothing is read for a record rejected up front
    delta = 0;
    return make_geo<kRun>(reinterpret_cast<const uint8_t*>(junk), 0u, 0u);
  }
  const uint8_t* rec = src + r.soff;
  delta = intptr_t(dst + r.doff) - intptr_t(rec);
  uint32_t aoff = 0u;
  if (DA && !r.edge && r.soff + kFileInfoSize + uint64_t(r.plen) + 128u <= src_len)
    aoff = uint32_t(-(delta & ~intptr_t(15))) & 127u;
  return make_geo<kRun>(rec + kFileInfoSize, r.plen, 0u, aoff);
}

template <bool DA>
__device__ __forceinline__ CState issue_crec(const CRec& r, const uint8_t* src, uint64_t src_len, uint8_t* dst,
                                             int lane, uintptr_t junk) {
  CState s;
  s.g = crec_geo<DA>(r, src, src_len, dst, junk, s.delta);
  if (r.pre == kSuccess) {
    s.hb = lane < kFileInfoSize && r.kind != 1u ? uint32_t(src[r.soff + uint32_t(lane)]) : 0u;
    s.h = load_head<kRun>(s.g, lane);
  } else {
    s.hb = 0u;
    s.h = Head<kRun>{};
  }
  return s;
}

// FileInfo dword k (bytes 4k..4k+3, k < 9) from the lanes' header bytes.
__device__ __forceinline__ uint32_t hdr_dword(uint32_t hb, uint32_t k) {
  return __builtin_amdgcn_readlane(hb, 4 * k) | __builtin_amdgcn_readlane(hb, 4 * k + 1) << 8 |
         __builtin_amdgcn_readlane(hb, 4 * k + 2) << 16 | __builtin_amdgcn_readlane(hb, 4 * k + 3) << 24;
}

// VERIFY: the verify-on-read form (sync_backup.cpp:345-435, block_console.cpp:
// 543-577) -- the same schedule and checks, no stores: `metas` (RawMeta, !WIDE)
// or `jobs` (CompactJob with the dest fields unused, WIDE: many blocks, 64-bit
// offsets) name the records, dst is unused.
// Payload copy for a destination not congruent to the source mod 4 (and tiny
// payloads), after the record's CRC pass: whole dwordx4 stores at 16-aligned
// destination chunks, each from ONE unaligned 16-byte load of the source (the
// HSA unaligned access mode: one global_load_dwordx4 at any byte address; the
// lines were just read by the CRC pass, so the re-read is mostly served by the
// caches).  At most 15 head and 15 tail bytes go byte by byte.
__device__ __forceinline__ void copy_unaligned(const uint8_t* s, uint8_t* d, uint32_t len, int lane) {
  const uintptr_t d0 = reinterpret_cast<uintptr_t>(d);
  const uintptr_t da = (d0 + 15u) & ~uintptr_t(15);
  const uint32_t head = uint32_t(da - d0) < len ? uint32_t(da - d0) : len;
  const uint32_t nch = (len - head) / 16u;
  const uint32_t t0 = head + 16u * nch;
  if (uint32_t(lane) < head) d[lane] = s[lane];
  if (uint32_t(lane) < len - t0) d[t0 + lane] = s[t0 + lane];
  const uint8_t* sa = s + head;
  uint32_t c = uint32_t(lane);
  for (; c + 3u * kWave < nch; c += 4u * kWave) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_memcpy(&v[k], sa + 16u * (c + uint32_t(k) * kWave), 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) st128_nt(da + 16u * (c + uint32_t(k) * kWave), v[k]);
  }
  for (; c < nch; c += kWave) {
    uint4 v;
    __builtin_memcpy(&v, sa + 16u * c, 16);
    st128_nt(da + 16u * c, v);
  }
}

// DIAG bits: 2 stripe grid anchored on destination lines (issue_crec<DA>), 3
// temporal payload loads (with the destination-anchored grid a source line is
// split between two stripes of the same wave; a temporal load keeps it in L2
// for the second).  The product is both (kCompactDiag).  Measurement only: bit
// 1 no payload CRC steps (variant 26: wrong CRCs and statuses; the kernel's own
// load/store schedule without the table lookups).
constexpr int kCompactDiag = 4 | 8;
// Record order of long device-compaction launches (FileCursor HS, round 4): the first
// 3/4 of the records go statically (wave w: w, w+W, ...), the rest by tickets.  Against
// one record per ticket, in one process on five boxes: -1.7, -1.7, 0.0, -1.8, -1.7 %
// (DESIGN.md §4.1).
constexpr int kCompactHS = 2;
// NW waves per workgroup, OCC workgroups per CU (LDS table layout LY must fit OCC
// times in 160 KiB): the product is 16 waves, one workgroup, layout 1.
// LR (measurement build): the stripes in flight in an LDS-DMA ring (LdsRing) instead of VGPRs.
template <bool WIDE, bool VERIFY = false, int DIAG = kCompactDiag, int CPF = kPF, int CF = 1, int TS = 0,
          bool SEG = false, int HS = 0, int NW = kBlock / kWave, int OCC = 1, int LY = kLY, bool LR = false>
__global__ void __launch_bounds__(NW * kWave, OCC * NW / 4) compact_pipe_kernel(
    const uint8_t* __restrict__ src, uint64_t src_len, const RawMeta* __restrict__ metas,
    const int32_t* __restrict__ flags, const int64_t* __restrict__ dest_off, const CompactJob* __restrict__ jobs,
    uint32_t n, uint8_t* __restrict__ dst, const Tables* __restrict__ tg, uint32_t* out_crc, int32_t* out_status,
    uint32_t* n_bad, uint32_t* sched, CSegArgs cs) {
  constexpr bool DA = !VERIFY && (DIAG & 4) != 0;
  constexpr bool LNT = (DIAG & 8) && !VERIFY ? false : kNT;  // the verify form keeps the headline's loads
  static_assert(OCC * (LdsLayout<LY>::bytes + (LR ? 1024u * NW * CPF : 0u)) <= 160u * 1024u,
                "OCC workgroups per CU must fit the LDS");
  __shared__ uint32_t lds_tables[LdsLayout<LY>::bytes / 4];
  load_tables<kRun, kPAR, LY>(lds_tables, tg);
  const int lane = threadIdx.x & (kWave - 1);
  LdsRing ring{nullptr, 0u, 0u};
  if constexpr (LR) {  // slot f of wave w: lds_ring[(f * NW + w) * 64 ..] (no LDS object in the product)
    __shared__ uint4 lds_ring[NW * CPF * kWave];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    ring.base = lds_ring + w * kWave;
    ring.addr = uint32_t(reinterpret_cast<uintptr_t>((lds_vp)(ring.base)));
    ring.stride = NW * kWave;
  }
  const LaneBase lb = lane_base_for<LY>(lane);
  const uint32_t wpb = NW;
  const uintptr_t junk = reinterpret_cast<uintptr_t>(tg->slice);
  // SEG: units are the jobs, then the ext segments of the split records (CSegArgs)
  const uint32_t njobs = n;
  uint8_t* plan = nullptr;  // stays null when nothing was split
  if (SEG && cs.plan) {
    const unsigned long long used = *reinterpret_cast<const unsigned long long*>(cs.plan);
    n = njobs + uint32_t(used < cs.cap ? used : cs.cap);
    if (used) plan = cs.plan;
  }
  auto unit = [&](uint32_t u) -> CRec {
    if constexpr (SEG) return load_cunit(u, njobs, src_len, jobs, plan, cs.cap, cs.lg);
    return load_crec<WIDE, VERIFY>(u, src_len, metas, flags, dest_off, jobs);
  };
  // CF > 1: chunks of CF records per ticket; HS: the static phase first
  FileCursor<kIL, CF, TS, HS> fc;
  constexpr bool FC = CF > 1 || HS > 0;  // files come from the cursor (chunks / the static phase)
  auto& tk = fc.tk;
  fc.init(sched, n, blockIdx.x & 7u, gridDim.x * wpb,
          blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave));
  if (FC) fc.start(lane);
  uint32_t bad = 0;
  do {
    uint32_t f = FC ? fc.take(lane) : tk.resolve(tk.issue(lane), lane);
    if (f >= n) break;
    uint32_t fn = FC ? fc.take(lane) : tk.resolve(tk.issue(lane), lane);
    CRec cur = unit(f);
    CState st = issue_crec<DA>(cur, src, src_len, dst, lane, junk);
    uint4 buf[CPF][kRun / 16];
    if constexpr (LR) load_ring_lds<kRun, CPF>(st.g, lane, ring, junk);
    else load_ring<kRun, CPF, LNT>(st.g, lane, buf, junk);
    CRec nxt = fn < n ? unit(fn) : CRec{};
    uint32_t jv = !FC && fn < n ? tk.issue(lane) : 0u;
    for (;;) {
      const bool more = fn < n;
      const CRec ncur = nxt;
      uint32_t c = st.g.nstripes ? lane_chain<kRun, CPF, LNT, LY, !VERIFY, true, 1, (DIAG & 2) != 0, LR>(
                                       lds_tables, lb, st.g, st.h, buf, lane, junk, st.delta, true, &ring)
                                 : 0u;
      // The next record's loads go out before this one is finished.
      CState ns = st;
      uint32_t fnn = n;
      if (more) {
        ns = issue_crec<DA>(ncur, src, src_len, dst, lane, junk);
        if constexpr (LR) load_ring_lds<kRun, CPF>(ns.g, lane, ring, junk);
        else load_ring<kRun, CPF, LNT>(ns.g, lane, buf, junk);
        fnn = FC ? fc.take(lane) : tk.resolve(jv, lane);
        if (fnn < n) {
          nxt = unit(fnn);
          if (!FC) jv = tk.issue(lane);
        }
      }
      int32_t status = cur.pre;
      if (status == kSuccess) {
        const uint8_t* rec = src + cur.soff;
        uint8_t* drec = dst + cur.doff;
        const uint32_t len = cur.plen;
        // FileInfo with offset_(8) size_(12) usize_(16) flag_(28) rewritten, the rest copied (task.cpp:753-759)
        if (!VERIFY && lane < kFileInfoSize && cur.kind != 1u) {
          const int fld = lane >> 2, sh = 8 * (lane & 3);
          uint32_t b = st.hb;
          if (fld == 2) b = uint32_t(cur.new_off) >> sh;
          else if (fld == 3 || fld == 4) b = uint32_t(cur.size) >> sh;
          else if (fld == 7) b = uint32_t(cur.flag) >> sh;
          drec[lane] = uint8_t(b);
        }
        if (VERIFY) {
        } else if (st.g.nstripes) {
          if (lane == 0) {  // tail [B16, end) from lane 0's registers
            const uint32_t ntw = uint32_t((st.g.end & ~uintptr_t(3)) - st.g.B16) / 4u;
            for (uint32_t i = 0; i < 3u; ++i)
              if (i < ntw) st32u(st.g.B16 + 4u * i + st.delta, st.h.tw[i]);
            const uintptr_t B = st.g.end & ~uintptr_t(3);
            for (uint32_t i = 0; i < 3u; ++i)
              if (B + i < st.g.end) *reinterpret_cast<uint8_t*>(B + i + st.delta) = uint8_t(st.h.tb[i]);
          }
        } else {  // tiny payload
          copy_unaligned(rec + kFileInfoSize, drec + kFileInfoSize, len, lane);
        }
        c = finish_file<kRun, LY>(lds_tables, lb, st.g, st.h, c, lane);
        const uint64_t hid = uint64_t(hdr_dword(st.hb, 0)) | uint64_t(hdr_dword(st.hb, 1)) << 32;
        if (cur.kind == 1u) {
        } else if (hid != cur.fid) status = kExitFileInfoError;
        else if (int32_t(hdr_dword(st.hb, 3)) != cur.size) status = kExitSyncFileError;
        else if (cur.kind == 0u && c != hdr_dword(st.hb, 8)) status = kExitCheckCrcError;
        if (SEG && cur.kind == 2u && lane == 0) {  // the fold decides the CRC check
          reinterpret_cast<uint32_t*>(plan + cseg_off_head(njobs))[f] = c;
          reinterpret_cast<uint32_t*>(plan + cseg_off_hdr(njobs))[f] = hdr_dword(st.hb, 8);
          reinterpret_cast<int32_t*>(plan + cseg_off_pre(njobs))[f] = status;
        }
      } else {
        c = 0u;
        if (SEG && cur.kind == 2u && lane == 0) reinterpret_cast<int32_t*>(plan + cseg_off_pre(njobs))[f] = status;
      }
      if (SEG && cur.kind == 1u) {
        if (lane == 0) reinterpret_cast<uint32_t*>(plan + cseg_off_ext_crc(njobs))[f - njobs] = c;
      } else if (SEG && cur.kind == 2u) {
      } else if (lane == 0) {
        if (out_crc) out_crc[f] = c;
        if (out_status) out_status[f] = status;
        bad += status != kSuccess ? 1u : 0u;
      }
      if (!more) break;
      f = fn;
      fn = fnn;
      cur = ncur;
      st = ns;
    }
  } while (false);
  if (lane == 0 && bad && n_bad) atomicAdd(n_bad, bad);
  if (lane == 0) launch_exit(sched, gridDim.x * wpb, nullptr, 0u);
}

// Segmented compaction plan (CSegArgs): one thread per job.  A live record whose
// payload is longer than one segment keeps its FileInfo and ragged first
// len - K*seg payload bytes in its own slot and gets K ext units for its whole
// segments, reserved as one range per workgroup (one atomic per 256 jobs); a
// workgroup whose range would pass `cap` leaves its records whole (and writes
// empty units into the part below cap).  Records the kernel rejects before
// reading (short, out of range: load_crec) are never split.
__global__ void __launch_bounds__(256) compact_seg_plan_kernel(const CompactJob* __restrict__ jobs, uint32_t n,
                                                               uint64_t src_len, CSegArgs cs) {
  __shared__ uint32_t wsum[4];
  __shared__ unsigned long long blk_base;
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t w = threadIdx.x / kWave;
  const uint32_t seg = 1024u << cs.lg;
  CompactJob j{};
  uint32_t K = 0;
  if (i < n) {
    j = jobs[i];
    const bool ok = j.size >= kFileInfoSize && j.src_offset + uint64_t(uint32_t(j.size)) <= src_len;
    const uint32_t L = ok ? uint32_t(j.size - kFileInfoSize) : 0u;
    K = L > seg ? (L - 1u) >> (10u + cs.lg) : 0u;
  }
  uint32_t x = K;  // inclusive scan over the wave
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == kWave - 1) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    before += k < w ? wsum[k] : 0u;
    total += wsum[k];
  }
  if (threadIdx.x == 0)
    blk_base = total ? atomicAdd(reinterpret_cast<unsigned long long*>(cs.plan), (unsigned long long)total) : 0ull;
  __syncthreads();
  const unsigned long long b0 = blk_base;
  const bool fits = b0 + total <= cs.cap;
  const unsigned long long my = b0 + before + (x - K);
  if (i < n) reinterpret_cast<uint32_t*>(cs.plan + cseg_off_base())[i] = (K && fits) ? uint32_t(my) : kNoSplit;
  if (!K) return;
  CSegUnit* ext = reinterpret_cast<CSegUnit*>(cs.plan + cseg_off_ext(n, cs.cap));
  if (fits) {
    const uint64_t head = uint64_t(uint32_t(j.size - kFileInfoSize)) - uint64_t(K) * seg;
    const uint64_t s0 = j.src_offset + kFileInfoSize + head, d0 = j.dest_offset + kFileInfoSize + head;
    // The record's edge bit rides on its last segment (the only one that ends
    // where the record ends): that unit never reads past the record either.
    const uint64_t edge = uint64_t(j.reserved) & 1u;
    for (uint32_t k = 0; k < K; ++k)
      ext[my + k] = CSegUnit{s0 + uint64_t(k) * seg, d0 + uint64_t(k) * seg, seg, i, k + 1 == K ? edge : 0u};
  } else {
    for (unsigned long long u = my; u < my + K && u < cs.cap; ++u) ext[u] = CSegUnit{0, 0, 0, 0, 0};
  }
}

// Segmented compaction fold: each split record's CRC from its head and segment
// CRCs (crc(A||B) = shift(crc(A), |B|) ^ crc(B), seed 0), then the record's CRC,
// status (the head's FileInfo checks first, then the CRC against the stored
// crc_) and mismatch count, as the record kernel writes them for whole records.
__global__ void __launch_bounds__(256) compact_seg_fold_kernel(const CompactJob* __restrict__ jobs, uint32_t n,
                                                               const Tables* __restrict__ tg, CSegArgs cs,
                                                               uint32_t* out_crc, int32_t* out_status,
                                                               uint32_t* n_bad) {
  __shared__ uint32_t T[uint32_t(kShiftChunks) * 32u];
  if (*reinterpret_cast<const unsigned long long*>(cs.plan) == 0ull) return;  // nothing was split
  const uint32_t* base = reinterpret_cast<const uint32_t*>(cs.plan + cseg_off_base());
  const uint32_t* head_crc = reinterpret_cast<const uint32_t*>(cs.plan + cseg_off_head(n));
  const uint32_t* hdr_crc = reinterpret_cast<const uint32_t*>(cs.plan + cseg_off_hdr(n));
  const int32_t* pre = reinterpret_cast<const int32_t*>(cs.plan + cseg_off_pre(n));
  const uint32_t* ext_crc = reinterpret_cast<const uint32_t*>(cs.plan + cseg_off_ext_crc(n));
  const uint32_t* tab = &tg->cseg_shift[cs.lg - kCSegLgMin][0][0];
  for (uint32_t k = threadIdx.x; k < uint32_t(kShiftChunks) * 32u; k += blockDim.x) T[k] = tab[k];
  __syncthreads();
  uint32_t bad = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t b = base[i];
    if (b == kNoSplit) continue;
    const uint32_t K = (uint32_t(jobs[i].size - kFileInfoSize) - 1u) >> (10u + cs.lg);
    uint32_t c = head_crc[i];
    for (uint32_t k = 0; k < K; ++k) c = shift5(T, 0u, c) ^ ext_crc[b + k];
    int32_t status = pre[i];
    if (status == kSuccess && c != hdr_crc[i]) status = kExitCheckCrcError;
    if (out_crc) out_crc[i] = c;
    if (out_status) out_status[i] = status;
    bad += status != kSuccess ? 1u : 0u;
  }
  if (n_bad) {  // one atomic per wave
#pragma unroll
    for (int m = kWave / 2; m >= 1; m >>= 1) bad += __shfl_xor(bad, m, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0 && bad) atomicAdd(n_bad, bad);
  }
}

// Packet frames in one pass (round 5): the throughput form of
// BasePacket::decode (verify, MODE 1) and BasePacket::copy + encode (seal, MODE 0)
// over n frames.  A wave takes frames by the file kernel's chunked tickets; it
// loads a frame's 24 header bytes (lanes 0..23, one byte each, only bytes inside
// the frame's `avail`) a frame ahead, parses them by getPacketInfo + decode's
// rules (parse_frame) when that frame comes up, checksums the body with seed
// TFS_PACKET_FLAG_V1 and writes the frame's final status and CRC itself (verify:
// against the header's crc_; seal: the CRC stored into the V1 header at +20).  No
// parse or finish launch and no descriptor scratch.  Bodies stay whole: a
// WriteDataMessage carries at most one 2 MiB segment (MAX_SEGMENT_SIZE,
// internal.h:157), so no body makes a launch's tail the way a 64 MiB file can.
template <int MODE>
__global__ void __launch_bounds__(kBlock) packet_files_kernel(uint8_t* __restrict__ base,
                                                              const PacketDesc* __restrict__ pd, uint32_t n,
                                                              const Tables* __restrict__ tg, uint32_t* out_crc,
                                                              int32_t* out_status, uint32_t* n_bad, uint32_t* sched) {
  constexpr int RUN = kRun, PF = kPF;
  __shared__ uint32_t lds_tables[LdsLayout<kLY>::bytes / 4];
  load_tables<RUN, false, kLY>(lds_tables, tg);
  const int lane = threadIdx.x & (kWave - 1);
  const LaneBase lb = lane_base_of(lane);
  const uint32_t wpb = kBlock / kWave;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uintptr_t junk = reinterpret_cast<uintptr_t>(tg->slice);
  FileCursor<kIL, kCF, kTS> frames;
  frames.init(sched, n, blockIdx.x & 7u, gridDim.x * wpb, blockIdx.x * wpb + wave);
  frames.start(lane);
  struct Issued {  // a frame whose header bytes are in flight
    uint64_t off;
    uint32_t avail, hb;  // hb: this lane's header byte (lanes 0..23)
  };
  struct Frame {
    Desc d;
    int32_t pre;
    uint32_t flag;
  };
  auto issue = [&](uint32_t u) -> Issued {
    const PacketDesc f = pd[u];
    Issued x{f.offset, f.len, 0u};
    if (uint32_t(lane) < 24u && uint32_t(lane) < f.len) x.hb = ld8(reinterpret_cast<uintptr_t>(base + f.offset) + lane);
    return x;
  };
  auto parse = [&](const Issued& x) -> Frame {
    uint32_t h[6];
#pragma unroll
    for (uint32_t k = 0; k < 6u; ++k) h[k] = hdr_dword(x.hb, k);
    Frame r;
    r.flag = h[0];
    r.pre = parse_frame(h, x.avail, x.off, MODE, r.d);
    return r;
  };
  uint32_t bad = 0;
  do {  // `break` = this wave has no (more) frames; every wave reaches launch_exit
    uint32_t f = frames.take(lane);
    if (f >= n) break;
    uint32_t fn = frames.take(lane);
    Frame cur = parse(issue(f));
    FileGeo<RUN> g = make_geo<RUN>(base + cur.d.offset, cur.d.len, kPacketFlagV1);
    Head<RUN> h = load_head<RUN>(g, lane);
    uint4 buf[PF][RUN / 16];
    load_ring<RUN, PF, kNT>(g, lane, buf, junk);
    Issued nx = fn < n ? issue(fn) : Issued{0, 0u, 0u};
    for (;;) {
      const bool more = fn < n;
      const uint32_t c = g.nstripes ? lane_chain<RUN, PF, kNT, kLY>(lds_tables, lb, g, h, buf, lane, junk) : 0u;
      // The next frame's header is in; its body loads go out before this one is finished.
      Frame ncur = cur;
      FileGeo<RUN> ng = g;
      Head<RUN> nh = h;
      uint32_t fnn = n;
      if (more) {
        ncur = parse(nx);
        ng = make_geo<RUN>(base + ncur.d.offset, ncur.d.len, kPacketFlagV1);
        nh = load_head<RUN>(ng, lane);
        load_ring<RUN, PF, kNT>(ng, lane, buf, junk);
        fnn = frames.take(lane);
        if (fnn < n) nx = issue(fnn);
      }
      const uint32_t crc = finish_file<RUN, kLY>(lds_tables, lb, g, h, c, lane);
      if (lane == 0) {
        int32_t st = cur.pre;
        uint32_t co = 0u;
        if (st == kPacketPending) {
          co = crc;
          if (MODE == 1) {
            st = crc == cur.d.aux ? kSuccess : kExitCheckCrcError;  // decode returns false (:142-148)
          } else {
            st = kSuccess;  // seal: only V1 headers carry a crc (base_packet_streamer.cpp:166-175)
            if (cur.flag == kPacketFlagV1) st32u(reinterpret_cast<uintptr_t>(base + cur.d.offset) - 4u, crc);
          }
        }
        if (out_crc) out_crc[f] = co;
        out_status[f] = st;
        bad += st != kSuccess ? 1u : 0u;
      }
      if (!more) break;
      f = fn;
      fn = fnn;
      cur = ncur;
      g = ng;
      h = nh;
    }
  } while (false);
  if (lane == 0 && bad && n_bad) atomicAdd(n_bad, bad);
  if (lane == 0) launch_exit(sched, gridDim.x * wpb, nullptr, 0u);
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

// Bench/test helper: unsealed V1 frame headers (crc 0) at rec_off[f] for bodies
// of len[f] bytes (TfsPacketNewHeaderV1::serialize order, little-endian).
__global__ void write_packet_headers_kernel(uint8_t* __restrict__ base, const uint64_t* __restrict__ rec_off,
                                            const uint32_t* __restrict__ len, uint32_t n, int32_t pcode,
                                            int32_t version, uint64_t first_id) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  uint8_t* p = base + rec_off[f];
  const uint64_t id = first_id + f;
  const uint32_t w[6] = {kPacketFlagV1, len[f], (uint32_t(pcode) & 0xFFFFu) | (uint32_t(version) << 16),
                         uint32_t(id), uint32_t(id >> 32), 0u};
  for (int i = 0; i < 24; ++i) p[i] = uint8_t(w[i >> 2] >> (8 * (i & 3)));
}

#ifdef TFS_CRC_MEASURE
// Calibration kernel (not on the product path): stream the same bytes without
// the CRC arithmetic.  run == 0: fully coalesced grid-stride, 16 B/lane.
// run > 0: the CRC kernel's pattern -- one wave per file, each lane reading
// `run` contiguous bytes of every 64*run-byte stripe (len multiple of 64*run).
// NT: non-temporal loads.
template <bool NT>
__global__ void __launch_bounds__(kBlock) membench_kernel(const uint8_t* __restrict__ base,
                                                          const Desc* __restrict__ desc, uint32_t n,
                                                          uint64_t nbytes, uint32_t run, uint32_t* out,
                                                          uint32_t align) {
  uint32_t acc = 0;
  if (run == 0) {
    const uintptr_t p = reinterpret_cast<uintptr_t>(base);
    const uint64_t nv = nbytes / 16;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nv; i += stride) {
      const uint4 v = ld128s<NT>(p + 16 * i);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  } else {
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wpb = kBlock / kWave;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    for (uint32_t f = blockIdx.x * wpb + wave; f < n; f += gridDim.x * wpb) {
      const Desc d = desc[f];
      const uintptr_t start = (reinterpret_cast<uintptr_t>(base + d.offset) + align - 1) & ~uintptr_t(align - 1);
      const uint32_t stripe = 64u * run, ns = (d.len - (align - 1)) / stripe;
      uint32_t r = 0;
      for (; r + 8 <= ns; r += 8) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = ld128s<NT>(start + uintptr_t(r + k) * stripe + uintptr_t(lane) * 16u);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
      }
      for (; r < ns; ++r) {
        const uint4 a = ld128s<NT>(start + uintptr_t(r) * stripe + uintptr_t(lane) * 16u);
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
      }
    }
  }
  if (acc == 0x9E3779B9u) out[0] = acc;  // keep the loads alive
}


// Calibration: copy with U 16-byte chunks per lane in flight per iteration
// (U loads, then U stores); LNT = nt loads; SK = store kind (0 plain, 1 nt).
template <bool LNT, int SK, int U>
__global__ void __launch_bounds__(kBlock) membench_copy2_kernel(const uint8_t* __restrict__ src,
                                                                uint8_t* __restrict__ dst, uint64_t nbytes) {
  const uint64_t nv = nbytes / 16;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  const uintptr_t s = reinterpret_cast<uintptr_t>(src), d = reinterpret_cast<uintptr_t>(dst);
  uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + uint64_t(U - 1) * stride < nv; i += uint64_t(U) * stride) {
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = ld128s<LNT>(s + 16 * (i + uint64_t(k) * stride));
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const u32x4 w = {v[k].x, v[k].y, v[k].z, v[k].w};
      gu128wp a = reinterpret_cast<gu128wp>(d + 16 * (i + uint64_t(k) * stride));
      if (SK == 1) __builtin_nontemporal_store(w, a);
      else *a = w;
    }
  }
  for (; i < nv; i += stride) {
    const uint4 v = ld128s<LNT>(s + 16 * i);
    const u32x4 w = {v.x, v.y, v.z, v.w};
    *reinterpret_cast<gu128wp>(d + 16 * i) = w;
  }
}
#endif  // TFS_CRC_MEASURE

}  // namespace tfscrc

// ---------------------------------------------------------------------------
// Launch wrappers (called from tfs_crc_abi.cpp; no HIP types leak past this TU
// except through that file).  `cap` is the workgroup count of a throughput
// launch: kMaxGrid, or fewer when CUs are left free for a resident kernel on
// the same device (tfs_crc_abi.cpp, throughput_cap).
//
// The product library (libtfs_crc.so) holds exactly one form of each kernel.
// The measurement build (-DTFS_CRC_MEASURE, libtfs_crc_measure.so) adds the A/B
// forms selected by TFS_CRC_VARIANT; the product never reads it.
// ---------------------------------------------------------------------------
namespace tfscrc {

static unsigned grid_for(uint32_t nwork, unsigned cap = kMaxGrid) {
  const uint32_t wpb = kBlock / kWave;
  uint64_t g = (uint64_t(nwork) + wpb - 1) / wpb;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  return unsigned(g);
}
// Workgroups of nw waves for nwork units, at most cap.
static unsigned grid_waves(uint32_t nwork, uint32_t nw, unsigned cap) {
  uint64_t g = (uint64_t(nwork) + nw - 1) / nw;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  return unsigned(g);
}

template <int MODE>
static hipError_t launch_variant(int variant, const uint8_t* base, const Desc* desc, uint32_t n, const Tables* tg,
                                 uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad, uint32_t* sched,
                                 hipStream_t stream, uint32_t vseed, uint32_t* done_flag, uint32_t seq, unsigned cap,
                                 const SplitArgs* split) {
  // Latency form for small batches (TFS_CRC_VARIANT 20 forces it for any n in
  // the measurement build).
  if (variant == 20 || n <= kWgMaxFiles) {
    const unsigned wg = n < kMaxGrid ? n : kMaxGrid;
    hipLaunchKernelGGL((crc_wg_kernel<MODE>), dim3(wg), dim3(kBlock), 0, stream, base, desc, n, tg, out_crc, out_ok,
                       n_bad, sched, vseed, done_flag, seq);
    return hipGetLastError();
  }
  if (!sched) return hipErrorInvalidValue;
  // Split files (tfs_crc_device.h): the address-ordered plan (count, scan, write)
  // before the main kernel, the fold after it, all on `stream`; the
  // completion-flag form (done_flag) never splits.  A split launch's work is its
  // files plus the segments the plan makes on the device (a few hundred 64 MiB
  // files are ~150 k units), so it takes the whole capped grid.
  const SplitArgs sa = split && !done_flag ? *split : SplitArgs{nullptr, 0u};
  const dim3 grid(sa.plan ? (cap < kMaxGrid ? cap : kMaxGrid) : grid_for(n, cap)), block(kBlock);
  if (sa.plan) {
    const uint32_t nb = ao_nblk(n);
    hipLaunchKernelGGL(split_ao_count_kernel, dim3(nb), dim3(kAoBlock), 0, stream, desc, n, sa);
    hipLaunchKernelGGL(split_ao_scan_kernel, dim3(1), dim3(1024), 0, stream, desc, n, sa);
    hipLaunchKernelGGL(split_ao_write_kernel, dim3(nb), dim3(kAoBlock), 0, stream, desc, n, sa);
    if (const hipError_t e = hipGetLastError()) return e;
  }
#ifdef TFS_CRC_MEASURE
  if (variant == 50)  // one file per ticket (the product before chunked tickets)
    hipLaunchKernelGGL((crc_files_kernel<MODE, 1, 0>), grid, block, 0, stream, base, desc, n, tg, out_crc, out_ok,
                       n_bad, sched, vseed, done_flag, seq, sa);
  else
#endif
    hipLaunchKernelGGL((crc_files_kernel<MODE>), grid, block, 0, stream, base, desc, n, tg, out_crc, out_ok, n_bad,
                       sched, vseed, done_flag, seq, sa);
  (void)variant;
  if (const hipError_t e = hipGetLastError()) return e;
  if (sa.plan) {
    const uint32_t fg = (n + 255u) / 256u;
    hipLaunchKernelGGL((split_ao_fold_kernel<MODE>), dim3(fg < 1024u ? fg : 1024u), dim3(256), 0, stream, desc, n, tg,
                       sa, out_crc, out_ok, n_bad);
  }
  return hipGetLastError();
}

hipError_t launch_crc_files(int mode, const uint8_t* base, const Desc* desc, uint32_t n, const Tables* tg,
                            uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad, uint32_t* sched, hipStream_t stream,
                            int variant, uint32_t vseed, uint32_t* done_flag, uint32_t seq, unsigned cap,
                            const SplitArgs* split) {
  if (n == 0) return hipSuccess;
  if (mode == 0)
    return launch_variant<0>(variant, base, desc, n, tg, out_crc, out_ok, n_bad, sched, stream, vseed, done_flag, seq,
                             cap, split);
  return launch_variant<1>(variant, base, desc, n, tg, out_crc, out_ok, n_bad, sched, stream, vseed, done_flag, seq,
                           cap, split);
}

hipError_t launch_resident(const Tables* tg, const ResHost* hs, uint32_t* left, uint32_t* dstate, unsigned grid,
                           uint32_t idle_ticks, uint32_t life_ticks, uint32_t gen, hipStream_t stream, uint64_t* trace) {
  hipLaunchKernelGGL(crc_resident_kernel, dim3(grid), dim3(kBlock), 0, stream, tg, hs, left, dstate, idle_ticks,
                     life_ticks, gen, trace);
  return hipGetLastError();
}

hipError_t launch_packet_parse(const uint8_t* base, const PacketDesc* pd, uint32_t n, int mode, Desc* desc,
                               int32_t* pre, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(packet_parse_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, base, pd, n, mode, desc, pre);
  return hipGetLastError();
}

hipError_t launch_packet_files(uint8_t* base, const PacketDesc* pd, uint32_t n, int mode, const Tables* tg,
                               uint32_t* crc, int32_t* status, uint32_t* n_bad, uint32_t* sched, hipStream_t stream,
                               unsigned cap) {
  if (n == 0) return hipSuccess;
  if (!sched) return hipErrorInvalidValue;
  if (mode == 1)
    hipLaunchKernelGGL(packet_files_kernel<1>, dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, base, pd, n, tg, crc,
                       status, n_bad, sched);
  else
    hipLaunchKernelGGL(packet_files_kernel<0>, dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, base, pd, n, tg, crc,
                       status, n_bad, sched);
  return hipGetLastError();
}

hipError_t launch_packet_finish(uint8_t* base, const PacketDesc* pd, const Desc* desc, uint32_t n, int mode,
                                const int32_t* pre, const uint8_t* ok, uint32_t* crc, int32_t* status,
                                uint32_t* n_bad, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(packet_finish_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, base, pd, desc, n, mode, pre,
                     ok, crc, status, n_bad);
  return hipGetLastError();
}


// Compaction of one block (RawMeta + flags + dest offsets): compact_pipe_kernel
// (dynamic tickets on the stream's slot, next-record prefetch).
hipError_t launch_compact_fused(const uint8_t* src, uint64_t src_len, const RawMeta* metas, const int32_t* flags,
                                const int64_t* dest_off, uint32_t n, uint8_t* dst, const Tables* tg, uint32_t* out_crc,
                                int32_t* out_status, uint32_t* n_bad, uint32_t* sched, hipStream_t stream,
                                int variant, unsigned cap) {
  if (n == 0) return hipSuccess;
  if (!sched) return hipErrorInvalidValue;
  hipLaunchKernelGGL(compact_pipe_kernel<false>, dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, src, src_len, metas,
                     flags, dest_off, nullptr, n, dst, tg, out_crc, out_status, n_bad, sched, CSegArgs{nullptr, 0u, 0u});
  (void)variant;
  return hipGetLastError();
}

// Compaction of many blocks (CompactJob, 64-bit offsets) in one launch.
hipError_t launch_compact_jobs(const uint8_t* src, uint64_t src_len, const CompactJob* jobs, uint32_t n, uint8_t* dst,
                               const Tables* tg, uint32_t* out_crc, int32_t* out_status, uint32_t* n_bad,
                               uint32_t* sched, hipStream_t stream, int variant, unsigned cap, const CSegArgs* seg) {
  if (n == 0) return hipSuccess;
  if (!sched) return hipErrorInvalidValue;
  const unsigned ccap = cap < kMaxGrid ? cap : kMaxGrid;
  if (seg && seg->plan) {
    // Segmented form: plan, the record kernel over jobs + segments (the whole
    // capped grid: the units are made on the device), fold -- all on `stream`.
    const CSegArgs cs = *seg;
    hipLaunchKernelGGL(compact_seg_plan_kernel, dim3((n + 255u) / 256u), dim3(256), 0, stream, jobs, n, src_len, cs);
    if (const hipError_t e = hipGetLastError()) return e;
    hipLaunchKernelGGL((compact_pipe_kernel<true, false, kCompactDiag, kPF, 1, 0, true>), dim3(ccap), dim3(kBlock), 0,
                       stream, src, src_len, nullptr, nullptr, nullptr, jobs, n, dst, tg, out_crc, out_status, n_bad,
                       sched, cs);
    if (const hipError_t e = hipGetLastError()) return e;
    const uint32_t fg = (n + 255u) / 256u;
    hipLaunchKernelGGL(compact_seg_fold_kernel, dim3(fg < 1024u ? fg : 1024u), dim3(256), 0, stream, jobs, n, tg, cs,
                       out_crc, out_status, n_bad);
    return hipGetLastError();
  }
#define TFS_CJR(NW_, OCC_, LY_, PF_, DIAG_, LR_)                                                                     \
  hipLaunchKernelGGL((compact_pipe_kernel<true, false, DIAG_, PF_, 1, 0, false, kCompactHS, NW_, OCC_, LY_, LR_>),   \
                     dim3(grid_waves(n, NW_, ccap * OCC_)), dim3(NW_ * kWave), 0, stream, src, src_len, nullptr,       \
                     nullptr, nullptr, jobs, n, dst, tg, out_crc, out_status, n_bad, sched, CSegArgs{nullptr, 0u, 0u})
#define TFS_CJ(NW_, OCC_, LY_, PF_, DIAG_) TFS_CJR(NW_, OCC_, LY_, PF_, DIAG_, false)
#ifdef TFS_CRC_MEASURE
  // Measurement forms: 26 the product without the payload CRC steps
  // (its own load/store schedule; wrong CRCs); 67 / 68 the record list through the
  // chunk copy's loop (dynamic / static order, calibration: no CRC, no headers).
  // Round 5, two workgroups per CU: 74 KiB of LDS tables
  // (LdsLayout<2>) and 12-wave (94-96: PF 5, 4, 3; 80 VGPRs), 10-wave (98: 96
  // VGPRs) or 16-wave (99: 64 VGPRs) workgroups; 97 the 74 KiB tables at one
  // 16-wave workgroup per CU (control).
  if (variant == 26) TFS_CJ(16, 1, kLY, kPF, kCompactDiag | 2);
  else if (variant == 67 || variant == 68)
    hipLaunchKernelGGL((variant == 67 ? compact_probe_copy_kernel<true, 128> : compact_probe_copy_kernel<false, 128>),
                       dim3(grid_for(n, cap)), dim3(kBlock), 0, stream, src, jobs, n, dst, sched);
  else if (variant == 94) TFS_CJ(12, 2, 2, kPF, kCompactDiag);
  else if (variant == 95) TFS_CJ(12, 2, 2, 4, kCompactDiag);
  else if (variant == 96) TFS_CJ(12, 2, 2, 3, kCompactDiag);
  else if (variant == 97) TFS_CJ(16, 1, 2, kPF, kCompactDiag);
  else if (variant == 98) TFS_CJ(10, 2, 2, kPF, kCompactDiag);
  else if (variant == 99) TFS_CJ(16, 2, 2, 3, kCompactDiag);
  // Round 6: the stripes in flight in an LDS-DMA ring
  // (LdsRing) beside the 74 KiB tables -- 120: 16 waves x 5 slots (154 KiB of LDS;
  // its VGPR-ring control is 97); 121: 8 waves x 8 slots (138 KiB).
  else if (variant == 120) TFS_CJR(16, 1, 2, kPF, kCompactDiag, true);
  else if (variant == 121) TFS_CJR(8, 1, 2, 8, kCompactDiag, true);
  else
#endif
    TFS_CJ(16, 1, kLY, kPF, kCompactDiag);
#undef TFS_CJ
#undef TFS_CJR
  (void)variant;
  return hipGetLastError();
}

// Verify-on-read of block records: the verify form of the record kernel
// (chunked tickets like the file kernel).  Measurement build: one record per
// ticket (50).
hipError_t launch_block_verify_pipe(const uint8_t* image, uint64_t image_len, const RawMeta* metas,
                                    const CompactJob* jobs, uint32_t n, const Tables* tg, uint32_t* out_crc,
                                    int32_t* out_status, uint32_t* n_bad, uint32_t* sched, hipStream_t stream,
                                    int variant, unsigned cap) {
  if (n == 0) return hipSuccess;
  if (!sched) return hipErrorInvalidValue;
  const dim3 grid(grid_for(n, cap));
#define TFS_BV(WIDE_, CF_, TS_)                                                                                     \
  hipLaunchKernelGGL((compact_pipe_kernel<WIDE_, true, kCompactDiag, kPF, CF_, TS_>), grid, dim3(kBlock), 0, stream, \
                     image, image_len, metas, nullptr, nullptr, jobs, n, nullptr, tg, out_crc, out_status, n_bad, sched, \
                     CSegArgs{nullptr, 0u, 0u})
#ifdef TFS_CRC_MEASURE
  if (variant == 50 && jobs) TFS_BV(true, 1, 0);
  else if (variant == 50) TFS_BV(false, 1, 0);
  else
#endif
  if (jobs) TFS_BV(true, kCF, kTS);
  else TFS_BV(false, kCF, kTS);
#undef TFS_BV
  (void)variant;
  return hipGetLastError();
}

hipError_t launch_synth_fill(uint64_t* dst, uint64_t nwords, uint64_t seed, uint64_t first_word, hipStream_t stream) {
  if (nwords == 0) return hipSuccess;
  uint64_t g = (nwords + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(synth_fill_kernel, dim3(unsigned(g)), dim3(256), 0, stream, dst, nwords, seed, first_word);
  return hipGetLastError();
}

#ifdef TFS_CRC_MEASURE
// Calibration: copy by wave-contiguous chunks of CH bytes (the record kernel's
// shape: one wave streams one range), chunk c to wave c mod W; each wave moves
// PF 1 KiB stripes per step (16 B per lane, nt loads, store kind SK).
// HOLE (round 4, partial-line writes): 1 leaves the chunk's first 16 bytes
// unwritten (one partial line per chunk), 2 also its last 16 bytes, 3 writes
// those two 16-byte pieces as byte stores (whole lines, assembled from partial
// stores of one wave) -- the record kernel's boundary-line pattern on a dense copy.
template <int PF, int SK, int HOLE = 0>
__global__ void __launch_bounds__(kBlock) membench_copy_chunk_kernel(const uint8_t* __restrict__ src,
                                                                     uint8_t* __restrict__ dst, uint64_t nbytes,
                                                                     uint64_t ch) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t wave = uint64_t(blockIdx.x) * (kBlock / kWave) + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t nw = uint64_t(gridDim.x) * (kBlock / kWave);
  const uint64_t nch = nbytes / ch;
  const uintptr_t s = reinterpret_cast<uintptr_t>(src), d = reinterpret_cast<uintptr_t>(dst);
  for (uint64_t c = wave; c < nch; c += nw) {
    const uint64_t b = c * ch + 16u * uint64_t(lane);
    for (uint64_t o = 0; o < ch; o += 1024u * PF) {
      uint4 v[PF];
#pragma unroll
      for (int k = 0; k < PF; ++k) v[k] = ld128s<true>(s + b + o + 1024u * k);
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const u32x4 w = {v[k].x, v[k].y, v[k].z, v[k].w};
        gu128wp a = reinterpret_cast<gu128wp>(d + b + o + 1024u * k);
        const bool first = o == 0 && k == 0 && lane == 0;
        const bool last = o + 1024u * (k + 1) >= ch && k == PF - 1 && lane == kWave - 1;
        if (HOLE && (first || (HOLE >= 2 && last))) {
          if (HOLE == 3) {
            uint8_t* bp = reinterpret_cast<uint8_t*>(d + b + o + 1024u * k);
            const uint32_t ww[4] = {w[0], w[1], w[2], w[3]};
#pragma unroll
            for (int i = 0; i < 16; ++i) bp[i] = uint8_t(ww[i >> 2] >> (8 * (i & 3)));
          }
          continue;
        }
        if (SK == 1) __builtin_nontemporal_store(w, a);
        else *a = w;
      }
    }
  }
}




hipError_t launch_membench(int pattern, const uint8_t* base, const Desc* desc, uint32_t n, uint64_t nbytes,
                           uint32_t* out, unsigned grid, hipStream_t stream) {
  if (pattern >= 53000 && pattern < 54000) {
    // 53SCC: chunked copy, S = store kind (0 plain, 1 nt), CC = chunk in 16 KiB units; PF 8, 256 workgroups
    const int S = (pattern / 100) % 10, CC = pattern % 100;
    const uint64_t ch = uint64_t(CC ? CC : 4) * 16384u;
    const uint64_t nb = nbytes / ch * ch;
    const dim3 g(grid ? grid : kMaxGrid);
    uint8_t* d = reinterpret_cast<uint8_t*>(out);
    if (S == 1)
      hipLaunchKernelGGL((membench_copy_chunk_kernel<8, 1>), g, dim3(kBlock), 0, stream, base, d, nb, ch);
    else if (S == 2)  // nt stores, one 16-byte hole per chunk (partial-line writes, round 4)
      hipLaunchKernelGGL((membench_copy_chunk_kernel<8, 1, 1>), g, dim3(kBlock), 0, stream, base, d, nb, ch);
    else if (S == 3)  // nt stores, holes at both ends of each chunk
      hipLaunchKernelGGL((membench_copy_chunk_kernel<8, 1, 2>), g, dim3(kBlock), 0, stream, base, d, nb, ch);
    else if (S == 4)  // nt stores, both ends written as byte stores
      hipLaunchKernelGGL((membench_copy_chunk_kernel<8, 1, 3>), g, dim3(kBlock), 0, stream, base, d, nb, ch);
    else
      hipLaunchKernelGGL((membench_copy_chunk_kernel<8, 0>), g, dim3(kBlock), 0, stream, base, d, nb, ch);
    return hipGetLastError();
  }
  // pattern: 0 = coalesced, 16 = stripe pattern (run 16); +1000 = non-temporal loads;
  // +10000 = stripes anchored at 128-byte boundaries (else 16)
  if (pattern >= 52000 && pattern < 53000) {
    // 52LSU: L = nt loads (0/1), S = store kind (0 plain, 1 nt), U = chunks in flight (1, 4, 8)
    const int L = (pattern / 100) % 10, S = (pattern / 10) % 10, U = pattern % 10;
    const dim3 g(grid ? grid : 2048u);
    uint8_t* d = reinterpret_cast<uint8_t*>(out);
#define TFS_COPY2(LL, SS, UU) \
  if (L == LL && S == SS && U == UU) hipLaunchKernelGGL((membench_copy2_kernel<LL == 1, SS, UU>), g, dim3(kBlock), 0, stream, base, d, nbytes)
    TFS_COPY2(0, 0, 1); TFS_COPY2(0, 0, 4); TFS_COPY2(0, 0, 8); TFS_COPY2(1, 0, 4); TFS_COPY2(1, 1, 4);
    TFS_COPY2(0, 1, 4); TFS_COPY2(1, 1, 8); TFS_COPY2(1, 0, 8);
#undef TFS_COPY2
    return hipGetLastError();
  }
  if (pattern < 0 || pattern >= 20000) return hipErrorInvalidValue;  // no other shape is built
  const uint32_t align = pattern >= 10000 ? 128u : 16u;
  pattern %= 10000;
  const bool nt = pattern >= 1000;
  const uint32_t run = uint32_t(pattern % 1000);
  // a stripe is 64 lanes x 16 B = 64 * run bytes: run 0 (grid-stride) or a multiple of 16
  if ((run != 0 && run % 16 != 0) || pattern >= 2000) return hipErrorInvalidValue;
  const dim3 g(grid ? grid : (run ? grid_for(n) : 2048u));
  if (nt)
    hipLaunchKernelGGL(membench_kernel<true>, g, dim3(kBlock), 0, stream, base, desc, n, nbytes, run, out, align);
  else
    hipLaunchKernelGGL(membench_kernel<false>, g, dim3(kBlock), 0, stream, base, desc, n, nbytes, run, out, align);
  return hipGetLastError();
}

#endif  // TFS_CRC_MEASURE

hipError_t launch_write_packet_headers(uint8_t* base, const uint64_t* rec_off, const uint32_t* len, uint32_t n,
                                       int32_t pcode, int32_t version, uint64_t first_id, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(write_packet_headers_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, base, rec_off, len, n,
                     pcode, version, first_id);
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
