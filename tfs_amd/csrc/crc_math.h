// crc_math.h -- GF(2) arithmetic for the reflected CRC-32 of Func::crc
// (src/common/func.cpp:426-435; poly 0xEDB88320, reflected, no inversion).
//
// Host-side only: builds the lookup tables the kernels stage into LDS / read
// from global memory.  Nothing here is on the per-byte path.
//
// Conventions (reflected domain, as in Func::crc): a 32-bit register value v
// holds the polynomial sum_{i} bit_i(v) * x^(31-i); multiplication is mod P.
// For seed-0 CRCs, crc(A||B) = shift(crc(A), |B|) ^ crc(B) where
// shift(c, n) = c * x^(8n) mod P; that identity is what lets a file be cut into
// independent lane segments and recombined.
#pragma once
#include <cstdint>

namespace tfscrc {

constexpr uint32_t kPoly = 0xEDB88320u;

// Standard byte table: the value of Func::crc(0, {b}) (== _crc32tab[b],
// src/common/func.h:128-154; pinned by tests/golden table_* vectors).
inline void make_byte_table(uint32_t t[256]) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : (c >> 1);
    t[i] = c;
  }
}

// Slice tables: s[k][b] = CRC contribution of byte b followed by k zero bytes.
// A dword step is c' = s[3][x&255] ^ s[2][(x>>8)&255] ^ s[1][(x>>16)&255] ^ s[0][x>>24]
// with x = c ^ w (w = 4 payload bytes, little-endian).
inline void make_slice_tables(uint32_t s[][256], int nslices) {
  make_byte_table(s[0]);
  for (int k = 1; k < nslices; ++k)
    for (int b = 0; b < 256; ++b) s[k][b] = (s[k - 1][b] >> 8) ^ s[0][s[k - 1][b] & 0xffu];
}

// a * b mod P (reflected).
inline uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1u) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

// x^(n * 2^k) mod P.
inline uint32_t x2nmodp(uint64_t n, unsigned k) {
  uint32_t p = 1u << 31;  // x^0
  uint32_t sq = 1u << 30; // x^1
  for (unsigned i = 0; i < k; ++i) sq = multmodp(sq, sq);
  while (n) {
    if (n & 1) p = multmodp(sq, p);
    n >>= 1;
    sq = multmodp(sq, sq);
  }
  return p;
}

// shift(c, nbytes) = CRC register after feeding nbytes zero bytes from state c.
inline uint32_t shift_bytes(uint32_t c, uint64_t nbytes) { return multmodp(x2nmodp(nbytes, 3), c); }

// Byte-indexed shift table for a fixed distance: shift(c, n) = XOR_j t[j][(c >> 8j) & 255].
inline void make_shift_table(uint32_t t[4][256], uint64_t nbytes) {
  const uint32_t k = x2nmodp(nbytes, 3);
  for (int j = 0; j < 4; ++j)
    for (uint32_t b = 0; b < 256; ++b) t[j][b] = multmodp(k, b << (8 * j));
}

// 5-bit-chunk shift table: shift(c, n) = XOR_k t[k][(c >> 5k) & 31], k = 0..6.
inline void make_shift_table5(uint32_t t[7][32], uint64_t nbytes) {
  const uint32_t k = x2nmodp(nbytes, 3);
  for (int j = 0; j < 7; ++j)
    for (uint32_t e = 0; e < 32; ++e) t[j][e] = (j == 6 && e >= 4) ? 0u : multmodp(k, e << (5 * j));
}

}  // namespace tfscrc
