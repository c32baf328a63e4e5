// ec_math.h -- host-side matrix work of TFS's erasure code,
// bit-identical to the reference's vendored jerasure/galois:
//
//   GF(2^8), primitive polynomial 0435 (x^8+x^4+x^3+x^2+1)   galois.cpp:48-57
//   encode matrix m[i][j] = 1 / (i XOR (pn + j))  (Cauchy)   erasure_code.cpp:58-67
//   bitmatrix: element e -> 8x8 bits, column x = e * 2^x,
//              bit l of column x at row l                       jerasure.cpp:261-287
//   decoding bitmatrix: the k*8 rows of the first k alive
//              devices (identity for data, bitmatrix rows for
//              parity), inverted over GF(2)                     jerasure.cpp:117-155,1033-1088
//
// The inverse of an invertible matrix is unique, so any correct GF(2)
// elimination reproduces jerasure's decoding matrix exactly.  Only the per-
// byte region work runs on the GPU (tfs_ec_kernels.hip); this is setup.
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace tfsec {

constexpr int kW = 8;            // ErasureCode::ws_ (erasure_code.cpp:33)
constexpr int kPacket = 128;     // ErasureCode::ps_ (erasure_code.cpp:34)
constexpr int kUnit = kW * kPacket;
constexpr int kMaxMembers = 12;  // MAX_MARSHALLING_NUM (common/internal.h:170)

struct Gf256 {
  int log[256];
  int exp[512];
  Gf256() {
    int b = 1;
    for (int j = 0; j < 255; ++j) {
      log[b] = j;
      exp[j] = exp[j + 255] = b;
      b <<= 1;
      if (b & 0x100) b ^= 0x11D;  // 0435
    }
    log[0] = -1;
    exp[510] = exp[511] = 0;
  }
  int mul(int a, int b) const { return (a == 0 || b == 0) ? 0 : exp[log[a] + log[b]]; }
  int div(int a, int b) const { return b == 0 ? -1 : (a == 0 ? 0 : exp[log[a] - log[b] + 255]); }
};

// k*8 x ... bit matrices are stored row-major as bytes (0/1).
using BitMat = std::vector<uint8_t>;

// m*8 rows x k*8 cols encode bitmatrix of the Cauchy matrix.
inline BitMat encode_bitmatrix(int k, int m) {
  static const Gf256 gf;
  BitMat bm(size_t(m) * kW * k * kW);
  const int cols = k * kW;
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) {
      int e = gf.div(1, i ^ (m + j));
      for (int x = 0; x < kW; ++x) {
        for (int l = 0; l < kW; ++l) bm[size_t(i * kW + l) * cols + j * kW + x] = (e >> l) & 1;
        e = gf.mul(e, 2);
      }
    }
  return bm;
}

// GF(2) inverse of an n x n bit matrix; false if singular.
inline bool invert_bits(BitMat a, int n, BitMat* inv) {
  inv->assign(size_t(n) * n, 0);
  for (int i = 0; i < n; ++i) (*inv)[size_t(i) * n + i] = 1;
  for (int c = 0; c < n; ++c) {
    int p = c;
    while (p < n && !a[size_t(p) * n + c]) ++p;
    if (p == n) return false;
    if (p != c)
      for (int x = 0; x < n; ++x) {
        std::swap(a[size_t(p) * n + x], a[size_t(c) * n + x]);
        std::swap((*inv)[size_t(p) * n + x], (*inv)[size_t(c) * n + x]);
      }
    for (int r = 0; r < n; ++r)
      if (r != c && a[size_t(r) * n + c])
        for (int x = 0; x < n; ++x) {
          a[size_t(r) * n + x] ^= a[size_t(c) * n + x];
          (*inv)[size_t(r) * n + x] ^= (*inv)[size_t(c) * n + x];
        }
  }
  return true;
}

// Decode plan: the k source devices (dm_ids: the first k alive, in index
// order) and, for every device to rebuild, its 8 bit-rows over those sources.
struct DecodePlan {
  std::vector<int> sources;   // dm_ids
  std::vector<int> outputs;   // devices rebuilt: erased data (erased != 0), then erased parity (erased == 1)
  BitMat rows;                // outputs.size()*8 rows x k*8 cols
};

// 0 ok, -1 not enough alive devices, -2 singular (erasure_code.cpp:90-118).
inline int make_decode_plan(int k, int m, const int* erased, DecodePlan* plan) {
  const int n = k * kW;
  int alive = 0;
  for (int i = 0; i < k + m; ++i) alive += erased[i] == 0;
  if (alive < k) return -1;
  plan->sources.clear();
  for (int i = 0; int(plan->sources.size()) < k; ++i)
    if (erased[i] == 0) plan->sources.push_back(i);
  const BitMat enc = encode_bitmatrix(k, m);
  BitMat a(size_t(n) * n, 0);
  for (int i = 0; i < k; ++i) {
    const int id = plan->sources[i];
    for (int r = 0; r < kW; ++r)
      for (int c = 0; c < n; ++c)
        a[size_t(i * kW + r) * n + c] = id < k ? uint8_t(c == id * kW + r) : enc[size_t((id - k) * kW + r) * n + c];
  }
  BitMat dec;
  if (!invert_bits(a, n, &dec)) return -2;
  // data device d = dec rows [d*8, d*8+8) applied to the sources
  plan->outputs.clear();
  plan->rows.clear();
  for (int d = 0; d < k; ++d)
    if (erased[d] != 0) {  // erasure_code.cpp:205 tests erased_[i] (1 or -1)
      plan->outputs.push_back(d);
      plan->rows.insert(plan->rows.end(), dec.begin() + size_t(d) * kW * n, dec.begin() + size_t(d + 1) * kW * n);
    }
  // parity p = enc rows of p applied to the data; data = dec applied to the
  // sources, so over the sources: enc_p * dec (GF(2) product).
  for (int p = 0; p < m; ++p)
    if (erased[k + p] == 1) {  // :214
      plan->outputs.push_back(k + p);
      for (int r = 0; r < kW; ++r) {
        const uint8_t* er = &enc[size_t(p * kW + r) * n];
        std::vector<uint8_t> row(n, 0);
        for (int t = 0; t < n; ++t)
          if (er[t])
            for (int c = 0; c < n; ++c) row[c] ^= dec[size_t(t) * n + c];
        plan->rows.insert(plan->rows.end(), row.begin(), row.end());
      }
    }
  return 0;
}

}  // namespace tfsec
