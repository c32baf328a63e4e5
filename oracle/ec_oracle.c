/*
 * oracle/ec_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of TFS's erasure code, the checker for
 * the GPU kernels behind include/tfs_ec.h.  Follows, loop for loop:
 *   galois.cpp:152-190    log/antilog tables of GF(2^8), polynomial 0435
 *   erasure_code.cpp:58-67  Cauchy matrix m[i][j] = 1 / (i ^ (pn + j))
 *   jerasure.cpp:261-287  matrix -> bitmatrix (column x of an element = e * 2^x)
 *   jerasure.cpp:304-348  bitmatrix dot product over packets (memcpy first, then XOR)
 *   jerasure.cpp:117-155  decoding bitmatrix (first k alive devices)
 *   jerasure.cpp:1033-1088 GF(2) inversion (upper triangular, then back-substitute)
 *   erasure_code.cpp:141-235 encode / decode (data first, then dead parity from data)
 * Pinned against the reference's own jerasure/galois sources compiled in the
 * survey container (oracle/build_ref.sh -> oracle/_ref/libref_ec.so,
 * tests/golden/ec_vectors.json via oracle/gen_golden_ec.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EC_W 8
#define EC_PS 128
#define EC_MAX 12
#define EXIT_DATA_INVALID (-16001)
#define EXIT_SIZE_INVALID (-16002)
#define EXIT_MATRIX_INVALID (-16003)
#define EXIT_NO_ENOUGH_DATA (-16004)

static int g_log[256], g_ilog[255 * 3];
static int g_ready;

static void gf_init(void) {
  int j, b = 1;
  if (g_ready) return;
  for (j = 0; j < 256; j++) g_log[j] = 255;
  for (j = 0; j < 255; j++) {
    g_log[b] = j;
    g_ilog[j] = b;
    b <<= 1;
    if (b & 256) b = (b ^ 0435) & 255;
  }
  for (j = 0; j < 255; j++) g_ilog[j + 255] = g_ilog[j + 510] = g_ilog[j];
  g_ready = 1;
}
static int gf_mul(int x, int y) { return (x == 0 || y == 0) ? 0 : g_ilog[g_log[x] + g_log[y]]; }
static int gf_div(int a, int b) { return b == 0 ? -1 : (a == 0 ? 0 : g_ilog[g_log[a] - g_log[b] + 255]); }

/* m*w x k*w bitmatrix, row-major ints */
static int* cauchy_bitmatrix(int k, int m) {
  int rowelts = k * EC_W, i, j, x, l;
  int* bm = (int*)calloc((size_t)k * m * EC_W * EC_W, sizeof(int));
  gf_init();
  for (i = 0; i < m; i++)
    for (j = 0; j < k; j++) {
      int elt = gf_div(1, i ^ (m + j));
      for (x = 0; x < EC_W; x++) {
        for (l = 0; l < EC_W; l++) bm[(i * EC_W + l) * rowelts + j * EC_W + x] = (elt >> l) & 1;
        elt = gf_mul(elt, 2);
      }
    }
  return bm;
}

static void dotprod(int k, const int* row, const int* src_ids, int dest, char** ptrs, int size) {
  int s, j, x, y, idx;
  char* dst = ptrs[dest];
  for (s = 0; s < size; s += EC_PS * EC_W) {
    idx = 0;
    for (j = 0; j < EC_W; j++) {
      int started = 0;
      char* p = dst + s + j * EC_PS;
      for (x = 0; x < k; x++) {
        const char* b = ptrs[src_ids ? src_ids[x] : x];
        for (y = 0; y < EC_W; y++, idx++) {
          if (!row[idx]) continue;
          if (!started) {
            memcpy(p, b + s + y * EC_PS, EC_PS);
            started = 1;
          } else {
            int t;
            for (t = 0; t < EC_PS; t++) p[t] ^= b[s + y * EC_PS + t];
          }
        }
      }
    }
  }
}

static int invert_bits(int* mat, int* inv, int n) {
  int i, j, k, t;
  for (i = 0; i < n; i++)
    for (j = 0; j < n; j++) inv[i * n + j] = i == j;
  for (i = 0; i < n; i++) {
    if (!mat[i * n + i]) {
      for (j = i + 1; j < n && !mat[j * n + i]; j++) {}
      if (j == n) return -1;
      for (k = 0; k < n; k++) {
        t = mat[i * n + k]; mat[i * n + k] = mat[j * n + k]; mat[j * n + k] = t;
        t = inv[i * n + k]; inv[i * n + k] = inv[j * n + k]; inv[j * n + k] = t;
      }
    }
    for (j = i + 1; j < n; j++)
      if (mat[j * n + i])
        for (k = 0; k < n; k++) { mat[j * n + k] ^= mat[i * n + k]; inv[j * n + k] ^= inv[i * n + k]; }
  }
  for (i = n - 1; i >= 0; i--)
    for (j = 0; j < i; j++)
      if (mat[j * n + i])
        for (k = 0; k < n; k++) { mat[j * n + k] ^= mat[i * n + k]; inv[j * n + k] ^= inv[i * n + k]; }
  return 0;
}

static int check(int k, int m, char** ptrs, const int* sizes, int size) {
  int i;
  if (size % (EC_W * EC_PS) != 0) return EXIT_SIZE_INVALID;
  for (i = 0; i < k + m; i++)
    if (!ptrs[i] || (sizes && sizes[i] < size)) return EXIT_DATA_INVALID;
  return 0;
}

int oracle_ec_encode(int k, int m, char** ptrs, const int* sizes, int size) {
  int i, rc = check(k, m, ptrs, sizes, size);
  int* bm;
  if (rc) return rc;
  bm = cauchy_bitmatrix(k, m);
  for (i = 0; i < m; i++) dotprod(k, bm + i * k * EC_W * EC_W, NULL, k + i, ptrs, size);
  free(bm);
  return 0;
}

int oracle_ec_decode(int k, int m, const int* erased, char** ptrs, const int* sizes, int size) {
  int i, j, alive = 0, n = k * EC_W, rc;
  int dm_ids[EC_MAX];
  int *bm, *tmp, *dec;
  for (i = 0; i < k + m; i++) alive += erased[i] == 0;
  if (alive < k) return EXIT_NO_ENOUGH_DATA;
  for (i = 0, j = 0; j < k; i++)
    if (erased[i] == 0) dm_ids[j++] = i;
  bm = cauchy_bitmatrix(k, m);
  tmp = (int*)calloc((size_t)n * n, sizeof(int));
  dec = (int*)calloc((size_t)n * n, sizeof(int));
  for (i = 0; i < k; i++) {
    if (dm_ids[i] < k) {
      for (j = 0; j < EC_W; j++) tmp[(i * EC_W + j) * n + dm_ids[i] * EC_W + j] = 1;
    } else {
      memcpy(tmp + (size_t)i * EC_W * n, bm + (size_t)(dm_ids[i] - k) * EC_W * n, sizeof(int) * EC_W * n);
    }
  }
  if (invert_bits(tmp, dec, n) < 0) {
    free(bm); free(tmp); free(dec);
    return EXIT_MATRIX_INVALID;
  }
  rc = check(k, m, ptrs, sizes, size);
  if (rc == 0) {
    for (i = 0; i < k; i++)
      if (erased[i]) dotprod(k, dec + (size_t)i * k * EC_W * EC_W, dm_ids, i, ptrs, size);
    for (i = 0; i < m; i++)
      if (erased[k + i] == 1) dotprod(k, bm + (size_t)i * k * EC_W * EC_W, NULL, k + i, ptrs, size);
  }
  free(bm); free(tmp); free(dec);
  return rc;
}
