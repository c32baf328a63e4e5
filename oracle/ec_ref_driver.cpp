// oracle/ec_ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
// Drives the reference's own vendored jerasure/galois sources (compiled from
// /root/reference/src/dataserver by build_ref.sh, never copied) the way
// ErasureCode::config/encode/decode do (erasure_code.cpp:49-235; that file
// itself needs tbsys and cannot be built here, so its dozen lines of glue are
// restated in this driver), to produce golden vectors for tests/golden/.
#include <cstdlib>
#include <cstring>

#include "galois.h"
#include "jerasure.h"

extern "C" int ref_ec_encode(int k, int m, char** ptrs, int size) {
  int* matrix = new int[k * m];
  for (int i = 0; i < m; i++)
    for (int j = 0; j < k; j++) matrix[i * k + j] = galois_single_divide(1, i ^ (m + j), 8);
  int* bm = jerasure_matrix_to_bitmatrix(k, m, 8, matrix);
  delete[] matrix;
  jerasure_bitmatrix_encode(k, m, 8, bm, ptrs, ptrs + k, size, 128);
  free(bm);
  return 0;
}

extern "C" int ref_ec_decode(int k, int m, int* erased, char** ptrs, int size) {
  int* matrix = new int[k * m];
  for (int i = 0; i < m; i++)
    for (int j = 0; j < k; j++) matrix[i * k + j] = galois_single_divide(1, i ^ (m + j), 8);
  int* bm = jerasure_matrix_to_bitmatrix(k, m, 8, matrix);
  delete[] matrix;
  int alive = 0;
  for (int i = 0; i < k + m; i++) alive += erased[i] == 0;
  if (alive < k) {
    free(bm);
    return -16004;
  }
  int* dec = new int[k * k * 64];
  int dm_ids[16];
  if (jerasure_make_decoding_bitmatrix(k, m, 8, bm, erased, dec, dm_ids) < 0) {
    delete[] dec;
    free(bm);
    return -16003;
  }
  for (int i = 0; i < k; i++)
    if (erased[i]) jerasure_bitmatrix_dotprod(k, 8, dec + i * k * 64, dm_ids, i, ptrs, ptrs + k, size, 128);
  for (int i = 0; i < m; i++)
    if (erased[k + i] == 1) jerasure_bitmatrix_dotprod(k, 8, bm + i * k * 64, NULL, k + i, ptrs, ptrs + k, size, 128);
  delete[] dec;
  free(bm);
  return 0;
}
