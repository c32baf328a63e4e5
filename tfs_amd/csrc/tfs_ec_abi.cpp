// tfs_ec_abi.cpp -- host side of include/tfs_ec.h: ErasureCode's setup on the
// host (ec_math.h), the region work on the GPU (tfs_ec_kernels.hip).  No CPU
// fallback: without a device every call fails with the ctx's error.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/tfs_ec.h"
#include "ec_math.h"

#include "tfs_ec_device.h"

extern "C" int tfs_crc32_dev_malloc(tfs_crc_ctx* ctx, uint64_t bytes, void** d_ptr);
extern "C" int tfs_crc32_dev_free(tfs_crc_ctx* ctx, void* d_ptr);
extern "C" void* tfs_crc32_stream(tfs_crc_ctx* ctx);

using namespace tfsec;

namespace {
// One launch plan: sources, outputs, expanded masks [O][8][S][8] (device).
struct Plan {
  std::vector<int> sources, outputs;
  uint32_t* d_masks = nullptr;
  bool valid = false;
};
}  // namespace

struct tfs_ec {
  tfs_crc_ctx* ctx = nullptr;
  int dn = 0, pn = 0;
  Plan enc, dec;
  int config_rc = TFS_SUCCESS;
  std::mutex mu;
  std::vector<void*> staging;  // host-form device buffers (dn+pn), grown on demand
  std::vector<uint64_t> staging_cap;
  int variant = 0;  // kernel form (TFS_EC_VARIANT at creation, measurement knob; 0 = product)
};

namespace {

int upload_plan(tfs_ec* ec, Plan* p, const std::vector<int>& sources, const std::vector<int>& outputs,
                const BitMat& rows) {
  const int S = int(sources.size()), O = int(outputs.size());
  const int cols = S * kW;
  std::vector<uint32_t> m(size_t(O) * 8 * S * 8);
  for (int o = 0; o < O; ++o)
    for (int r = 0; r < 8; ++r)
      for (int s = 0; s < S; ++s)
        for (int c = 0; c < 8; ++c)
          m[((size_t(o) * 8 + r) * S + s) * 8 + c] = rows[size_t(o * kW + r) * cols + s * kW + c] ? 0xFFFFFFFFu : 0u;
  void* d = nullptr;
  int rc = tfs_crc32_dev_malloc(ec->ctx, m.size() * 4 + 4, &d);
  if (rc) return rc;
  if (hipMemcpy(d, m.data(), m.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    tfs_crc32_dev_free(ec->ctx, d);
    return TFS_CRC_EXIT_DEVICE_ERROR;
  }
  p->sources = sources;
  p->outputs = outputs;
  p->d_masks = static_cast<uint32_t*>(d);
  p->valid = true;
  return TFS_SUCCESS;
}

// Checks of ErasureCode::encode/decode (erasure_code.cpp:145-172, 181-201).
int check_call(tfs_ec* ec, const Plan& p, void* const* members, const int* sizes, int size) {
  if (!p.valid) return TFS_EXIT_MATRIX_INVALID;
  if (size < 0 || size % kUnit != 0) return TFS_EXIT_SIZE_INVALID;
  if (!members) return TFS_EXIT_DATA_INVALID;
  for (int i = 0; i < ec->dn + ec->pn; ++i)
    if (!members[i] || (sizes && sizes[i] < size)) return TFS_EXIT_DATA_INVALID;
  return TFS_SUCCESS;
}

int run_plan(tfs_ec* ec, const Plan& p, void* const* members, int size, hipStream_t st) {
  const uint64_t units = uint64_t(size) / kUnit;
  if (units == 0 || p.outputs.empty()) return TFS_SUCCESS;
  const int S = int(p.sources.size());
  for (size_t o0 = 0; o0 < p.outputs.size(); o0 += 4) {
    const int og = int(std::min<size_t>(4, p.outputs.size() - o0));
    EcArgs a;
    memset(&a, 0, sizeof a);
    for (int s = 0; s < S; ++s) a.src[s] = static_cast<const uint8_t*>(members[p.sources[s]]);
    for (int o = 0; o < og; ++o) a.dst[o] = static_cast<uint8_t*>(members[p.outputs[o0 + o]]);
    a.masks = p.d_masks + o0 * 8 * size_t(S) * 8;
    a.S = uint32_t(S);
    a.units = units;
    if (launch_ec_apply(a, og, ec->variant, st) != hipSuccess) return TFS_CRC_EXIT_DEVICE_ERROR;
  }
  return TFS_SUCCESS;
}

// Host form: members staged through device buffers; sources up, outputs down.
int run_host(tfs_ec* ec, const Plan& p, char* const* members, const int* sizes, int size) {
  std::lock_guard<std::mutex> g(ec->mu);
  void* const* mv = reinterpret_cast<void* const*>(members);
  int rc = check_call(ec, p, mv, sizes, size);
  if (rc) return rc;
  const int n = ec->dn + ec->pn;
  if (ec->staging.empty()) {
    ec->staging.assign(n, nullptr);
    ec->staging_cap.assign(n, 0);
  }
  hipStream_t st = static_cast<hipStream_t>(tfs_crc32_stream(ec->ctx));
  std::vector<void*> dm(n, nullptr);
  auto need = [&](int i) -> int {
    if (ec->staging_cap[i] < uint64_t(size)) {
      if (ec->staging[i]) tfs_crc32_dev_free(ec->ctx, ec->staging[i]);
      ec->staging[i] = nullptr;
      ec->staging_cap[i] = 0;
      const int r = tfs_crc32_dev_malloc(ec->ctx, uint64_t(size) + 64, &ec->staging[i]);
      if (r) return r;
      ec->staging_cap[i] = uint64_t(size);
    }
    dm[i] = ec->staging[i];
    return TFS_SUCCESS;
  };
  for (int s : p.sources) {
    if ((rc = need(s))) return rc;
    if (hipMemcpyAsync(dm[s], members[s], size_t(size), hipMemcpyHostToDevice, st) != hipSuccess)
      return TFS_CRC_EXIT_DEVICE_ERROR;
  }
  for (int o : p.outputs)
    if ((rc = need(o))) return rc;
  for (int i = 0; i < n; ++i)
    if (!dm[i]) dm[i] = ec->staging[p.sources[0]];  // members the plan does not touch
  rc = run_plan(ec, p, dm.data(), size, st);
  if (rc) return rc;
  for (int o : p.outputs)
    if (hipMemcpyAsync(members[o], dm[o], size_t(size), hipMemcpyDeviceToHost, st) != hipSuccess)
      return TFS_CRC_EXIT_DEVICE_ERROR;
  return hipStreamSynchronize(st) == hipSuccess ? TFS_SUCCESS : TFS_CRC_EXIT_DEVICE_ERROR;
}

}  // namespace

extern "C" {

int tfs_ec_config(tfs_crc_ctx* ctx, int dn, int pn, const int* erased, tfs_ec** out) {
  if (!ctx || !out) return TFS_EXIT_PARAMETER_ERROR;
  *out = nullptr;
  if (dn <= 0 || pn <= 0 || dn + pn > kMaxMembers) return TFS_EXIT_PARAMETER_ERROR;
  tfs_ec* ec = new tfs_ec();
  ec->ctx = ctx;
  ec->dn = dn;
  ec->pn = pn;
#ifdef TFS_CRC_MEASURE
  if (const char* v = getenv("TFS_EC_VARIANT")) ec->variant = atoi(v);
#endif
  *out = ec;
  std::vector<int> data(dn), parity(pn);
  for (int j = 0; j < dn; ++j) data[j] = j;
  for (int i = 0; i < pn; ++i) parity[i] = dn + i;
  int rc = upload_plan(ec, &ec->enc, data, parity, encode_bitmatrix(dn, pn));
  if (rc == TFS_SUCCESS && erased) {
    DecodePlan dp;
    const int r = make_decode_plan(dn, pn, erased, &dp);
    if (r == -1) rc = TFS_EXIT_NO_ENOUGH_DATA;
    else if (r == -2) rc = TFS_EXIT_MATRIX_INVALID;
    else rc = upload_plan(ec, &ec->dec, dp.sources, dp.outputs, dp.rows);
  }
  ec->config_rc = rc;
  return rc;
}

int tfs_ec_free(tfs_ec* ec) {
  if (!ec) return TFS_EXIT_PARAMETER_ERROR;
  (void)hipStreamSynchronize(static_cast<hipStream_t>(tfs_crc32_stream(ec->ctx)));
  if (ec->enc.d_masks) tfs_crc32_dev_free(ec->ctx, ec->enc.d_masks);
  if (ec->dec.d_masks) tfs_crc32_dev_free(ec->ctx, ec->dec.d_masks);
  for (void* p : ec->staging)
    if (p) tfs_crc32_dev_free(ec->ctx, p);
  delete ec;
  return TFS_SUCCESS;
}

int tfs_ec_encode_device(tfs_ec* ec, void* const* d_members, const int* sizes, int size, void* stream) {
  if (!ec) return TFS_EXIT_PARAMETER_ERROR;
  const int rc = check_call(ec, ec->enc, d_members, sizes, size);
  if (rc) return rc;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : static_cast<hipStream_t>(tfs_crc32_stream(ec->ctx));
  return run_plan(ec, ec->enc, d_members, size, st);
}

int tfs_ec_decode_device(tfs_ec* ec, void* const* d_members, const int* sizes, int size, void* stream) {
  if (!ec) return TFS_EXIT_PARAMETER_ERROR;
  const int rc = check_call(ec, ec->dec, d_members, sizes, size);
  if (rc) return rc;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : static_cast<hipStream_t>(tfs_crc32_stream(ec->ctx));
  return run_plan(ec, ec->dec, d_members, size, st);
}

int tfs_ec_encode(tfs_ec* ec, char* const* members, const int* sizes, int size) {
  if (!ec) return TFS_EXIT_PARAMETER_ERROR;
  return run_host(ec, ec->enc, members, sizes, size);
}

int tfs_ec_decode(tfs_ec* ec, char* const* members, const int* sizes, int size) {
  if (!ec) return TFS_EXIT_PARAMETER_ERROR;
  return run_host(ec, ec->dec, members, sizes, size);
}

}  // extern "C"
