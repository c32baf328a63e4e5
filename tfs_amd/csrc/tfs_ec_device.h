// tfs_ec_device.h -- launch arguments shared by tfs_ec_kernels.hip and tfs_ec_abi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tfsec {

constexpr int kMaxMembersDev = 12;  // MAX_MARSHALLING_NUM
constexpr int kMaxOutGroup = 4;     // outputs accumulated in registers per launch

struct EcArgs {
  const uint8_t* src[kMaxMembersDev];
  uint8_t* dst[kMaxOutGroup];
  const uint32_t* masks;  // [OG][8][S][8] words (0 or 0xffffffff) for this launch's outputs
  uint32_t S;
  uint64_t units;         // size / 1024
};

hipError_t launch_ec_apply(const EcArgs& a, int og, int variant, hipStream_t stream);

}  // namespace tfsec
