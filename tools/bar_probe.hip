// bar_probe.hip -- can the host write device memory directly (large BAR), and how
// fast?  Fine-grained device memory (hipDeviceMallocFinegrained) mapped for the CPU:
// the host copies a body into it with streaming stores, fences, and a kernel reads it
// back with system-coherent loads; the bytes must match on every round (the body
// changes every round).  Prints one JSON object.
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/bar_probe.hip -o tools/bar_probe
#include <hip/hip_runtime.h>
#include <emmintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void sum_kernel(const uint32_t* p, uint32_t n, uint32_t* out) {
  uint32_t s = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) s += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (threadIdx.x == 0) out[0] = s;
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  void* d = nullptr;
  hipError_t e = hipExtMallocWithFlags(&d, 1 << 20, hipDeviceMallocFinegrained);
  if (e != hipSuccess) {
    printf("{\"alloc\": \"%s\"}\n", hipGetErrorString(e));
    return 0;
  }
  hipPointerAttribute_t a{};
  (void)hipPointerGetAttributes(&a, d);
  uint32_t* out = nullptr;
  (void)hipHostMalloc(reinterpret_cast<void**>(&out), 64, hipHostMallocCoherent | hipHostMallocMapped);
  std::vector<uint32_t> src(1024);
  int bad = 0;
  std::vector<double> wr_us[3];
  const uint32_t sizes[3] = {256, 1024, 4096};
  for (int round = 0; round < 300; ++round) {
    for (int k = 0; k < 3; ++k) {
      const uint32_t bytes = sizes[k], n = bytes / 4;
      uint32_t want = 0;
      for (uint32_t i = 0; i < n; ++i) want += (src[i] = uint32_t(round * 2654435761u + i * 40503u + k));
      const auto t0 = std::chrono::steady_clock::now();
      for (uint32_t i = 0; i < n; i += 4)
        _mm_stream_si128(reinterpret_cast<__m128i*>(static_cast<uint32_t*>(d) + i),
                         _mm_loadu_si128(reinterpret_cast<const __m128i*>(&src[i])));
      _mm_sfence();
      const auto t1 = std::chrono::steady_clock::now();
      wr_us[k].push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      out[0] = 0;
      hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(64), 0, 0, static_cast<const uint32_t*>(d), n, out);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("{\"kernel\": \"failed\"}\n");
        return 1;
      }
      bad += out[0] != want;
    }
  }
  printf("{\"alloc\": \"ok\", \"type\": %d, \"host_ptr_same\": %d, \"mismatches\": %d, \"write_us_p50\": {\"256\": %.3f, \"1024\": %.3f, \"4096\": %.3f}}\n",
         int(a.type), int(a.hostPointer == d), bad, med(wr_us[0]), med(wr_us[1]), med(wr_us[2]));
  return 0;
}
