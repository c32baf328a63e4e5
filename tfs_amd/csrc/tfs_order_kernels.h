// tfs_order_kernels.h -- size-ordered launches for crc_files_kernel (included
// by tfs_crc_kernels.hip).  A counting sort of the descriptors by size class
// floor(log2(len)), largest class first (LPT: no wave starts a big file after
// the rest of the grid has drained).  Three small kernels over the 16-byte
// descriptors: count per class, counts -> cursors, scatter.  Order inside a
// class is arbitrary (no result depends on it).  One class only (uniform
// sizes): the flag stays 0 and the CRC kernel keeps the identity order.
#pragma once

namespace tfscrc {

__device__ __forceinline__ uint32_t size_class(uint32_t len) { return 31u - __builtin_clz(len | 1u); }

__global__ void __launch_bounds__(1024) order_count_kernel(const Desc* __restrict__ desc, uint32_t n,
                                                           uint32_t* __restrict__ ctr) {
  __shared__ uint32_t h[kSizeClasses];
  if (threadIdx.x < kSizeClasses) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    atomicAdd(&h[size_class(desc[i].len)], 1u);
  __syncthreads();
  if (threadIdx.x < kSizeClasses && h[threadIdx.x]) atomicAdd(&ctr[threadIdx.x * kOrderStride], h[threadIdx.x]);
}

__global__ void order_scan_kernel(uint32_t* __restrict__ ctr) {
  if (threadIdx.x != 0) return;
  uint32_t run = 0, classes = 0;
  for (int c = int(kSizeClasses) - 1; c >= 0; --c) {
    const uint32_t k = ctr[c * kOrderStride];
    ctr[c * kOrderStride] = run;
    run += k;
    classes += k ? 1u : 0u;
  }
  ctr[kSizeClasses * kOrderStride] = classes > 1u ? 1u : 0u;
}

// One descriptor per thread; per workgroup one global atomic per class.
__global__ void __launch_bounds__(1024) order_scatter_kernel(const Desc* __restrict__ desc, uint32_t n,
                                                             uint32_t* __restrict__ ctr, uint32_t* __restrict__ order) {
  if (ctr[kSizeClasses * kOrderStride] == 0u) return;
  __shared__ uint32_t h[kSizeClasses], base[kSizeClasses];
  if (threadIdx.x < kSizeClasses) h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c = 0, r = 0;
  if (i < n) {
    c = size_class(desc[i].len);
    r = atomicAdd(&h[c], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kSizeClasses && h[threadIdx.x])
    base[threadIdx.x] = atomicAdd(&ctr[threadIdx.x * kOrderStride], h[threadIdx.x]);
  __syncthreads();
  if (i < n) order[base[c] + r] = i;
}

}  // namespace tfscrc
