// Snapshot staging copy: device buffer -> contiguous staging
// buffer (HBM or pinned host memory mapped into the GPU) with 16-byte-per-lane
// non-temporal loads, so a snapshot of actor state / the registry mirror does
// not evict the routing working set from L2 / Infinity Cache.
#include "common.hpp"

namespace ptype {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void snapshot_copy_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                            int64_t n16) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = __builtin_nontemporal_load(src + i);
}

void launch_snapshot_copy(uintptr_t dst, uintptr_t src, int64_t n16, uintptr_t stream) {
  if (n16 <= 0) return;
  int64_t g = (n16 + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(snapshot_copy_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), (u32x4*)dst,
                     (const u32x4*)src, n16);
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
