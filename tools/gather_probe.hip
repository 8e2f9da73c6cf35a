// Directory-gather floor on MI355X: what one random 4-B lookup per message costs
// against a streaming copy of the same column.  Every mailbox / exchange Send
// resolves each message's actor through the route directory, so this is the
// floor under the count / enqueue passes.
//
//   copy       out[i] = act[i]                       (8 Mi u32: 33 MB read + 33 MB written)
//   gather     out[i] = dir[act[i]]   dir 512 KB     (131072 actors: the bench's registry)
//   gather4m   out[i] = dir[act[i]]   dir 4 MB       (1 Mi actors)
//   lds8       out[i] = sdir[act[i]]  1-B shard table of 131072 actors staged in LDS
//              (128 KB per block, one persistent block per CU)
//
// build: hipcc -O3 --offload-arch=gfx950 tools/gather_probe.hip -o /tmp/gather_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));           \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

template <int IPT>
__global__ __launch_bounds__(256) void copy_k(const uint32_t* __restrict__ a, uint32_t* __restrict__ o, int64_t n) {
  const int64_t b = (int64_t)blockIdx.x * 256 * IPT + threadIdx.x;
  uint32_t v[IPT];
#pragma unroll
  for (int k = 0; k < IPT; ++k) v[k] = b + k * 256 < n ? __builtin_nontemporal_load(a + b + k * 256) : 0u;
#pragma unroll
  for (int k = 0; k < IPT; ++k)
    if (b + k * 256 < n) o[b + k * 256] = v[k];
}

template <int IPT>
__global__ __launch_bounds__(256) void gather_k(const uint32_t* __restrict__ a, const uint32_t* __restrict__ dir,
                                                uint32_t* __restrict__ o, int64_t n) {
  const int64_t b = (int64_t)blockIdx.x * 256 * IPT + threadIdx.x;
  uint32_t v[IPT];
#pragma unroll
  for (int k = 0; k < IPT; ++k) v[k] = b + k * 256 < n ? __builtin_nontemporal_load(a + b + k * 256) : 0u;
#pragma unroll
  for (int k = 0; k < IPT; ++k) v[k] = dir[v[k]];
#pragma unroll
  for (int k = 0; k < IPT; ++k)
    if (b + k * 256 < n) o[b + k * 256] = v[k];
}

// persistent: one 1024-thread block per CU stages the 1-B table, then strides the batch
__global__ __launch_bounds__(1024) void lds8_k(const uint32_t* __restrict__ a, const uint8_t* __restrict__ sdir,
                                               uint32_t nd, uint32_t* __restrict__ o, int64_t n) {
  extern __shared__ __align__(16) uint8_t t[];
  for (uint32_t j = threadIdx.x * 16; j < nd; j += blockDim.x * 16)
    *reinterpret_cast<uint4*>(t + j) = *reinterpret_cast<const uint4*>(sdir + j);
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 8;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x * 8 + threadIdx.x; b < n; b += stride) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = b + k * 1024 < n ? __builtin_nontemporal_load(a + b + k * 1024) : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = t[v[k]];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (b + k * 1024 < n) o[b + k * 1024] = v[k];
  }
}

int main() {
  const int64_t n = 8 << 20;
  const uint32_t nd_small = 131072, nd_big = 1 << 20;
  std::vector<uint32_t> h(n), hs(n), dirh(nd_big);
  uint64_t x = 88172645463325252ull;
  for (int64_t i = 0; i < n; ++i) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    h[i] = (uint32_t)(x % nd_big);
    hs[i] = (uint32_t)(x % nd_small);
  }
  for (uint32_t i = 0; i < nd_big; ++i) dirh[i] = i * 2654435761u;
  uint32_t *a, *as, *dir, *o;
  uint8_t* sdir;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&as, n * 4));
  CK(hipMalloc(&o, n * 4));
  CK(hipMalloc(&dir, nd_big * 4));
  CK(hipMalloc(&sdir, nd_small));
  CK(hipMemcpy(a, h.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(as, hs.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dir, dirh.data(), nd_big * 4, hipMemcpyHostToDevice));
  CK(hipMemset(sdir, 3, nd_small));
  CK(hipFuncSetAttribute((const void*)lds8_k, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    for (int r = 0; r < 3; ++r) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int reps = 20;
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %8.2f us\n", name, ms * 1000 / reps);
  };
  for (int ipt : {1, 2, 4, 8}) {
    const int64_t g = (n + 256 * ipt - 1) / (256 * ipt);
    char nm[64];
    snprintf(nm, sizeof nm, "copy ipt=%d", ipt);
    timeit(nm, [&] {
      if (ipt == 1) hipLaunchKernelGGL(copy_k<1>, dim3(g), dim3(256), 0, 0, a, o, n);
      if (ipt == 2) hipLaunchKernelGGL(copy_k<2>, dim3(g), dim3(256), 0, 0, a, o, n);
      if (ipt == 4) hipLaunchKernelGGL(copy_k<4>, dim3(g), dim3(256), 0, 0, a, o, n);
      if (ipt == 8) hipLaunchKernelGGL(copy_k<8>, dim3(g), dim3(256), 0, 0, a, o, n);
    });
    snprintf(nm, sizeof nm, "gather512k ipt=%d", ipt);
    timeit(nm, [&] {
      if (ipt == 1) hipLaunchKernelGGL(gather_k<1>, dim3(g), dim3(256), 0, 0, as, dir, o, n);
      if (ipt == 2) hipLaunchKernelGGL(gather_k<2>, dim3(g), dim3(256), 0, 0, as, dir, o, n);
      if (ipt == 4) hipLaunchKernelGGL(gather_k<4>, dim3(g), dim3(256), 0, 0, as, dir, o, n);
      if (ipt == 8) hipLaunchKernelGGL(gather_k<8>, dim3(g), dim3(256), 0, 0, as, dir, o, n);
    });
    snprintf(nm, sizeof nm, "gather4m ipt=%d", ipt);
    timeit(nm, [&] {
      if (ipt == 1) hipLaunchKernelGGL(gather_k<1>, dim3(g), dim3(256), 0, 0, a, dir, o, n);
      if (ipt == 2) hipLaunchKernelGGL(gather_k<2>, dim3(g), dim3(256), 0, 0, a, dir, o, n);
      if (ipt == 4) hipLaunchKernelGGL(gather_k<4>, dim3(g), dim3(256), 0, 0, a, dir, o, n);
      if (ipt == 8) hipLaunchKernelGGL(gather_k<8>, dim3(g), dim3(256), 0, 0, a, dir, o, n);
    });
  }
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  timeit("lds8 (1 block/CU)", [&] { hipLaunchKernelGGL(lds8_k, dim3(cus), dim3(1024), 131072, 0, as, sdir, nd_small, o, n); });
  CK(hipDeviceSynchronize());
  return 0;
}
