// Throughput of device-scope atomicAdd on a few hot counters (the one-pass sort's
// run reservations: every tile adds its run length to each of the view's 8 shard
// counters and waits for the old value).  G blocks of 512 threads; lanes 0..K-1 of
// each block add to K counters and store the returned offset; timed with events
// against the same grid without the atomics.
//   hipcc --offload-arch=gfx950 -O3 -o tools/atomic_contention_probe.bin tools/atomic_contention_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// stride: words between counters (1: one cache line, 32: a 128-B line each)
// sets: block b adds to counter set b % sets, the sets set_words apart (other
// memory channels?)
__global__ __launch_bounds__(512) void reserve_kernel(unsigned* ctr, unsigned* out, int K, int stride, int on, int sets,
                                                      int set_words) {
  __shared__ unsigned base[64];
  const int k = threadIdx.x;
  if (k < K) {
    const unsigned n = 200 + (blockIdx.x * 7 + k) % 113;  // a run length
    base[k] = on ? atomicAdd(ctr + (size_t)(blockIdx.x % sets) * set_words + k * stride, n) : n;
  }
  __syncthreads();
  // every lane uses its shard's base (the scatter's dependency)
  if (threadIdx.x < 64) out[blockIdx.x * 64 + threadIdx.x] = base[threadIdx.x % K] + threadIdx.x;
}

int main() {
  unsigned *ctr, *out;
  const size_t ctr_words = (size_t)64 * 16384;
  CK(hipMalloc(&ctr, ctr_words * 4));
  CK(hipMalloc(&out, 8192 * 64 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grids[] = {256, 512, 1024, 2048, 4096};
  struct Cfg { int K, stride, sets, set_words; };
  const Cfg cfgs[] = {{8, 1, 1, 0}, {8, 32, 1, 0}, {64, 32, 1, 0}, {8, 1, 8, 32}, {8, 1, 8, 1024},
                      {8, 1, 8, 16384}, {8, 1, 64, 16384}, {8, 32, 8, 4096}};
  for (const Cfg& c : cfgs)
      for (int G : grids) {
        const int K = c.K, stride = c.stride;
        float us[2];
        for (int on = 0; on < 2; ++on) {
          CK(hipMemset(ctr, 0, ctr_words * 4));
          for (int w = 0; w < 3; ++w)
            hipLaunchKernelGGL(reserve_kernel, dim3(G), dim3(512), 0, 0, ctr, out, K, stride, on, c.sets, c.set_words);
          CK(hipEventRecord(a, 0));
          const int reps = 20;
          for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(reserve_kernel, dim3(G), dim3(512), 0, 0, ctr, out, K, stride, on, c.sets, c.set_words);
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, a, b));
          us[on] = ms * 1000.f / reps;
        }
        printf("{\"counters\": %d, \"stride_words\": %d, \"sets\": %d, \"set_words\": %d, \"blocks\": %d, "
               "\"us_no_atomics\": %.2f, \"us_atomics\": %.2f, \"ns_per_block\": %.1f}\n",
               K, stride, c.sets, c.set_words, G, us[0], us[1], (us[1] - us[0]) * 1000.f / G);
      }
  return 0;
}
