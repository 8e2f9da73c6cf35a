// Cost of cross-stream hand-offs between back-to-back kernels on gfx950: the
// epoch engine orders its compute and comm streams with HIP events (4 per chunk),
// and a loopback R = 8 kernel trace shows 6-14 us idle gaps exactly there.
//
// Modes (40 copy kernels of ~10 us each):
//   plain     : kernels back-to-back on one stream
//   record    : + hipEventRecord after every kernel (same stream, nobody waits)
//   handoff   : + another stream waits on every event (no work there)
//   pingpong  : kernels alternate between two streams, each waiting on the other's event
//   waitvalue : pingpong ordered by hipStreamWriteValue32 / hipStreamWaitValue32 on a flag word
// for event flags default, DisableSystemFence, ReleaseToDevice.
//
// build: hipcc --offload-arch=gfx950 -O2 tools/event_gap_bench.hip -o build/event_gap_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

int main() {
  const size_t bytes = 32ull << 20, n = bytes / 16;
  uint4 *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  uint32_t* flag;
  CK(hipMalloc(&flag, 4096));
  CK(hipMemset(flag, 0, 4096));
  const int K = 40;
  const unsigned flag_sets[3] = {hipEventDisableTiming, hipEventDisableTiming | hipEventDisableSystemFence,
                                 hipEventDisableTiming | hipEventReleaseToDevice};
  const char* flag_names[3] = {"default", "no-system-fence", "release-to-device"};
  auto launch = [&](hipStream_t s) { copy_kernel<<<2048, 256, 0, s>>>(a, b, n); };
  uint32_t seq = 0;
  auto run = [&](int mode, unsigned fl) {
    std::vector<hipEvent_t> ev(2 * K);
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, fl));
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < K; ++k) {
      hipStream_t s = (mode >= 3 && (k & 1)) ? s2 : s1;
      launch(s);
      if (mode == 1) CK(hipEventRecord(ev[k], s));
      if (mode == 2) {
        CK(hipEventRecord(ev[k], s1));
        CK(hipStreamWaitEvent(s2, ev[k], 0));
      }
      if (mode == 3) {
        hipStream_t o = (k & 1) ? s1 : s2;
        CK(hipEventRecord(ev[k], s));
        CK(hipStreamWaitEvent(o, ev[k], 0));
      }
      if (mode == 4) {
        hipStream_t o = (k & 1) ? s1 : s2;
        ++seq;
        CK(hipStreamWriteValue32(s, flag, seq, 0));
        CK(hipStreamWaitValue32(o, flag, seq, hipStreamWaitValueGte, 0xffffffffu));
      }
    }
    CK(hipStreamSynchronize(s1));
    CK(hipStreamSynchronize(s2));
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    for (auto& e : ev) CK(hipEventDestroy(e));
    return us / K;
  };
  const char* modes[5] = {"plain", "record", "handoff", "pingpong", "waitvalue"};
  for (int rep = 0; rep < 2; ++rep)  // first pass warms up
    for (int m = 0; m < 5; ++m)
      for (int f = 0; f < 3; ++f) {
        if ((m == 0 || m == 4) && f) continue;
        const double us = run(m, flag_sets[f]);
        if (rep) printf("{\"mode\": \"%s\", \"event_flags\": \"%s\", \"us_per_kernel\": %.2f}\n", modes[m],
                        flag_names[f], us);
      }
  return 0;
}
