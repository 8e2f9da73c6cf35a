// The optimus coordinator's gather on the device (BASELINE config 4).
//
// Reference: example/optimus/coordinator/coordinator.go:91-98 (watchReplies):
// the first reply that is not the target wins, else the target (prime).  The
// fan-out is one Send of every target's 10-wide ranges (splitWork, :67-73);
// its replies come back in message order, so target j's ranges are a
// contiguous run [first[j], first[j] + n[j]) in ascending range order and the
// first non-target reply in that order is the smallest divisor -- the answer
// the reference's gather returns once every range has replied.
//
// One wave per target scans its run 64 replies at a time and stops at the
// first hit (early exit: the rest of the run is never read).  A reply whose
// status is not OK before the hit fails the target (the reference log.Fatal()s
// on a failed Call, :85-88): out_st gets that status.
#include "common.hpp"

namespace ptype {

__global__ __launch_bounds__(256) void prime_gather_kernel(const int64_t* __restrict__ val,
                                                           const int32_t* __restrict__ st,
                                                           const int64_t* __restrict__ first,
                                                           const int64_t* __restrict__ n,
                                                           const int64_t* __restrict__ target, int64_t T,
                                                           int64_t* __restrict__ out, int32_t* __restrict__ out_st,
                                                           unsigned long long* __restrict__ scanned) {
  const int64_t j = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  if (j >= T) return;  // (wave-uniform)
  const unsigned lane = lane_id();
  const int64_t f = first[j], cnt = n[j], tg = target[j];
  int64_t ans = tg;
  int32_t status = kStatusOk;
  int64_t read = 0;
  for (int64_t b = 0; b < cnt; b += kWave) {
    const int64_t i = b + lane;
    const bool in = i < cnt;
    const int64_t v = in ? val[f + i] : tg;
    const int32_t s = in ? st[f + i] : kStatusOk;
    read += in;
    const uint64_t bad = __ballot(s != kStatusOk), hit = __ballot(s == kStatusOk && v != tg);
    const uint64_t stop = bad | hit;
    if (stop) {
      const int k = __builtin_ctzll(stop);  // the first reply in range order that decides
      if ((bad >> k) & 1) status = __shfl(s, k);
      else ans = __shfl(v, k);
      break;
    }
  }
  if (lane == 0) {
    out[j] = ans;
    out_st[j] = status;
  }
  if (scanned) {
    for (int off = 32; off > 0; off >>= 1) read += __shfl_xor(read, off);
    if (lane == 0) atomicAdd(scanned, (unsigned long long)read);
  }
}

void launch_prime_gather(uintptr_t val, uintptr_t st, uintptr_t first, uintptr_t n, uintptr_t target, int64_t T,
                         uintptr_t out, uintptr_t out_st, uintptr_t scanned, uintptr_t stream) {
  if (T <= 0) return;
  const int per = 256 / kWave;
  hipLaunchKernelGGL(prime_gather_kernel, dim3((unsigned)((T + per - 1) / per)), dim3(256), 0, as_stream(stream),
                     (const int64_t*)val, (const int32_t*)st, (const int64_t*)first, (const int64_t*)n,
                     (const int64_t*)target, T, (int64_t*)out, (int32_t*)out_st, (unsigned long long*)scanned);
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
