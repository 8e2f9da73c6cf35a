// Host <-> GPU ping-pong floor for the single-call (latency) path: where should
// the request ring live?  One resident lane polls a request word and answers
// into pinned host memory; the host times write -> answer.
//
//   host    : request word in pinned host memory (hipHostMalloc coherent) -- the
//             dispatcher's current ring; every GPU poll is a PCIe read
//   devfine : request word in fine-grained DEVICE memory written by the host
//             through its BAR mapping (hipExtMallocWithFlags finegrained); GPU
//             polls are local
//   devbar  : hipMalloc'd device memory opened to the CPU agent with
//             hsa_amd_agents_allow_access (large-BAR mapping)
//
// Each mode runs in its own child process (forked before any HIP call), so a
// mode the platform does not support (host fault on the mapping) only ends its
// child.  The GPU lane gives up after 2 s without a request (bounded spin).
// build: hipcc --offload-arch=gfx950 -O2 tools/ring_latency_probe.hip -lhsa-runtime64 -o tools/ring_latency_probe.bin
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      fflush(stdout), _exit(3);                                                                        \
    }                                                                                    \
  } while (0)

__global__ void pong_kernel(uint32_t* req, uint32_t* rep, int iters, uint64_t timeout_ticks, int sleep) {
  if (threadIdx.x != 0) return;
  for (int i = 1; i <= iters; ++i) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != (uint32_t)i) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        __hip_atomic_store(rep, 0xdeadu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
      if (sleep) __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(rep, (uint32_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static hsa_agent_t g_cpu{};
static hsa_status_t find_cpu(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU) {
    g_cpu = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

static int run_mode(const char* mode, int sleep) {
  CK(hipSetDevice(0));
  uint32_t* rep;
  CK(hipHostMalloc((void**)&rep, 4096, hipHostMallocCoherent | hipHostMallocMapped));
  uint32_t* req = nullptr;
  if (!strcmp(mode, "host")) {
    CK(hipHostMalloc((void**)&req, 4096, hipHostMallocCoherent | hipHostMallocMapped));
  } else if (!strcmp(mode, "devfine")) {
    CK(hipExtMallocWithFlags((void**)&req, 4096, hipDeviceMallocFinegrained));
  } else {
    CK(hipMalloc((void**)&req, 4096));
    hsa_iterate_agents(find_cpu, nullptr);
    const hsa_status_t st = hsa_amd_agents_allow_access(1, &g_cpu, nullptr, req);
    if (st != HSA_STATUS_SUCCESS) {
      printf("{\"mode\": \"%s\", \"error\": \"hsa_amd_agents_allow_access %d\"}\n", mode, (int)st);
      return 0;
    }
  }
  CK(hipMemset(req, 0, 4096));
  *(volatile uint32_t*)rep = 0;
  // the host write path itself: a fault here ends this child only
  *(volatile uint32_t*)(req + 8) = 1;
  _mm_sfence();
  CK(hipDeviceSynchronize());
  const int iters = 20000;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(pong_kernel, dim3(1), dim3(64), 0, s, req, rep, iters, (uint64_t)200000000, sleep);
  CK(hipGetLastError());
  std::vector<double> lat;
  lat.reserve(iters);
  bool ok = true;
  for (int i = 1; i <= iters && ok; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n((volatile uint32_t*)req, (uint32_t)i, __ATOMIC_RELEASE);
    _mm_sfence();
    while (true) {
      const uint32_t v = __atomic_load_n((volatile uint32_t*)rep, __ATOMIC_ACQUIRE);
      if (v == (uint32_t)i) break;
      if (v == 0xdeadu || std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
        ok = false;
        break;
      }
    }
    lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  CK(hipStreamSynchronize(s));  // the lane exits after iters or its 2 s timeout
  if (!ok) {
    printf("{\"mode\": \"%s\", \"sleep\": %d, \"error\": \"GPU lane never saw the host's write\"}\n", mode, sleep);
    return 0;
  }
  lat.erase(lat.begin(), lat.begin() + 1000);
  std::sort(lat.begin(), lat.end());
  auto q = [&](double f) { return lat[(size_t)(f * (lat.size() - 1))]; };
  printf("{\"mode\": \"%s\", \"sleep\": %d, \"p50_us\": %.3f, \"p90_us\": %.3f, \"p99_us\": %.3f}\n", mode, sleep,
         q(0.5), q(0.9), q(0.99));
  return 0;
}

int main() {
  for (const char* mode : {"host", "devfine", "devbar"})
    for (int sleep : {0, 1}) {
      fflush(stdout);
      const pid_t pid = fork();
      if (pid == 0) {
        const int rc = run_mode(mode, sleep);
        fflush(stdout);
        _exit(rc);
      }
      int st = 0;
      waitpid(pid, &st, 0);
      if (!WIFEXITED(st) || WEXITSTATUS(st))
        printf("{\"mode\": \"%s\", \"sleep\": %d, \"error\": \"child status %d\"}\n", mode, sleep, st);
      fflush(stdout);
    }
  return 0;
}
