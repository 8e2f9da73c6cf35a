// Cross-process single-call floor: can a client PROCESS write a
// request word that lives in another process's DEVICE memory, so the server's
// polling lane never reads host memory?
//
// server : one fine-grained device word (hipExtMallocWithFlags finegrained),
//          exported with hipIpcGetMemHandle through a POSIX shm segment; one
//          resident lane echoes every new value of the word into a reply word
//          in that shm segment (registered with HIP, mapped).
// client : hipIpcOpenMemHandle on the handle, then the CPU writes the imported
//          word directly (mode "ipc"), or after hsa_amd_agents_allow_access
//          (mode "ipc-allow"); "shm" is the old path -- the request word in the
//          shm segment itself, polled by the GPU over PCIe.
//
// Every role runs in its own child process forked before any HIP call, so a
// client mode the platform does not support (host fault on the mapping) ends
// that child only.  The server lane gives up after 2 s without a request and
// the server relaunches it until told to stop (bounded).
// build: hipcc --offload-arch=gfx950 -O2 tools/ipc_ring_probe.hip -lhsa-runtime64 -o tools/ipc_ring_probe.bin
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <errno.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <sys/un.h>
#include <sys/select.h>
#include <sys/wait.h>
#include <unistd.h>

#include <stddef.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      fflush(stdout), _exit(3);                                                          \
    }                                                                                    \
  } while (0)

struct alignas(64) Shared {
  hipIpcMemHandle_t handle;
  std::atomic<uint32_t> ready, stop, mode_shm, pad;
  int32_t pid, dmabuf_fd;
  uint64_t dmabuf_off;
  int32_t dmabuf_status, pad2;
  alignas(64) uint32_t rep;      // written by the GPU lane
  alignas(64) uint32_t shm_req;  // the "shm" mode's request word
};

__global__ void echo_kernel(uint32_t* req, uint32_t* rep, uint32_t last, uint64_t idle_ticks, uint32_t* out_last) {
  if (threadIdx.x != 0) return;
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const uint32_t v = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v != last) {
      __hip_atomic_store(rep, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      last = v;
      t0 = __builtin_amdgcn_s_memrealtime();
      continue;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
    __builtin_amdgcn_s_sleep(1);
  }
  __hip_atomic_store(out_last, last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

// dma-buf fd hand-off over an abstract unix socket (SCM_RIGHTS): works between
// sibling processes, where pidfd_getfd needs ptrace rights (Yama scope 1 denies it).
static sockaddr_un abstract_addr(int pid, socklen_t* len) {
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  const int n = snprintf(a.sun_path + 1, sizeof(a.sun_path) - 1, "ptype-ipc-probe-%d", pid);
  *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n);
  return a;
}

static void serve_fd(int fd, Shared* sh) {
  const int ls = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  socklen_t len;
  sockaddr_un a = abstract_addr(getpid(), &len);
  if (ls < 0 || bind(ls, (sockaddr*)&a, len) != 0 || listen(ls, 8) != 0) {
    fprintf(stderr, "server: fd socket: %s\n", strerror(errno));
    return;
  }
  while (!sh->stop.load()) {
    timeval tv{0, 200000};
    fd_set rs;
    FD_ZERO(&rs);
    FD_SET(ls, &rs);
    if (select(ls + 1, &rs, nullptr, nullptr, &tv) <= 0) continue;
    const int c = accept(ls, nullptr, nullptr);
    if (c < 0) continue;
    char b = 'f';
    iovec io{&b, 1};
    char ctl[CMSG_SPACE(sizeof(int))] = {};
    msghdr m{};
    m.msg_iov = &io;
    m.msg_iovlen = 1;
    m.msg_control = ctl;
    m.msg_controllen = sizeof ctl;
    cmsghdr* cm = CMSG_FIRSTHDR(&m);
    cm->cmsg_level = SOL_SOCKET;
    cm->cmsg_type = SCM_RIGHTS;
    cm->cmsg_len = CMSG_LEN(sizeof(int));
    memcpy(CMSG_DATA(cm), &fd, sizeof(int));
    if (sendmsg(c, &m, 0) != 1) fprintf(stderr, "server: sendmsg: %s\n", strerror(errno));
    close(c);
  }
  close(ls);
}

static int recv_fd(int pid) {
  const int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  socklen_t len;
  sockaddr_un a = abstract_addr(pid, &len);
  if (s < 0 || connect(s, (sockaddr*)&a, len) != 0) return -1;
  char b = 0;
  iovec io{&b, 1};
  char ctl[CMSG_SPACE(sizeof(int))] = {};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = ctl;
  m.msg_controllen = sizeof ctl;
  int fd = -1;
  if (recvmsg(s, &m, 0) == 1)
    for (cmsghdr* cm = CMSG_FIRSTHDR(&m); cm; cm = CMSG_NXTHDR(&m, cm))
      if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) memcpy(&fd, CMSG_DATA(cm), sizeof(int));
  close(s);
  return fd;
}

static int server(Shared* sh) {
  CK(hipSetDevice(0));
  CK(hipHostRegister(sh, sizeof(Shared), hipHostRegisterMapped));
  Shared* dsh = nullptr;
  CK(hipHostGetDevicePointer((void**)&dsh, sh, 0));
  uint32_t* req = nullptr;
  CK(hipExtMallocWithFlags((void**)&req, 4096, hipDeviceMallocFinegrained));
  CK(hipMemset(req, 0, 4096));
  CK(hipDeviceSynchronize());
  CK(hipIpcGetMemHandle(&sh->handle, req));
  sh->pid = (int32_t)getpid();
  int fd = -1;
  uint64_t off = 0;
  sh->dmabuf_status = (int32_t)hsa_amd_portable_export_dmabuf(req, 4096, &fd, &off);
  sh->dmabuf_fd = fd;
  sh->dmabuf_off = off;
  std::thread fd_thread([fd, sh] { if (fd >= 0) serve_fd(fd, sh); });
  uint32_t* last = nullptr;
  CK(hipHostMalloc((void**)&last, 64, hipHostMallocCoherent | hipHostMallocMapped));
  *last = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  sh->ready.store(1);
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(60);
  uint32_t cur_shm = 2;  // unknown
  while (!sh->stop.load() && std::chrono::steady_clock::now() < t_end) {
    const uint32_t m = sh->mode_shm.load();
    uint32_t* word = m ? &dsh->shm_req : req;
    if (m != cur_shm) {
      cur_shm = m;
      *last = m ? sh->shm_req : 0;
    }
    hipLaunchKernelGGL(echo_kernel, dim3(1), dim3(64), 0, s, word, &dsh->rep, *last, (uint64_t)20000000,
                       last);  // 0.2 s idle
    CK(hipGetLastError());
    CK(hipStreamSynchronize(s));
  }
  fd_thread.join();
  CK(hipFree(req));
  return 0;
}

static int client(Shared* sh, const char* mode, int tag) {
  uint32_t* req = nullptr;
  if (!strcmp(mode, "shm")) {
    sh->mode_shm.store(1);
    req = &sh->shm_req;
    std::this_thread::sleep_for(std::chrono::milliseconds(400));  // server lane switches over
  } else if (!strcmp(mode, "dmabuf")) {
    sh->mode_shm.store(0);
    std::this_thread::sleep_for(std::chrono::milliseconds(400));
    fprintf(stderr, "client dmabuf: export status %d fd %d off %lu\n", sh->dmabuf_status, sh->dmabuf_fd,
            (unsigned long)sh->dmabuf_off);
    const int fd = recv_fd(sh->pid);
    if (fd < 0) {
      printf("{\"mode\": \"%s\", \"error\": \"fd hand-off: %s\"}\n", mode, strerror(errno));
      return 0;
    }
    const size_t pg = 4096;
    void* p = mmap(nullptr, pg, PROT_READ | PROT_WRITE, MAP_SHARED, fd, (off_t)(sh->dmabuf_off & ~(pg - 1)));
    if (p == MAP_FAILED) {
      printf("{\"mode\": \"%s\", \"error\": \"mmap: %s\"}\n", mode, strerror(errno));
      return 0;
    }
    req = reinterpret_cast<uint32_t*>(static_cast<char*>(p) + (sh->dmabuf_off & (pg - 1)));
    fprintf(stderr, "client dmabuf: mapped %p, word %u\n", p, *(volatile uint32_t*)req);
  } else {
    sh->mode_shm.store(0);
    std::this_thread::sleep_for(std::chrono::milliseconds(400));
    CK(hipSetDevice(0));
    void* p = nullptr;
    CK(hipIpcOpenMemHandle(&p, sh->handle, hipIpcMemLazyEnablePeerAccess));
    req = static_cast<uint32_t*>(p);
    hsa_amd_pointer_info_t info{};
    info.size = sizeof(info);
    uint32_t n = 0;
    hsa_agent_t* agents = nullptr;
    const hsa_status_t pst = hsa_amd_pointer_info(p, &info, malloc, &n, &agents);
    fprintf(stderr, "client %s: imported %p, pointer_info %d type %d agents %u hostptr %p\n", mode, p, (int)pst,
            (int)info.type, n, info.hostBaseAddress);
    free(agents);
    if (!strcmp(mode, "ipc-allow")) {
      hsa_iterate_agents(find_cpu, nullptr);
      const hsa_status_t st = hsa_amd_agents_allow_access(1, &g_cpu, nullptr, p);
      fprintf(stderr, "client %s: allow_access(cpu) -> %d\n", mode, (int)st);
    }
  }
  const int iters = 20000;
  std::vector<double> lat;
  lat.reserve(iters);
  bool ok = true;
  for (int i = 1; i <= iters && ok; ++i) {
    const uint32_t v = ((uint32_t)tag << 24) | (uint32_t)i;
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n((volatile uint32_t*)req, v, __ATOMIC_RELEASE);
    _mm_sfence();
    while (__atomic_load_n((volatile uint32_t*)&sh->rep, __ATOMIC_ACQUIRE) != v) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
        ok = false;
        break;
      }
    }
    lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  if (!ok) {
    printf("{\"mode\": \"%s\", \"error\": \"the server lane never saw the client's write\"}\n", mode);
    return 0;
  }
  lat.erase(lat.begin(), lat.begin() + 1000);
  std::sort(lat.begin(), lat.end());
  auto q = [&](double f) { return lat[(size_t)(f * (lat.size() - 1))]; };
  printf("{\"mode\": \"%s\", \"p50_us\": %.3f, \"p90_us\": %.3f, \"p99_us\": %.3f}\n", mode, q(0.5), q(0.9), q(0.99));
  return 0;
}

int main() {
  void* m = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) return 2;
  memset(m, 0, sizeof(Shared));
  Shared* sh = static_cast<Shared*>(m);
  fflush(stdout);
  const pid_t srv = fork();
  if (srv == 0) _exit(server(sh));
  for (int w = 0; w < 600 && !sh->ready.load(); ++w) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  if (!sh->ready.load()) {
    printf("{\"error\": \"server not ready\"}\n");
    sh->stop.store(1);
    waitpid(srv, nullptr, 0);
    return 1;
  }
  int tag = 1;
  for (const char* mode : {"shm", "dmabuf", "ipc", "ipc-allow"}) {
    fflush(stdout);
    const pid_t pid = fork();
    if (pid == 0) {
      const int rc = client(sh, mode, tag);
      fflush(stdout);
      _exit(rc);
    }
    int st = 0;
    waitpid(pid, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st)) printf("{\"mode\": \"%s\", \"error\": \"client status %d\"}\n", mode, st);
    fflush(stdout);
    ++tag;
  }
  sh->stop.store(1);
  int st = 0;
  waitpid(srv, &st, 0);
  printf("{\"server_status\": %d}\n", st);
  return 0;
}
