#include "shmring.hpp"

#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <stddef.h>
#include <sys/mman.h>
#include <sys/select.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>

#include "ringproto.hpp"
#include "util.hpp"

namespace ptype {

void shm_futex_wake(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, 1, nullptr, nullptr, 0);
}

void shm_futex_wait(std::atomic<uint32_t>* w, uint32_t expect, int64_t timeout_us) {
  timespec ts{(time_t)(timeout_us / 1000000), (long)((timeout_us % 1000000) * 1000)};
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, expect, timeout_us >= 0 ? &ts : nullptr, nullptr,
          0);
}

static std::string shm_path(const std::string& name) { return name[0] == '/' ? name : "/" + name; }

std::shared_ptr<ShmSegment> ShmSegment::create(const std::string& name, size_t bytes) {
  const std::string p = shm_path(name);
  shm_unlink(p.c_str());  // a stale segment of a dead server
  const int fd = shm_open(p.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) fail(Errc::kGeneric, "shm_open(" + p + "): " + std::strerror(errno));
  if (ftruncate(fd, (off_t)bytes) != 0) {
    close(fd);
    shm_unlink(p.c_str());
    fail(Errc::kGeneric, "ftruncate(" + p + "): " + std::strerror(errno));
  }
  void* b = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (b == MAP_FAILED) {
    shm_unlink(p.c_str());
    fail(Errc::kGeneric, "mmap(" + p + "): " + std::strerror(errno));
  }
  std::memset(b, 0, bytes);
  auto s = std::shared_ptr<ShmSegment>(new ShmSegment());
  s->name_ = p;
  s->base_ = b;
  s->size_ = bytes;
  s->unlink_ = true;
  return s;
}

std::shared_ptr<ShmSegment> ShmSegment::attach(const std::string& name) {
  const std::string p = shm_path(name);
  const int fd = shm_open(p.c_str(), O_RDWR, 0600);
  if (fd < 0) return nullptr;
  struct stat st {};
  if (fstat(fd, &st) != 0 || st.st_size <= 0) {
    close(fd);
    return nullptr;
  }
  void* b = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (b == MAP_FAILED) return nullptr;
  auto s = std::shared_ptr<ShmSegment>(new ShmSegment());
  s->name_ = p;
  s->base_ = b;
  s->size_ = (size_t)st.st_size;
  return s;
}

void ShmSegment::unlink_now() {
  shm_unlink(name_.c_str());
  unlink_ = false;
}

ShmSegment::~ShmSegment() {
  if (base_) munmap(base_, size_);
  if (unlink_) shm_unlink(name_.c_str());
}

bool xproc_device_ring_enabled() {
  const char* v = getenv("PTYPE_XPROC_RING");
  return !(v && std::string(v) == "host");
}

// ---- dma-buf fd hand-off (abstract unix socket, SCM_RIGHTS).  pidfd_getfd
// would need ptrace rights over the server (Yama scope 1 denies it between
// sibling processes); a socket the server answers works for any same-uid peer.
static sockaddr_un abstract_addr(const std::string& name, socklen_t* len) {
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  const size_t n = std::min(name.size(), sizeof(a.sun_path) - 2);
  std::memcpy(a.sun_path + 1, name.data(), n);  // sun_path[0] = 0: abstract namespace
  *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n);
  return a;
}

FdHandoff::FdHandoff(const std::string& name, int fd) : fd_(fd) {
  listen_fd_ = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  socklen_t len;
  const sockaddr_un a = abstract_addr(name, &len);
  if (listen_fd_ < 0 || bind(listen_fd_, (const sockaddr*)&a, len) != 0 || listen(listen_fd_, 64) != 0) {
    const std::string e = std::strerror(errno);
    if (listen_fd_ >= 0) close(listen_fd_);
    fail(Errc::kGeneric, "fd hand-off socket " + name + ": " + e);
  }
  thread_ = std::thread([this] { loop(); });
}

FdHandoff::~FdHandoff() {
  stop_.store(true);
  if (thread_.joinable()) thread_.join();
  close(listen_fd_);
}

void FdHandoff::loop() {
  while (!stop_.load()) {
    fd_set rs;
    FD_ZERO(&rs);
    FD_SET(listen_fd_, &rs);
    timeval tv{0, 100000};
    if (select(listen_fd_ + 1, &rs, nullptr, nullptr, &tv) <= 0) continue;
    const int c = accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (c < 0) continue;
    ucred cred{};
    socklen_t cl = sizeof cred;
    if (getsockopt(c, SOL_SOCKET, SO_PEERCRED, &cred, &cl) == 0 && cred.uid == getuid()) {
      char b = 'r';
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
      std::memcpy(CMSG_DATA(cm), &fd_, sizeof(int));
      if (sendmsg(c, &m, MSG_NOSIGNAL) == 1) handed_.fetch_add(1);
    }
    close(c);
  }
}

int shm_receive_fd(const std::string& name, std::string* why) {
  const int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  socklen_t len;
  const sockaddr_un a = abstract_addr(name, &len);
  if (s < 0 || connect(s, (const sockaddr*)&a, len) != 0) {
    if (why) *why = std::string("connect: ") + std::strerror(errno);
    if (s >= 0) close(s);
    return -1;
  }
  timeval tv{2, 0};
  setsockopt(s, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  char b = 0;
  iovec io{&b, 1};
  char ctl[CMSG_SPACE(sizeof(int))] = {};
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = ctl;
  m.msg_controllen = sizeof ctl;
  int fd = -1;
  if (recvmsg(s, &m, MSG_CMSG_CLOEXEC) == 1)
    for (cmsghdr* cm = CMSG_FIRSTHDR(&m); cm; cm = CMSG_NXTHDR(&m, cm))
      if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) std::memcpy(&fd, CMSG_DATA(cm), sizeof(int));
  if (fd < 0 && why) *why = "no fd received (different user?)";
  close(s);
  return fd;
}

std::shared_ptr<DevRingMap> DevRingMap::attach(const ShmHeader* h, std::string* why) {
  if (!h->req_dev) {
    if (why) *why = "the server's ring is in the segment";
    return nullptr;
  }
  const std::string name(h->req_sock, strnlen(h->req_sock, sizeof h->req_sock));
  const int fd = shm_receive_fd(name, why);
  if (fd < 0) return nullptr;
  const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
  const uint64_t off = h->req_dev_off;
  const size_t lead = (size_t)(off & (pg - 1));
  const size_t len = (lead + (size_t)h->req_dev_bytes + pg - 1) & ~(pg - 1);
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, (off_t)(off - lead));
  const int err = errno;
  close(fd);  // the mapping holds the buffer
  if (p == MAP_FAILED) {
    if (why) *why = std::string("mmap of the device ring: ") + std::strerror(err);
    return nullptr;
  }
  auto m = std::shared_ptr<DevRingMap>(new DevRingMap());
  m->map_ = p;
  m->len_ = len;
  m->req_ = reinterpret_cast<RingSlot*>(static_cast<char*>(p) + lead);
  return m;
}

DevRingMap::~DevRingMap() {
  if (map_) munmap(map_, len_);
}

ShmView shm_attach_view(const std::shared_ptr<ShmSegment>& seg, std::shared_ptr<DevRingMap>* devmap) {
  const ShmHeader* h = static_cast<const ShmHeader*>(seg->base());
  if (seg->size() < sizeof(ShmHeader) || h->magic != kShmMagic || seg->size() < shm_bytes(h->ring))
    fail(Errc::kUnavailable, "shared-memory segment " + seg->name() + " is not a ptype dispatcher");
  ShmView v = shm_view(seg->base(), h->ring);
  if (h->req_dev) {
    std::string why;
    *devmap = DevRingMap::attach(h, &why);
    if (!*devmap) fail(Errc::kUnavailable, "dispatcher " + seg->name() + ": device request ring: " + why);
    v.req = (*devmap)->req();
    v.bar = true;
  }
  return v;
}

static uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static void poke_if_parked(const ShmView& v) {
  if (__atomic_load_n(&v.ctrl->state, __ATOMIC_SEQ_CST) != kRunning) {
    v.hdr->wake.store(1, std::memory_order_seq_cst);
    shm_futex_wake(&v.hdr->wake);
  }
}

ReplyRecord shm_call(const ShmView& v, const MsgRecord& m, double timeout_s) {
  RingRefs r;
  r.req = v.req;
  r.rep = v.rep;
  r.owner = v.owner;
  r.takers = v.takers;
  r.next_seq = &v.hdr->next_seq;
  r.ring = v.hdr->ring;
  r.bar = v.bar;
  r.poke = [&v] { poke_if_parked(v); };
  RingTicket t = ring_take(r, 1, timeout_s);
  RingTicketGuard guard{r, t};
  const uint64_t seq = t.seq;
  ring_test_stop("took");
  if (!ring_claim(r, seq, timeout_s))
    fail(Errc::kTimeout, "device actor call: request slot not free in time (left for rescue)");
  ring_test_stop("claimed");
  ring_write(r, seq, m, now_ns());
  poke_if_parked(v);
  int64_t value = 0;
  uint32_t status = 0;
  if (getenv("PTYPE_RING_TEST_STOP")) {  // test hook: stop once the reply has landed, before reading it
    const uint64_t t0 = now_ns();
    while (!reply_landed(r, seq) && (now_ns() - t0) * 1e-9 < timeout_s) std::this_thread::yield();
    ring_test_stop("landed");
  }
  if (!ring_wait(r, seq, timeout_s, &value, &status)) fail(Errc::kTimeout, "device actor call: reply timeout");
  ReplyRecord out;
  out.value = value;
  out.status = (int32_t)status;
  out.actor = m.actor;
  return out;
}

// ---- locator: "/ptype-port-<port>" holds {pid, segment name}
static std::string locator_name(int port) { return "/ptype-port-" + std::to_string(port); }

void shm_locator_publish(int port, const std::string& segment) {
  auto s = ShmSegment::create(locator_name(port), 256);
  char* b = static_cast<char*>(s->base());
  const int32_t pid = (int32_t)getpid();
  std::memcpy(b, &pid, sizeof pid);
  std::strncpy(b + 8, segment.c_str(), 240);
  // keep the mapping alive for the process lifetime; shm_locator_remove unlinks
  static std::mutex mu;
  static std::vector<std::shared_ptr<ShmSegment>> keep;
  std::lock_guard<std::mutex> g(mu);
  keep.push_back(s);
}

void shm_locator_remove(int port) { shm_unlink(locator_name(port).c_str()); }

std::string shm_locator_lookup(int port) {
  auto s = ShmSegment::attach(locator_name(port));
  if (!s || s->size() < 256) return "";
  const char* b = static_cast<const char*>(s->base());
  int32_t pid = 0;
  std::memcpy(&pid, b, sizeof pid);
  if (pid <= 0 || (kill(pid, 0) != 0 && errno == ESRCH)) return "";  // its server is gone
  return std::string(b + 8, strnlen(b + 8, 240));
}

}  // namespace ptype

namespace ptype {

// ---- HostDispatcher
HostDispatcher::HostDispatcher(const std::string& name, uint32_t ring) {
  if (ring < 2 || (ring & (ring - 1))) throw std::invalid_argument("HostDispatcher: ring must be a power of two");
  seg_ = ShmSegment::create(name, shm_bytes(ring));
  seg_->unlink_on_close();
  v_ = shm_view(seg_->base(), ring);
  for (uint32_t i = 0; i < ring; ++i) v_.owner[i].store(i, std::memory_order_relaxed);
  v_.hdr->ring = ring;
  v_.hdr->owner_pid = (int32_t)getpid();
  __atomic_store_n(&v_.ctrl->state, (uint64_t)kRunning, __ATOMIC_SEQ_CST);
  __atomic_store_n(&v_.hdr->magic, kShmMagic, __ATOMIC_RELEASE);
  thread_ = std::thread([this] { loop(); });
}

HostDispatcher::~HostDispatcher() {
  stop_.store(true);
  if (thread_.joinable()) thread_.join();
}

void HostDispatcher::loop() {
  const uint32_t ring = v_.hdr->ring;
  uint64_t head = 0;
  unsigned idle = 0;
  while (!stop_.load(std::memory_order_relaxed)) {
    RingSlot* sl = &v_.req[head & (ring - 1)];
    if (__atomic_load_n(&sl->tag, __ATOMIC_ACQUIRE) != head + 1) {
      if (++idle > 4096) std::this_thread::sleep_for(std::chrono::microseconds(50));
      else std::this_thread::yield();
      continue;
    }
    idle = 0;
    const MsgRecord m = sl->msg;
    if (ring_csum(head, m) != sl->csum) continue;  // payload not yet visible with its tag: read again
    int64_t value = 0;
    uint32_t st = kStatusOk;
    switch (m.method) {
      case kCalculatorMultiply: value = m.a0 * m.a1; break;
      case kEcho: value = m.a0; break;
      default: st = kStatusNoMethod; break;
    }
    if (m.method == kMethodNone) noops_.fetch_add(1);
    ReplySlot* o = &v_.rep[head & (ring - 1)];
    o->value = value;
    __atomic_store_n(&o->tag, reply_tag(head, st), __ATOMIC_RELEASE);
    processed_.fetch_add(1);
    ++head;
  }
}

}  // namespace ptype
