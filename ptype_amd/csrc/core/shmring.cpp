#include "shmring.hpp"

#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
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

ShmSegment::~ShmSegment() {
  if (base_) munmap(base_, size_);
  if (unlink_) shm_unlink(name_.c_str());
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
  r.ring = v.hdr->ring;
  r.poke = [&v] { poke_if_parked(v); };
  const uint64_t seq = v.hdr->next_seq.fetch_add(1);
  if (!ring_claim(r, seq, timeout_s))
    fail(Errc::kTimeout, "device actor call: request slot not free in time (left for rescue)");
  ring_write(r, seq, m, now_ns());
  poke_if_parked(v);
  int64_t value = 0;
  uint32_t status = 0;
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
