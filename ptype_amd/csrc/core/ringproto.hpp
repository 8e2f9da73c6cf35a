// Host side of the single-call request ring (the persistent dispatcher's
// latency path), shared by the in-process DeviceServer (csrc/hip/server.hpp)
// and same-node client processes (shmring.cpp).
//
// The dispatcher consumes strictly in sequence order, so every sequence number
// that is taken MUST end up published, and a slot may only be reused once its
// previous occupant's reply has been taken.  owner[slot] is the slot's state:
//
//   s              free for sequence s (nobody has claimed it yet)
//   s | kBusy      claimed by s's caller: published, or about to be; freed
//                  (-> s + ring) by that caller once it has read s's reply
//   s | kRescued   s's caller is gone (or gave up): a rescuer published a no-op
//                  (method 0 -> kStatusNoMethod) in its place, or the caller timed
//                  out waiting and marked its reply unwanted
//
// Liveness, not timers, decides takeovers.  A caller records
// the sequence numbers it holds in a TAKER entry of this ring (its process token
// = pid + process start time, and the range) BEFORE they exist: numbers are
// taken by a compare-and-swap on the shared counter after the entry names
// them, so a caller killed at any instruction leaves its numbers attributable.
// Another caller may then
//   * take over a slot whose previous reply landed but was never freed only if
//     that reply's caller marked it unwanted or holds no live entry any more
//     (a descheduled or SIGSTOPped caller is alive: its slot waits for it);
//   * rescue an unclaimed number in front of its own only if no live entry
//     holds it (its taker died, or gave up claiming and released the entry).
// (the grace-period takeover could overwrite a live caller's reply,
// and a number stranded behind an abandoned slot was never rescued.)
#pragma once
#include <errno.h>
#include <immintrin.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/types.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <functional>
#include <stdexcept>
#include <string>
#include <thread>

#include "records.hpp"

// The request ring's real synchronisation runs through its consumer -- a GPU
// wave in production, another mapping of the segment in the stress test --
// which ThreadSanitizer cannot see: a slot taken over after its reply landed is
// ordered behind the previous occupant's request only by that consumer.  These
// annotations state that edge (publish = release of the slot, reply observed
// before a takeover = acquire of it).
#if defined(__SANITIZE_THREAD__)
#define PT_TSAN_RING 1
#elif defined(__has_feature)
#if __has_feature(thread_sanitizer)
#define PT_TSAN_RING 1
#endif
#endif
#ifdef PT_TSAN_RING
#include <sanitizer/tsan_interface.h>
#endif

namespace ptype {

inline void ring_tsan_release(const void* slot) {
#ifdef PT_TSAN_RING
  __tsan_release(const_cast<void*>(slot));
#else
  (void)slot;
#endif
}
inline void ring_tsan_acquire(const void* slot) {
#ifdef PT_TSAN_RING
  __tsan_acquire(const_cast<void*>(slot));
#else
  (void)slot;
#endif
}

constexpr uint64_t kOwnerBusy = 1ull << 62;
constexpr uint64_t kOwnerRescued = 1ull << 63;
constexpr uint64_t kOwnerSeq = kOwnerBusy - 1;

// A caller's record of the sequence numbers it holds.  range = first << 16 | n.
constexpr uint32_t kRingTakers = 256;
constexpr uint32_t kRingMaxTake = 0xffffu;
enum RingTakerState : uint32_t { kTakerIdle = 0, kTakerHolds = 1 };
struct alignas(32) RingTaker {
  std::atomic<uint64_t> token;  // 0: free; else the holder's process token
  std::atomic<uint64_t> range;  // first seq << 16 | count (valid while state == kTakerHolds)
  std::atomic<uint32_t> state;
  uint32_t pad0;
  uint64_t pad1;
};
static_assert(sizeof(RingTaker) == 32, "RingTaker layout");

struct RingRefs {
  RingSlot* req = nullptr;      // host-writable view of the request ring
  ReplySlot* rep = nullptr;     // host view of the reply ring
  std::atomic<uint64_t>* owner = nullptr;
  RingTaker* takers = nullptr;  // kRingTakers entries
  std::atomic<uint64_t>* next_seq = nullptr;  // the shared sequence counter
  uint32_t ring = 0;            // power of two
  bool bar = false;             // request ring is device memory written through the BAR
  std::function<void()> poke;   // make sure the dispatcher runs (relaunch / wake its server)
};

inline uint64_t ring_now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// ---- process identity and liveness
// /proc/<pid>/stat: state (field 3) and start time in clock ticks (field 22).
inline bool ring_proc_stat(int pid, char* state, uint64_t* start) {
  char path[64], buf[1024];
  snprintf(path, sizeof path, "/proc/%d/stat", pid);
  FILE* f = fopen(path, "r");
  if (!f) return false;
  const size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* p = strrchr(buf, ')');  // the command name may hold spaces and parens
  if (!p || p[1] != ' ') return false;
  *state = p[2];
  p += 2;
  for (int field = 3; field < 22; ++field) {
    p = strchr(p, ' ');
    if (!p) return false;
    ++p;
  }
  *start = strtoull(p, nullptr, 10);
  return true;
}

// pid << 32 | low 32 bits of the process start time: a recycled pid does not
// look like the process that died.
// Cached per pid (a forked child computes its own).
inline uint64_t ring_self_token() {
  static std::atomic<uint64_t> cached{0};
  const uint32_t pid = (uint32_t)getpid();
  uint64_t tok = cached.load(std::memory_order_relaxed);
  if ((tok >> 32) == pid) return tok;
  char st = 0;
  uint64_t start = 0;
  (void)ring_proc_stat((int)pid, &st, &start);
  tok = ((uint64_t)pid << 32) | (uint32_t)start;
  cached.store(tok, std::memory_order_relaxed);
  return tok;
}

// Whether the process of `tok` still exists (stopped counts as alive; a zombie
// or a different process under a recycled pid does not).
inline bool ring_token_alive(uint64_t tok) {
  const int pid = (int)(tok >> 32);
  if (pid == (int)getpid()) return true;
  if (pid <= 0) return false;
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  char st = 0;
  uint64_t start = 0;
  if (!ring_proc_stat(pid, &st, &start)) return false;  // gone between the two checks
  if (st == 'Z' || st == 'X') return false;
  return (uint32_t)start == (uint32_t)tok;
}

// Whether a live caller holds sequence number p (took it and has not released it).
inline bool ring_holder_alive(const RingRefs& r, uint64_t p) {
  for (uint32_t i = 0; i < kRingTakers; ++i) {
    RingTaker& e = r.takers[i];
    if (e.state.load(std::memory_order_acquire) != kTakerHolds) continue;
    const uint64_t tok = e.token.load(std::memory_order_acquire);
    const uint64_t rg = e.range.load(std::memory_order_acquire);
    const uint64_t first = rg >> 16, n = rg & 0xffffu;
    if (tok && p >= first && p < first + n && ring_token_alive(tok)) return true;
  }
  return false;
}

// ---- taking sequence numbers
struct RingTicket {
  uint64_t seq = 0;  // first number of the range
  uint32_t n = 0;
  int32_t taker = -1;
};

// Acquire a taker entry of this process and take n consecutive numbers through
// it.  Entries of dead processes are reclaimed when none is free.
inline RingTicket ring_take(const RingRefs& r, uint32_t n, double timeout_s = 30.0) {
  if (n == 0 || n > kRingMaxTake) throw std::invalid_argument("ring_take: 1..65535 numbers");
  RingTicket t;
  t.n = n;
  const uint64_t me = ring_self_token();
  static thread_local uint32_t hint = (uint32_t)(std::hash<std::thread::id>()(std::this_thread::get_id()) % kRingTakers);
  const uint64_t t0 = ring_now_ns();
  for (uint32_t scan = 0; t.taker < 0; ++scan) {
    const uint32_t i = (hint + scan) % kRingTakers;
    uint64_t z = 0;
    if (r.takers[i].token.load(std::memory_order_relaxed) == 0 &&
        r.takers[i].token.compare_exchange_strong(z, me, std::memory_order_acq_rel)) {
      t.taker = (int32_t)i;
      hint = i;
      break;
    }
    if (scan % kRingTakers == kRingTakers - 1) {  // a full pass found none free: reclaim the dead's
      for (uint32_t j = 0; j < kRingTakers; ++j) {
        uint64_t tok = r.takers[j].token.load(std::memory_order_acquire);
        if (tok && !ring_token_alive(tok)) {
          r.takers[j].state.store(kTakerIdle, std::memory_order_release);
          r.takers[j].token.compare_exchange_strong(tok, 0, std::memory_order_acq_rel);
        }
      }
      if ((ring_now_ns() - t0) * 1e-9 > timeout_s) throw std::runtime_error("request ring: no free taker entry");
      std::this_thread::yield();
    }
  }
  RingTaker& e = r.takers[t.taker];
  for (;;) {
    uint64_t c = r.next_seq->load(std::memory_order_acquire);
    e.range.store((c << 16) | n, std::memory_order_relaxed);
    e.state.store(kTakerHolds, std::memory_order_seq_cst);  // names c..c+n-1 before they are taken
    if (r.next_seq->compare_exchange_weak(c, c + n, std::memory_order_seq_cst)) {
      t.seq = c;
      return t;
    }
  }
}

// The numbers are published and waited for (or given up): the entry is free.
// Numbers of the range that were never claimed become rescuable.
inline void ring_release(const RingRefs& r, RingTicket& t) {
  if (t.taker < 0) return;
  RingTaker& e = r.takers[t.taker];
  e.state.store(kTakerIdle, std::memory_order_release);
  e.token.store(0, std::memory_order_release);
  t.taker = -1;
}

// RAII: releases the ticket's entry on every exit path.
struct RingTicketGuard {
  const RingRefs& r;
  RingTicket& t;
  ~RingTicketGuard() { ring_release(r, t); }
};

// ---- publish / reply
// Write request `m` for `seq` into its slot (the slot is claimed) and publish the tag.
inline void ring_write(const RingRefs& r, uint64_t seq, const MsgRecord& m, uint64_t t_ns) {
  RingSlot* s = &r.req[seq & (r.ring - 1)];
  s->msg = m;
  s->csum = ring_csum(seq, m);  // before the tag (release below)
  s->t_pub_ns = t_ns;
  // a BAR mapping is write-combined: the payload must be out before the tag
  if (r.bar) _mm_sfence();
  ring_tsan_release(s);
  __atomic_store_n(&s->tag, seq + 1, __ATOMIC_RELEASE);
  if (r.bar) {
    _mm_sfence();
    // a posted write can still be in flight when the caller checks whether the
    // dispatcher is running (Dekker hand-off); a read of the same line is
    // non-posted and returns only after it has landed
    (void)__atomic_load_n(&s->tag, __ATOMIC_ACQUIRE);
  }
}

inline bool reply_landed(const RingRefs& r, uint64_t seq) {
  return reply_tag_is(__atomic_load_n(&r.rep[seq & (r.ring - 1)].tag, __ATOMIC_ACQUIRE), seq);
}

// Publish a no-op for `p` if its caller is gone: p unclaimed with no live holder;
// p claimed but never published by a caller that died; or p's slot still held
// by an abandoned / dead previous occupant whose reply has landed.  True if
// this call did.
inline bool ring_rescue(const RingRefs& r, uint64_t p) {
  std::atomic<uint64_t>& o = r.owner[p & (r.ring - 1)];
  uint64_t cur = o.load(std::memory_order_acquire);
  const uint64_t prev = p - r.ring;
  bool gone = false;
  if (cur == p) {
    gone = !ring_holder_alive(r, p);
  } else if (cur == (p | kOwnerBusy)) {
    if (reply_landed(r, p) || __atomic_load_n(&r.req[p & (r.ring - 1)].tag, __ATOMIC_ACQUIRE) == p + 1) return false;
    gone = !ring_holder_alive(r, p);
  } else if (p >= r.ring && (cur == (prev | kOwnerRescued) || cur == (prev | kOwnerBusy)) && reply_landed(r, prev)) {
    gone = !ring_holder_alive(r, p) && (cur == (prev | kOwnerRescued) || !ring_holder_alive(r, prev));
  }
  if (!gone || !o.compare_exchange_strong(cur, p | kOwnerRescued, std::memory_order_acq_rel)) return false;
  if (cur != p) ring_tsan_acquire(&r.req[p & (r.ring - 1)]);
  MsgRecord noop{};
  noop.method = kMethodNone;
  noop.flags = kFlagValid;
  ring_write(r, p, noop, ring_now_ns());
  return true;
}

// Rescue every number in front of `seq` whose caller is gone.  Replies land in
// sequence order, so the scan walks down from seq - 1 and stops at the first
// number whose reply has landed.
inline void ring_rescue_scan(const RingRefs& r, uint64_t seq) {
  const uint64_t lo = seq >= r.ring ? seq - r.ring + 1 : 0;
  for (uint64_t p = seq; p-- > lo;) {
    if (reply_landed(r, p)) break;
    const uint64_t w = r.owner[p & (r.ring - 1)].load(std::memory_order_acquire);
    if (w == p || w == (p | kOwnerBusy) || (p >= r.ring && (w & kOwnerSeq) == p - r.ring && w != p - r.ring))
      ring_rescue(r, p);
  }
}

// Claim the slot of `seq` (the caller holds seq in a taker entry).  Returns false
// if `seq` was rescued in its place (the call must fail) or the wait exceeded
// `timeout_s` (the caller then releases its entry: seq becomes rescuable).
inline bool ring_claim(const RingRefs& r, uint64_t seq, double timeout_s) {
  std::atomic<uint64_t>& o = r.owner[seq & (r.ring - 1)];
  const uint64_t prev = seq - r.ring;
  const uint64_t t0 = ring_now_ns();
  double next_scan = 0.01;
  for (unsigned spins = 0;; ++spins) {
    uint64_t cur = o.load(std::memory_order_acquire);
    if (cur == seq) {
      if (o.compare_exchange_strong(cur, seq | kOwnerBusy, std::memory_order_acq_rel)) return true;
      continue;
    }
    if (cur == (seq | kOwnerRescued)) return false;
    if ((spins & 255) == 255) {
      // the previous occupant's reply landed but was never freed: take the slot
      // over if that reply is unwanted (its caller timed out) or its caller is gone
      if (seq >= r.ring && (cur == (prev | kOwnerRescued) || cur == (prev | kOwnerBusy)) && reply_landed(r, prev) &&
          (cur == (prev | kOwnerRescued) || !ring_holder_alive(r, prev))) {
        if (o.compare_exchange_strong(cur, seq | kOwnerBusy, std::memory_order_acq_rel)) {
          ring_tsan_acquire(&r.req[seq & (r.ring - 1)]);  // prev's request was consumed before its reply
          return true;
        }
        continue;
      }
      if (r.poke) r.poke();
      const double waited = (ring_now_ns() - t0) * 1e-9;
      if (waited > next_scan) {  // the dispatcher may be stuck on a number whose caller is gone
        next_scan = waited + 0.01;
        if (seq >= r.ring && (cur == prev || cur == (prev | kOwnerBusy))) ring_rescue(r, prev);  // this slot's
        ring_rescue_scan(r, seq);
      }
      if (waited > timeout_s) return false;
      std::this_thread::yield();
    }
  }
}

// Wait for the reply of `seq`; true with the slot freed, false on timeout (the
// slot is marked unwanted: the next occupant takes it over once the late reply
// lands).  While the reply is overdue, numbers in front of `seq` whose callers
// are gone are rescued (the dispatcher runs in order and would wait for them).
inline bool ring_wait(const RingRefs& r, uint64_t seq, double timeout_s, int64_t* value, uint32_t* status) {
  ReplySlot* out = &r.rep[seq & (r.ring - 1)];
  const uint64_t t0 = ring_now_ns();
  const double scan_every = 0.01;  // how often to look for dead callers in front (liveness decides, not age)
  double next_scan = scan_every;
  uint64_t tag;
  for (unsigned spins = 0;; ++spins) {
    tag = __atomic_load_n(&out->tag, __ATOMIC_ACQUIRE);
    if (reply_tag_is(tag, seq)) {
      const int64_t v = out->value;  // written with the tag (one 16-B device store)
      // re-read: the value belongs to this tag only if the slot still carries it
      if (__atomic_load_n(&out->tag, __ATOMIC_ACQUIRE) != tag) continue;
      *value = v;
      break;
    }
    if ((spins & 1023) == 1023) {
      if (r.poke) r.poke();
      const double waited = (ring_now_ns() - t0) * 1e-9;
      if (waited > next_scan) {
        next_scan = waited + scan_every;
        ring_rescue_scan(r, seq);
      }
      if (waited > timeout_s) {
        uint64_t mine = seq | kOwnerBusy;
        r.owner[seq & (r.ring - 1)].compare_exchange_strong(mine, seq | kOwnerRescued, std::memory_order_acq_rel);
        return false;
      }
      std::this_thread::yield();
    }
  }
  *status = (uint32_t)(tag & 0xff);
  // Free the slot only if it is still ours (a CAS, never a blind store: a slot
  // taken over meanwhile must not be handed back as unclaimed).
  uint64_t mine = seq | kOwnerBusy;
  r.owner[seq & (r.ring - 1)].compare_exchange_strong(mine, seq + r.ring, std::memory_order_acq_rel);
  return true;
}

// Test hook (PTYPE_RING_TEST_STOP=took|claimed|landed): the calling process stops
// itself (SIGSTOP) at that point of its next call, once -- lets a test freeze a
// caller mid-call and resume (SIGCONT) or kill it.
inline void ring_test_stop(const char* point) {
  static const char* want = getenv("PTYPE_RING_TEST_STOP");
  static std::atomic<bool> fired{false};
  if (want && strcmp(want, point) == 0 && !fired.exchange(true)) raise(SIGSTOP);
}

}  // namespace ptype
