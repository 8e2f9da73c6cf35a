// Host side of the single-call request ring (the persistent dispatcher's
// latency path), shared by the in-process DeviceServer (csrc/hip/server.hpp)
// and same-node client processes (shmring.cpp).
//
// Publishers take sequence numbers from one shared counter; the dispatcher
// consumes strictly in sequence order, so every taken sequence number MUST end
// up published, and a slot may only be reused once its previous occupant's
// reply has landed.  owner[slot] is the slot's state word:
//
//   s              free for sequence s (nobody has claimed it yet)
//   s | kBusy      claimed by s's publisher: published, or about to be; freed
//                  (-> s + ring) when s's reply has been taken
//   s | kRescued   s's publisher stalled or died before publishing; a rescuer
//                  published a no-op (method 0 -> kStatusNoMethod) in its place;
//                  or s's caller timed out waiting (nobody reads s's reply)
//
// A timed-out caller does NOT free its slot (the dispatcher may not have read
// the request yet): the slot stays busy until the late reply lands, and the
// next occupant takes it over then.  A caller whose reply is overdue rescues
// the unclaimed sequence numbers in front of it, so a publisher that died
// between taking a number and publishing wedges the ring for a bounded time
// only.  (the old protocol freed a timed-out slot at once and
// waited for owners without a bound.)
#pragma once
#include <immintrin.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <functional>
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

struct RingRefs {
  RingSlot* req = nullptr;      // host-writable view of the request ring
  ReplySlot* rep = nullptr;     // host view of the reply ring
  std::atomic<uint64_t>* owner = nullptr;
  uint32_t ring = 0;            // power of two
  bool bar = false;             // request ring is device memory written through the BAR
  std::function<void()> poke;   // make sure the dispatcher runs (relaunch / wake its server)
};

inline uint64_t ring_now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

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

// Publish a no-op for `p` if nobody has claimed it; true if this call did.
inline bool ring_rescue(const RingRefs& r, uint64_t p) {
  uint64_t exp = p;
  if (!r.owner[p & (r.ring - 1)].compare_exchange_strong(exp, p | kOwnerRescued, std::memory_order_acq_rel))
    return false;
  MsgRecord noop{};
  noop.method = kMethodNone;
  noop.flags = kFlagValid;
  ring_write(r, p, noop, ring_now_ns());
  return true;
}

// Claim the slot of `seq` (its previous occupant's reply taken, or taken over).
// Returns false if `seq` was rescued by someone else (the call must fail) or the
// wait exceeded `timeout_s` (then `seq` stays unclaimed; a later caller rescues it).
inline bool ring_claim(const RingRefs& r, uint64_t seq, double timeout_s) {
  std::atomic<uint64_t>& o = r.owner[seq & (r.ring - 1)];
  const uint64_t prev = seq - r.ring;
  const uint64_t t0 = ring_now_ns();
  const double takeover_after = timeout_s < 2.0 ? timeout_s / 2 : 1.0;
  for (unsigned spins = 0;; ++spins) {
    uint64_t cur = o.load(std::memory_order_acquire);
    if (cur == seq) {
      if (o.compare_exchange_strong(cur, seq | kOwnerBusy, std::memory_order_acq_rel)) return true;
      continue;
    }
    if (cur == (seq | kOwnerRescued)) return false;
    if ((spins & 255) == 255) {
      // the previous occupant's reply landed but nobody took it.  Rescued (a no-op
      // nobody waits for) or abandoned (its caller timed out and marked it): take
      // the slot over now.  Merely busy: its caller may be alive and just slow to
      // read the reply -- taking over at once let the next reply overwrite it (a
      // lost call under load) -- so only after a grace period (a caller that died)
      const bool gone = cur == (prev | kOwnerRescued) ||
                        (cur == (prev | kOwnerBusy) && (ring_now_ns() - t0) * 1e-9 > takeover_after);
      if (seq >= r.ring && gone && reply_landed(r, prev)) {
        if (o.compare_exchange_strong(cur, seq | kOwnerBusy, std::memory_order_acq_rel)) {
          ring_tsan_acquire(&r.req[seq & (r.ring - 1)]);  // prev's request was consumed before its reply
          return true;
        }
        continue;
      }
      if (r.poke) r.poke();
      if ((ring_now_ns() - t0) * 1e-9 > timeout_s) return false;
      std::this_thread::yield();
    }
  }
}

// Wait for the reply of `seq`; true with the slot freed, false on timeout (the
// slot stays busy: the late reply lands before the next occupant takes over).
// While the reply is overdue, unclaimed sequence numbers in front of `seq` are
// rescued: the dispatcher runs in order and would otherwise wait for them forever.
inline bool ring_wait(const RingRefs& r, uint64_t seq, double timeout_s, int64_t* value, uint32_t* status) {
  ReplySlot* out = &r.rep[seq & (r.ring - 1)];
  const uint64_t t0 = ring_now_ns();
  const double rescue_every = timeout_s < 0.2 ? timeout_s / 2 : 0.1;
  // the scan repeats: a number that was not yet rescuable at one scan (its slot
  // still held by the previous occupant) can be stranded later, when its
  // publisher gives up claiming -- a single early scan left the ring wedged
  double next_rescue = rescue_every;
  uint64_t tag;
  for (unsigned spins = 0; !reply_tag_is(tag = __atomic_load_n(&out->tag, __ATOMIC_ACQUIRE), seq); ++spins) {
    if ((spins & 1023) == 1023) {
      if (r.poke) r.poke();
      const double waited = (ring_now_ns() - t0) * 1e-9;
      if (waited > next_rescue) {
        next_rescue = waited + rescue_every;
        const uint64_t lo = seq >= r.ring ? seq - r.ring + 1 : 0;
        for (uint64_t p = seq; p-- > lo;)
          if ((r.owner[p & (r.ring - 1)].load(std::memory_order_acquire) & kOwnerSeq) == p) ring_rescue(r, p);
      }
      if (waited > timeout_s) {
        // abandoned: the next occupant may take the slot over as soon as the late
        // reply lands (nobody will read it)
        uint64_t mine = seq | kOwnerBusy;
        r.owner[seq & (r.ring - 1)].compare_exchange_strong(mine, seq | kOwnerRescued, std::memory_order_acq_rel);
        return false;
      }
      std::this_thread::yield();
    }
  }
  *value = out->value;  // landed with the tag (one 16-B device store)
  *status = (uint32_t)(tag & 0xff);
  // Free the slot only if it is still ours: once the reply has landed, the next
  // occupant may already have taken the slot over (ring_claim's takeover for a
  // caller that looks gone).  A blind store here handed its claimed slot back as
  // unclaimed, and a rescuer then overwrote its published request with a no-op
  // (a lost call and two writers on one slot: TSan / ASan stress under load).
  uint64_t mine = seq | kOwnerBusy;
  r.owner[seq & (r.ring - 1)].compare_exchange_strong(mine, seq + r.ring, std::memory_order_acq_rel);
  return true;
}

}  // namespace ptype
