// Fixed binary message records shared by the host control plane (_core) and
// the gfx950 device runtime (_hip).
//
// These replace the reference's per-call gob payloads on the data plane
// (reference: cluster/rpc.go:59-105 hands `args`/`reply` to stdlib net/rpc; the
// calculator payload is example/calculator/calculator.go:3-5 `Args{A, B int}` and
// the optimus payload example/optimus/prime.go:7-11 `Args{Min, Max, Target int}`).
// A request is 32 bytes: an 8-byte header plus three machine ints, which covers
// every payload the reference sends.  Replies are 16 bytes.  Both are sized so a
// wave moves them with 16-byte (dwordx4) accesses.
#pragma once
#include <stdint.h>

namespace ptype {

// Well-known method ids of the compiled-in device handlers (switch in dispatch).
enum MethodId : uint16_t {
  kMethodNone = 0,
  kCalculatorMultiply = 1,  // reply = a0 * a1                      (calculator.go:9-12)
  kPrimeCheck = 2,          // reply = first divisor in [a0,min(a1,a2)) or a2 (prime.go:15-25)
  kEcho = 3,                // reply = a0
  kRetryTest = 4,           // stateful: fails until per-actor count >= a0 (rpc_test.go:55-77)
  kCounterAdd = 5,          // stateful: state += a0; reply = new state
  kForward = 6,             // actor-to-actor "tell": state += 1; if a1 > 0 emit Forward to actor a0
                            // with (next = (a0 + stride) % n, a1 - 1, a2); a2 = stride | n << 32
  kSeqFold = 7,             // ORDERED stateful: reply = state; state = state * kFoldMul + a0 (wrapping).
                            // Non-commutative, so the final state and the replies expose the exact
                            // order an actor processed its messages in (mailbox FIFO audit)
  kMethodCount = 8,
};

// Served only by a persistent dispatcher that holds a relay table (xcall.hpp
// PeerRelay): the request (actor = remote actor, a0 = remote method, a1, a2 =
// its arguments) is forwarded from the dispatcher wave through a GPU peer lane
// to ANOTHER process's dispatcher, and that actor's reply is this call's reply
// -- a call a handler makes to a remote actor, with no host on its path.
// Outside a dispatcher with a relay table: kStatusNoMethod.
constexpr uint16_t kMethodRelay = 0x7e;

// An actor handler that decides to call another actor and continues on its reply
// (the optimus coordinator: coordinator.go:75-89 fans candidates out to Prime
// workers and counts the primes).  Local actor A, a0 = candidate n, a1 = worker
// count W, a2 = first worker id B (remote actors B .. B + W - 1 of the relay
// peer).  The handler picks the worker itself (B + hash(n) % W), asks it
// PrimeCheck(2, isqrt(n) + 1, n) through the relay, and on the reply adds 1 to
// A's state if n is prime; this call's reply is A's tally after it.  Served like
// kMethodRelay (a dispatcher with a relay table); elsewhere kStatusNoMethod.
constexpr uint16_t kMethodCoordPrime = 0x7d;

// Multiplier of kSeqFold (odd, so the fold is a bijection of the prior state).
constexpr uint64_t kFoldMul = 0x100000001b3ull;

// Methods whose handler is a non-commutative read-modify-write of actor state:
// they must run one at a time per actor, in mailbox order (HBM mailboxes, K2/K3).
inline constexpr bool method_ordered(uint32_t m) { return m == kSeqFold; }

// Methods whose handler reads no actor state at all (the reply is a function of
// the arguments): a message only has to reach its actor's GPU, so a sender may
// resolve just the destination rank (the route directory's rank byte table) and
// carry the actor id instead of the destination mailbox.
inline constexpr bool method_stateless(uint32_t m) {
  return m == kCalculatorMultiply || m == kPrimeCheck || m == kEcho;
}

enum RecordFlags : uint16_t {
  kFlagValid = 1,
  kFlagRouted = 2,  // `actor` holds the destination's local mailbox index
  kFlagIdentity = 4,  // slot header: slot position == message index (R = 1, no gaps)
  kFlagA2 = 8,        // mailbox record: the third argument is in the ring's a2 side array
  kFlagSharded = 16,  // sorted-exchange region header: records sorted by actor shard (shard table at its end)
  kFlagActorIds = 32,  // sorted-exchange region header: the mailbox field carries actor ids (stateless method)
};

enum ReplyStatus : int32_t {
  kStatusOk = 0,
  kStatusNoMethod = 1,      // rpc: can't find method
  kStatusFailed = 2,        // handler returned an error ("failed", rpc_test.go:76)
  kStatusNoActor = 3,       // registry lookup miss
  kStatusOverflow = 4,      // epoch bucket full; message deferred to the next epoch
  kStatusNotDelivered = 5,  // reply slot never written
  kStatusRankLost = 6,      // the actor's rank died with the message in flight (re-homed since: re-send)
};

struct alignas(16) MsgRecord {
  uint32_t actor;   // global actor key before routing, local mailbox index after
  uint16_t method;  // MethodId
  uint16_t flags;   // RecordFlags
  int64_t a0, a1, a2;
};
static_assert(sizeof(MsgRecord) == 32, "MsgRecord must be 32 bytes");

struct alignas(16) ReplyRecord {
  int64_t value;
  int32_t status;
  uint32_t actor;  // echoes the serving mailbox (debug / audit)
};
static_assert(sizeof(ReplyRecord) == 16, "ReplyRecord must be 16 bytes");

// Host<->device latency-path ring slot (fine-grained host memory).  The tag is
// written last with release semantics; the consumer polls the tag only.
struct alignas(64) RingSlot {
  MsgRecord msg;
  uint64_t tag;       // sequence number + 1 of the request published in this slot
  uint64_t t_pub_ns;  // host steady-clock time of publication (latency tracing)
  uint64_t csum;      // ring_csum(seq, msg): lets the device read msg in the same trip as the tag
  uint64_t pad;
};

#ifdef __HIPCC__
#define PT_HD __host__ __device__
#else
#define PT_HD
#endif
// Checksum binding a ring slot's message words to its sequence number.  The
// dispatcher reads tag, message and checksum in ONE batch of loads (one PCIe
// round trip, not two): individual 8-B reads of host memory may be served in
// any order, so a message word can be older than the tag it was read with --
// the checksum, written before the tag, exposes that (mismatch -> read again).
inline PT_HD uint64_t ring_csum(uint64_t seq, uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3) {
  uint64_t h = seq * 0x9e3779b97f4a7c15ull;
  for (uint64_t w : {w0, w1, w2, w3}) {
    h ^= w + 0x632be59bd9b4e019ull + (h << 6) + (h >> 2);
    h ^= h >> 31;
    h *= 0xbf58476d1ce4e5b9ull;
  }
  return h ^ (h >> 29);
}
inline uint64_t ring_csum(uint64_t seq, const MsgRecord& m) {
  uint64_t w[4];
  static_assert(sizeof(MsgRecord) == sizeof(w), "MsgRecord is four words");
  __builtin_memcpy(w, &m, sizeof(w));
  return ring_csum(seq, w[0], w[1], w[2], w[3]);
}
#undef PT_HD

// One traced request of the persistent dispatcher (host-visible trace ring).
struct TraceRec {
  uint64_t seq;
  uint64_t t_pub_ns;      // host: request published
  uint64_t t_seen_ticks;  // device s_memrealtime (100 MHz): batch picked up
  uint64_t t_done_ticks;  // device: reply published
};
static_assert(sizeof(RingSlot) == 64, "RingSlot must be 64 bytes");

// Reply slot of the latency path.  The value and the tag share one aligned
// 16-B unit that the device writes with ONE 16-byte store: one PCIe write that
// lands whole, so the host that sees the tag sees the value -- no system fence
// and no second write for the tag (that pair cost ~0.6 us per call).  The tag
// carries the status in its low byte: (seq + 1) << 8 | status.
struct alignas(32) ReplySlot {
  int64_t value;
  uint64_t tag;    // reply_tag(seq, status)
  uint64_t pad[2];
};
static_assert(sizeof(ReplySlot) == 32, "ReplySlot must be 32 bytes");

inline constexpr uint64_t reply_tag(uint64_t seq, uint32_t status) { return ((seq + 1) << 8) | (status & 0xffu); }
inline constexpr bool reply_tag_is(uint64_t tag, uint64_t seq) { return (tag >> 8) == ((seq + 1) & (~0ull >> 8)); }

// Device-side backend entry point that the host net/rpc server uses to execute a
// call on a GPU actor (exported by _hip as a C function pointer).
typedef int (*DeviceSubmitFn)(void* ctx, const MsgRecord* req, ReplyRecord* rep, int n);

// Control block of the persistent dispatcher (host-visible; the device polls it).
enum ServerState : uint64_t { kStopped = 0, kRunning = 1, kLaunching = 2 };

struct alignas(64) ServerCtrl {
  uint64_t stop;
  uint64_t state;
  uint64_t resume_head;
  uint64_t processed;
  uint64_t exits_idle;
  uint64_t exits_lifetime;
  uint64_t trace_mask;   // 0: tracing off; else trace ring capacity - 1
  uint64_t trace_ring;   // device address of the TraceRec ring
  uint64_t calib_req;    // host sets 1; the kernel answers with calib_ticks and clears it
  uint64_t calib_ticks;
  uint64_t xl_n;         // GPU peer lanes to poll (0 while none is registered: no cost on the ring's path)
  uint64_t relay;        // device address of a RelayTable (server.hpp): kMethodRelay calls go through it
  uint64_t pad[4];
};
static_assert(sizeof(ServerCtrl) == 128, "ServerCtrl layout");

}  // namespace ptype
