// Sorted exchange: the multi-GPU Send with mailbox delivery, where the sender's
// counting sort does the receiver's enqueue.
//
// Every rank sorts its batch stably straight into the per-peer request regions
// of the all-to-all (count / scan / scatter, the building blocks of
// sort_common.hpp): by destination rank alone when its batch carries no ordered
// method, by (destination rank, destination actor shard) when it may.  A region
// therefore arrives as the SENDER'S part of the receiver's actor mailboxes --
// one message-ordered queue, or 64 shard runs (an actor's messages in message
// order within its run) plus a shard table (header flag kFlagSharded).  The
// receiver runs no enqueue pass at all -- its drains read the received regions
// as its mailboxes, chosen per region:
//   * parallel drain (unsharded regions): every record runs independently,
//     replies land at the record's position of the reply region (coalesced);
//   * ordered drain (sharded regions): one block per shard takes that shard's
//     runs of every sharded region in source-rank order, actors' state in LDS,
//     each actor's records one at a time in ring order (LDS bins), so every
//     (sender, actor) pair is FIFO.
// The sender's completion gathers each message's reply through the position
// the scatter recorded (perm).  Per message on the wire: the wire-v3 packed
// record (packed.hpp) and a packed reply.
//
// No host wait per Send.  Region geometry (record layout L, per-peer capacity
// C) cannot be agreed within a Send without a host round trip (RCCL's sizes
// are host arguments), so Send k uses the agreement of Send k - 2: every Send
// folds its own column maxima and busiest bucket into a 16-word vector on the
// device, all-reduces it (MAX) on the comm stream and copies it to pinned host
// memory; two Sends later every rank derives the same L and C from it (the lag
// is fixed, so ranks never disagree on a geometry).  Sends 0 and 1 use the
// widest layout.  A message that does not fit the layout in force (a field
// wider than agreed, or its bucket past C) is answered STATUS_OVERFLOW --
// send_all re-sends it -- and its slot carries a null record (mailbox field all
// ones, which no real mailbox uses: the agreed width leaves room for it).
// The all-to-alls need no host sizes of their own either: padded regions
// (ncclAllToAll, equal split) while traffic is even, and under skew the agreed
// per-(sender, destination) capacities -- the same lag-2 agreement carries the
// R x R matrix of region totals -- whose region prefixes move by grouped
// ncclSend / ncclRecv (each region is [header][shard table][records], so its
// used part is a prefix).  Either way the step captures into a hipGraph.
//
// Reference: the batched fan-out this replaces is the optimus coordinator's
// goroutine-per-range Calls (example/optimus/coordinator/coordinator.go:67-98)
// over cluster/rpc.go:69-105; the per-request server goroutine of net/rpc
// (example/calculator/server/server.go:16-20) is the mailbox drain.
#pragma once
#include <memory>
#include <vector>

#include "engine.hpp"
#include "packed.hpp"

namespace ptype {

constexpr int kSxShardBits = 6;  // actor shards per rank on the wire: mailbox & 63
constexpr int kSxShards = 1 << kSxShardBits;
constexpr int kSxMaxRanks = 16;
constexpr int kSxMaxChunks = 4;
constexpr int64_t kSxSmallSend = 2 << 20;  // Sends of up to this many messages: collectives on the caller's stream
constexpr int kSxTableWords = (kSxShards + 1 + 3) & ~3;  // shard table, right after a request region's header
constexpr int kSxRecOff = 4 + kSxTableWords;             // records start here: a region's used part is a prefix
// request region words for n records of S dwords: [header 4][shard table][n * S], 16-B padded
__host__ __device__ inline int64_t sx_req_words(int64_t n, int S) { return (kSxRecOff + n * S + 3) & ~3ll; }
// The agreement vector: the packed meta words, then the R x R matrix of
// per-(sender, destination) region totals (row = sender; the MAX all-reduce
// fills every row) -- the per-pair capacities of Send + 2.
constexpr int kSxMetaPair = kMetaWords;
constexpr int kSxMetaWords = kMetaWords + kSxMaxRanks * kSxMaxRanks;
struct SxCaps {  // per-destination capacities (records), by value into the sender's kernels
  uint32_t c[kSxMaxRanks];
};

struct SxSend {
  uintptr_t actor = 0, a0 = 0, a1 = 0, a2 = 0, method_col = 0;
  int method_uniform = 0;
  int64_t M = 0;
  uintptr_t table = 0;
  uint64_t cap = 0;
  uintptr_t dir = 0;
  uintptr_t dir_rank = 0;  // the directory's rank byte table (stateless batches: rank-only gathers)
  uint32_t n_dir = 0, affine_w = 0;
  uintptr_t out_val = 0, out_st = 0, state = 0;
  uint32_t n_state = 0;
  uint64_t delay_ticks = 0;
  bool ordered = false;  // receivers run each actor's records one at a time in ring order
  uintptr_t stream = 0;
};

struct SxWire {
  PackedLayout L{};
  int S = 0;                // dwords per request record as moved (L.S rounded to a kernel variant)
  int64_t C = 0;            // per-peer capacity (records) of this Send
  int64_t req_words = 0;    // region stride (per peer, per chunk; the moved prefix may be shorter)
  int64_t rep_words = 0;
  int64_t req_moved = 0;    // words this rank sends per chunk, all peers (requests / replies)
  int64_t rep_moved = 0;
  bool pairs = false;       // per-pair capacities in force (prefixes moved by grouped send / recv)
  uint32_t cap_out[kSxMaxRanks] = {};  // this rank's capacity per destination
  uint32_t cap_in[kSxMaxRanks] = {};   // per source
  bool agreed = false;      // L and C came from an agreement (else the start-up wide layout)
  bool shard_ok = true;     // sharded (ordered) regions may be sent this Send (else ordered messages overflow)
  int route_mode = 0;       // sender resolution: 0 hash, 1 directory, 2 affine, 3 rank byte table
  int64_t spec_from = -1;   // the Send whose agreement they came from
  uint64_t meta[kMetaWords] = {};
};

class SortedExchange {
 public:
  // R ranks (comm: the process group's ncclComm_t, or fake), batches of up to
  // chunks * max_chunk messages; C_alloc: per-peer capacity the buffers hold;
  // C0: the start-up capacity (until the first agreement applies).
  SortedExchange(int device, uintptr_t comm, int R, int rank, int64_t max_chunk, int chunks, int64_t C_alloc,
                 int64_t C0, std::shared_ptr<HostComm> fake = nullptr);
  ~SortedExchange();
  void send(const SxSend& a);
  const SxWire& last_wire() const { return wire_; }
  int64_t sends() const { return sends_; }
  int ranks() const { return R_; }
  // receiver counters: handler failures, replies wider than agreed; sender: one-pass look-backs that gave up (0)
  std::vector<uint64_t> stats() const;
  // Messages answered STATUS_OVERFLOW by the last Send, max over the ranks (0: no
  // rank must re-send).  Waits for that Send's agreement copy -- one host wait on
  // an event already queued, no collective of its own.
  uint64_t last_overflow() const;
  // The same count for Send k (its agreement buffer is reused by Send k + 2: valid
  // until then).  Send k's copy completes before Send k + 2 can even pick its
  // layout, so a caller that resolves Send k just before Send k + 2 waits on
  // nothing the pipeline would not wait on anyway.
  uint64_t overflow_of(int64_t k) const;
  // host time: every send() call, and the part of it spent waiting for an
  // agreement (pick_spec: Send k - 2's; last_overflow / overflow_of: counted apart)
  struct HostProfile {
    uint64_t sends = 0, total_ns = 0, spec_wait_ns = 0, overflow_waits = 0, overflow_wait_ns = 0;
  };
  HostProfile host_profile() const { return prof_; }
  // the one-pass sort's epoch counter (tests: preset near the 2^24 tag wrap); synchronous
  void set_epoch_counter(uint32_t v);
  uint32_t epoch_counter() const;

 private:
  struct Bufs {
    uint32_t *send = nullptr, *recv = nullptr, *reply = nullptr, *back = nullptr;
    int32_t* perm = nullptr;
  };
  void pick_spec(hipStream_t cs);
  void wait_event(hipEvent_t e) const;
  void adopt(const uint64_t* meta, int64_t from);
  // regions `stride` bytes apart; send[q] / recv[q] bytes of each (nullptr: whole regions)
  void a2a(const void* src, void* dst, size_t stride, const size_t* send, const size_t* recv, bool grouped_p2p);
  void allreduce_meta(uint64_t* dev, hipStream_t s);
  bool collectives() const { return cell_ != nullptr || fake_ != nullptr; }

  int device_;
  CommCell* cell_;  // the data plane's RCCL communicator (dp_link.hpp), or null
  std::shared_ptr<HostComm> fake_;
  int R_, rank_, chunks_;
  int64_t max_chunk_, C_alloc_;
  hipStream_t comm_stream_ = nullptr;
  hipStream_t cur_comm_ = nullptr;  // the stream this Send's collectives go on (comm_stream_, or the caller's)
  hipStream_t last_comm_ = nullptr;  // comm_stream_ when the last eager Send's collectives went there
  Bufs bufs_[kSxMaxChunks];
  uint32_t* hist_ = nullptr;  // [G][R * K] per-block bucket counts -> prefixes (K = 64 or 1)
  uint32_t* boff_ = nullptr;  // [R * K] bucket offsets within their region
  unsigned long long* desc_ = nullptr;  // [tiles][R] one-pass look-back descriptors (rank-only batches)
  unsigned* tctr_ = nullptr;    // [0] one-pass tile counter (self-resetting), [1] its epoch tag
  unsigned* ticket_ = nullptr;  // last-block ticket of the one-pass kernel (self-resetting)
  uint32_t* rcnt_ = nullptr;    // [chunks][kSxMaxRanks] one-pass run reservations per region (self-resetting)
  uint32_t* first_ovf_ = nullptr;  // sharded Sends: per-bucket first overflowed message index (+ an any-word)
  uint64_t* meta_dev_ = nullptr;   // [2][kSxMetaWords] agreement vectors (device)
  uint64_t* meta_host_ = nullptr;  // [2][kSxMetaWords] pinned copies
  unsigned long long* stats_ = nullptr;  // [2] receiver counters
  hipEvent_t ev_meta_[2]{};
  hipEvent_t ev_join_{};  // device-side comms: the comm stream joined back into the caller's
  int64_t meta_send_[2] = {-1, -1};  // the Send whose agreement each buffer holds
  bool meta_zeroed_[2] = {false, false};  // cleared by the previous Send's first completion launch
  hipEvent_t ev_routed_[kSxMaxChunks]{}, ev_req_in_[kSxMaxChunks]{}, ev_served_[kSxMaxChunks]{},
      ev_rep_in_[kSxMaxChunks]{};
  // the layout and capacity in force
  PackedLayout L_{};
  int64_t C_ = 0;
  bool agreed_ = false;
  int64_t spec_from_ = -1;
  uint64_t spec_meta_[kMetaWords] = {};
  static constexpr int kNeedWindow = 4;      // capacity: the busiest bucket of the last 4 agreements
  uint64_t need_hist_[kNeedWindow] = {};
  uint64_t pair_hist_[kNeedWindow][kSxMaxRanks * kSxMaxRanks] = {};  // per-pair totals of the same agreements
  int need_n_ = 0;
  // per-pair capacities in force (row = sender); pairs_: they differ enough from
  // the uniform C that moving prefixes pays (the same decision on every rank)
  uint32_t cap_[kSxMaxRanks * kSxMaxRanks] = {};
  bool pairs_ = false;
  bool self_copy_ = false;  // tune sx_self_copy (read per Send)
  int64_t sends_ = 0;
  SxWire wire_;
  mutable HostProfile prof_;
};

// The layout of an agreement: packed_layout with a mailbox field one bit wider
// than the largest mailbox, so the all-ones value is free for null records.
PackedLayout sx_layout(const uint64_t* meta);

}  // namespace ptype
