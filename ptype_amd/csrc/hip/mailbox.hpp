// HBM actor mailboxes (SURVEY K2 `mailbox_enqueue`, K3 `dispatch` in epoch and
// persistent form): the queue between a message's arrival on a GPU and its
// actor running it.
//
// Reference: net/rpc gives every request its own goroutine on the server
// (stdlib; registered at example/calculator/server/server.go:16-20, served at
// :38; calls leave the client at cluster/rpc.go:65 and :88).  Here the queue is
// explicit and lives in HBM:
//
//   * S shards per GPU (power of two); actor (local mailbox) m belongs to shard
//     m & (S - 1), so an actor's messages always meet in one ring.
//   * each shard is a ring of Q 32-B records:  half A {tag, mbox, origin,
//     method | flags << 16}, half B {a0, a1}; a2 (3-argument methods) in a side
//     array.  tag = (position >> log2 Q) + 1: the lap the slot was published in,
//     so a consumer tells a fresh record from last lap's without any flag word.
//   * per-shard counters on their own cache lines: tail (reservations), done
//     (positions a producer has finished: written, or given up as overflow),
//     head (consumed; the consumer's, read by producers for the capacity check).
//
// Producers (K2) reserve ring positions with ONE atomicAdd per (tile, shard):
// a block stages a tile of messages, ranks them per shard with LDS atomics and
// reserves each shard's run at once.  A position that would overwrite an
// unconsumed record is not written: that message is answered
// kStatusOverflow on the spot (the Send re-sends it), its position becomes a
// hole, and `done` still counts it.  A consumer treats a position whose tag
// never arrives as a hole once the shard is quiescent (done == tail).
//
// Consumers (K3) run handlers in ring order per actor:
//   * epoch form: launched behind the enqueue on the same stream (graph-
//     capturable); stateless / commutative methods drain every shard with the
//     whole grid, ordered methods (records.hpp method_ordered) one wave per
//     shard;
//   * persistent form: a grid well below residency (RCCL keeps its CUs) whose
//     waves each own a set of shards, poll tags + s_sleep, and drain
//     concurrently with producers on other streams; the host's stop flag makes
//     them drain what is left and exit.  Producers store records write-through
//     (sc1, B half drained before the tag half); the consumer reads tags,
//     counters and records with no-op atomics, which execute at the memory side:
//     an sc1 load is served by the reading XCD's own (non-coherent) L2, and a
//     line it cached before the producer wrote stays stale there (observed: a
//     consumer that never saw its records).
// Within a 64-record window the owning wave finds actors that appear twice
// (an LDS owner table) and runs just those lanes one at a time, in lane = ring
// order; everything else runs in parallel.
#pragma once
#include <memory>
#include <vector>

#include "common.hpp"
#include "handlers.hpp"

namespace ptype {

constexpr int kMboxCtrStride = 32;  // u64 words per shard: [0] tail, [1] done (one line), [16] head (another)
constexpr int kMboxCtrTicket = 24;  // [24]: the epoch drain's per-shard last-block ticket (self-resetting)
constexpr int kMboxMaxShards = 4096;
// Sorted epoch mailboxes (mailbox_sort.hip): shard limit, and the per-(block,
// shard) histogram's size -- it bounds the count / scatter grid (G <= words / S)
constexpr int kMboxSortMaxShards = 1024;
constexpr uint32_t kMboxSortHistWords = 1u << 18;
constexpr uint32_t kMboxSortGroups = 32;  // group sums of 32 blocks each (G <= 1024)
enum MboxStat : int {
  kMbEnqueued = 0,   // records written into rings
  kMbOverflow = 1,   // messages answered kStatusOverflow (ring full)
  kMbNoActor = 2,    // registry miss / not this rank's actor
  kMbProcessed = 3,  // records run by a consumer
  kMbFailed = 4,     // handler status != ok
  kMbHoles = 5,      // positions skipped as holes
  kMbSerial = 6,     // records run serialised (same actor twice in a window)
  kMbSpilled = 7,    // stateless messages whose ring was full, run from the batch by the drain
  kMbTicket = 8,     // reserved (the epoch drain's tickets are per shard: kMboxCtrTicket)
  kMbLookback = 9,   // one-pass sort: look-backs that gave up waiting (a bug guard; must stay 0)
  kMbStatWords = 16,
};
constexpr int kMbStripes = 32;  // stats copies (block-striped atomics; stats() sums them)

struct MboxView {
  // records: half A {tag, mailbox, origin, method | flags}, half B {a0, a1}, 16 B
  // each; `planar`: [2][S * Q][4] words (two planes), else [S * Q][8] (32-B records)
  uint32_t* rec = nullptr;
  int64_t* a2 = nullptr;    // [S * Q]
  unsigned long long* ctr = nullptr;
  unsigned long long* stats = nullptr;
  uint32_t log_s = 0, log_q = 0;
  uint32_t planar = 0;
  uint64_t b_off = 0;  // planar: word offset of plane B (past plane A + a de-aliasing pad)
  // one-pass sorts of stateless batches: per-shard run reservations, one counter per
  // 128-B line (kResvStride words; null: the epoch totals are in the group sums)
  uint32_t* resv = nullptr;
};
constexpr int kResvStride = 32;

// Host-visible control block of the persistent consumer.
struct alignas(64) MboxCtrl {
  uint64_t stop;
  uint64_t live_waves;  // waves still running
  uint64_t processed;
  uint64_t exits_idle;
  uint64_t exits_lifetime;
  uint64_t pad[3];
};

// Where replies go, indexed by the record's origin (< n): SoA outputs (a local
// Send: origin = message index), or -- mailbox delivery on receipt at N > 1 --
// the epoch's wire-v2 reply regions (origin = source rank * C + slot position),
// which the reverse all-to-all takes back to the senders.
struct ReplyView {
  int64_t* val = nullptr;
  int32_t* st = nullptr;
  uint64_t n = 0;
  uint32_t* slots = nullptr;
  int64_t rep_words = 0;
  uint32_t C = 0;
};

struct PackedLayout;
void launch_mailbox_enqueue_slots_packed(const MboxView& mv, uintptr_t recv, int R, int64_t C, const PackedLayout& L,
                                         const ReplyView& rv, int64_t expected_per_rank, bool arrival,
                                         uintptr_t stream);
void launch_mailbox_enqueue(const MboxView& mv, uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2,
                            uintptr_t method_col, int method_uniform, int64_t M, uintptr_t table, uint64_t cap,
                            uintptr_t dir, uint32_t n_dir, uint32_t affine_w, int rank_self, uint32_t origin_base,
                            const ReplyView& rv, bool live, uintptr_t stream, bool arrival = false);
void launch_mailbox_enqueue_slots(const MboxView& mv, uintptr_t recv, int R, int64_t C, int nargs, bool mc,
                                  const ReplyView& rv, int64_t expected_per_rank, bool arrival, uintptr_t stream);
void launch_mailbox_drain(const MboxView& mv, uintptr_t state, uint32_t n_state, uint64_t delay_ticks,
                          const OutboxView& ob, const ReplyView& rv, bool ordered, uintptr_t stream,
                          int fixed_method = 0);
void launch_mailbox_consumer(const MboxView& mv, MboxCtrl* ctrl, uintptr_t state, uint32_t n_state,
                             uint64_t delay_ticks, const ReplyView& rv, int blocks, uint64_t idle_ticks,
                             uint64_t max_ticks, uintptr_t stream);

// One epoch Send through the sorted mailboxes (Mailboxes::send_sorted).
struct MboxSend {
  uintptr_t actor = 0, a0 = 0, a1 = 0, a2 = 0, method_col = 0;
  int method_uniform = 0;
  int64_t M = 0;
  uintptr_t table = 0;
  uint64_t cap = 0;
  uintptr_t dir = 0;
  uint32_t n_dir = 0, affine_w = 0;
  int rank_self = 0;
  uint32_t origin_base = 0;
  uintptr_t out_val = 0, out_st = 0;
  uint64_t out_n = 0;
  uintptr_t state = 0;
  uint32_t n_state = 0;
  uint64_t delay_ticks = 0;
  std::vector<uintptr_t> outbox;
  uint64_t outbox_cap = 0;
  bool arrival = false;  // shard by arrival tile (batches without ordered methods)
  bool ordered = true;   // ordered drain: per-actor serial, FIFO; else the parallel drain
  int fixed_method = 0;  // every message carries this method (constant-folded handler)
  // sort kernels: 0 auto (tune mbox_sort, else one-pass for stateless batches and from 1024
  // tiles on), 1 one-pass (stateless: run reservations; ordered: look-back), 2 count + scatter
  int sort_mode = 0;
  uintptr_t stream = 0;
  // the directory's rank byte table (one byte per id): a stateless uniform batch
  // resolves only its rank (1 MB at 1 M ids, L2-resident, against the 4 MB
  // directory) and its records carry the actor id, which no stateless handler reads
  uintptr_t dir_rank = 0;
  // route mode 4's presence map of the directory, kept by the registry mirror for
  // rank pres_rank (rebuilt with the directory; RegistryTable.presence): used when it is
  // this Send's rank, else the Send folds its own from dir_rank
  uintptr_t pres = 0;
  int pres_rank = -1;
};

// Route mode 4's presence map: 2 bits per directory id for rank `rank` (mailbox_sort.hip)
uint32_t presence_words(uint32_t n_dir);
void launch_presence(uintptr_t dir_rank, uint32_t n_dir, int rank, uintptr_t out, uintptr_t stream);

class Mailboxes {
 public:
  Mailboxes(int device, uint32_t shards, uint32_t slots, bool with_a2);
  ~Mailboxes();

  // Epoch Send (mailbox_sort.hip): K2 as a stable counting sort of the batch into
  // the shard rings (count, scan, scatter: every ring in message order), then
  // the ordered or parallel K3 drain; replies at origin_base + message index.
  // The rings must be empty of live records (no persistent session running).
  void send_sorted(const MboxSend& a);

  // K2 from a SoA client batch resolved against the registry mirror (this rank's
  // actors only); origin of message i = origin_base + i.  `live`: a persistent
  // consumer may be draining concurrently (write-through, ordered publication).
  // `arrival`: shard by arrival tile, not by actor (batches without ordered methods).
  void enqueue(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col, int method_uniform,
               int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir, uint32_t affine_w,
               int rank_self, uint32_t origin_base, uintptr_t out_val, uintptr_t out_st, uint64_t out_n, bool live,
               uintptr_t stream, bool arrival = false);
  // K3 epoch form: drain everything enqueued before it on `stream`.
  void drain(uintptr_t state, uint32_t n_state, uint64_t delay_ticks, uintptr_t out_val, uintptr_t out_st,
             uint64_t out_n, bool ordered, uintptr_t stream, const std::vector<uintptr_t>& outbox = {},
             uint64_t outbox_cap = 0, int fixed_method = 0);
  // K3 persistent form on its own stream.
  void start(uintptr_t state, uint32_t n_state, uint64_t delay_ticks, uintptr_t out_val, uintptr_t out_st,
             uint64_t out_n, int blocks, double idle_ms, double max_s);
  // Ask the persistent consumer to drain what is queued and exit; waits for it.
  void stop();
  bool running() const;
  void reset(uintptr_t stream);  // counters and rings to empty (no consumer may be running)

  std::vector<uint64_t> stats() const;            // kMbStatWords device counters
  // the one-pass sort's epoch counter (tests: preset near the 2^24 tag wrap); synchronous
  void set_epoch_counter(uint32_t v);
  uint32_t epoch_counter() const;
  std::vector<uint64_t> shard_counters() const;   // [tail, done, head] per shard
  uint32_t shards() const { return 1u << mv_.log_s; }
  uint32_t slots() const { return 1u << mv_.log_q; }
  uint64_t bytes() const { return bytes_; }
  // ring record bytes of the last sorted Send (8: 8-B records, 16: compact, 32: long records in use)
  int last_record_bytes() const { return last_rec_bytes_; }
  // shards the last sorted Send's rings were viewed as (stateless batches: a coarser view, 8 by default)
  uint32_t last_view_shards() const { return last_view_shards_; }
  // the last sorted Send's route: 0 hash probe, 1 directory, 2 affine rule, 3 rank byte table
  int last_route() const { return last_route_; }
  uint64_t consumer_processed() const;
  uint64_t launches() const { return launches_; }
  const MboxView& view() const { return mv_; }

 private:
  int device_;
  MboxView mv_;
  uint64_t bytes_ = 0;
  uint64_t rec_bytes_ = 0;  // the record planes (+ pad)
  MboxCtrl* ctrl_ = nullptr;   // pinned host
  MboxCtrl* dctrl_ = nullptr;  // its device address
  hipStream_t stream_ = nullptr;
  bool started_ = false;
  uint64_t launches_ = 0;
  uint32_t* sort_hist_ = nullptr;   // [G][S] per-block shard counts (send_sorted)
  uint32_t* sort_gsum_ = nullptr;   // [kMboxSortGroups][S] group sums (zero between Sends: the drains clear them)
  unsigned* sort_ticket_ = nullptr; // last-block ticket of the parallel drain (self-resetting)
  uint32_t* sort_rw_ = nullptr;     // [M] each message's mailbox (route word), count -> scatter
  uint32_t* sort_sidx_ = nullptr;   // [M] each message's ring slot (message-order drain; spilled tiles)
  uint32_t* sort_tinfo_ = nullptr;  // [tiles][2][S] each tile's runs: slot bias, count (ring-order drain / completion)
  unsigned long long* sort_desc_ = nullptr;  // [tiles][S] one-pass sort: per-tile shard counts / prefixes (look-back)
  unsigned* sort_tctr_ = nullptr;   // [0] one-pass sort's tile counter (self-resetting), [1] its epoch tag
  uint64_t sort_cap_ = 0;           // messages the two arrays hold
  int last_rec_bytes_ = 0;
  uint32_t last_view_shards_ = 0;
  int last_route_ = -1;
  uint32_t* sort_resv_ = nullptr;   // [S][kResvStride] one-pass run reservations (zero between Sends)
  uint32_t* pres_ = nullptr;        // route mode 4: 2-bit presence map of the route directory (per Send)
  const uint32_t* pres_view_ = nullptr;  // the map this Send reads (pres_, or the registry mirror's)
  void build_presence(const MboxSend& a, hipStream_t st);
  uint64_t pres_words_ = 0;
  // 8-B ring records: [0] the field widths in force (device; updated by each Send's
  // last block), per-tile field bit lengths, and a pinned mirror of [0] (bit 31: the
  // fields no longer fit 64 bits -- the host then keeps 16-B records)
  uint32_t* r8w_ = nullptr;
  uint32_t* r8max_ = nullptr;
  uint32_t* r8host_ = nullptr;
  int64_t* r8esc_ = nullptr;  // ordered 8-B records: escape records' {a0, mailbox} by ring slot
  uint64_t r8_tiles_ = 0;
  // ordered drain: replies staged at ring slots [S * Q], one 16-B word each
  // (value lo, value hi, status, 0) -- one gather per message in the completion
  void* stage_rep_ = nullptr;
};

}  // namespace ptype
