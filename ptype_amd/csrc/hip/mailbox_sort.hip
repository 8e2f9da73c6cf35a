// Sorted epoch mailboxes: K2 as a stable counting sort into the shard rings,
// K3 as a ring-order parallel drain or an LDS-binned ordered drain.
//
// The epoch form of a Send (mailbox.hpp has the ring layout) runs
//
//   sort     every message goes into its shard's ring at (tail + prefix + rank),
//            the rank computed in message order (wave match on the shard bits +
//            per-wave counts), so each ring holds its messages in MESSAGE ORDER:
//            every actor's mailbox is FIFO by construction, with no atomic per
//            message.  Two forms:
//              one pass (batches of >= 1024 tiles): a block claims the next tile,
//              resolves it (one route-directory gather per message), ranks it,
//              and finds its prefix by a decoupled look-back over earlier tiles'
//              descriptors (mbx_onesweep_kernel);
//              count + scatter: the count resolves and histograms per block
//              (+ group sums over 32 blocks); each scatter block's prefix is the
//              group sums before its group plus at most 31 rows inside it (no
//              scan pass);
//            either records each tile's runs (slot bias + count per shard) for
//            the drains;
//   drain    parallel (batches without ordered methods): one block per tile reads
//            the tile's runs in ring order (whole lines), stages the replies in
//            LDS at their place in the tile and writes them out coalesced;
//            ordered: one block owns one shard -- its actors' state staged in
//            LDS -- and runs each actor's records one at a time in ring order,
//            distinct actors side by side (LDS bins), replies staged at their
//            ring slots; a ring-order completion puts them in message order.
//
// Stateless batches use an 8-shard view of the rings (every ring is empty
// between epoch Sends): longer runs per tile and shard.  Arrival sharding
// (stateless only) skips the sort: tile t's messages sit at fixed positions of
// ring t mod S.
//
// Records are 16 B in the common case (compact form, plane A only):
//   w0 = origin | kCompactMark    (bit 31 marks an epoch record; a live ring's
//                                  lap tags never have it)
//   w1 = mailbox (24 bits) | method << 24 (7 bits)
//   w2, w3 = a0, a1 as int32
// 8 B for stateless batches of one method with two arguments (in.rec8, set by
// the host: one u64 per slot of plane A viewed as 8-B cells):
//   bits [0, 12) place in the tile (the drains know the tile) | mailbox (wm bits)
//   | zigzag a0 (w0 bits) | zigzag a1 (w1 bits),   12 + wm + w0 + w1 = 64
// where a message whose mailbox or arguments do not fit the fields SPILLS (its
// tile is drained in message order, the message run straight from the batch).
// The widths are a device word the previous Send's last block sets from that
// Send's per-tile field maxima (no host read): a batch whose values grow spills
// for one Send, then fits;
// and 32 B (+ the a2 side array) when an argument needs 64 bits or a third
// argument is present (long form: w1 bit 31, w2 = method | flags << 16, plane B
// {a0, a1}).  The tagged 32-B records of mailbox.hip stay the format of live
// sessions (persistent consumer) and of delivery on receipt.
//
// XCD-aware placement (MI355X: 8 XCDs, per-XCD L2s, blocks dealt round-robin):
// count / scatter block b takes the range of virtual block (b % 8) * G/8 + b / 8,
// so each XCD owns one contiguous eighth of the batch -- and therefore one
// contiguous part of every shard's run, whose partially written lines meet in
// ONE L2.
//
// Reference: the server's per-request goroutine of stdlib net/rpc
// (example/calculator/server/server.go:16-20, :38; handler
// example/calculator/calculator.go:9-12) -- here an explicit FIFO queue in HBM.
#include "mailbox_sort_dev.hpp"

namespace ptype {

static bool fused_ok(int64_t tiles) {
  const int f = tune().mbox_fused;
  return f == 1 || (f < 0 && tiles <= 512);
}

// Removed variants (measured slower or flat; A/B rows in profiles/r4_mailbox_ab.md and
// profiles/r5_mailbox_ab.md): the look-back sort for stateless batches (run reservations
// won), the persistent reserving sort (42.8 vs 50.5 G msg/s), 1024- and 2048-message tiles
// for the fused / separate sort, arguments loaded after the look-back, the LDS-table count,
// the group look-back, non-temporal directory gathers and reply stores, the binned ordered
// drain (233 vs 175 us), 2048-record ordered windows, the ordered drain without the
// register fold or the prefetched window, 16-B ordered records at 8 Mi, the wide ring
// drain and the 8 / 16 / 32-shard stateless views other than 8.
uint32_t presence_words(uint32_t n_dir) { return n_dir <= kPresMax ? pres_words(n_dir) : 0u; }
void launch_presence(uintptr_t dir_rank, uint32_t n_dir, int rank, uintptr_t out, uintptr_t stream) {
  if (n_dir == 0 || n_dir > kPresMax || !dir_rank || !out) throw std::invalid_argument("presence: 1 <= n_dir <= 2^18");
  const uint32_t nw = pres_words(n_dir);
  hipLaunchKernelGGL(mbx_presence_kernel<>, dim3((nw + 255) / 256), dim3(256), 0, as_stream(stream),
                     (const uint8_t*)dir_rank, n_dir, rank, (uint32_t*)out);
  PT_HIP_CHECK(hipGetLastError());
}

// Route mode 4's presence map of this Send's directory: the registry mirror's (rebuilt
// with the directory) when it is kept for this Send's rank, else folded here, every Send
// (the directory may have changed since the last one; 128 KB read for 131072 ids).
void Mailboxes::build_presence(const MboxSend& a, hipStream_t st) {
  if (a.pres && a.pres_rank == a.rank_self) {
    pres_view_ = (const uint32_t*)a.pres;
    return;
  }
  const uint32_t nw = pres_words(a.n_dir);
  if (nw > pres_words_) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      throw std::runtime_error("mailbox send: first presence-map Send inside a graph capture (warm up first)");
    PT_HIP_CHECK(hipStreamSynchronize(st));
    if (pres_) PT_HIP_CHECK(hipFree(pres_));
    PT_HIP_CHECK(hipMalloc((void**)&pres_, (size_t)nw * 4));
    pres_words_ = nw;
  }
  pres_view_ = pres_;
  hipLaunchKernelGGL(mbx_presence_kernel<>, dim3((nw + 255) / 256), dim3(256), 0, st, (const uint8_t*)a.dir_rank,
                     a.n_dir, a.rank_self, pres_);
  PT_HIP_CHECK(hipGetLastError());
}

void Mailboxes::send_sorted(const MboxSend& a) {
  const uint32_t S = shards();
  if (S > (uint32_t)kMboxSortMaxShards) throw std::invalid_argument("sorted mailboxes: at most 1024 shards");
  if ((uint64_t)S * slots() > 0xfffffffeull) throw std::invalid_argument("sorted mailboxes: shards * slots < 2^32");
  if (started_ && running()) throw std::runtime_error("mailbox send: a persistent consumer owns the rings");
  if (a.M <= 0) return;
  if (!a.actor || !a.a0) throw std::invalid_argument("mailbox send: missing column");
  if (a.a2 && !mv_.a2) throw std::invalid_argument("mailbox send: 3-argument batch but the rings have no a2 array");
  if (a.cap == 0 || (a.cap & (a.cap - 1))) throw std::invalid_argument("table capacity must be a power of two");
  if (!a.out_val || !a.out_st) throw std::invalid_argument("mailbox send: reply outputs required");
  if ((uint64_t)a.origin_base + (uint64_t)a.M > a.out_n) throw std::invalid_argument("mailbox send: reply view too small");
  if ((uint64_t)a.origin_base + (uint64_t)a.M > 0x7fffffffull) throw std::invalid_argument("mailbox send: origin >= 2^31");
  if (a.arrival && a.ordered) throw std::invalid_argument("mailbox send: arrival sharding cannot serve ordered methods");
  PT_HIP_CHECK(hipSetDevice(device_));
  hipStream_t st = as_stream(a.stream);
  const Tune tn = tune();
  auto capturing = [&] {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
  };
  const int64_t tiles = (a.M + kSTile - 1) / kSTile;
  if (tiles > 0xffffffffll) throw std::invalid_argument("mailbox send: batch too large");
  // per-message workspace (route words, ring slots) and per-tile runs: grown outside graph capture
  if (!a.arrival && (uint64_t)a.M > sort_cap_) {
    if (capturing()) throw std::runtime_error("mailbox send: a larger batch than before inside a graph capture (warm up first)");
    PT_HIP_CHECK(hipStreamSynchronize(st));
    for (void** p : {(void**)&sort_rw_, (void**)&sort_sidx_, (void**)&sort_tinfo_, (void**)&sort_desc_})
      if (*p) {
        PT_HIP_CHECK(hipFree(*p));
        *p = nullptr;
      }
    PT_HIP_CHECK(hipMalloc((void**)&sort_rw_, (size_t)a.M * 4));
    PT_HIP_CHECK(hipMalloc((void**)&sort_sidx_, (size_t)a.M * 4));
    PT_HIP_CHECK(hipMalloc((void**)&sort_tinfo_, (size_t)tiles * 2 * S * 4));
    // look-back descriptors: zero = no tag (every Send's tag is >= 1)
    PT_HIP_CHECK(hipMalloc((void**)&sort_desc_, (size_t)tiles * S * 8));
    PT_HIP_CHECK(hipMemsetAsync(sort_desc_, 0, (size_t)tiles * S * 8, st));
    PT_HIP_CHECK(hipStreamSynchronize(st));
    sort_cap_ = (uint64_t)a.M;
  }
  if (a.ordered && !stage_rep_) {
    if (capturing()) throw std::runtime_error("mailbox send: first ordered Send inside a graph capture (warm up first)");
    const uint64_t n = (uint64_t)S * slots();
    PT_HIP_CHECK(hipMalloc(&stage_rep_, n * 16));
    bytes_ += n * 16;
  }
  SortIn in{};
  in.actor = (const uint32_t*)a.actor;
  in.a0 = (const int64_t*)a.a0;
  in.a1 = (const int64_t*)a.a1;
  in.a2 = (const int64_t*)a.a2;
  in.mcol = (const uint16_t*)a.method_col;
  in.method_uniform = (uint32_t)a.method_uniform;
  in.M = a.M;
  in.table = (const TableEntry*)a.table;
  in.mask = a.cap - 1;
  in.dir = (const uint32_t*)a.dir;
  in.dirr = (const uint8_t*)a.dir_rank;
  in.n_dir = a.n_dir;
  in.aw = a.affine_w;
  in.aw_shift = (a.affine_w && (a.affine_w & (a.affine_w - 1)) == 0) ? __builtin_ctz(a.affine_w) : -1;
  in.rank_self = a.rank_self;
  in.origin_base = a.origin_base;
  in.tiles = (uint32_t)tiles;
  // blocks: as many as the histogram holds (it stays L2-resident for the prefixes),
  // a multiple of 8 (one contiguous eighth of the batch per XCD)
  int64_t G = std::min<int64_t>({tiles, (int64_t)(kMboxSortHistWords / S), (int64_t)1024,
                                 (int64_t)kMboxSortGroups * kGroupBlocks});
  if (G >= 8) G -= G % 8;
  G = std::max<int64_t>(G, 1);
  in.G = (uint32_t)G;
  in.tpb = (uint32_t)((tiles + G - 1) / G);
  // one block per tile (tile-granular kernels), dealt XCD by XCD: a multiple of 8
  const uint32_t tile_grid = (uint32_t)(tiles >= 8 ? (tiles + 7) / 8 * 8 : tiles);
  // the sort: one pass, or count + scatter.  Stateless batches always take the one pass (each
  // tile reserves its runs: no look-back); ordered ones look back, which a grid under 1024
  // tiles cannot hide (8 Mi msgs 0.212-0.221 vs 0.228-0.230 ms per Send; 1 Mi msgs 0.047-0.049
  // vs 0.043 for count + scatter).  Tune mbox_sort=1 / 2 forces either.
  const int sort_mode = a.sort_mode ? a.sort_mode
                        : tn.mbox_sort ? tn.mbox_sort
                        : (tiles >= 1024 || (!a.ordered && !a.arrival)) ? 1 : 2;
  if (sort_mode < 1 || sort_mode > 2) throw std::invalid_argument("mailbox send: sort_mode 0..2");
  const bool two_pass = sort_mode == 2;
  const uint32_t ngroups = two_pass ? (uint32_t)((G + kGroupBlocks - 1) / kGroupBlocks) : 1u;
  const int mode = (a.affine_w && a.n_dir) ? 2 : (a.dir && a.n_dir) ? 1 : 0;
  ReplyView rv{(int64_t*)a.out_val, (int32_t*)a.out_st, a.out_n};
  OutboxView ob;
  if (a.outbox_cap) {
    if (a.outbox.size() != 6) throw std::invalid_argument("outbox: [actor, a0, a1, a2, method, count]");
    ob.actor = (uint32_t*)a.outbox[0];
    ob.a0 = (int64_t*)a.outbox[1];
    ob.a1 = (int64_t*)a.outbox[2];
    ob.a2 = (int64_t*)a.outbox[3];
    ob.method = (uint16_t*)a.outbox[4];
    ob.count = (unsigned long long*)a.outbox[5];
    ob.cap = a.outbox_cap;
  }
  const bool fixed_mul = a.fixed_method == kCalculatorMultiply;

  if (a.arrival) {  // fixed positions: enqueue + drain, no count pass
    last_rec_bytes_ = (a.a2 || a.method_col) ? 32 : 16;
    last_view_shards_ = S;
    last_route_ = mode;
    // both in one launch (mbx_arrival_fused_kernel): an arrival run belongs to one tile, so the
    // fused form needs no grid-wide phase at any size (tune mbox_fused=0: the two kernels)
    if (!a.a2 && !a.method_col && tn.mbox_fused != 0) {
      // rank byte routes for a stateless method on the directory: the records carry actor ids
      const bool rank_arr = mode == 1 && a.dir_rank && a.n_dir <= kMaxMbox && method_stateless((uint32_t)a.method_uniform);
      if (rank_arr) last_route_ = 3;
      // route mode 4 (the directory's presence map in LDS) when it fits -- for batches past 512
      // tiles: below, the map's staging per block (1024 blocks x 32 KB at 1 Mi) outweighs the
      // gathers it replaces (config 2: 31.2 vs 29.5 G msg/s)
      const bool pres_arr = rank_arr && a.n_dir <= kPresMax && tiles > 512;
      size_t af_lds = 0;
      if (pres_arr) {
        build_presence(a, st);
        in.pres = pres_view_;
        last_route_ = 4;
        af_lds = (size_t)pres_words(a.n_dir) * 4;
        static bool attr = false;
        if (!attr) {  // (past the 64 KB default for the largest maps)
          for (const void* k : {(const void*)mbx_arrival_fused_kernel<4, kCalculatorMultiply, 2>,
                                (const void*)mbx_arrival_fused_kernel<4, kCalculatorMultiply>,
                                (const void*)mbx_arrival_fused_kernel<4, 0, 2>, (const void*)mbx_arrival_fused_kernel<4, 0>})
            PT_HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)((size_t)pres_words(kPresMax) * 4)));
          attr = true;
        }
      }
      // 8-B records past 512 tiles (tune mbox_rec8: the sort's rule; per wave, 16 B when a value
      // of the wave does not fit)
      const bool allow8 = mv_.planar && (tn.mbox_rec8 == 1 || (tn.mbox_rec8 < 0 && tiles > 512));
      if (allow8) last_rec_bytes_ = 8;
      // batches of up to 512 4096-message tiles: 1024-message tiles (four times the blocks)
      SortIn in1 = in;
      const bool small_tiles = tiles <= 512;
      if (small_tiles) in1.tiles = (uint32_t)((a.M + kST * 2 - 1) / (kST * 2));
      const uint32_t grid1 = in1.tiles >= 8 ? (in1.tiles + 7) / 8 * 8 : in1.tiles;
#define PT_AFUSED(MO, FX)                                                                                             \
  do {                                                                                                                \
    if (small_tiles)                                                                                                  \
      hipLaunchKernelGGL((mbx_arrival_fused_kernel<MO, FX, 2>), dim3(grid1), dim3(kST), af_lds, st, in1, mv_,         \
                         (int64_t*)a.state, a.n_state, a.delay_ticks, ob, rv, sort_ticket_, allow8);                  \
    else                                                                                                              \
      hipLaunchKernelGGL((mbx_arrival_fused_kernel<MO, FX>), dim3(grid1), dim3(kST), af_lds, st, in1, mv_,            \
                         (int64_t*)a.state, a.n_state, a.delay_ticks, ob, rv, sort_ticket_, allow8);                  \
  } while (0)
      if (fixed_mul) {
        if (pres_arr) PT_AFUSED(4, kCalculatorMultiply);
        else if (rank_arr) PT_AFUSED(3, kCalculatorMultiply);
        else if (mode == 2) PT_AFUSED(2, kCalculatorMultiply);
        else if (mode == 1) PT_AFUSED(1, kCalculatorMultiply);
        else PT_AFUSED(0, kCalculatorMultiply);
      } else {
        if (pres_arr) PT_AFUSED(4, 0);
        else if (rank_arr) PT_AFUSED(3, 0);
        else if (mode == 2) PT_AFUSED(2, 0);
        else if (mode == 1) PT_AFUSED(1, 0);
        else PT_AFUSED(0, 0);
      }
#undef PT_AFUSED
      PT_HIP_CHECK(hipGetLastError());
      return;
    }
#define PT_AENQ(MO)                                                                                        \
  do {                                                                                                     \
    if (a.a2 && a.method_col)                                                                              \
      hipLaunchKernelGGL((mbx_arrival_enqueue_kernel<MO, true, true>), dim3(tile_grid), dim3(kST), 0, st, in, mv_, rv);  \
    else if (a.a2)                                                                                         \
      hipLaunchKernelGGL((mbx_arrival_enqueue_kernel<MO, true, false>), dim3(tile_grid), dim3(kST), 0, st, in, mv_, rv); \
    else if (a.method_col)                                                                                 \
      hipLaunchKernelGGL((mbx_arrival_enqueue_kernel<MO, false, true>), dim3(tile_grid), dim3(kST), 0, st, in, mv_, rv); \
    else                                                                                                   \
      hipLaunchKernelGGL((mbx_arrival_enqueue_kernel<MO, false, false>), dim3(tile_grid), dim3(kST), 0, st, in, mv_, rv); \
  } while (0)
#define PT_ADRAIN(FX, MO)                                                                                   \
  hipLaunchKernelGGL((mbx_arrival_drain_kernel<FX, MO>), dim3(tile_grid), dim3(kST), 0, st, mv_, in, (int64_t*)a.state, \
                     a.n_state, a.delay_ticks, ob, rv, sort_ticket_)
    if (mode == 2) PT_AENQ(2); else if (mode == 1) PT_AENQ(1); else PT_AENQ(0);
    PT_HIP_CHECK(hipGetLastError());
    if (fixed_mul) {
      if (mode == 2) PT_ADRAIN(kCalculatorMultiply, 2); else if (mode == 1) PT_ADRAIN(kCalculatorMultiply, 1);
      else PT_ADRAIN(kCalculatorMultiply, 0);
    } else {
      if (mode == 2) PT_ADRAIN(0, 2); else if (mode == 1) PT_ADRAIN(0, 1); else PT_ADRAIN(0, 0);
    }
#undef PT_AENQ
#undef PT_ADRAIN
    PT_HIP_CHECK(hipGetLastError());
    return;
  }

  // Stateless batches run on a COARSER view of the same rings: 8 shards of Q * S / 8
  // slots (every ring is empty between epoch Sends, so any view keeps each actor's
  // messages in one ring, in message order; ordered batches keep the full S for the
  // ordered drain's one block per shard).  Longer runs per tile and shard: whole lines
  // for the sort's stores and the drain's loads (8 Mi msgs, 256 shards -> 32 / 16 / 8:
  // 0.222 -> 0.186 / 0.179 / 0.180 ms per Send; round 4 with run reservations and 8-B
  // records: 8 shards 2-3 % faster per bench step than 16, profiles/r4_mailbox_ab.md).
  MboxView mv = mv_;
  uint32_t Sv = S;
  constexpr uint32_t kStatelessShards = 8;
  if (!a.ordered && kStatelessShards < S) {
    const uint32_t k = mv.log_s - (uint32_t)__builtin_ctz(kStatelessShards);
    mv.log_s -= k;
    mv.log_q += k;
    Sv = kStatelessShards;
  }
  last_view_shards_ = Sv;
  // the stateless drain: ring order (default) or message order (tune mbox_drain_msg: every slot index written)
  const bool msg_drain = tn.mbox_drain_msg != 0;
  const bool all_sidx = msg_drain && !a.ordered;
  const bool reserve = !a.ordered && sort_mode == 1;  // (one-pass stateless: tiles reserve runs)
  if (reserve) {
    if (!sort_resv_) {
      if (capturing()) throw std::runtime_error("mailbox send: first reserving Send inside a graph capture (warm up first)");
      PT_HIP_CHECK(hipMalloc((void**)&sort_resv_, (size_t)kMboxSortMaxShards * kResvStride * 4));
      PT_HIP_CHECK(hipMemset(sort_resv_, 0, (size_t)kMboxSortMaxShards * kResvStride * 4));
    }
    mv.resv = sort_resv_;
  }
  // Rank byte gathers (route mode 3) for a stateless uniform one-pass Send on the
  // directory: 1 B per id (L2-resident) instead of the 4-B route word, and the
  // records carry the actor id -- every actor's messages still meet in one ring
  // (the shard is a function of the id), and no stateless handler reads a mailbox.
  const bool rank_route = mode == 1 && a.dir_rank && a.n_dir <= kMaxMbox && !a.ordered && !all_sidx && !a.a2 &&
                          !a.method_col && method_stateless((uint32_t)a.method_uniform) && sort_mode == 1;
  last_route_ = rank_route ? 3 : mode;
  // 8-B ring records: one-pass sort of a batch of one method, at most two arguments for
  // stateless batches (the ring-order drain) and one for ordered ones (the windowed drain:
  // 25.5 vs 24.5 G msg/s per 8 Mi SeqFold step, round 5).  Batches up to 512 tiles, which
  // take the fused kernel, keep 16-B records (1 Mi bench step 24.1 vs 21.9 G msg/s).  Field
  // widths: the mailbox from the state size or the directory, the rest split between the
  // zigzag arguments; a stateless record that does not fit spills, an ordered one escapes.
  const bool r8 = (tn.mbox_rec8 == 1 || (tn.mbox_rec8 < 0 && tiles > 512)) && sort_mode == 1 &&
                  (!a.ordered || !a.a1) && !a.a2 && !a.method_col && mv.planar && !all_sidx;
  if (r8 && (!r8w_ || r8_tiles_ < (uint64_t)tiles)) {  // (outside a capture: grown with the sort workspace)
    if (capturing())
      throw std::runtime_error("mailbox send: first 8-B-record Send of this size inside a graph capture (warm up first)");
    PT_HIP_CHECK(hipStreamSynchronize(st));
    if (!r8w_) {
      // the first Send's widths: the mailbox from the state size or the directory, the rest split
      const uint32_t nmb = std::max(a.n_state, a.n_dir);
      uint32_t wm = 20;
      if (nmb > 1) wm = 32u - (uint32_t)__builtin_clz(nmb - 1);
      wm = std::max(1u, std::min(wm, 24u));
      const uint32_t w0 = (52u - wm) / 2, w = wm | (w0 << 8) | ((52u - wm - w0) << 16);
      PT_HIP_CHECK(hipMalloc((void**)&r8w_, 16));
      PT_HIP_CHECK(hipMemcpy(r8w_, &w, 4, hipMemcpyHostToDevice));
      PT_HIP_CHECK(hipHostMalloc((void**)&r8host_, 64, hipHostMallocMapped));
      *r8host_ = w;
    }
    if (r8max_) PT_HIP_CHECK(hipFree(r8max_));
    PT_HIP_CHECK(hipMalloc((void**)&r8max_, (size_t)tiles * 4));
    r8_tiles_ = (uint64_t)tiles;
  }
  // fields that outgrew 64 bits (the last Send's widths, bit 31): 16-B records from here on
  const bool r8_on = r8 && !(__atomic_load_n(r8host_, __ATOMIC_RELAXED) & 0x80000000u);
  // fields that outgrew 8 B in a stateless batch of a PURE method (its handler reads no actor):
  // wide pure records, 16 B {a0, a1} + a u16 place, instead of the 32-B long form (the 8 Mi
  // full-range int64 step writes and reads 18 B per message, not 32)
  const bool rw_on = r8 && !r8_on && rank_route;  // (rank routes: stateless methods only)
  last_rec_bytes_ = r8_on ? 8 : rw_on ? 18 : ((a.a2 || a.method_col) ? 32 : 16);  // (16: compact unless a value is wide)
  if (r8_on && a.ordered && !r8esc_) {  // escape side array: {a0, mailbox} per ring slot
    if (capturing())
      throw std::runtime_error("mailbox send: first ordered 8-B-record Send inside a graph capture (warm up first)");
    const uint64_t n = (uint64_t)S * slots();
    PT_HIP_CHECK(hipMalloc((void**)&r8esc_, n * 16));
    bytes_ += n * 16;
  }
  if (r8_on) {
    in.rec8 = 1;
    in.r8w = r8w_;
    in.r8max = r8max_;
    in.r8esc = r8esc_;
  } else if (rw_on) {
    in.recw = 1;
    in.r8w = r8w_;
    in.r8max = r8max_;
  }
  const int rf = r8_on ? 1 : rw_on ? 2 : 0;
  uint32_t* tinfo = all_sidx ? nullptr : sort_tinfo_;
  if (two_pass) {
#define PT_COUNT(MO) \
  hipLaunchKernelGGL((mbx_count_kernel<MO>), dim3(in.G), dim3(kST), 0, st, in, mv.log_s, sort_hist_, sort_gsum_, sort_rw_)
    if (mode == 2) PT_COUNT(2); else if (mode == 1) PT_COUNT(1); else PT_COUNT(0);
#undef PT_COUNT
    PT_HIP_CHECK(hipGetLastError());
#define PT_SCAT(A2, MC)                                                                                           \
  hipLaunchKernelGGL((mbx_scatter_kernel<A2, MC>), dim3(in.G), dim3(kST), scatter_lds_bytes(Sv), st, in, mv,     \
                     (const uint32_t*)sort_hist_, (const uint32_t*)sort_gsum_, sort_rw_, sort_sidx_, tinfo, rv,      \
                     !a.ordered, all_sidx)
    if (a.a2 && a.method_col) PT_SCAT(true, true);
    else if (a.a2) PT_SCAT(true, false);
    else if (a.method_col) PT_SCAT(false, true);
    else PT_SCAT(false, false);
#undef PT_SCAT
  } else if (!a.ordered && !all_sidx && fused_ok(tiles)) {
    // one-pass sort + ring-order drain in ONE launch (mbx_sortdrain_kernel, mailbox_sort_fused.hip)
    MbxFusedLaunch f{in, mv, sort_desc_, sort_tctr_, sort_gsum_, sort_sidx_, sort_tinfo_, sort_rw_, rv,
                     (int64_t*)a.state, a.n_state, a.delay_ticks, ob, sort_ticket_, reserve, r8host_,
                     std::max(onesweep_lds_bytes(Sv), ring_drain_lds_bytes(Sv, kSTile)), st, rf, mode, fixed_mul,
                     rank_route, a.a2 != 0, a.method_col != 0};
    mbx_launch_fused(f);
    return;
  } else {
    // route mode 4: a rank-routed Send on a directory whose presence map fits LDS
    const bool pres_route = rank_route && a.n_dir <= kPresMax;
    if (pres_route) {
      build_presence(a, st);
      in.pres = pres_view_;
      last_route_ = 4;
    }
    const size_t os_lds = pres_route ? ((onesweep_lds_bytes(Sv) + 15) & ~(size_t)15) + (size_t)pres_words(a.n_dir) * 4
                                     : onesweep_lds_bytes(Sv);
    if (pres_route) {
      static bool attr = false;
      if (!attr) {  // (past the 64 KB default for the largest maps)
        PT_HIP_CHECK(hipFuncSetAttribute((const void*)mbx_onesweep_kernel<4, false, false>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)(((onesweep_lds_bytes(kMboxSortMaxShards) + 15) & ~(size_t)15) +
                                               (size_t)pres_words(kPresMax) * 4)));
        attr = true;
      }
    }
    // one block per tile, claimed in launch order (the grid is exactly the tile count)
#define PT_OS1(MO, A2, MC)                                                                                        \
  hipLaunchKernelGGL((mbx_onesweep_kernel<MO, A2, MC>), dim3(in.tiles), dim3(kST), os_lds, st, in,                 \
                     mv, sort_desc_, sort_tctr_, sort_gsum_, sort_sidx_, tinfo, sort_rw_, rv, !a.ordered, all_sidx,  \
                     reserve)
#define PT_OS(MO)                                   \
  do {                                              \
    if (a.a2 && a.method_col) PT_OS1(MO, true, true); \
    else if (a.a2) PT_OS1(MO, true, false);         \
    else if (a.method_col) PT_OS1(MO, false, true); \
    else PT_OS1(MO, false, false);                  \
  } while (0)
    if (pres_route) PT_OS1(4, false, false);
    else if (rank_route) PT_OS1(3, false, false);
    else if (mode == 2) PT_OS(2); else if (mode == 1) PT_OS(1); else PT_OS(0);
#undef PT_OS
#undef PT_OS1
  }
  PT_HIP_CHECK(hipGetLastError());
  if (a.ordered) {
    // the ordered drain + the ring-order completion (mailbox_sort_ordered.hip)
    MbxOrderedLaunch o{};
    o.in = in, o.mv = mv, o.gsum = sort_gsum_, o.ngroups = ngroups, o.state = (int64_t*)a.state;
    o.n_state = a.n_state, o.delay_ticks = a.delay_ticks, o.ob = ob, o.stage_rep = (u32x4*)stage_rep_;
    o.origin_base = a.origin_base, o.Sv = Sv, o.r8_on = r8_on, o.a12 = a.a1 || a.a2;
    o.fold = a.fixed_method == kSeqFold && !a.method_col;
    if (r8_on) {
      o.r8a.r8w = r8w_;
      o.r8a.method = (uint32_t)a.method_uniform;
      o.r8a.esc = r8esc_;
    }
    o.r8max = r8max_, o.r8w = r8w_, o.r8host = r8host_, o.tinfo = sort_tinfo_, o.rv = rv, o.tctr = sort_tctr_;
    o.tile_grid = tile_grid, o.st = st;
    mbx_launch_ordered(o);
  } else if (msg_drain) {
#define PT_DMSG(FX)                                                                                              \
  hipLaunchKernelGGL((mbx_drain_msg_kernel<FX>), dim3(in.G), dim3(kST), 0, st, mv, in, (const uint32_t*)sort_sidx_, \
                     (const uint32_t*)sort_rw_, (int64_t*)a.state, a.n_state, a.delay_ticks, ob, rv, sort_gsum_,  \
                     ngroups, sort_ticket_, sort_tctr_)
    if (fixed_mul) PT_DMSG(kCalculatorMultiply);
    else PT_DMSG(0);
#undef PT_DMSG
  } else {
    // the ring-order drain; its LDS stage is sized by the 8-shard view (narrow form)
#define PT_DRING(FX, RF)                                                                                          \
  hipLaunchKernelGGL((mbx_drain_ring_kernel<FX, true, RF>), dim3(tile_grid), dim3(kST), ring_drain_lds_bytes(Sv, kSTile), \
                     st, mv, in, (const uint32_t*)sort_tinfo_, (const uint32_t*)sort_sidx_, (const uint32_t*)sort_rw_, \
                     (int64_t*)a.state, a.n_state, a.delay_ticks, ob, rv, sort_gsum_, ngroups, sort_ticket_,        \
                     sort_tctr_, r8host_)
    if (fixed_mul) {
      if (rf == 1) PT_DRING(kCalculatorMultiply, 1);
      else if (rf == 2) PT_DRING(kCalculatorMultiply, 2);
      else PT_DRING(kCalculatorMultiply, 0);
    } else {
      if (rf == 1) PT_DRING(0, 1);
      else if (rf == 2) PT_DRING(0, 2);
      else PT_DRING(0, 0);
    }
#undef PT_DRING
  }
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
