// Sorted epoch mailboxes: K2 as a stable counting sort into the shard rings,
// K3 as an XCD-aware parallel drain or an LDS-binned ordered drain.
//
// The epoch form of a Send (mailbox.hpp has the ring layout) runs
//
//   count    each block resolves its contiguous range of the batch against the
//            registry mirror (route directory / hash probe) and counts its
//            messages per shard: hist[block][shard];
//   scan     exclusive prefix of hist over blocks, per shard; column totals;
//   scatter  each block re-resolves its range and writes every message into its
//            shard's ring at (tail + prefix + rank), the rank computed in message
//            order (wave match on the shard bits + per-wave counts), so each
//            ring holds its messages in MESSAGE ORDER: every actor's mailbox is
//            FIFO by construction, with no atomic per message or per tile;
//   drain    parallel (batches without ordered methods): every record runs
//            independently; ordered: one block owns one shard -- its actors'
//            state staged in LDS -- and runs each actor's records one at a time
//            in ring order, distinct actors side by side (LDS bins).
//
// Records are 16 B in the common case (compact form, plane A only):
//   w0 = origin | kCompactMark    (bit 31 marks an epoch record; a live ring's
//                                  lap tags never have it)
//   w1 = mailbox (24 bits) | method << 24 (7 bits)
//   w2, w3 = a0, a1 as int32
// and 32 B (+ the a2 side array) when an argument needs 64 bits or a third
// argument is present (long form: w1 bit 31, w2 = method | flags << 16, plane B
// {a0, a1}).  The tagged 32-B records of mailbox.hip stay the format of live
// sessions (persistent consumer) and of delivery on receipt.
//
// XCD-aware placement (MI355X: 8 XCDs, per-XCD L2s, blocks dealt round-robin):
// count / scatter block b takes the range of virtual block (b % 8) * G/8 + b / 8,
// so each XCD owns one contiguous eighth of the batch -- and therefore one
// contiguous part of every shard's run, whose partially written lines meet in
// ONE L2.  The parallel drain gives XCD x the same part x of every shard: the
// origins of that part are (the rings being message-ordered) one eighth of the
// batch, so the scattered reply stores of one output line come from one XCD.
//
// Reference: the server's per-request goroutine of stdlib net/rpc
// (example/calculator/server/server.go:16-20, :38; handler
// example/calculator/calculator.go:9-12) -- here an explicit FIFO queue in HBM.
#include <algorithm>
#include <vector>

#include "mailbox.hpp"
#include "mailbox_dev.hpp"
#include "route_common.hpp"

namespace ptype {

namespace {
constexpr int kST = 256;             // count / scatter threads per block
constexpr int kSK = 8;               // messages per thread per tile
constexpr int kSTile = kST * kSK;    // 2048 messages
constexpr int kSWave = kSK * kWave;  // a wave's contiguous run of a tile (512)
constexpr uint32_t kCompactMark = 0x80000000u;
constexpr uint32_t kCompactLong = 0x80000000u;
constexpr int kOrdThreads = 512;  // ordered drain: one block per shard, one bin per thread
constexpr int kOrdK = 4;
constexpr int kOrdWin = kOrdThreads * kOrdK;  // records per window (2048)
constexpr int kOrdWaves = kOrdThreads / kWave;
constexpr uint32_t kOrdStateMax = 4096;  // a shard's actors whose state is staged in LDS (32 KB)
constexpr int kDrainThreads = 256;
constexpr int kDrainK = 4;
}  // namespace

// ---------------------------------------------------------------- inputs
struct SortIn {  // by value
  const uint32_t* actor;
  const int64_t* a0;
  const int64_t* a1;
  const int64_t* a2;
  const uint16_t* mcol;
  uint32_t method_uniform;
  int64_t M;
  const TableEntry* table;
  uint64_t mask;
  const uint32_t* dir;
  uint32_t n_dir;
  uint32_t aw;
  int aw_shift;
  int rank_self;
  uint32_t origin_base;
  uint32_t G;      // blocks
  uint32_t tiles;  // ceil(M / kSTile)
  uint32_t tpb;    // tiles per block
};

// Block b's range: XCD (b % 8) owns virtual blocks [x * G/8, (x+1) * G/8).
__device__ __forceinline__ uint32_t virt_block(uint32_t b, uint32_t G) {
  return (G >= 8 && (G & 7) == 0) ? (b & 7) * (G >> 3) + (b >> 3) : b;
}

template <int MODE>
__device__ __forceinline__ void resolve_k(const SortIn& in, const uint32_t (&a)[kSK], int (&r)[kSK],
                                          uint32_t (&mb)[kSK]) {
  if constexpr (MODE == 1) {
    uint32_t w[kSK];
#pragma unroll
    for (int k = 0; k < kSK; ++k) w[k] = a[k] < in.n_dir ? in.dir[a[k]] : kDirFallback;
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      r[k] = w[k] == kDirMissing ? -1 : (int)(w[k] & 0xff);
      mb[k] = w[k] >> 8;
      if (w[k] == kDirFallback) {
        if (a[k] != 0xffffffffu) lookup_entry(in.table, in.mask, actor_key(a[k]), r[k], mb[k]);
        else r[k] = -1;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      if (MODE == 2 && a[k] < in.n_dir) {
        r[k] = in.aw_shift >= 0 ? (int)(a[k] & (in.aw - 1)) : (int)(a[k] % in.aw);
        mb[k] = in.aw_shift >= 0 ? a[k] >> in.aw_shift : a[k] / in.aw;
      } else if (a[k] == 0xffffffffu) {
        r[k] = -1;
        mb[k] = 0;
      } else {
        lookup_entry(in.table, in.mask, actor_key(a[k]), r[k], mb[k]);
      }
    }
  }
}

// Message i of tile t for (item k, lane) of wave w: a wave owns a contiguous run
// of the tile, so message order within a tile is (wave, item, lane).
__device__ __forceinline__ int64_t tile_index(uint32_t t, int k) {
  return (int64_t)t * kSTile + (threadIdx.x / kWave) * kSWave + k * kWave + lane_id();
}

__device__ __forceinline__ void load_actors(const SortIn& in, uint32_t t, uint32_t (&a)[kSK]) {
#pragma unroll
  for (int k = 0; k < kSK; ++k) {
    const int64_t i = tile_index(t, k);
    a[k] = i < in.M ? __builtin_nontemporal_load(in.actor + i) : 0xffffffffu;
  }
}

// Lanes of this wave whose `key` (log_bits bits) equals this lane's, among `act`.
__device__ __forceinline__ uint64_t match_bits(uint32_t key, uint32_t log_bits, uint64_t act) {
  uint64_t m = act;
  for (uint32_t b = 0; b < log_bits; ++b) {
    const uint64_t bb = __ballot((key >> b) & 1u);
    m &= ((key >> b) & 1u) ? bb : ~bb;
  }
  return m;
}

// ---------------------------------------------------------------- K2s pass 1: count
template <int MODE, bool ARRIVAL>
__global__ __launch_bounds__(kST) void mbx_count_kernel(SortIn in, uint32_t log_s, uint32_t* __restrict__ hist) {
  __shared__ uint32_t cnt[kMboxSortMaxShards];
  const uint32_t S = 1u << log_s;
  const uint32_t v = virt_block(blockIdx.x, in.G);
  for (uint32_t s = threadIdx.x; s < S; s += kST) cnt[s] = 0;
  __syncthreads();
  const uint32_t t0 = v * in.tpb, t1 = min(t0 + in.tpb, in.tiles);
  uint32_t a[kSK];
  if (t0 < t1) load_actors(in, t0, a);
  for (uint32_t t = t0; t < t1; ++t) {
    int r[kSK];
    uint32_t mb[kSK];
    resolve_k<MODE>(in, a, r, mb);
    if (t + 1 < t1) load_actors(in, t + 1, a);  // next tile's loads in flight while this one counts
    if constexpr (ARRIVAL) {
      unsigned c = 0;
#pragma unroll
      for (int k = 0; k < kSK; ++k) c += (r[k] == in.rank_self && mb[k] < kMaxMbox) ? 1u : 0u;
      c = (unsigned)__builtin_amdgcn_readlane((int)wave_incl_scan(c), 63);
      if (lane_id() == 0 && c) atomicAdd(&cnt[t & (S - 1)], c);
    } else {
#pragma unroll
      for (int k = 0; k < kSK; ++k)
        if (r[k] == in.rank_self && mb[k] < kMaxMbox) atomicAdd(&cnt[mb[k] & (S - 1)], 1u);
    }
  }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < S; s += kST) hist[(size_t)v * S + s] = cnt[s];
}

// ---------------------------------------------------------------- K2s pass 2: scan
// hist [G][S] -> exclusive prefix over blocks per shard, in place; etot[s] = the
// shard's total.  Block: 64 shards x 16 row groups (coalesced 256-B row reads).
__global__ __launch_bounds__(1024) void mbx_scan_kernel(uint32_t* __restrict__ hist, uint32_t G, uint32_t log_s,
                                                        uint32_t* __restrict__ etot) {
  __shared__ uint32_t part[16][64];
  const uint32_t S = 1u << log_s;
  const uint32_t lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const uint32_t c = blockIdx.x * 64 + lane;
  const uint32_t rows = (G + 15) / 16, r0 = min(G, g * rows), r1 = min(G, r0 + rows);
  uint32_t sum = 0;
  if (c < S) {
    uint32_t r = r0;
    for (; r + 8 <= r1; r += 8) {
      uint32_t x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = hist[(size_t)(r + j) * S + c];
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += x[j];
    }
    for (; r < r1; ++r) sum += hist[(size_t)r * S + c];
  }
  part[g][lane] = sum;
  __syncthreads();
  uint32_t run = 0;
  for (uint32_t j = 0; j < g; ++j) run += part[j][lane];
  if (c < S) {
    if (g == 15) etot[c] = run + sum;
    for (uint32_t r = r0; r < r1; ++r) {
      const uint32_t x = hist[(size_t)r * S + c];
      hist[(size_t)r * S + c] = run;
      run += x;
    }
  }
}

// ---------------------------------------------------------------- K2s pass 3: scatter
struct SortTileIn {
  uint32_t a[kSK];
  int64_t x0[kSK], x1[kSK], x2[kSK];
};

__device__ __forceinline__ void load_args(const SortIn& in, uint32_t t, SortTileIn& x) {
#pragma unroll
  for (int k = 0; k < kSK; ++k) {
    const int64_t i = tile_index(t, k);
    const bool ok = i < in.M;
    x.a[k] = ok ? __builtin_nontemporal_load(in.actor + i) : 0xffffffffu;
    x.x0[k] = ok ? __builtin_nontemporal_load(in.a0 + i) : 0;
    x.x1[k] = ok && in.a1 ? __builtin_nontemporal_load(in.a1 + i) : 0;
    x.x2[k] = ok && in.a2 ? __builtin_nontemporal_load(in.a2 + i) : 0;
  }
}

__device__ __forceinline__ bool fits_i32(int64_t v) { return v == (int64_t)(int32_t)v; }

template <int MODE, bool ARRIVAL>
__global__ __launch_bounds__(kST) void mbx_scatter_kernel(SortIn in, MboxView mv, const uint32_t* __restrict__ hist,
                                                          ReplyView rv) {
  __shared__ uint32_t run[kMboxSortMaxShards];   // this block's next offset per shard
  __shared__ uint32_t room[kMboxSortMaxShards];  // offset limit per shard (free ring slots)
  __shared__ unsigned long long base[kMboxSortMaxShards];  // ring position of offset 0 (the tail)
  __shared__ uint32_t wcnt[kST / kWave][kMboxSortMaxShards];  // per-wave counts -> wave offsets
  const uint32_t S = 1u << mv.log_s;
  const uint64_t Q = 1ull << mv.log_q;
  const uint32_t v = virt_block(blockIdx.x, in.G);
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  for (uint32_t s = threadIdx.x; s < S; s += kST) {
    run[s] = hist[(size_t)v * S + s];
    const uint64_t tl = *ctr_tail(mv, s), hd = *ctr_head(mv, s);
    base[s] = tl;
    const uint64_t free = hd + Q > tl ? hd + Q - tl : 0;
    room[s] = (uint32_t)(free < 0xffffffffull ? free : 0xffffffffull);
  }
  unsigned long long n_enq = 0, n_ovf = 0, n_miss = 0;
  const uint32_t t0 = v * in.tpb, t1 = min(t0 + in.tpb, in.tiles);
  SortTileIn x;
  if (t0 < t1) load_args(in, t0, x);
  for (uint32_t t = t0; t < t1; ++t) {
    for (uint32_t s = lane; s < S; s += kWave) wcnt[w][s] = 0;  // this wave's row only
    int r[kSK];
    uint32_t mb[kSK];
    resolve_k<MODE>(in, x.a, r, mb);
    int64_t v0[kSK], v1[kSK], v2[kSK];
    uint32_t meth[kSK];
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      v0[k] = x.x0[k], v1[k] = x.x1[k], v2[k] = x.x2[k];
      const int64_t i = tile_index(t, k);
      meth[k] = in.mcol && i < in.M ? (uint32_t)in.mcol[i] : in.method_uniform;
    }
    if (t + 1 < t1) load_args(in, t + 1, x);  // next tile's loads in flight across this tile's barriers
    // rank of each message among this wave's earlier messages of its shard
    uint32_t wr[kSK], sh[kSK];
    bool ok[kSK];
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      ok[k] = r[k] == in.rank_self && mb[k] < kMaxMbox;
      sh[k] = ARRIVAL ? (t & (S - 1)) : (mb[k] & (S - 1));
      const uint64_t act = __ballot(ok[k]);
      const uint64_t peers = ARRIVAL ? act : match_bits(sh[k], mv.log_s, act);
      const unsigned below = mbcnt64(peers);
      const int leader = peers ? __builtin_ctzll(peers) : 0;
      unsigned old = 0;
      if (ok[k] && below == 0) {  // group leader: one plain LDS read-add per distinct shard of the wave
        old = wcnt[w][sh[k]];
        wcnt[w][sh[k]] = old + (unsigned)__popcll(peers);
      }
      old = (unsigned)__shfl((int)old, leader);
      wr[k] = old + below;
    }
    __syncthreads();
    for (uint32_t s = threadIdx.x; s < S; s += kST) {  // wave offsets in message order, then the block's run
      uint32_t rr = run[s];
#pragma unroll
      for (int ww = 0; ww < kST / kWave; ++ww) {
        const uint32_t c = wcnt[ww][s];
        wcnt[ww][s] = rr;
        rr += c;
      }
      run[s] = rr;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const int64_t i = tile_index(t, k);
      if (i >= in.M) continue;
      const uint32_t origin = in.origin_base + (uint32_t)i;
      if (!ok[k]) {
        ++n_miss;
        write_status(rv, origin, kStatusNoActor);
        continue;
      }
      const uint32_t off = wcnt[w][sh[k]] + wr[k];
      if (off >= room[sh[k]]) {  // the ring is full: answered now, re-sent by send_all
        ++n_ovf;
        write_status(rv, origin, kStatusOverflow);
        continue;
      }
      const uint64_t slot = slot_at(mv, sh[k], base[sh[k]] + off);
      const bool compact = meth[k] < 128u && fits_i32(v0[k]) && fits_i32(v1[k]) && v2[k] == 0;
      if (compact) {
        *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
            u32x4{origin | kCompactMark, mb[k] | (meth[k] << 24), (uint32_t)v0[k], (uint32_t)v1[k]};
      } else {
        const uint32_t fl = v2[k] != 0 ? (uint32_t)kFlagA2 : 0u;
        *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
            u32x4{origin | kCompactMark, mb[k] | kCompactLong, (meth[k] & 0xffffu) | (fl << 16), 0u};
        *reinterpret_cast<u32x4*>(rec_b(mv, slot)) =
            u32x4{(uint32_t)v0[k], (uint32_t)((uint64_t)v0[k] >> 32), (uint32_t)v1[k], (uint32_t)((uint64_t)v1[k] >> 32)};
        if (fl) mv.a2[slot] = v2[k];
      }
      ++n_enq;
    }
    __syncthreads();  // wcnt rows are reused by the next tile
  }
  block_add_stats(mv.stats, n_enq, kMbEnqueued, n_ovf, kMbOverflow, n_miss, kMbNoActor);
}

// ---------------------------------------------------------------- compact record decode
struct SortRec {
  uint32_t origin, mb, method, flags;
  int64_t a0, a1, a2;
  bool valid;
};

__device__ __forceinline__ bool rec_is_long(const u32x4& ha) { return (ha.y & kCompactLong) != 0; }

__device__ __forceinline__ SortRec decode_sorted(const u32x4& ha, const u32x4& hb, int64_t a2v) {
  SortRec x;
  x.valid = (ha.x & kCompactMark) != 0;
  x.origin = ha.x & ~kCompactMark;
  if (!rec_is_long(ha)) {
    x.mb = ha.y & 0xffffffu;
    x.method = (ha.y >> 24) & 0x7fu;
    x.flags = 0;
    x.a0 = (int64_t)(int32_t)ha.z;
    x.a1 = (int64_t)(int32_t)ha.w;
    x.a2 = 0;
  } else {
    x.mb = ha.y & 0xffffffu;
    x.method = ha.z & 0xffffu;
    x.flags = ha.z >> 16;
    x.a0 = (int64_t)(((uint64_t)hb.y << 32) | hb.x);
    x.a1 = (int64_t)(((uint64_t)hb.w << 32) | hb.z);
    x.a2 = (x.flags & kFlagA2) ? a2v : 0;
  }
  return x;
}

// Range of shard s this epoch: [tail, tail + min(total, free slots)).
__device__ __forceinline__ void epoch_range(const MboxView& mv, const uint32_t* etot, uint32_t s, uint64_t& lo,
                                            uint64_t& n, uint32_t& tot) {
  const uint64_t Q = 1ull << mv.log_q;
  lo = *ctr_tail(mv, s);
  const uint64_t hd = *ctr_head(mv, s);
  const uint64_t free = hd + Q > lo ? hd + Q - lo : 0;
  tot = etot[s];
  n = tot < free ? tot : free;
}

// The epoch's positions of shard s are consumed: head = tail = tail + total
// (overflowed positions were never written and are skipped with them).
__device__ __forceinline__ void epoch_commit(const MboxView& mv, uint32_t s, uint64_t lo, uint32_t tot) {
  *ctr_tail(mv, s) = lo + tot;
  *ctr_done(mv, s) = lo + tot;
  *ctr_head(mv, s) = lo + tot;
}

// ---------------------------------------------------------------- K3s parallel drain
// Grid X * S blocks: shard s, part p of X.  XCD x (= block % 8) takes parts
// [x * X/8, (x+1) * X/8) of every shard.  The last block of a shard commits it.
template <int FIXED>
__global__ __launch_bounds__(kDrainThreads) void mbx_drain_par_kernel(MboxView mv, const uint32_t* __restrict__ etot,
                                                                      uint32_t X, int64_t* __restrict__ state,
                                                                      uint32_t n_state, uint64_t delay_ticks,
                                                                      OutboxView ob, ReplyView rv) {
  const uint32_t L = blockIdx.x;
  uint32_t s, p;
  if ((X & 7) == 0) {
    const uint32_t px = X >> 3, j = L >> 3, x = L & 7;
    s = j / px;
    p = x * px + j % px;
  } else {
    s = L / X;
    p = L % X;
  }
  uint64_t lo, n;
  uint32_t tot;
  epoch_range(mv, etot, s, lo, n, tot);
  const uint64_t b0 = lo + n * p / X, b1 = lo + n * (p + 1) / X;
  unsigned long long done = 0, failed = 0, holes = 0;
  for (uint64_t p0 = b0; p0 < b1; p0 += (uint64_t)kDrainK * kDrainThreads) {
    u32x4 ha[kDrainK];
#pragma unroll
    for (int k = 0; k < kDrainK; ++k) {
      const uint64_t q = p0 + (uint64_t)k * kDrainThreads + threadIdx.x;
      ha[k] = q < b1 ? *reinterpret_cast<const u32x4*>(rec_a(mv, slot_at(mv, s, q))) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int k = 0; k < kDrainK; ++k) {
      const uint64_t q = p0 + (uint64_t)k * kDrainThreads + threadIdx.x;
      if (q >= b1) continue;
      u32x4 hb = {0u, 0u, 0u, 0u};
      int64_t a2v = 0;
      const uint64_t slot = slot_at(mv, s, q);
      if (rec_is_long(ha[k])) {
        hb = *reinterpret_cast<const u32x4*>(rec_b(mv, slot));
        if (((ha[k].z >> 16) & kFlagA2) && mv.a2) a2v = mv.a2[slot];
      }
      const SortRec x = decode_sorted(ha[k], hb, a2v);
      if (!x.valid) {
        ++holes;
        continue;
      }
      MsgRecord m;
      m.actor = x.mb;
      m.method = (uint16_t)(FIXED ? FIXED : x.method);
      m.flags = (uint16_t)x.flags;
      m.a0 = x.a0, m.a1 = x.a1, m.a2 = x.a2;
      const ReplyRecord rr = run_handler(m, state, n_state, delay_ticks, ob);
      failed += rr.status != kStatusOk;
      write_reply(rv, x.origin, rr);
      ++done;
    }
  }
  block_add_stats(mv.stats, done, kMbProcessed, failed, kMbFailed, holes, kMbHoles);
  // the last block of this shard commits it (every block of the shard has read
  // the counters by the time it takes its ticket)
  __shared__ int last;
  unsigned long long* tk = mv.ctr + (uint64_t)s * kMboxCtrStride + kMboxCtrTicket;
  if (threadIdx.x == 0) last = atomicAdd(tk, 1ull) == X - 1;
  __syncthreads();
  if (last && threadIdx.x == 0) {
    epoch_commit(mv, s, lo, tot);
    *tk = 0;
  }
}

// ---------------------------------------------------------------- K3s ordered drain
// One block owns shard s: its actors' state is staged in LDS (when it fits), and
// the shard's records are taken in windows of kOrdWin in ring order.  A window
// is sorted stably in LDS into kOrdThreads bins by actor (bin = local actor index
// mod bins), then thread b runs bin b's records one at a time in ring order: an
// actor's messages run serially and in FIFO order, distinct bins in parallel.
// Every method of the shard runs here (so a batch mixing ordered and other
// methods keeps per-actor FIFO across all of them).
struct OrdLds {
  uint32_t wcnt[kOrdWaves][kOrdThreads];  // per-wave bin counts -> offsets
  uint32_t bstart[kOrdThreads];
  uint32_t bcount[kOrdThreads];
  uint32_t wsum[kOrdWaves];
  uint32_t org[kOrdWin];
  uint32_t act[kOrdWin];  // actor index for the handler (LDS-local or global mailbox)
  uint32_t meth[kOrdWin];  // method | flags << 16
  int64_t a0[kOrdWin], a1[kOrdWin], a2[kOrdWin];
};

__global__ __launch_bounds__(kOrdThreads) void mbx_drain_ordered_kernel(MboxView mv, const uint32_t* __restrict__ etot,
                                                                        int64_t* __restrict__ state, uint32_t n_state,
                                                                        uint64_t delay_ticks, OutboxView ob,
                                                                        ReplyView rv) {
  extern __shared__ __align__(16) unsigned char smem_ord[];
  OrdLds& L = *reinterpret_cast<OrdLds*>(smem_ord);
  int64_t* st_lds = reinterpret_cast<int64_t*>(smem_ord + sizeof(OrdLds));
  const uint32_t s = blockIdx.x;
  const uint32_t S = 1u << mv.log_s;
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  uint64_t lo, n;
  uint32_t tot;
  epoch_range(mv, etot, s, lo, n, tot);
  // this shard's actors are mailboxes s, s + S, s + 2S, ...: local index j = mb >> log_s
  const uint32_t n_loc = (state && s < n_state) ? (n_state - 1 - s) / S + 1 : 0;
  const bool in_lds = state && n_loc <= kOrdStateMax;
  if (in_lds)
    for (uint32_t j = threadIdx.x; j < n_loc; j += kOrdThreads) st_lds[j] = state[s + (uint64_t)j * S];
  __syncthreads();
  unsigned long long done = 0, failed = 0, holes = 0, serial = 0;
  for (uint64_t w0 = lo; w0 < lo + n; w0 += kOrdWin) {
    const uint64_t w1 = lo + n < w0 + kOrdWin ? lo + n : w0 + kOrdWin;
    for (uint32_t b = lane; b < kOrdThreads; b += kWave) L.wcnt[w][b] = 0;
    SortRec x[kOrdK];
    uint32_t bin[kOrdK], wr[kOrdK];
#pragma unroll
    for (int k = 0; k < kOrdK; ++k) {  // wave w owns window positions [w * 64K, (w+1) * 64K)
      const uint64_t q = w0 + (uint64_t)w * (kWave * kOrdK) + (uint64_t)k * kWave + lane;
      u32x4 ha = {0u, 0u, 0u, 0u}, hb = {0u, 0u, 0u, 0u};
      int64_t a2v = 0;
      if (q < w1) {
        const uint64_t slot = slot_at(mv, s, q);
        ha = *reinterpret_cast<const u32x4*>(rec_a(mv, slot));
        if (rec_is_long(ha)) {
          hb = *reinterpret_cast<const u32x4*>(rec_b(mv, slot));
          if (((ha.z >> 16) & kFlagA2) && mv.a2) a2v = mv.a2[slot];
        }
      }
      x[k] = decode_sorted(ha, hb, a2v);
      if (q < w1 && !x[k].valid) ++holes;
      x[k].valid = x[k].valid && q < w1;
    }
#pragma unroll
    for (int k = 0; k < kOrdK; ++k) {
      bin[k] = (x[k].mb >> mv.log_s) & (kOrdThreads - 1);
      const uint64_t peers = match_bits(bin[k], 9, __ballot(x[k].valid));
      const unsigned below = mbcnt64(peers);
      const int leader = peers ? __builtin_ctzll(peers) : 0;
      unsigned old = 0;
      if (x[k].valid && below == 0) {
        old = L.wcnt[w][bin[k]];
        L.wcnt[w][bin[k]] = old + (unsigned)__popcll(peers);
      }
      wr[k] = (unsigned)__shfl((int)old, leader) + below;
    }
    __syncthreads();
    {  // bin totals and wave offsets (thread b owns bin b), then an exclusive scan over bins
      const unsigned b = threadIdx.x;
      unsigned r = 0;
#pragma unroll
      for (int ww = 0; ww < kOrdWaves; ++ww) {
        const unsigned c = L.wcnt[ww][b];
        L.wcnt[ww][b] = r;
        r += c;
      }
      L.bcount[b] = r;
      const unsigned inc = wave_incl_scan(r);
      if (lane == kWave - 1) L.wsum[w] = inc;
      __syncthreads();
      unsigned off = inc - r;
      for (unsigned ww = 0; ww < w; ++ww) off += L.wsum[ww];
      L.bstart[b] = off;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kOrdK; ++k) {
      if (!x[k].valid) continue;
      const unsigned d = L.bstart[bin[k]] + L.wcnt[w][bin[k]] + wr[k];
      L.org[d] = x[k].origin;
      L.act[d] = in_lds ? (x[k].mb >> mv.log_s) : x[k].mb;
      L.meth[d] = x[k].method | (x[k].flags << 16);
      L.a0[d] = x[k].a0;
      L.a1[d] = x[k].a1;
      L.a2[d] = x[k].a2;
    }
    __syncthreads();
    {  // this thread's bin, serially in ring order
      const unsigned b = threadIdx.x, e = L.bstart[b] + L.bcount[b];
      if (L.bcount[b] > 1) serial += L.bcount[b] - 1;  // records that waited behind their bin's earlier ones
      int64_t* st = in_lds ? st_lds : state;
      const uint32_t nst = in_lds ? n_loc : n_state;
      for (unsigned d = L.bstart[b]; d < e; ++d) {
        MsgRecord m;
        m.actor = L.act[d];
        m.method = (uint16_t)(L.meth[d] & 0xffffu);
        m.flags = (uint16_t)(L.meth[d] >> 16);
        m.a0 = L.a0[d], m.a1 = L.a1[d], m.a2 = L.a2[d];
        const ReplyRecord rr = run_handler(m, st, nst, delay_ticks, ob, true);
        failed += rr.status != kStatusOk;
        write_reply(rv, L.org[d], rr);
        ++done;
        if (!in_lds) vm_drain();  // global state: this store lands before the bin's next load
      }
    }
    __syncthreads();  // the window's LDS is reused
  }
  if (in_lds)
    for (uint32_t j = threadIdx.x; j < n_loc; j += kOrdThreads) state[s + (uint64_t)j * S] = st_lds[j];
  block_add_stats(mv.stats, done, kMbProcessed, failed, kMbFailed, holes, kMbHoles);
  __syncthreads();  // block_add_stats' LDS partials are reused
  block_add_stats(mv.stats, serial, kMbSerial, 0, -1, 0, -1);
  if (threadIdx.x == 0) epoch_commit(mv, s, lo, tot);
}

// ---------------------------------------------------------------- host
void Mailboxes::send_sorted(const MboxSend& a) {
  const uint32_t S = shards();
  if (S > (uint32_t)kMboxSortMaxShards) throw std::invalid_argument("sorted mailboxes: at most 1024 shards");
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
  in.n_dir = a.n_dir;
  in.aw = a.affine_w;
  in.aw_shift = (a.affine_w && (a.affine_w & (a.affine_w - 1)) == 0) ? __builtin_ctz(a.affine_w) : -1;
  in.rank_self = a.rank_self;
  in.origin_base = a.origin_base;
  const int64_t tiles = (a.M + kSTile - 1) / kSTile;
  if (tiles > 0xffffffffll) throw std::invalid_argument("mailbox send: batch too large");
  in.tiles = (uint32_t)tiles;
  // blocks: as many as the histogram holds (it stays L2-resident for the scan),
  // a multiple of 8 (one contiguous eighth of the batch per XCD)
  static const int64_t g_env = getenv("PTYPE_SORT_BLOCKS") ? atoll(getenv("PTYPE_SORT_BLOCKS")) : 0;
  int64_t G = std::min<int64_t>({tiles, (int64_t)(kMboxSortHistWords / S), g_env > 0 ? g_env : (int64_t)1024});
  if (G >= 8) G -= G % 8;
  G = std::max<int64_t>(G, 1);
  in.G = (uint32_t)G;
  in.tpb = (uint32_t)((tiles + G - 1) / G);
  const int mode = (a.affine_w && a.n_dir) ? 2 : (a.dir && a.n_dir) ? 1 : 0;
  const ReplyView rv{(int64_t*)a.out_val, (int32_t*)a.out_st, a.out_n};
#define PT_SORT_K(KERNEL, MO, AR, ...) hipLaunchKernelGGL((KERNEL<MO, AR>), __VA_ARGS__)
#define PT_SORT(KERNEL, ...)                                             \
  do {                                                                   \
    if (a.arrival) {                                                     \
      if (mode == 2) PT_SORT_K(KERNEL, 2, true, __VA_ARGS__);            \
      else if (mode == 1) PT_SORT_K(KERNEL, 1, true, __VA_ARGS__);       \
      else PT_SORT_K(KERNEL, 0, true, __VA_ARGS__);                      \
    } else {                                                             \
      if (mode == 2) PT_SORT_K(KERNEL, 2, false, __VA_ARGS__);           \
      else if (mode == 1) PT_SORT_K(KERNEL, 1, false, __VA_ARGS__);      \
      else PT_SORT_K(KERNEL, 0, false, __VA_ARGS__);                     \
    }                                                                    \
  } while (0)
  PT_SORT(mbx_count_kernel, dim3(in.G), dim3(kST), 0, st, in, mv_.log_s, sort_hist_);
  PT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(mbx_scan_kernel, dim3((S + 63) / 64), dim3(1024), 0, st, sort_hist_, in.G, mv_.log_s, sort_tot_);
  PT_HIP_CHECK(hipGetLastError());
  PT_SORT(mbx_scatter_kernel, dim3(in.G), dim3(kST), 0, st, in, mv_, (const uint32_t*)sort_hist_, rv);
  PT_HIP_CHECK(hipGetLastError());
#undef PT_SORT
#undef PT_SORT_K
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
  if (a.ordered) {
    const size_t lds = sizeof(OrdLds) + (size_t)kOrdStateMax * sizeof(int64_t);
    static bool attr = false;
    if (!attr) {  // above the 64 KB default dynamic LDS
      PT_HIP_CHECK(hipFuncSetAttribute((const void*)mbx_drain_ordered_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      attr = true;
    }
    hipLaunchKernelGGL(mbx_drain_ordered_kernel, dim3(S), dim3(kOrdThreads), lds, st, mv_, (const uint32_t*)sort_tot_,
                       (int64_t*)a.state, a.n_state, a.delay_ticks, ob, rv);
  } else {
    // X parts per shard, a multiple of 8 (XCD-aware), ~2048 blocks in all
    const uint32_t X = 8u * std::max<uint32_t>(1u, 256u / S);
    if (a.fixed_method == kCalculatorMultiply)
      hipLaunchKernelGGL((mbx_drain_par_kernel<kCalculatorMultiply>), dim3(X * S), dim3(kDrainThreads), 0, st, mv_,
                         (const uint32_t*)sort_tot_, X, (int64_t*)a.state, a.n_state, a.delay_ticks, ob, rv);
    else
      hipLaunchKernelGGL((mbx_drain_par_kernel<0>), dim3(X * S), dim3(kDrainThreads), 0, st, mv_,
                         (const uint32_t*)sort_tot_, X, (int64_t*)a.state, a.n_state, a.delay_ticks, ob, rv);
  }
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
