// Sorted epoch mailboxes: K2 as a stable counting sort into the shard rings,
// K3 as an XCD-aware parallel drain or an LDS-binned ordered drain.
//
// The epoch form of a Send (mailbox.hpp has the ring layout) runs
//
//   count    each block resolves its contiguous range of the batch against the
//            registry mirror (route directory / hash probe), keeps each
//            message's mailbox (route word) and counts its messages per shard:
//            hist[block][shard], plus group sums over 32 blocks (atomics);
//   scatter  each block's prefix per shard is the group sums before its group
//            plus the rows before it inside its group (at most 31 + 31 L2-hot
//            rows: no scan pass); it writes every message into its shard's ring
//            at (tail + prefix + rank), the rank computed in message order (wave
//            match on the shard bits + per-wave counts), so each ring holds its
//            messages in MESSAGE ORDER: every actor's mailbox is FIFO by
//            construction, with no atomic per message; it records each
//            message's ring slot;
//   drain    parallel (batches without ordered methods): each record is taken
//            from its ring slot in message order -- the replies are written
//            coalesced (draining in ring order scattered every reply: 273 us of
//            random stores per 8 Mi); ordered: one block owns one shard -- its
//            actors' state staged in LDS -- and runs each actor's records one at
//            a time in ring order, distinct actors side by side (LDS bins),
//            replies staged at their ring slots; a completion pass gathers them
//            into message order.
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
// ONE L2.
//
// Reference: the server's per-request goroutine of stdlib net/rpc
// (example/calculator/server/server.go:16-20, :38; handler
// example/calculator/calculator.go:9-12) -- here an explicit FIFO queue in HBM.
#include <algorithm>
#include <vector>

#include "mailbox.hpp"
#include "mailbox_dev.hpp"
#include "route_common.hpp"
#include "sort_common.hpp"

namespace ptype {

namespace {
constexpr uint32_t kCompactMark = 0x80000000u;
constexpr uint32_t kCompactLong = 0x80000000u;
constexpr int kOrdThreads = 512;  // ordered drain: one block per shard, one bin per thread
constexpr int kOrdK = 4;
constexpr int kOrdWin = kOrdThreads * kOrdK;  // records per window (2048)
constexpr int kOrdWaves = kOrdThreads / kWave;
constexpr uint32_t kOrdStateMax = 4096;  // a shard's actors whose state is staged in LDS (32 KB)
}  // namespace

// ---------------------------------------------------------------- K2s pass 1: count
constexpr uint32_t kGroupBlocks = 32;  // the scatter's prefix: group sums + rows inside the group
constexpr uint32_t kNoSlot = 0xffffffffu;
// A stateless batch's message whose shard ring is full SPILLS: the parallel drain
// runs it straight from the batch (its route word + argument columns) in message
// order, like any other -- no STATUS_OVERFLOW, so no re-send round and no host
// read of an overflow count.  Ordered batches keep the ring's
// FIFO and answer kStatusOverflow (send_all re-sends the tail).
constexpr uint32_t kSpillSlot = 0xfffffffeu;

template <int MODE, bool ARRIVAL>
__global__ __launch_bounds__(kST) void mbx_count_kernel(SortIn in, uint32_t log_s, uint32_t* __restrict__ hist,
                                                        uint32_t* __restrict__ gsum, uint32_t* __restrict__ rw) {
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
    unsigned c = 0;
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const int64_t i = tile_index(t, k);
      const bool ok = r[k] == in.rank_self && mb[k] < kMaxMbox;
      if (i < in.M) rw[i] = ok ? mb[k] : kNoSlot;
      if constexpr (ARRIVAL) {
        c += ok ? 1u : 0u;
      } else if (ok) {
        atomicAdd(&cnt[mb[k] & (S - 1)], 1u);
      }
    }
    if constexpr (ARRIVAL) {
      c = (unsigned)__builtin_amdgcn_readlane((int)wave_incl_scan(c), 63);
      if (lane_id() == 0 && c) atomicAdd(&cnt[t & (S - 1)], c);
    }
  }
  __syncthreads();
  uint32_t* g = gsum + (size_t)(v / kGroupBlocks) * S;
  for (uint32_t s = threadIdx.x; s < S; s += kST) {
    const uint32_t c = cnt[s];
    hist[(size_t)v * S + s] = c;
    if (c) atomicAdd(&g[s], c);
  }
}

// ---------------------------------------------------------------- K2s pass 2: scatter
// The tile's arguments are loaded with its route words, before the ranking (in
// flight across it).  Loading them only once the ranks are known (a smaller
// register file, occupancy 4 -> 5) measured slower: 124 -> 164 us per 8 Mi.
template <bool A2, bool MC>
__device__ __forceinline__ void load_routed(const SortIn& in, const uint32_t* __restrict__ rw, uint32_t t,
                                            uint32_t (&m)[kSK], int64_t (&x0)[kSK], int64_t (&x1)[kSK],
                                            int64_t (&x2)[kSK], uint32_t (&meth)[kSK]) {
#pragma unroll
  for (int k = 0; k < kSK; ++k) {
    const int64_t i = tile_index(t, k);
    const bool ok = i < in.M;
    m[k] = ok ? __builtin_nontemporal_load(rw + i) : kNoSlot;
    x0[k] = ok ? __builtin_nontemporal_load(in.a0 + i) : 0;
    x1[k] = ok && in.a1 ? __builtin_nontemporal_load(in.a1 + i) : 0;
    x2[k] = 0;
    if constexpr (A2) x2[k] = ok ? __builtin_nontemporal_load(in.a2 + i) : 0;
    meth[k] = in.method_uniform;
    if constexpr (MC) meth[k] = ok ? (uint32_t)in.mcol[i] : 0u;
  }
}

// STAGED (per-actor rings, opt-in: PTYPE_SCATTER_STAGED=1): a tile's records
// are first placed in LDS in ring order -- grouped by shard, message order
// within a shard -- and then written out by consecutive threads, so a wave's
// stores cover a few whole runs instead of 64 scattered 16-B records.
// Measured SLOWER on MI355X (8 Mi msgs, 256 shards: 117 -> 161 us): the 80 KB
// stage halves the resident blocks and adds three barriers and a binary search
// per record, which costs more than the scattered stores (L2 merges them).
constexpr size_t kStageBytes = (size_t)kSTile * 16;
__host__ __device__ constexpr size_t scatter_lds_bytes(uint32_t S, bool staged) {
  return (size_t)S * (16 + 4 * (kST / kWave)) + (staged ? (size_t)S * 12 + kStageBytes : 0);
}

template <bool ARRIVAL, bool A2, bool MC, bool STAGED>
__global__ __launch_bounds__(kST) void mbx_scatter_kernel(SortIn in, MboxView mv, const uint32_t* __restrict__ hist,
                                                          const uint32_t* __restrict__ gsum,
                                                          const uint32_t* __restrict__ rw,
                                                          uint32_t* __restrict__ sidx, ReplyView rv, bool spill) {
  // LDS sized by the shard count (16 + 4 * waves B per shard, + 12 B and the stage
  // when STAGED): occupancy is not capped by the 1024-shard maximum
  extern __shared__ __align__(16) unsigned char smem_sc[];
  const uint32_t S = 1u << mv.log_s;
  u32x4* stage = reinterpret_cast<u32x4*>(smem_sc);  // STAGED: the tile's records in ring order
  unsigned long long* base =
      reinterpret_cast<unsigned long long*>(smem_sc + (STAGED ? kStageBytes : 0));  // ring position of offset 0 (tail)
  uint32_t* run = reinterpret_cast<uint32_t*>(base + S);  // this block's next offset per shard
  uint32_t* room = run + S;                               // offset limit (free ring slots)
  uint32_t* wcnt_all = room + S;                          // [kST / kWave][S] per-wave counts -> wave offsets
  uint32_t* rb = wcnt_all + (kST / kWave) * S;            // STAGED: run[] before this tile
  uint32_t* tc = rb + S;                                  // STAGED: this tile's count per shard
  uint32_t* tpre = tc + S;                                // STAGED: exclusive prefix of tc (stage offsets)
  __shared__ uint32_t scan_w[kST / kWave];
  auto wcnt = [&](unsigned ww, uint32_t sh) -> uint32_t& { return wcnt_all[ww * S + sh]; };
  const uint64_t Q = 1ull << mv.log_q;
  const uint32_t v = virt_block(blockIdx.x, in.G);
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  const uint32_t g0 = v / kGroupBlocks, v0 = g0 * kGroupBlocks;
  for (uint32_t s = threadIdx.x; s < S; s += kST) {
    // this block's prefix: whole groups before it, then the rows before it in its group
    uint32_t p = 0;
    for (uint32_t g = 0; g < g0; ++g) p += gsum[(size_t)g * S + s];
    for (uint32_t u = v0; u < v; ++u) p += hist[(size_t)u * S + s];
    run[s] = p;
    const uint64_t tl = *ctr_tail(mv, s), hd = *ctr_head(mv, s);
    base[s] = tl;
    const uint64_t free = hd + Q > tl ? hd + Q - tl : 0;
    room[s] = (uint32_t)(free < 0xffffffffull ? free : 0xffffffffull);
  }
  unsigned long long n_enq = 0, n_ovf = 0, n_miss = 0, n_spill = 0;
  const uint32_t t0 = v * in.tpb, t1 = min(t0 + in.tpb, in.tiles);
  for (uint32_t t = t0; t < t1; ++t) {
    for (uint32_t s = lane; s < S; s += kWave) wcnt(w, s) = 0;  // this wave's row only
    uint32_t mb[kSK], meth[kSK];
    int64_t v0[kSK], v1[kSK], v2[kSK];
    load_routed<A2, MC>(in, rw, t, mb, v0, v1, v2, meth);
    // rank of each message among this wave's earlier messages of its shard
    uint32_t wr[kSK], sh[kSK];
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const bool ok = mb[k] != kNoSlot;
      sh[k] = ARRIVAL ? (t & (S - 1)) : (mb[k] & (S - 1));
      const uint64_t act = __ballot(ok);
      const uint64_t peers = ARRIVAL ? act : match_bits(sh[k], mv.log_s, act);
      const unsigned below = mbcnt64(peers);
      const int leader = peers ? __builtin_ctzll(peers) : 0;
      unsigned old = 0;
      if (ok && below == 0) {  // group leader: one plain LDS read-add per distinct shard of the wave
        old = wcnt(w, sh[k]);
        wcnt(w, sh[k]) = old + (unsigned)__popcll(peers);
      }
      wr[k] = (unsigned)__shfl((int)old, leader) + below;
    }
    __syncthreads();
    for (uint32_t s = threadIdx.x; s < S; s += kST) {  // wave offsets in message order, then the block's run
      uint32_t rr = run[s];
      if constexpr (STAGED) rb[s] = rr;
#pragma unroll
      for (int ww = 0; ww < kST / kWave; ++ww) {
        const uint32_t c = wcnt(ww, s);
        wcnt(ww, s) = rr;
        rr += c;
      }
      if constexpr (STAGED) tc[s] = rr - run[s];
      run[s] = rr;
    }
    if constexpr (STAGED) {  // stage offsets: exclusive prefix of the tile's shard counts
      __syncthreads();
      const uint32_t per = (S + kST - 1) / kST, s0 = threadIdx.x * per, s1 = min(S, s0 + per);
      uint32_t mine = 0;
      for (uint32_t s = s0; s < s1; ++s) mine += tc[s];
      const uint32_t incl = wave_incl_scan(mine);
      if (lane == kWave - 1) scan_w[w] = incl;
      __syncthreads();
      uint32_t acc = incl - mine;
      for (unsigned ww = 0; ww < w; ++ww) acc += scan_w[ww];
      for (uint32_t s = s0; s < s1; ++s) {
        tpre[s] = acc;
        acc += tc[s];
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const int64_t i = tile_index(t, k);
      if (i >= in.M) continue;
      const uint32_t origin = in.origin_base + (uint32_t)i;
      if (mb[k] == kNoSlot) {
        ++n_miss;
        sidx[i] = kNoSlot;
        write_status(rv, origin, kStatusNoActor);
        continue;
      }
      const uint32_t off = wcnt(w, sh[k]) + wr[k];
      if (off >= room[sh[k]]) {  // the ring is full
        if (spill) {  // stateless batch: the drain runs it from the batch
          ++n_spill;
          sidx[i] = kSpillSlot;
          continue;
        }
        ++n_ovf;  // answered now, re-sent by send_all
        sidx[i] = kNoSlot;
        write_status(rv, origin, kStatusOverflow);
        continue;
      }
      const int64_t x0 = v0[k], x1 = v1[k], x2 = v2[k];
      const uint32_t mt = meth[k];
      const uint64_t slot = slot_at(mv, sh[k], base[sh[k]] + off);
      sidx[i] = (uint32_t)slot;
      const bool compact = mt < 128u && fits_i32(x0) && fits_i32(x1) && x2 == 0;
      if (STAGED) {  // the write-out below stores it (a wide record goes out now; its stage entry says so)
        const uint32_t lpos = tpre[sh[k]] + (off - rb[sh[k]]);
        stage[lpos] = compact ? u32x4{origin | kCompactMark, mb[k] | (mt << 24), (uint32_t)x0, (uint32_t)x1}
                              : u32x4{0u, 0u, 0u, 0u};
      }
      if (STAGED && compact) {
      } else if (compact) {
        *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
            u32x4{origin | kCompactMark, mb[k] | (mt << 24), (uint32_t)x0, (uint32_t)x1};
      } else {
        const uint32_t fl = x2 != 0 ? (uint32_t)kFlagA2 : 0u;
        *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
            u32x4{origin | kCompactMark, mb[k] | kCompactLong, (mt & 0xffffu) | (fl << 16), 0u};
        *reinterpret_cast<u32x4*>(rec_b(mv, slot)) =
            u32x4{(uint32_t)x0, (uint32_t)((uint64_t)x0 >> 32), (uint32_t)x1, (uint32_t)((uint64_t)x1 >> 32)};
        if (fl) mv.a2[slot] = x2;
      }
      ++n_enq;
    }
    if constexpr (STAGED) {  // write-out in ring order: thread j stores stage position j
      __syncthreads();
      const uint32_t total = tpre[S - 1] + tc[S - 1];
      for (uint32_t j = threadIdx.x; j < total; j += kST) {
        uint32_t lo = 0, hi = S - 1;  // the last shard whose stage offset is <= j (a non-empty one)
        while (lo < hi) {
          const uint32_t mid = (lo + hi + 1) >> 1;
          if (tpre[mid] <= j) lo = mid;
          else hi = mid - 1;
        }
        const uint32_t off = rb[lo] + (j - tpre[lo]);
        if (off >= room[lo]) continue;  // spilled / overflowed: never staged
        const u32x4 r = stage[j];
        if (r.x) *reinterpret_cast<u32x4*>(rec_a(mv, slot_at(mv, lo, base[lo] + off))) = r;
      }
    }
    __syncthreads();  // wcnt rows (and the stage) are reused by the next tile
  }
  block_add_stats(mv.stats, n_enq, kMbEnqueued, n_ovf, kMbOverflow, n_miss, kMbNoActor);
  if (spill) {
    __syncthreads();  // block_add_stats' LDS partials are reused
    block_add_stats(mv.stats, n_spill, kMbSpilled, 0, -1, 0, -1);
  }
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

__device__ __forceinline__ SortRec load_sorted(const MboxView& mv, uint64_t slot) {
  const u32x4 ha = *reinterpret_cast<const u32x4*>(rec_a(mv, slot));
  u32x4 hb = {0u, 0u, 0u, 0u};
  int64_t a2v = 0;
  if (rec_is_long(ha)) {
    hb = *reinterpret_cast<const u32x4*>(rec_b(mv, slot));
    if (((ha.z >> 16) & kFlagA2) && mv.a2) a2v = mv.a2[slot];
  }
  return decode_sorted(ha, hb, a2v);
}

// The epoch's total of shard s (group sums) -- and the group words zeroed for
// the next Send once read (`clear`: the caller is the shard's last reader).
__device__ __forceinline__ uint32_t epoch_total(uint32_t* gsum, uint32_t ngroups, uint32_t S, uint32_t s, bool clear) {
  uint32_t t = 0;
  for (uint32_t g = 0; g < ngroups; ++g) {
    t += gsum[(size_t)g * S + s];
    if (clear) gsum[(size_t)g * S + s] = 0u;
  }
  return t;
}

// The epoch's positions of shard s are consumed: head = tail = tail + total
// (overflowed positions were never written and are skipped with them).
__device__ __forceinline__ void epoch_commit(const MboxView& mv, uint32_t s, uint32_t tot) {
  const uint64_t t = *ctr_tail(mv, s) + tot;
  *ctr_tail(mv, s) = t;
  *ctr_done(mv, s) = t;
  *ctr_head(mv, s) = t;
}

// ---------------------------------------------------------------- K3s parallel drain
// Batches without ordered methods: every record runs on its own, so the drain
// takes each message's record from its ring slot in MESSAGE order (the slot the
// scatter recorded) -- the record reads are gathers, the replies land
// coalesced.  The last block commits every shard (and clears the group sums).
template <int FIXED>
__global__ __launch_bounds__(kST) void mbx_drain_msg_kernel(MboxView mv, SortIn in, const uint32_t* __restrict__ sidx,
                                                            const uint32_t* __restrict__ rw,
                                                            int64_t* __restrict__ state, uint32_t n_state,
                                                            uint64_t delay_ticks, OutboxView ob, ReplyView rv,
                                                            uint32_t* __restrict__ gsum, uint32_t ngroups,
                                                            unsigned* __restrict__ ticket) {
  // the scatter's block -> tile ranges: a tile's records sit in ~S short runs that
  // this block's waves read whole (line reuse in L1 / L2), not one record per block
  unsigned long long done = 0, failed = 0, holes = 0;
  const uint32_t v = virt_block(blockIdx.x, in.G);
  const uint32_t t0 = v * in.tpb, t1 = min(t0 + in.tpb, in.tiles);
  for (uint32_t t = t0; t < t1; ++t) {
    uint32_t sl[kSK];
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const int64_t i = tile_index(t, k);
      sl[k] = i < in.M ? __builtin_nontemporal_load(sidx + i) : kNoSlot;
    }
    u32x4 ha[kSK];
#pragma unroll
    for (int k = 0; k < kSK; ++k)
      ha[k] = sl[k] < kSpillSlot ? *reinterpret_cast<const u32x4*>(rec_a(mv, sl[k])) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      if (sl[k] == kNoSlot) continue;  // answered by the scatter (no actor / ring full)
      SortRec x;
      if (sl[k] == kSpillSlot) {  // its ring was full: the message runs straight from the batch
        const int64_t i = tile_index(t, k);
        x.valid = true;
        x.mb = rw[i];
        x.method = in.mcol ? (uint32_t)in.mcol[i] : in.method_uniform;
        x.flags = 0;
        x.a0 = in.a0[i];
        x.a1 = in.a1 ? in.a1[i] : 0;
        x.a2 = in.a2 ? in.a2[i] : 0;
      } else {
        u32x4 hb = {0u, 0u, 0u, 0u};
        int64_t a2v = 0;
        if (rec_is_long(ha[k])) {
          hb = *reinterpret_cast<const u32x4*>(rec_b(mv, sl[k]));
          if (((ha[k].z >> 16) & kFlagA2) && mv.a2) a2v = mv.a2[sl[k]];
        }
        x = decode_sorted(ha[k], hb, a2v);
      }
      const uint32_t origin = in.origin_base + (uint32_t)tile_index(t, k);
      if (!x.valid) {
        ++holes;
        write_status(rv, origin, kStatusNotDelivered);
        continue;
      }
      MsgRecord m;
      m.actor = x.mb;
      m.method = (uint16_t)(FIXED ? FIXED : x.method);
      m.flags = (uint16_t)x.flags;
      m.a0 = x.a0, m.a1 = x.a1, m.a2 = x.a2;
      const ReplyRecord rr = run_handler(m, state, n_state, delay_ticks, ob);
      failed += rr.status != kStatusOk;
      write_reply(rv, origin, rr);
      ++done;
    }
  }
  block_add_stats(mv.stats, done, kMbProcessed, failed, kMbFailed, holes, kMbHoles);
  __shared__ bool last;
  if (threadIdx.x == 0) last = last_block_ticket(ticket);
  __syncthreads();
  if (last) {  // every block's records are read: the rings are consumed
    const uint32_t S = 1u << mv.log_s;
    for (uint32_t s = threadIdx.x; s < S; s += kST) epoch_commit(mv, s, epoch_total(gsum, ngroups, S, s, true));
  }
}

// ---------------------------------------------------------------- K3s ordered drain
// One block owns shard s: its actors' state is staged in LDS (when it fits), and
// the shard's records are taken in windows of kOrdWin in ring order.  A window
// is sorted stably in LDS into kOrdThreads bins by actor (bin = local actor index
// mod bins), then thread b runs bin b's records one at a time in ring order: an
// actor's messages run serially and in FIFO order, distinct bins in parallel.
// Every method of the shard runs here (so a batch mixing ordered and other
// methods keeps per-actor FIFO across all of them).  Replies are staged at the
// records' ring slots (a window's slots are contiguous: whole lines), and
// mbx_complete_kernel gathers them into message order.
struct OrdLds {
  uint32_t wcnt[kOrdWaves][kOrdThreads];  // per-wave bin counts -> offsets
  uint32_t bstart[kOrdThreads];
  uint32_t bcount[kOrdThreads];
  uint32_t wsum[kOrdWaves];
  uint32_t slot[kOrdWin];
  uint32_t act[kOrdWin];  // actor index for the handler (LDS-local or global mailbox)
  uint32_t meth[kOrdWin];  // method | flags << 16
  int64_t a0[kOrdWin], a1[kOrdWin], a2[kOrdWin];
};

__global__ __launch_bounds__(kOrdThreads) void mbx_drain_ordered_kernel(MboxView mv, uint32_t* __restrict__ gsum,
                                                                        uint32_t ngroups, int64_t* __restrict__ state,
                                                                        uint32_t n_state, uint64_t delay_ticks,
                                                                        OutboxView ob, u32x4* __restrict__ srep) {
  extern __shared__ __align__(16) unsigned char smem_ord[];
  OrdLds& L = *reinterpret_cast<OrdLds*>(smem_ord);
  int64_t* st_lds = reinterpret_cast<int64_t*>(smem_ord + sizeof(OrdLds));
  const uint32_t s = blockIdx.x;
  const uint32_t S = 1u << mv.log_s;
  const uint64_t Q = 1ull << mv.log_q;
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  __shared__ uint32_t tot_s;
  if (threadIdx.x == 0) tot_s = epoch_total(gsum, ngroups, S, s, true);
  const uint64_t lo = *ctr_tail(mv, s), hd = *ctr_head(mv, s);
  const uint64_t free = hd + Q > lo ? hd + Q - lo : 0;
  // this shard's actors are mailboxes s, s + S, s + 2S, ...: local index j = mb >> log_s
  const uint32_t n_loc = (state && s < n_state) ? (n_state - 1 - s) / S + 1 : 0;
  const bool in_lds = state && n_loc <= kOrdStateMax;
  if (in_lds)
    for (uint32_t j = threadIdx.x; j < n_loc; j += kOrdThreads) st_lds[j] = state[s + (uint64_t)j * S];
  __syncthreads();
  const uint32_t tot = tot_s;
  const uint64_t n = tot < free ? tot : free;
  const uint64_t sbase = (uint64_t)s << mv.log_q, qmask = Q - 1, rot = shard_rot(mv, s);  // slot_at, hoisted
  unsigned long long done = 0, failed = 0, holes = 0, serial = 0;
  // (loading the next window ahead, during this one's serial bins, measured no
  // faster -- 188 -> 200 us -- and spilled registers to scratch)
  for (uint64_t w0 = lo; w0 < lo + n; w0 += kOrdWin) {
    const uint64_t w1 = lo + n < w0 + kOrdWin ? lo + n : w0 + kOrdWin;
    for (uint32_t b = lane; b < kOrdThreads; b += kWave) L.wcnt[w][b] = 0;
    SortRec x[kOrdK];
    uint32_t bin[kOrdK], wr[kOrdK];
    uint64_t slot[kOrdK];
#pragma unroll
    for (int k = 0; k < kOrdK; ++k) {  // wave w owns window positions [w * 64K, (w+1) * 64K)
      const uint64_t q = w0 + (uint64_t)w * (kWave * kOrdK) + (uint64_t)k * kWave + lane;
      slot[k] = sbase | ((q + rot) & qmask);
      if (q < w1) {
        x[k] = load_sorted(mv, slot[k]);
        if (!x[k].valid) ++holes;
      } else {
        x[k].valid = false;
      }
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
      L.slot[d] = (uint32_t)slot[k];
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
        srep[L.slot[d]] = u32x4{(uint32_t)rr.value, (uint32_t)((uint64_t)rr.value >> 32), (uint32_t)rr.status, 0u};
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
  if (threadIdx.x == 0) epoch_commit(mv, s, tot);
}

// Ordered drain's replies, staged at ring slots, gathered into message order.
// Tile-granular like the parallel drain: block b gathers the tiles whose
// records scatter block b wrote, so its reads hit ~S short runs of contiguous
// slots (lines shared by the block's waves) instead of one line per message.
__global__ __launch_bounds__(kST) void mbx_complete_kernel(SortIn in, const uint32_t* __restrict__ sidx,
                                                           const u32x4* __restrict__ srep, ReplyView rv) {
  const uint32_t v = virt_block(blockIdx.x, in.G);
  const uint32_t t0 = v * in.tpb, t1 = min(t0 + in.tpb, in.tiles);
  for (uint32_t t = t0; t < t1; ++t) {
    uint32_t sl[kSK];
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const int64_t i = tile_index(t, k);
      sl[k] = i < in.M ? __builtin_nontemporal_load(sidx + i) : kNoSlot;
    }
    u32x4 r[kSK];
#pragma unroll
    for (int k = 0; k < kSK; ++k)
      if (sl[k] < kSpillSlot) r[k] = srep[sl[k]];  // one 16-B gather per message
#pragma unroll
    for (int k = 0; k < kSK; ++k)
      if (sl[k] < kSpillSlot)
        put_reply(rv, in.origin_base + (uint32_t)tile_index(t, k), (int64_t)(((uint64_t)r[k].y << 32) | r[k].x),
                  (int32_t)r[k].z);
  }
}

// ---------------------------------------------------------------- host
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
  // per-message workspace (route words, ring slots): grown outside graph capture
  if ((uint64_t)a.M > sort_cap_) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      throw std::runtime_error("mailbox send: a larger batch than before inside a graph capture (warm up first)");
    PT_HIP_CHECK(hipStreamSynchronize(st));
    if (sort_rw_) PT_HIP_CHECK(hipFree(sort_rw_));
    if (sort_sidx_) PT_HIP_CHECK(hipFree(sort_sidx_));
    PT_HIP_CHECK(hipMalloc((void**)&sort_rw_, (size_t)a.M * 4));
    PT_HIP_CHECK(hipMalloc((void**)&sort_sidx_, (size_t)a.M * 4));
    sort_cap_ = (uint64_t)a.M;
  }
  if (a.ordered && !stage_rep_) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      throw std::runtime_error("mailbox send: first ordered Send inside a graph capture (warm up first)");
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
  in.n_dir = a.n_dir;
  in.aw = a.affine_w;
  in.aw_shift = (a.affine_w && (a.affine_w & (a.affine_w - 1)) == 0) ? __builtin_ctz(a.affine_w) : -1;
  in.rank_self = a.rank_self;
  in.origin_base = a.origin_base;
  static const bool dir_nt = getenv("PTYPE_DIR_NT") && atoi(getenv("PTYPE_DIR_NT")) != 0;
  in.dir_nt = dir_nt;
  const int64_t tiles = (a.M + kSTile - 1) / kSTile;
  if (tiles > 0xffffffffll) throw std::invalid_argument("mailbox send: batch too large");
  in.tiles = (uint32_t)tiles;
  // blocks: as many as the histogram holds (it stays L2-resident for the prefixes),
  // a multiple of 8 (one contiguous eighth of the batch per XCD)
  static const int64_t g_env = getenv("PTYPE_SORT_BLOCKS") ? atoll(getenv("PTYPE_SORT_BLOCKS")) : 0;
  int64_t G = std::min<int64_t>({tiles, (int64_t)(kMboxSortHistWords / S), g_env > 0 ? g_env : (int64_t)1024,
                                 (int64_t)kMboxSortGroups * kGroupBlocks});
  if (G >= 8) G -= G % 8;
  G = std::max<int64_t>(G, 1);
  in.G = (uint32_t)G;
  in.tpb = (uint32_t)((tiles + G - 1) / G);
  const uint32_t ngroups = (uint32_t)((G + kGroupBlocks - 1) / kGroupBlocks);
  const int mode = (a.affine_w && a.n_dir) ? 2 : (a.dir && a.n_dir) ? 1 : 0;
  const ReplyView rv{(int64_t*)a.out_val, (int32_t*)a.out_st, a.out_n};
#define PT_COUNT(MO, AR) \
  hipLaunchKernelGGL((mbx_count_kernel<MO, AR>), dim3(in.G), dim3(kST), 0, st, in, mv_.log_s, sort_hist_, sort_gsum_, sort_rw_)
  if (a.arrival) {
    if (mode == 2) PT_COUNT(2, true); else if (mode == 1) PT_COUNT(1, true); else PT_COUNT(0, true);
  } else {
    if (mode == 2) PT_COUNT(2, false); else if (mode == 1) PT_COUNT(1, false); else PT_COUNT(0, false);
  }
#undef PT_COUNT
  PT_HIP_CHECK(hipGetLastError());
  // per-actor rings, records staged in LDS and written out in ring order: opt-in (measured slower)
  static const bool staged_ok = getenv("PTYPE_SCATTER_STAGED") && atoi(getenv("PTYPE_SCATTER_STAGED")) != 0;
  const bool staged = staged_ok && !a.arrival && !a.a2;
#define PT_SCAT1(AR, A2, MC, ST)                                                                                  \
  do {                                                                                                            \
    const size_t lds_ = scatter_lds_bytes(S, ST);                                                                 \
    if (ST) {                                                                                                     \
      static bool attr_ = false;                                                                                  \
      if (!attr_) { /* above the 64 KB default dynamic LDS */                                                     \
        PT_HIP_CHECK(hipFuncSetAttribute((const void*)mbx_scatter_kernel<AR, A2, MC, ST>,                         \
                                         hipFuncAttributeMaxDynamicSharedMemorySize,                              \
                                         (int)scatter_lds_bytes(kMboxSortMaxShards, true)));                      \
        attr_ = true;                                                                                             \
      }                                                                                                           \
    }                                                                                                             \
    hipLaunchKernelGGL((mbx_scatter_kernel<AR, A2, MC, ST>), dim3(in.G), dim3(kST), lds_, st, in, mv_,           \
                       (const uint32_t*)sort_hist_, (const uint32_t*)sort_gsum_, (const uint32_t*)sort_rw_,       \
                       sort_sidx_, rv, !a.ordered);                                                               \
  } while (0)
#define PT_SCAT(AR, A2, MC)                                  \
  do {                                                       \
    if (!(AR) && !(A2) && staged) PT_SCAT1(AR, A2, MC, true); \
    else PT_SCAT1(AR, A2, MC, false);                         \
  } while (0)
#define PT_SCAT_AR(AR)                                  \
  do {                                                  \
    if (a.a2 && a.method_col) PT_SCAT(AR, true, true);   \
    else if (a.a2) PT_SCAT(AR, true, false);            \
    else if (a.method_col) PT_SCAT(AR, false, true);    \
    else PT_SCAT(AR, false, false);                     \
  } while (0)
  if (a.arrival) PT_SCAT_AR(true);
  else PT_SCAT_AR(false);
#undef PT_SCAT_AR
#undef PT_SCAT
#undef PT_SCAT1
  PT_HIP_CHECK(hipGetLastError());
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
    hipLaunchKernelGGL(mbx_drain_ordered_kernel, dim3(S), dim3(kOrdThreads), lds, st, mv_, sort_gsum_, ngroups,
                       (int64_t*)a.state, a.n_state, a.delay_ticks, ob, (u32x4*)stage_rep_);
    PT_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(mbx_complete_kernel, dim3(in.G), dim3(kST), 0, st, in, (const uint32_t*)sort_sidx_,
                       (const u32x4*)stage_rep_, rv);
  } else {
    if (a.fixed_method == kCalculatorMultiply)
      hipLaunchKernelGGL((mbx_drain_msg_kernel<kCalculatorMultiply>), dim3(in.G), dim3(kST), 0, st, mv_, in,
                         (const uint32_t*)sort_sidx_, (const uint32_t*)sort_rw_, (int64_t*)a.state, a.n_state,
                         a.delay_ticks, ob, rv, sort_gsum_,
                         ngroups, sort_ticket_);
    else
      hipLaunchKernelGGL((mbx_drain_msg_kernel<0>), dim3(in.G), dim3(kST), 0, st, mv_, in,
                         (const uint32_t*)sort_sidx_, (const uint32_t*)sort_rw_, (int64_t*)a.state, a.n_state,
                         a.delay_ticks, ob, rv, sort_gsum_,
                         ngroups, sort_ticket_);
  }
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
