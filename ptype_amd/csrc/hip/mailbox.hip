// HBM actor mailboxes: K2 enqueue, K3 epoch drain, K3 persistent consumer.
// Design and protocol: mailbox.hpp.
#include <string.h>

#include <vector>

#include "mailbox.hpp"
#include "mailbox_dev.hpp"
#include "packed.hpp"
#include "route_common.hpp"

#include <algorithm>

namespace ptype {

int64_t wire_req_words(int64_t C, int nargs, bool mc);

// ---------------------------------------------------------------- K2 enqueue
// The common part of K2 for one tile of K * 256 messages already resolved to
// (ok, mailbox, method, args, origin): per-shard ranks in LDS, ONE reservation
// per (tile, shard), capacity check against the shard's head, the records
// (B half + a2 first; with a live consumer drained before any tag half).
// `hist` must hold zeros for this tile when called (the caller zeroed it
// before its own loads; the barrier below orders that).
template <bool LIVE, int K, bool ARRIVAL>
__device__ __forceinline__ void enqueue_tile(const MboxView& mv, unsigned long long* base, unsigned long long* lim,
                                             unsigned* hist, uint32_t tile_index, const bool (&in)[K],
                                             const bool (&ok)[K], const uint32_t (&mb)[K],
                                             const uint32_t (&meth)[K], const int64_t (&x0)[K],
                                             const int64_t (&x1)[K], const int64_t (&x2)[K],
                                             const uint32_t (&origin)[K], bool has_a2, const ReplyView& rv,
                                             unsigned long long& n_enq, unsigned long long& n_ovf,
                                             unsigned long long& n_miss) {
  const uint32_t S = 1u << mv.log_s;
  const uint64_t Q = 1ull << mv.log_q;
  __syncthreads();  // hist zeroed
  unsigned off[K];
  const uint32_t tile_shard = tile_index & (S - 1);
  if constexpr (ARRIVAL) {
    // message-order compaction: rank = (item k, wave, lane) prefix of the valid flags
    __shared__ unsigned wcnt[K][4];
    const unsigned w = threadIdx.x / kWave;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t bal = __ballot(ok[k]);
      off[k] = ok[k] ? mbcnt64(bal) : 0xffffffffu;
      if (lane_id() == 0) wcnt[k][w] = (unsigned)__popcll(bal);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned run = 0;
      for (int k = 0; k < K; ++k)
        for (int q = 0; q < 4; ++q) {
          const unsigned c = wcnt[k][q];
          wcnt[k][q] = run;
          run += c;
        }
      hist[tile_shard] = run;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (off[k] != 0xffffffffu) off[k] += wcnt[k][w];
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) off[k] = ok[k] ? atomicAdd(&hist[mb[k] & (S - 1)], 1u) : 0xffffffffu;
  }
  __syncthreads();
  uint32_t sh[K];  // ring of each message
#pragma unroll
  for (int k = 0; k < K; ++k) sh[k] = ARRIVAL ? tile_shard : mb[k] & (S - 1);
  // ONE reservation per (tile, shard), and the capacity limit from the shard's head
  for (uint32_t s = threadIdx.x; s < S; s += blockDim.x) {
    const unsigned c = hist[s];
    if (c) {
      if constexpr (LIVE) {
        // clamped to the ring's free space (a CAS bounded by head + Q): a full ring
        // reserves nothing, so overflow leaves no hole a live consumer would have
        // to wait out -- under producers that never pause it never could
        // (the unclamped add made consumption crawl under overload)
        unsigned long long t = ld_fresh(ctr_tail(mv, s)), take = 0;
        for (;;) {
          const unsigned long long room = ld_fresh(ctr_head(mv, s)) + Q;
          take = t < room ? (room - t < c ? room - t : c) : 0ull;
          if (!take) break;
          const unsigned long long seen = atomicCAS(ctr_tail(mv, s), t, t + take);
          if (seen == t) break;
          t = seen;
        }
        base[s] = t;
        lim[s] = t + take;  // offsets >= take overflow (answered now, never reserved)
      } else {
        base[s] = atomicAdd(ctr_tail(mv, s), (unsigned long long)c);
        lim[s] = *ctr_head(mv, s) + Q;
      }
    }
  }
  __syncthreads();
  uint64_t pos[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    pos[k] = ~0ull;
    if (!in[k]) continue;
    if (off[k] == 0xffffffffu) {
      ++n_miss;
      write_status(rv, origin[k], kStatusNoActor);
      continue;
    }
    const uint32_t s = sh[k];
    const uint64_t p = base[s] + off[k];
    if (p >= lim[s]) {  // would overwrite an unconsumed record: a hole, answered now
      ++n_ovf;
      write_status(rv, origin[k], kStatusOverflow);
      continue;
    }
    pos[k] = p;
    const uint64_t slot = slot_at(mv, s, p);
    const u32x4 hb = {(uint32_t)x0[k], (uint32_t)((uint64_t)x0[k] >> 32), (uint32_t)x1[k],
                      (uint32_t)((uint64_t)x1[k] >> 32)};
    if constexpr (LIVE) {
      st16_sc1(rec_b(mv, slot), hb);
      if (has_a2)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(mv.a2 + slot), (unsigned long long)x2[k],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      *reinterpret_cast<u32x4*>(rec_b(mv, slot)) = hb;
      if (has_a2) mv.a2[slot] = x2[k];
    }
  }
  if constexpr (LIVE) vm_drain();  // every B half of this wave is out before its tags
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (pos[k] == ~0ull) continue;
    const u32x4 ha = {lap_tag(mv, pos[k]), mb[k], origin[k],
                      (meth[k] & 0xffffu) | ((uint32_t)(kFlagValid | kFlagRouted | (has_a2 ? kFlagA2 : 0)) << 16)};
    uint32_t* rc = rec_at(mv, sh[k], pos[k]);
    if constexpr (LIVE) st16_sc1(rc, ha);
    else *reinterpret_cast<u32x4*>(rc) = ha;
    ++n_enq;
  }
  if constexpr (LIVE) vm_drain();
  __syncthreads();  // every wave's records are out: the tile's positions are done
  if constexpr (LIVE) {  // the reserved positions are written: done catches up with tail
    for (uint32_t s = threadIdx.x; s < S; s += blockDim.x)
      if (hist[s] && lim[s] > base[s]) atomicAdd(ctr_done(mv, s), lim[s] - base[s]);
  }
  __syncthreads();  // LDS reused by the next tile
}


// One tile = K * 256 messages per block (item-major, coalesced).  LDS holds the
// tile's per-shard counts, then each shard's reserved base and capacity limit.
//
// ARRIVAL: shard by arrival instead of by actor -- the whole tile goes to ring
// (tile index & (S - 1)) in message order, compacted by a block scan, with ONE
// reservation per tile.  Only for batches without ordered methods (an actor's
// messages then meet in no single ring): the rings stay a queue, but enqueue
// and drain are both streaming passes and the drain's replies land coalesced
// (actor sharding scatters every reply: 0.49 ms vs ~0.1 ms per 8 Mi messages).
template <int MODE, bool LIVE, int K, bool ARRIVAL = false>
__global__ __launch_bounds__(256) void mailbox_enqueue_kernel(
    MboxView mv, const uint32_t* __restrict__ actor, const int64_t* __restrict__ a0, const int64_t* __restrict__ a1,
    const int64_t* __restrict__ a2, const uint16_t* __restrict__ mcol, uint32_t method_uniform, int64_t M,
    const TableEntry* __restrict__ table, uint64_t mask, const uint32_t* __restrict__ dir, uint32_t n_dir,
    uint32_t aw, int aw_shift, int rank_self, uint32_t origin_base, ReplyView rv) {
  extern __shared__ unsigned long long lds_mb[];
  const uint32_t S = 1u << mv.log_s;
  unsigned long long* base = lds_mb;      // [S]
  unsigned long long* lim = lds_mb + S;   // [S]
  unsigned* hist = reinterpret_cast<unsigned*>(lds_mb + 2 * S);  // [S]
  const int64_t tile = (int64_t)K * blockDim.x;
  unsigned long long n_enq = 0, n_ovf = 0, n_miss = 0;
  for (int64_t tb = blockIdx.x * tile; tb < M; tb += (int64_t)gridDim.x * tile) {
    for (uint32_t s = threadIdx.x; s < S; s += blockDim.x) hist[s] = 0;
    uint32_t a[K];
    int64_t x0[K], x1[K], x2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = tb + k * (int64_t)blockDim.x + threadIdx.x;
      const bool in = i < M;
      a[k] = in ? __builtin_nontemporal_load(actor + i) : 0xffffffffu;
      x0[k] = in ? __builtin_nontemporal_load(a0 + i) : 0;
      x1[k] = in && a1 ? __builtin_nontemporal_load(a1 + i) : 0;
      x2[k] = in && a2 ? __builtin_nontemporal_load(a2 + i) : 0;
    }
    int r[K];
    uint32_t mb[K];
    if constexpr (MODE == 1) {
      uint32_t w[K];
#pragma unroll
      for (int k = 0; k < K; ++k) w[k] = a[k] < n_dir ? dir[a[k]] : kDirFallback;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        r[k] = w[k] == kDirMissing ? -1 : (int)(w[k] & 0xff);
        mb[k] = w[k] >> 8;
        if (w[k] == kDirFallback) {
          if (a[k] != 0xffffffffu) lookup_entry(table, mask, actor_key(a[k]), r[k], mb[k]);
          else r[k] = -1;
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (MODE == 2 && a[k] < n_dir) {
          r[k] = aw_shift >= 0 ? (int)(a[k] & (aw - 1)) : (int)(a[k] % aw);
          mb[k] = aw_shift >= 0 ? a[k] >> aw_shift : a[k] / aw;
        } else if (a[k] == 0xffffffffu) {
          r[k] = -1;
          mb[k] = 0;
        } else {
          lookup_entry(table, mask, actor_key(a[k]), r[k], mb[k]);
        }
      }
    }
    bool in[K], ok[K];
    uint32_t meth[K], org[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = tb + k * (int64_t)blockDim.x + threadIdx.x;
      in[k] = i < M;
      ok[k] = in[k] && r[k] == rank_self && mb[k] < kMaxMbox;
      meth[k] = in[k] ? (mcol ? (uint32_t)mcol[i] : method_uniform) : 0u;
      org[k] = origin_base + (uint32_t)i;
    }
    enqueue_tile<LIVE, K, ARRIVAL>(mv, base, lim, hist, (uint32_t)(tb / tile), in, ok, mb, meth, x0, x1, x2, org,
                                   a2 != nullptr, rv, n_enq, n_ovf, n_miss);
  }
  block_add_stats(mv.stats, n_enq, kMbEnqueued, n_ovf, kMbOverflow, n_miss, kMbNoActor);
}

// ---------------------------------------------------------------- K2 on receipt
// At N > 1 the records arrive in the epoch's request regions (wire v2, already
// routed by the sender: word 0 is the local mailbox).  grid (X, R): block (x, d)
// tiles source rank d's region; origin = d * C + slot position, so the drain
// answers straight into the reply region the reverse all-to-all returns.
template <int NARGS, bool MC, int K, bool ARRIVAL>
__global__ __launch_bounds__(256) void mailbox_enqueue_slots_kernel(MboxView mv, const uint32_t* __restrict__ recv,
                                                                    int64_t req_words, uint32_t C, ReplyView rv) {
  extern __shared__ unsigned long long lds_mb[];
  const uint32_t S = 1u << mv.log_s;
  unsigned long long* base = lds_mb;
  unsigned long long* lim = lds_mb + S;
  unsigned* hist = reinterpret_cast<unsigned*>(lds_mb + 2 * S);
  constexpr int kStride = 1 + (MC ? 1 : 0) + 2 * NARGS;
  const int d = blockIdx.y;
  const uint32_t* rq = recv + (int64_t)d * req_words;
  const uint4 h = *reinterpret_cast<const uint4*>(rq);
  const bool valid = (h.w >> 16) & kFlagValid;
  const int64_t count = valid ? (int64_t)(h.x < C ? h.x : C) : 0;
  const uint32_t hm = h.w & 0xffffu;
  if (blockIdx.x == 0 && threadIdx.x == 0)  // reply header: delivered count (as the dispatch writes it)
    *reinterpret_cast<uint4*>(rv.slots + (int64_t)d * rv.rep_words) = make_uint4((uint32_t)count, 0u, 0u, 0u);
  const int64_t tile = (int64_t)K * blockDim.x;
  unsigned long long n_enq = 0, n_ovf = 0, n_miss = 0;
  for (int64_t tb = blockIdx.x * tile; tb < count; tb += (int64_t)gridDim.x * tile) {
    for (uint32_t s = threadIdx.x; s < S; s += blockDim.x) hist[s] = 0;
    bool in[K], ok[K];
    uint32_t mb[K], meth[K], org[K];
    int64_t x0[K], x1[K], x2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = tb + k * (int64_t)blockDim.x + threadIdx.x;
      in[k] = i < count;
      uint32_t wv[kStride];
      if (in[k]) {
        load_words<kStride>(rq + 4 + i * kStride, wv);
      } else {
#pragma unroll
        for (int j = 0; j < kStride; ++j) wv[j] = 0;
      }
      constexpr int o = 1 + (MC ? 1 : 0);
      mb[k] = wv[0];
      meth[k] = MC ? (wv[1] & 0xffffu) : hm;
      x0[k] = (int64_t)(((uint64_t)wv[o + 1] << 32) | wv[o]);
      x1[k] = NARGS > 1 ? (int64_t)(((uint64_t)wv[o + 3] << 32) | wv[o + 2]) : 0;
      x2[k] = NARGS > 2 ? (int64_t)(((uint64_t)wv[o + 5] << 32) | wv[o + 4]) : 0;
      ok[k] = in[k] && mb[k] < kMaxMbox;
      org[k] = (uint32_t)d * C + (uint32_t)i;
    }
    enqueue_tile<false, K, ARRIVAL>(mv, base, lim, hist, (uint32_t)(d * 4096 + tb / tile), in, ok, mb, meth, x0, x1,
                                    x2, org, NARGS > 2, rv, n_enq, n_ovf, n_miss);
  }
  block_add_stats(mv.stats, n_enq, kMbEnqueued, n_ovf, kMbOverflow, n_miss, kMbNoActor);
}

// The same from wire v3 request regions (packed.hpp): S dwords per record, fields
// at the agreed bit offsets, arguments zigzag-coded.  The drain still answers in
// wire v2 geometry (into a staging region set); pack_replies then writes the v3
// reply regions the reverse all-to-all moves.
template <int S, int K, bool ARRIVAL>
__global__ __launch_bounds__(256) void mailbox_enqueue_slots_packed_kernel(MboxView mv,
                                                                           const uint32_t* __restrict__ recv,
                                                                           int64_t req_words, uint32_t C,
                                                                           PackedLayout L, ReplyView rv) {
  extern __shared__ unsigned long long lds_mb[];
  const uint32_t NS = 1u << mv.log_s;
  unsigned long long* base = lds_mb;
  unsigned long long* lim = lds_mb + NS;
  unsigned* hist = reinterpret_cast<unsigned*>(lds_mb + 2 * NS);
  const int d = blockIdx.y;
  const uint32_t* rq = recv + (int64_t)d * req_words;
  const uint4 h = *reinterpret_cast<const uint4*>(rq);
  const bool valid = (h.w >> 16) & kFlagValid;
  const int64_t count = valid ? (int64_t)(h.x < C ? h.x : C) : 0;
  const uint32_t hm = h.w & 0xffffu;
  if (blockIdx.x == 0 && threadIdx.x == 0)
    *reinterpret_cast<uint4*>(rv.slots + (int64_t)d * rv.rep_words) = make_uint4((uint32_t)count, 0u, 0u, 0u);
  const int64_t tile = (int64_t)K * blockDim.x;
  const bool has_a2 = L.w[4] != 0;
  unsigned long long n_enq = 0, n_ovf = 0, n_miss = 0;
  for (int64_t tb = blockIdx.x * tile; tb < count; tb += (int64_t)gridDim.x * tile) {
    for (uint32_t s = threadIdx.x; s < NS; s += blockDim.x) hist[s] = 0;
    bool in[K], ok[K];
    uint32_t mb[K], meth[K], org[K];
    int64_t x0[K], x1[K], x2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = tb + k * (int64_t)blockDim.x + threadIdx.x;
      in[k] = i < count;
      uint32_t wv[S];
      if (in[k]) {
        load_words<S>(rq + 4 + i * S, wv);
      } else {
#pragma unroll
        for (int j = 0; j < S; ++j) wv[j] = 0;
      }
      mb[k] = (uint32_t)packed_field<S>(L, 1, wv);
      meth[k] = L.w[0] ? (uint32_t)packed_field<S>(L, 0, wv) : hm;
      x0[k] = zz_dec(packed_field<S>(L, 2, wv));
      x1[k] = zz_dec(packed_field<S>(L, 3, wv));
      x2[k] = zz_dec(packed_field<S>(L, 4, wv));
      ok[k] = in[k] && mb[k] < kMaxMbox;
      org[k] = (uint32_t)d * C + (uint32_t)i;
    }
    enqueue_tile<false, K, ARRIVAL>(mv, base, lim, hist, (uint32_t)(d * 4096 + tb / tile), in, ok, mb, meth, x0, x1,
                                    x2, org, has_a2, rv, n_enq, n_ovf, n_miss);
  }
  block_add_stats(mv.stats, n_enq, kMbEnqueued, n_ovf, kMbOverflow, n_miss, kMbNoActor);
}

// Run one window of up to 64 records (lane l holds ring position h + l) in ring
// order per actor.  Lanes whose actor appears once in the window run together;
// lanes of an actor that appears more than once (found through a 128-entry LDS
// owner table per wave) run one at a time in lane order afterwards.
__device__ __forceinline__ unsigned long long run_window_ordered(const MboxMsg& x, int64_t* __restrict__ state,
                                                                  uint32_t n_state, uint64_t delay_ticks,
                                                                  OutboxView ob, const ReplyView& rv,
                                                                  volatile uint32_t* owner, volatile uint32_t* conf,
                                                                  unsigned long long& failed, uint32_t log_s) {
  const unsigned lane = lane_id();
  const uint32_t h = (x.m.actor >> log_s) & 127u;
  if (x.valid) conf[h] = 0u;
  if (x.valid) owner[h] = lane;
  const bool lost = x.valid && owner[h] != lane;
  if (lost) conf[h] = 1u;
  const bool serial = x.valid && conf[h] != 0u;
  uint64_t ser = __ballot(serial);
  if (x.valid && !serial) {
    const ReplyRecord r = run_handler(x.m, state, n_state, delay_ticks, ob, true);
    failed += r.status != kStatusOk;
    write_reply(rv, x.origin, r);
  }
  const unsigned long long n_serial = (unsigned long long)__popcll(ser);
  while (ser) {
    vm_drain();  // the previous lane's state store has landed before the next one reads
    const int l = __builtin_ctzll(ser);
    if ((int)lane == l) {
      const ReplyRecord r = run_handler(x.m, state, n_state, delay_ticks, ob, true);
      failed += r.status != kStatusOk;
      write_reply(rv, x.origin, r);
    }
    ser &= ser - 1;
  }
  vm_drain();  // this window's state stores land before the next window's loads
  return n_serial;
}

// ---------------------------------------------------------------- K3 epoch drain (parallel)
// grid (X, S): block (x, s) strides over shard s's queued positions.  Stateless
// and commutative methods only (the host picks the ordered form otherwise).  The
// last block of each shard commits that shard's head (per-shard ticket, self-resetting).
template <int FIXED, int K>
__global__ __launch_bounds__(256) void mailbox_drain_kernel(MboxView mv, int64_t* __restrict__ state,
                                                            uint32_t n_state, uint64_t delay_ticks, OutboxView ob,
                                                            ReplyView rv) {
  const uint32_t s = blockIdx.y;
  const uint64_t Q = 1ull << mv.log_q;
  const uint64_t h = *ctr_head(mv, s), t = *ctr_tail(mv, s);
  const uint64_t end = t < h + Q ? t : h + Q;
  unsigned long long done = 0, failed = 0, holes = 0;
  const uint64_t step = (uint64_t)gridDim.x * K * blockDim.x;
  for (uint64_t p0 = h + (uint64_t)blockIdx.x * K * blockDim.x; p0 < end; p0 += step) {
    u32x4 ha[K], hb[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t p = p0 + (uint64_t)k * blockDim.x + threadIdx.x;
      if (p < end) {
        const uint64_t slot = slot_at(mv, s, p);
        ha[k] = *reinterpret_cast<const u32x4*>(rec_a(mv, slot));
        hb[k] = *reinterpret_cast<const u32x4*>(rec_b(mv, slot));
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t p = p0 + (uint64_t)k * blockDim.x + threadIdx.x;
      if (p >= end) continue;
      if (ha[k].x != lap_tag(mv, p)) {
        ++holes;
        continue;
      }
      const uint64_t slot = slot_at(mv, s, p);
      MboxMsg x = decode(ha[k], hb[k], mv.a2 ? mv.a2 + slot : nullptr);
      if (FIXED) x.m.method = FIXED;
      const ReplyRecord r = run_handler(x.m, state, n_state, delay_ticks, ob);
      failed += r.status != kStatusOk;
      write_reply(rv, x.origin, r);
      ++done;
    }
  }
  // `processed` is counted per shard by its last block (positions - holes), not by
  // every block: 1024 same-address atomics at the kernel's end serialise (~9 ns
  // each) in its tail.  A block with holes takes them back out of the count.
  (void)done;
  block_add_stats(mv.stats, holes ? (unsigned long long)(-(long long)holes) : 0ull, kMbProcessed, failed, kMbFailed,
                  holes, kMbHoles);
  // the last block of this shard commits its head (every block of the shard has
  // read the head by now).  A ticket per shard: one word for the whole grid
  // serialised 1024 returning atomics.  No fence: nothing is handed over but the
  // ticket itself, and an agent release per block wrote back the XCD's L2 --
  // half-written reply lines included -- 2048 times per drain
  __shared__ int last;
  unsigned long long* tk = mv.ctr + (uint64_t)s * kMboxCtrStride + kMboxCtrTicket;
  if (threadIdx.x == 0) last = atomicAdd(tk, 1ull) == gridDim.x - 1;
  __syncthreads();
  if (last && threadIdx.x == 0) {
    *ctr_head(mv, s) = t;
    *ctr_done(mv, s) = t;  // epoch enqueues do not count `done`; the drain settles it
    if (end > h) atomicAdd(&mv.stats[kMbProcessed], (unsigned long long)(end - h));
    *tk = 0;
  }
}

// ---------------------------------------------------------------- K3 epoch drain (ordered)
// One wave per shard; windows of 64 consecutive positions in ring order.
__global__ __launch_bounds__(256) void mailbox_drain_ordered_kernel(MboxView mv, int64_t* __restrict__ state,
                                                                    uint32_t n_state, uint64_t delay_ticks,
                                                                    OutboxView ob, ReplyView rv) {
  __shared__ uint32_t owner_tab[4][128], conf_tab[4][128];
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  const uint32_t s = blockIdx.x * 4 + w;
  const uint32_t S = 1u << mv.log_s;
  if (s >= S) return;  // whole wave: no barrier follows
  const uint64_t Q = 1ull << mv.log_q;
  const uint64_t h = *ctr_head(mv, s), t = *ctr_tail(mv, s);
  const uint64_t end = t < h + Q ? t : h + Q;
  unsigned long long done = 0, failed = 0, holes = 0, serial = 0;
  for (uint64_t p0 = h; p0 < end; p0 += kWave) {
    const uint64_t p = p0 + lane;
    MboxMsg x;
    x.valid = false;
    if (p < end) {
      const uint64_t slot = slot_at(mv, s, p);
      const u32x4 ha = *reinterpret_cast<const u32x4*>(rec_a(mv, slot));
      const u32x4 hb = *reinterpret_cast<const u32x4*>(rec_b(mv, slot));
      if (ha.x == lap_tag(mv, p)) {
        x = decode(ha, hb, mv.a2 ? mv.a2 + slot : nullptr);
        ++done;
      } else {
        ++holes;
      }
    }
    serial += run_window_ordered(x, state, n_state, delay_ticks, ob, rv, owner_tab[w], conf_tab[w], failed,
                                 mv.log_s);
  }
  if (lane == 0) *ctr_head(mv, s) = t, *ctr_done(mv, s) = t;
  for (int off = 32; off > 0; off >>= 1) {
    done += __shfl_xor(done, off);
    failed += __shfl_xor(failed, off);
    holes += __shfl_xor(holes, off);
  }
  if (lane == 0) {
    if (done) atomicAdd(&mv.stats[kMbProcessed], done);
    if (failed) atomicAdd(&mv.stats[kMbFailed], failed);
    if (holes) atomicAdd(&mv.stats[kMbHoles], holes);
    if (serial) atomicAdd(&mv.stats[kMbSerial], serial);
  }
}

// ---------------------------------------------------------------- K3 persistent consumer
// Wave g of G owns shards g, g + G, ...  Polls the next window's tags with sc1
// loads; a window is the run of consecutive published records (up to 64).  A
// position whose tag has not arrived while the shard is quiescent (done ==
// tail, read after the tag) is a hole and is skipped.  Exits on: the host's
// stop flag once its shards are empty and quiescent, `idle_ticks` without work,
// or `max_ticks` (hard bound: nothing can spin forever).
__global__ __launch_bounds__(256) void mailbox_consumer_kernel(MboxView mv, MboxCtrl* __restrict__ ctrl,
                                                               int64_t* __restrict__ state, uint32_t n_state,
                                                               uint64_t delay_ticks, ReplyView rv,
                                                               uint64_t idle_ticks, uint64_t max_ticks) {
  __shared__ uint32_t owner_tab[4][128], conf_tab[4][128];
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  const uint32_t g = blockIdx.x * 4 + w, G = gridDim.x * 4;
  const uint32_t S = 1u << mv.log_s;
  const uint64_t t_start = realtime_ticks();
  uint64_t last_work = t_start;
  unsigned long long processed = 0, failed = 0, holes = 0, serial = 0;
  bool stopping = false, lifetime = false;
  unsigned sweeps = 0;
  for (;;) {
    bool work = false, pending = false;
    for (uint32_t s = g; s < S; s += G) {
      unsigned long long* hp = ctr_head(mv, s);
      const uint64_t h = ld_fresh(hp);
      const uint64_t p = h + lane;
      uint32_t* rc = rec_at(mv, s, p);
      const u32x4 ha = ld16_fresh(rc);
      const bool ready = ha.x == lap_tag(mv, p);
      const uint64_t m = __ballot(ready);
      unsigned n = m == ~0ull ? 64u : (unsigned)__builtin_ctzll(~m);
      if (n == 0) {
        const uint64_t t = ld_fresh(ctr_tail(mv, s));
        if (h < t) {
          pending = true;
          // quiescent shard (every reserved position finished) and still no tag: a hole
          const uint64_t d = ld_fresh(ctr_done(mv, s));
          if (d == t && ld16_fresh(rec_at(mv, s, h)).x != lap_tag(mv, h)) {
            if (lane == 0) __hip_atomic_exchange(hp, (unsigned long long)(h + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ++holes;
            work = true;
          }
        }
        continue;
      }
      MboxMsg x;
      x.valid = false;
      if (lane < n) {
        const uint64_t slot = slot_at(mv, s, p);
        const u32x4 hb = ld16_fresh(rec_b(mv, slot));
        int64_t a2v = 0;
        if (((ha.w >> 16) & kFlagA2) && mv.a2) a2v = (int64_t)ld_fresh(reinterpret_cast<unsigned long long*>(mv.a2 + slot));
        x = decode(ha, hb, &a2v);
      }
      serial += run_window_ordered(x, state, n_state, delay_ticks, OutboxView(), rv, owner_tab[w], conf_tab[w],
                                   failed, mv.log_s);
      processed += n;
      if (lane == 0) __hip_atomic_exchange(hp, (unsigned long long)(h + n), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // slots free again
      work = true;
    }
    const uint64_t now = realtime_ticks();
    if (work) {
      last_work = now;
      continue;
    }
    if ((++sweeps & 15) == 0 && !stopping) stopping = sys_ld64(&ctrl->stop) != 0;
    lifetime = now - t_start > max_ticks;
    if ((stopping && !pending) || lifetime || (idle_ticks && now - last_work > idle_ticks && !pending)) break;
    __builtin_amdgcn_s_sleep(2);
  }
  for (int off = 32; off > 0; off >>= 1) failed += __shfl_xor(failed, off);
  if (lane == 0) {
    atomicAdd(&mv.stats[kMbProcessed], processed);
    if (failed) atomicAdd(&mv.stats[kMbFailed], failed);
    if (holes) atomicAdd(&mv.stats[kMbHoles], holes);
    if (serial) atomicAdd(&mv.stats[kMbSerial], serial);
    __hip_atomic_fetch_add(&ctrl->processed, (uint64_t)processed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_fetch_add(lifetime ? &ctrl->exits_lifetime : &ctrl->exits_idle, (uint64_t)1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_fetch_add(&ctrl->live_waves, (uint64_t)-1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Before a persistent session: positions reserved by epoch enqueues (which do
// not count `done`) are all finished once those kernels have completed.
__global__ void mailbox_settle_kernel(MboxView mv) {
  const uint32_t S = 1u << mv.log_s;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < S; s += gridDim.x * blockDim.x)
    *ctr_done(mv, s) = *ctr_tail(mv, s);
}

// ---------------------------------------------------------------- launchers
static unsigned mb_grid(int64_t work, int per, unsigned cap) {
  int64_t g = (work + per - 1) / per;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

void launch_mailbox_enqueue(const MboxView& mv, uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2,
                            uintptr_t method_col, int method_uniform, int64_t M, uintptr_t table, uint64_t cap,
                            uintptr_t dir, uint32_t n_dir, uint32_t affine_w, int rank_self, uint32_t origin_base,
                            const ReplyView& rv, bool live, uintptr_t stream, bool arrival) {
  if (M <= 0) return;
  if (arrival && live) throw std::invalid_argument("mailbox enqueue: a live session shards by actor");
  if (!actor || !a0) throw std::invalid_argument("mailbox enqueue: missing column");
  if (a2 && !mv.a2) throw std::invalid_argument("mailbox enqueue: 3-argument batch but the rings have no a2 array");
  if (cap == 0 || (cap & (cap - 1))) throw std::invalid_argument("table capacity must be a power of two");
  if ((uint64_t)origin_base + (uint64_t)M > rv.n) throw std::invalid_argument("mailbox enqueue: reply view too small");
  if ((uint64_t)origin_base + (uint64_t)M > 0xffffffffull) throw std::invalid_argument("mailbox enqueue: origin > u32");
  constexpr int K = 8;   // actor sharding: a big tile amortises the (tile, shard) reservations
  // arrival sharding: 4 items per thread (one reservation per tile; 64 VGPRs, 8
  // waves/SIMD); 1 and 2 measured slower at 1 Mi and 8 Mi messages
  // (profiles/r2_enq_items_sweep.txt).
  constexpr int KA = 4;
  const int aw_shift = (affine_w && (affine_w & (affine_w - 1)) == 0) ? __builtin_ctz(affine_w) : -1;
  const int mode = (affine_w && n_dir) ? 2 : (dir && n_dir) ? 1 : 0;
  const uint32_t S = 1u << mv.log_s;
  const size_t lds = (size_t)S * (8 + 8 + 4);
  constexpr unsigned enq_blocks = 4096u;
  const dim3 g(mb_grid(M, 256 * (arrival ? KA : K), enq_blocks));
#define PT_ENQ(MO, LV)                                                                                                \
  hipLaunchKernelGGL((mailbox_enqueue_kernel<MO, LV, K>), g, dim3(256), lds, as_stream(stream), mv,                \
                     (const uint32_t*)actor, (const int64_t*)a0, (const int64_t*)a1, (const int64_t*)a2,           \
                     (const uint16_t*)method_col, (uint32_t)method_uniform, M, (const TableEntry*)table, cap - 1,  \
                     (const uint32_t*)dir, n_dir, affine_w, aw_shift, rank_self, origin_base, rv)
#define PT_ENQA_K(MO, KV)                                                                                             \
  hipLaunchKernelGGL((mailbox_enqueue_kernel<MO, false, KV, true>), g, dim3(256), lds, as_stream(stream), mv,       \
                     (const uint32_t*)actor, (const int64_t*)a0, (const int64_t*)a1, (const int64_t*)a2,           \
                     (const uint16_t*)method_col, (uint32_t)method_uniform, M, (const TableEntry*)table, cap - 1,  \
                     (const uint32_t*)dir, n_dir, affine_w, aw_shift, rank_self, origin_base, rv)
#define PT_ENQA(MO)     \
  do {                  \
    if (KA == 1)        \
      PT_ENQA_K(MO, 1); \
    else if (KA == 2)   \
      PT_ENQA_K(MO, 2); \
    else                \
      PT_ENQA_K(MO, 4); \
  } while (0)
  if (live) {
    if (mode == 2) PT_ENQ(2, true); else if (mode == 1) PT_ENQ(1, true); else PT_ENQ(0, true);
  } else if (arrival) {
    if (mode == 2) PT_ENQA(2); else if (mode == 1) PT_ENQA(1); else PT_ENQA(0);
  } else {
    if (mode == 2) PT_ENQ(2, false); else if (mode == 1) PT_ENQ(1, false); else PT_ENQ(0, false);
  }
#undef PT_ENQ
#undef PT_ENQA
#undef PT_ENQA_K
  PT_HIP_CHECK(hipGetLastError());
}

void launch_mailbox_enqueue_slots(const MboxView& mv, uintptr_t recv, int R, int64_t C, int nargs, bool mc,
                                  const ReplyView& rv, int64_t expected_per_rank, bool arrival, uintptr_t stream) {
  if (R < 1 || C < 1 || !rv.slots || rv.C != (uint32_t)C) throw std::invalid_argument("mailbox enqueue slots: geometry");
  if (nargs > 2 && !mv.a2) throw std::invalid_argument("mailbox enqueue: 3-argument records but no a2 array");
  if ((uint64_t)R * (uint64_t)C > 0xffffffffull) throw std::invalid_argument("mailbox enqueue: origin > u32");
  constexpr int K = 4;
  const int64_t req_words = wire_req_words(C, nargs, mc);
  const uint32_t S = 1u << mv.log_s;
  const size_t lds = (size_t)S * (8 + 8 + 4);
  const int64_t per = expected_per_rank > 0 ? expected_per_rank : C;
  const dim3 g(mb_grid(per, 256 * K, (unsigned)std::max(1, 4096 / R)), (unsigned)R);
#define PT_ENQS(NA, MCV)                                                                                           \
  if (arrival)                                                                                                    \
    hipLaunchKernelGGL((mailbox_enqueue_slots_kernel<NA, MCV, K, true>), g, dim3(256), lds, as_stream(stream), mv, \
                       (const uint32_t*)recv, req_words, (uint32_t)C, rv);                                        \
  else                                                                                                            \
    hipLaunchKernelGGL((mailbox_enqueue_slots_kernel<NA, MCV, K, false>), g, dim3(256), lds, as_stream(stream), mv, \
                       (const uint32_t*)recv, req_words, (uint32_t)C, rv);
  switch (nargs * 2 + (mc ? 1 : 0)) {
    case 2: PT_ENQS(1, false) break;
    case 3: PT_ENQS(1, true) break;
    case 4: PT_ENQS(2, false) break;
    case 5: PT_ENQS(2, true) break;
    case 6: PT_ENQS(3, false) break;
    default: PT_ENQS(3, true) break;
  }
#undef PT_ENQS
  PT_HIP_CHECK(hipGetLastError());
}

void launch_mailbox_enqueue_slots_packed(const MboxView& mv, uintptr_t recv, int R, int64_t C, const PackedLayout& L,
                                         const ReplyView& rv, int64_t expected_per_rank, bool arrival,
                                         uintptr_t stream) {
  if (R < 1 || C < 1 || !rv.slots || rv.C != (uint32_t)C) throw std::invalid_argument("mailbox enqueue slots: geometry");
  if (L.w[4] && !mv.a2) throw std::invalid_argument("mailbox enqueue: 3-argument records but no a2 array");
  if (L.S < 1 || L.S > 8) throw std::invalid_argument("mailbox enqueue: packed record of 1..8 dwords");
  if ((uint64_t)R * (uint64_t)C > 0xffffffffull) throw std::invalid_argument("mailbox enqueue: origin > u32");
  constexpr int K = 4;
  const int64_t req_words = packed_req_words(C, L.S);
  const uint32_t NS = 1u << mv.log_s;
  const size_t lds = (size_t)NS * (8 + 8 + 4);
  const int64_t per = expected_per_rank > 0 ? expected_per_rank : C;
  const dim3 g(mb_grid(per, 256 * K, (unsigned)std::max(1, 4096 / R)), (unsigned)R);
#define PT_ENQP(SV)                                                                                                  \
  if (arrival)                                                                                                       \
    hipLaunchKernelGGL((mailbox_enqueue_slots_packed_kernel<SV, K, true>), g, dim3(256), lds, as_stream(stream), mv, \
                       (const uint32_t*)recv, req_words, (uint32_t)C, L, rv);                                        \
  else                                                                                                               \
    hipLaunchKernelGGL((mailbox_enqueue_slots_packed_kernel<SV, K, false>), g, dim3(256), lds, as_stream(stream),    \
                       mv, (const uint32_t*)recv, req_words, (uint32_t)C, L, rv);
  switch (L.S) {
    case 1: PT_ENQP(1) break;
    case 2: PT_ENQP(2) break;
    case 3: PT_ENQP(3) break;
    case 4: PT_ENQP(4) break;
    case 5: PT_ENQP(5) break;
    case 6: PT_ENQP(6) break;
    case 7: PT_ENQP(7) break;
    default: PT_ENQP(8) break;
  }
#undef PT_ENQP
  PT_HIP_CHECK(hipGetLastError());
}

void launch_mailbox_drain(const MboxView& mv, uintptr_t state, uint32_t n_state, uint64_t delay_ticks,
                          const OutboxView& ob, const ReplyView& rv, bool ordered, uintptr_t stream,
                          int fixed_method) {
  const uint32_t S = 1u << mv.log_s;
  hipStream_t st = as_stream(stream);
  if (ordered) {
    hipLaunchKernelGGL(mailbox_drain_ordered_kernel, dim3((S + 3) / 4), dim3(256), 0, st, mv, (int64_t*)state,
                       n_state, delay_ticks, ob, rv);
  } else {
    // ~1024 blocks over the shards (each block strides over its shard's queue).
    // Measured (8 Mi records, 256 shards): 1024 / 2048 / 4096 blocks 0.232 / 0.237 /
    // 0.240 ms per mailbox step; 4 records per thread instead of 2: no change.
    constexpr unsigned target = 1024u;
    const unsigned X = S >= target ? 1u : target / S;
    // a Send that knows every queued record's method (uniform batch) drains with
    // that handler constant-folded
    if (fixed_method == kCalculatorMultiply)
      hipLaunchKernelGGL((mailbox_drain_kernel<kCalculatorMultiply, 2>), dim3(X, S), dim3(256), 0, st, mv,
                         (int64_t*)state, n_state, delay_ticks, ob, rv);
    else
      hipLaunchKernelGGL((mailbox_drain_kernel<0, 2>), dim3(X, S), dim3(256), 0, st, mv, (int64_t*)state, n_state,
                         delay_ticks, ob, rv);
  }
  PT_HIP_CHECK(hipGetLastError());
}

void launch_mailbox_consumer(const MboxView& mv, MboxCtrl* ctrl, uintptr_t state, uint32_t n_state,
                             uint64_t delay_ticks, const ReplyView& rv, int blocks, uint64_t idle_ticks,
                             uint64_t max_ticks, uintptr_t stream) {
  hipLaunchKernelGGL(mailbox_consumer_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), mv, ctrl,
                     (int64_t*)state, n_state, delay_ticks, rv, idle_ticks, max_ticks);
  PT_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- host class
static uint32_t log2_exact(uint32_t v, const char* what) {
  if (v == 0 || (v & (v - 1))) throw std::invalid_argument(std::string(what) + " must be a power of two");
  return (uint32_t)__builtin_ctz(v);
}

Mailboxes::Mailboxes(int device, uint32_t shards, uint32_t slots, bool with_a2) : device_(device) {
  mv_.log_s = log2_exact(shards, "mailbox shards");
  mv_.log_q = log2_exact(slots, "mailbox slots per shard");
  mv_.planar = true;  // (the interleaved 32-B record form measured slower; the flag stays for the live rings)
  if (shards > (uint32_t)kMboxMaxShards) throw std::invalid_argument("mailbox shards <= 4096");
  if (slots < 64) throw std::invalid_argument("mailbox slots per shard >= 64");
  PT_HIP_CHECK(hipSetDevice(device_));
  stream_ = dedicated_stream(device_);  // the persistent consumer runs here
  const uint64_t n = (uint64_t)shards * slots;
  // plane B starts past plane A plus a pad: A[slot] and B[slot] are read together,
  // and a power-of-two distance between them aliases in the HBM address mapping.
  // Measured (bench mailbox step, pad sweep): pad 0 / 4.3 KB / 65 KB / 2 MB / 8 MB /
  // 128 MB: 0.234-0.238 ms; 1 MB + 3.4 KB: 0.215-0.217; 33 MB: 0.219.
  const uint64_t pad = 1052032ull;
  mv_.b_off = (n * 16 + pad) / 4;
  rec_bytes_ = n * 32 + pad;
  PT_HIP_CHECK(hipMalloc((void**)&mv_.rec, rec_bytes_));
  PT_HIP_CHECK(hipMemsetAsync(mv_.rec, 0, rec_bytes_, stream_));  // tag 0 = never published
  bytes_ = rec_bytes_;
  if (with_a2) {
    PT_HIP_CHECK(hipMalloc((void**)&mv_.a2, n * 8));
    bytes_ += n * 8;
  }
  const size_t ctr_bytes = (size_t)shards * kMboxCtrStride * 8;
  PT_HIP_CHECK(hipMalloc((void**)&mv_.ctr, ctr_bytes));
  PT_HIP_CHECK(hipMemsetAsync(mv_.ctr, 0, ctr_bytes, stream_));
  PT_HIP_CHECK(hipMalloc((void**)&sort_hist_, (size_t)kMboxSortHistWords * sizeof(uint32_t)));
  PT_HIP_CHECK(hipMalloc((void**)&sort_gsum_, (size_t)kMboxSortGroups * shards * sizeof(uint32_t)));
  PT_HIP_CHECK(hipMemsetAsync(sort_gsum_, 0, (size_t)kMboxSortGroups * shards * sizeof(uint32_t), stream_));
  PT_HIP_CHECK(hipMalloc((void**)&sort_ticket_, kTicketWords * sizeof(unsigned)));
  PT_HIP_CHECK(hipMemsetAsync(sort_ticket_, 0, kTicketWords * sizeof(unsigned), stream_));
  PT_HIP_CHECK(hipMalloc((void**)&sort_tctr_, 2 * sizeof(unsigned)));
  PT_HIP_CHECK(hipMemsetAsync(sort_tctr_, 0, 2 * sizeof(unsigned), stream_));
  bytes_ += (size_t)kMboxSortHistWords * sizeof(uint32_t) + (size_t)kMboxSortGroups * shards * sizeof(uint32_t);
  PT_HIP_CHECK(hipMalloc((void**)&mv_.stats, kMbStripes * kMbStatWords * 8));
  PT_HIP_CHECK(hipMemsetAsync(mv_.stats, 0, kMbStripes * kMbStatWords * 8, stream_));
  bytes_ += ctr_bytes + kMbStripes * kMbStatWords * 8;
  const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable;
  PT_HIP_CHECK(hipHostMalloc((void**)&ctrl_, sizeof(MboxCtrl), fl));
  memset((void*)ctrl_, 0, sizeof(MboxCtrl));
  PT_HIP_CHECK(hipHostGetDevicePointer((void**)&dctrl_, ctrl_, 0));
  // (not a device-wide sync: a persistent dispatcher may be running)
  PT_HIP_CHECK(hipStreamSynchronize(stream_));
}

Mailboxes::~Mailboxes() {
  try {
    if (started_) stop();
  } catch (...) {
  }
  (void)hipSetDevice(device_);
  if (stream_) (void)hipStreamDestroy(stream_);
  (void)hipFree(mv_.rec);
  if (mv_.a2) (void)hipFree(mv_.a2);
  (void)hipFree(mv_.ctr);
  (void)hipFree(mv_.stats);
  for (void* p : {(void*)sort_hist_, (void*)sort_gsum_, (void*)sort_ticket_, (void*)sort_rw_, (void*)sort_sidx_,
                  (void*)sort_tinfo_, (void*)sort_desc_, (void*)sort_tctr_, stage_rep_,
                  (void*)r8w_, (void*)r8max_, (void*)r8esc_, (void*)sort_resv_, (void*)pres_})
    if (p) (void)hipFree(p);
  if (ctrl_) (void)hipHostFree(ctrl_);
  if (r8host_) (void)hipHostFree(r8host_);
}

void Mailboxes::enqueue(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                        int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir,
                        uint32_t affine_w, int rank_self, uint32_t origin_base, uintptr_t out_val, uintptr_t out_st,
                        uint64_t out_n, bool live, uintptr_t stream, bool arrival) {
  ReplyView rv{(int64_t*)out_val, (int32_t*)out_st, out_n};
  if (!out_val || !out_st) throw std::invalid_argument("mailbox enqueue: reply outputs required");
  launch_mailbox_enqueue(mv_, actor, a0, a1, a2, method_col, method_uniform, M, table, cap, dir, n_dir, affine_w,
                         rank_self, origin_base, rv, live, stream, arrival);
}

void Mailboxes::drain(uintptr_t state, uint32_t n_state, uint64_t delay_ticks, uintptr_t out_val, uintptr_t out_st,
                      uint64_t out_n, bool ordered, uintptr_t stream, const std::vector<uintptr_t>& outbox,
                      uint64_t outbox_cap, int fixed_method) {
  if (started_ && running()) throw std::runtime_error("mailbox drain: a persistent consumer owns the rings");
  OutboxView ob;
  if (outbox_cap) {
    if (outbox.size() != 6) throw std::invalid_argument("outbox: [actor, a0, a1, a2, method, count]");
    ob.actor = (uint32_t*)outbox[0];
    ob.a0 = (int64_t*)outbox[1];
    ob.a1 = (int64_t*)outbox[2];
    ob.a2 = (int64_t*)outbox[3];
    ob.method = (uint16_t*)outbox[4];
    ob.count = (unsigned long long*)outbox[5];
    ob.cap = outbox_cap;
  }
  launch_mailbox_drain(mv_, state, n_state, delay_ticks, ob, ReplyView{(int64_t*)out_val, (int32_t*)out_st, out_n},
                       ordered, stream, fixed_method);
}

void Mailboxes::start(uintptr_t state, uint32_t n_state, uint64_t delay_ticks, uintptr_t out_val, uintptr_t out_st,
                      uint64_t out_n, int blocks, double idle_ms, double max_s) {
  if (started_ && running()) throw std::runtime_error("mailbox consumer already running");
  if (blocks < 1 || blocks > 256) throw std::invalid_argument("consumer blocks: 1..256 (stay below residency)");
  PT_HIP_CHECK(hipSetDevice(device_));
  PT_HIP_CHECK(hipStreamSynchronize(stream_));
  __atomic_store_n(&ctrl_->stop, 0ull, __ATOMIC_SEQ_CST);
  __atomic_store_n(&ctrl_->live_waves, (uint64_t)blocks * 4, __ATOMIC_SEQ_CST);
  hipLaunchKernelGGL(mailbox_settle_kernel, dim3(1), dim3(256), 0, stream_, mv_);
  launch_mailbox_consumer(mv_, dctrl_, state, n_state, delay_ticks,
                          ReplyView{(int64_t*)out_val, (int32_t*)out_st, out_n}, blocks,
                          (uint64_t)(idle_ms * 1e5), (uint64_t)(max_s * 1e8), (uintptr_t)stream_);
  started_ = true;
  ++launches_;
}

void Mailboxes::stop() {
  if (!started_) return;
  __atomic_store_n(&ctrl_->stop, 1ull, __ATOMIC_SEQ_CST);
  PT_HIP_CHECK(hipSetDevice(device_));
  PT_HIP_CHECK(hipStreamSynchronize(stream_));
  started_ = false;
}

bool Mailboxes::running() const { return __atomic_load_n(&ctrl_->live_waves, __ATOMIC_ACQUIRE) != 0; }

uint64_t Mailboxes::consumer_processed() const { return __atomic_load_n(&ctrl_->processed, __ATOMIC_ACQUIRE); }

void Mailboxes::reset(uintptr_t stream) {
  if (started_ && running()) throw std::runtime_error("mailbox reset: consumer running");
  hipStream_t s = as_stream(stream);
  const uint64_t n = (uint64_t)shards() * slots();
  PT_HIP_CHECK(hipMemsetAsync(mv_.rec, 0, rec_bytes_, s));
  PT_HIP_CHECK(hipMemsetAsync(mv_.ctr, 0, (size_t)shards() * kMboxCtrStride * 8, s));
  PT_HIP_CHECK(hipMemsetAsync(mv_.stats, 0, kMbStripes * kMbStatWords * 8, s));
  PT_HIP_CHECK(hipMemsetAsync(sort_gsum_, 0, (size_t)kMboxSortGroups * shards() * sizeof(uint32_t), s));
  PT_HIP_CHECK(hipMemsetAsync(sort_ticket_, 0, kTicketWords * sizeof(unsigned), s));
}

void Mailboxes::set_epoch_counter(uint32_t v) {
  PT_HIP_CHECK(hipSetDevice(device_));
  PT_HIP_CHECK(hipDeviceSynchronize());
  PT_HIP_CHECK(hipMemcpy(sort_tctr_ + 1, &v, sizeof v, hipMemcpyHostToDevice));
}

uint32_t Mailboxes::epoch_counter() const {
  uint32_t v = 0;
  PT_HIP_CHECK(hipSetDevice(device_));
  PT_HIP_CHECK(hipMemcpy(&v, sort_tctr_ + 1, sizeof v, hipMemcpyDeviceToHost));
  return v;
}

std::vector<uint64_t> Mailboxes::stats() const {
  std::vector<uint64_t> raw((size_t)kMbStripes * kMbStatWords), v(kMbStatWords, 0);
  PT_HIP_CHECK(hipSetDevice(device_));
  PT_HIP_CHECK(hipMemcpy(raw.data(), mv_.stats, raw.size() * 8, hipMemcpyDeviceToHost));
  for (int k = 0; k < kMbStripes; ++k)
    for (int w = 0; w < kMbStatWords; ++w) v[w] += raw[(size_t)k * kMbStatWords + w];
  return v;
}

std::vector<uint64_t> Mailboxes::shard_counters() const {
  const uint32_t S = shards();
  std::vector<uint64_t> raw((size_t)S * kMboxCtrStride), out((size_t)S * 3);
  PT_HIP_CHECK(hipSetDevice(device_));
  PT_HIP_CHECK(hipMemcpy(raw.data(), mv_.ctr, raw.size() * 8, hipMemcpyDeviceToHost));
  for (uint32_t s = 0; s < S; ++s) {
    out[3 * s] = raw[(size_t)s * kMboxCtrStride];
    out[3 * s + 1] = raw[(size_t)s * kMboxCtrStride + 1];
    out[3 * s + 2] = raw[(size_t)s * kMboxCtrStride + 16];
  }
  return out;
}

}  // namespace ptype
