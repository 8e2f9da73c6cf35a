// Device side of the sorted epoch mailboxes (design notes: mailbox_sort.hip):
// the kernels and their helpers, all templates, compiled into the launcher TUs
// that instantiate them -- mailbox_sort.hip (sorts, ring / message-order drains,
// arrival sharding), mailbox_sort_fused.hip (the fused sort + drain) and
// mailbox_sort_ordered.hip (the ordered drain and the ring-order completion) --
// so the variants build in parallel instead of as one long object.
#pragma once
#include <algorithm>
#include <type_traits>
#include <vector>

#include "mailbox.hpp"
#include "mailbox_dev.hpp"
#include "route_common.hpp"
#include "sort_common.hpp"
#include "tune.hpp"

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
constexpr uint32_t kRunSpilled = 0x80000000u;  // tinfo count word: the run did not fit the ring's room

template <int MODE>
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
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const int64_t i = tile_index(t, k);
      const bool ok = r[k] == in.rank_self && mb[k] < kMaxMbox;
      if (i < in.M) rw[i] = ok ? mb[k] : kNoSlot;
      if (ok) atomicAdd(&cnt[mb[k] & (S - 1)], 1u);
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

// Per-tile runs (`tinfo`, [tiles][2][S] u32): tile t's records of shard s sit at
// ring slots s | ((bias + j) & (Q - 1)), j < count (bias = epoch-start tail +
// the run's offset + the shard's rotation; count clamped to the free room, its
// top bit set when the run spilled / overflowed the room) -- what the ring-order
// drain and completion read instead of a per-message slot index.  The slot
// index `sidx` is written only where a consumer needs it: every message with
// `all_sidx` (the message-order drain, tune mbox_drain_msg=1), and the whole
// tile when some message of it spilled (the drain runs that tile in message
// order).  (An opt-in LDS-staged write-out in ring order measured slower,
// 117 -> 161 us per 8 Mi msgs: the 80 KB stage halved the resident blocks;
// removed, see git history 4c4ea76.)
__host__ __device__ constexpr size_t scatter_lds_bytes(uint32_t S) { return (size_t)S * (16 + 4 * (kST / kWave)); }

template <bool A2, bool MC>
__global__ __launch_bounds__(kST) void mbx_scatter_kernel(SortIn in, MboxView mv, const uint32_t* __restrict__ hist,
                                                          const uint32_t* __restrict__ gsum,
                                                          uint32_t* __restrict__ rw,
                                                          uint32_t* __restrict__ sidx, uint32_t* __restrict__ tinfo,
                                                          ReplyView rv, bool spill, bool all_sidx) {
  // LDS sized by the shard count (16 + 4 * waves B per shard): occupancy is not
  // capped by the 1024-shard maximum
  extern __shared__ __align__(16) unsigned char smem_sc[];
  const uint32_t S = 1u << mv.log_s;
  unsigned long long* base = reinterpret_cast<unsigned long long*>(smem_sc);  // ring position of offset 0 (tail)
  uint32_t* run = reinterpret_cast<uint32_t*>(base + S);  // this block's next offset per shard
  uint32_t* room = run + S;                               // offset limit (free ring slots)
  uint32_t* wcnt_all = room + S;                          // [kST / kWave][S] per-wave counts -> wave offsets
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
      sh[k] = mb[k] & (S - 1);
      const uint64_t peers = match_bits(sh[k], mv.log_s, __ballot(ok));
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
    int sp = 0;
    for (uint32_t s = threadIdx.x; s < S; s += kST) {  // wave offsets in message order, then the block's run
      uint32_t rr = run[s];
#pragma unroll
      for (int ww = 0; ww < kST / kWave; ++ww) {
        const uint32_t c = wcnt(ww, s);
        wcnt(ww, s) = rr;
        rr += c;
      }
      run[s] = rr;
      sp |= rr > room[s];
    }
    bool tile_spill = false;  // (either barrier publishes the wave offsets too)
    if (spill) tile_spill = __syncthreads_or(sp) != 0;
    else __syncthreads();
    const bool wsidx = all_sidx || tile_spill;
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const int64_t i = tile_index(t, k);
      if (i >= in.M) continue;
      const uint32_t origin = in.origin_base + (uint32_t)i;
      if (mb[k] == kNoSlot) {
        ++n_miss;
        if (wsidx) sidx[i] = kNoSlot;
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
        if (wsidx) sidx[i] = kNoSlot;
        write_status(rv, origin, kStatusOverflow);
        continue;
      }
      const int64_t x0 = v0[k], x1 = v1[k], x2 = v2[k];
      const uint32_t mt = meth[k];
      const uint64_t slot = slot_at(mv, sh[k], base[sh[k]] + off);
      if (wsidx) sidx[i] = (uint32_t)slot;
      if (mt < 128u && fits_i32(x0) && fits_i32(x1) && x2 == 0) {
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
    if (tinfo) {  // the tile's runs (after the stores: the messages' registers are dead by now -- +25 VGPRs above)
      // slot bias from the epoch-start tail (a drain may commit before the completion reads it)
      for (uint32_t s = threadIdx.x; s < S; s += kST) {
        const uint32_t r0 = wcnt(0, s), rr = run[s];  // wave 0's offset = the run before this tile
        const uint32_t cc = r0 >= room[s] ? 0u : min(rr - r0, room[s] - r0);
        tinfo[(size_t)t * 2 * S + s] = (uint32_t)(base[s] + r0) + shard_rot(mv, s);
        tinfo[(size_t)t * 2 * S + S + s] = cc | (rr > room[s] ? kRunSpilled : 0u);
      }
    }
    __syncthreads();  // wcnt rows are reused by the next tile
  }
  block_add_stats(mv.stats, n_enq, kMbEnqueued, n_ovf, kMbOverflow, n_miss, kMbNoActor);
  if (spill) {
    __syncthreads();  // block_add_stats' LDS partials are reused
    block_add_stats(mv.stats, n_spill, kMbSpilled, 0, -1, 0, -1);
  }
}

// ---------------------------------------------------------------- K2s one pass: resolve + look-back + scatter
// The count and scatter passes as ONE kernel (a single-pass counting sort with
// decoupled look-back): each block claims the next tile in launch order (a tile
// counter, so every earlier tile's block is already running), resolves its
// messages through the route directory ONCE (the gather is the expensive part:
// 8 Mi random 4-B lookups cost ~27 us of L2 request rate on MI355X,
// tools/gather_probe.hip), ranks them per shard in message order (wave match),
// publishes its per-shard counts, and finds its offset in each shard's epoch run
// by looking back over earlier tiles' descriptors until one carries an
// inclusive prefix.  Descriptors are u64 {epoch tag 24 | status 2 | value 38},
// published and read with memory-side atomics (the per-XCD L2s are not coherent
// within a kernel); the tag (from a device word the drain advances) makes a
// previous Send's descriptors invalid without clearing them, graph replays
// included.  The last tile leaves each shard's epoch total in gsum[0][s] for the
// drains' commit.  The batch's inputs are read once and the route words never
// leave registers (the two-pass form wrote and re-read 4 B per message).
__host__ __device__ constexpr size_t onesweep_lds_bytes(uint32_t S) { return (size_t)S * (8 + 4 + 4 + 4 * (kST / kWave)); }

template <bool A2, bool MC, int SK = kSK>
__device__ __forceinline__ void load_cols(const SortIn& in, uint32_t t, int64_t (&v0)[SK], int64_t (&v1)[SK],
                                          int64_t (&v2)[SK], uint32_t (&meth)[SK]) {
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int64_t i = tile_index<SK>(t, k);
    const bool ok = i < in.M;
    v0[k] = ok ? __builtin_nontemporal_load(in.a0 + i) : 0;
    v1[k] = ok && in.a1 ? __builtin_nontemporal_load(in.a1 + i) : 0;
    v2[k] = 0;
    if constexpr (A2) v2[k] = ok ? __builtin_nontemporal_load(in.a2 + i) : 0;
    meth[k] = in.method_uniform;
    if constexpr (MC) meth[k] = ok ? (uint32_t)in.mcol[i] : 0u;
  }
}

__device__ __forceinline__ uint32_t bitlen64(uint64_t x) { return x ? 64u - (uint32_t)__clzll(x) : 0u; }
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
  return v;
}

// The next Send's 8-B field widths from this Send's per-tile bit lengths (the last
// block, after every tile's maxima are out): each field as wide as its largest
// value, the slack of the 52 bits split between the arguments.  Fields that no
// longer fit set bit 31 (the host then keeps 16-B records).
__device__ __forceinline__ void rec8_next_from(const uint32_t* r8max, uint32_t* r8w, uint32_t* host, uint32_t tiles);
__device__ __forceinline__ void rec8_next(const SortIn& in, uint32_t* r8w, uint32_t* host, uint32_t tiles) {
  rec8_next_from(in.r8max, r8w, host, tiles);
}
__device__ __forceinline__ void rec8_next_from(const uint32_t* r8max, uint32_t* r8w, uint32_t* host, uint32_t tiles) {
  __shared__ uint32_t mx[3];
  if (threadIdx.x < 3) mx[threadIdx.x] = 0;
  __syncthreads();
  uint32_t bm = 0, b0 = 0, b1 = 0;
  for (uint32_t t = threadIdx.x; t < tiles; t += blockDim.x) {
    const uint32_t x = __hip_atomic_fetch_add(const_cast<uint32_t*>(r8max) + t, 0u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    bm = max(bm, x & 0xffu), b0 = max(b0, (x >> 8) & 0xffu), b1 = max(b1, (x >> 16) & 0xffu);
  }
  bm = wave_max_u32(bm), b0 = wave_max_u32(b0), b1 = wave_max_u32(b1);
  if (lane_id() == 0) {
    atomicMax(&mx[0], bm);
    atomicMax(&mx[1], b0);
    atomicMax(&mx[2], b1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t wm = max(mx[0], 1u), n0 = max(mx[1], 1u), n1 = max(mx[2], 1u);
    uint32_t w = 0;
    if (wm <= 24 && wm + n0 + n1 <= 52) {
      const uint32_t w0 = n0 + (52 - wm - n0 - n1) / 2;
      w = wm | (w0 << 8) | ((52 - wm - w0) << 16);
    } else {
      const uint32_t wmc = min(wm, 24u), w0 = (52 - wmc) / 2;
      w = wmc | (w0 << 8) | ((52 - wmc - w0) << 16) | 0x80000000u;
    }
    *r8w = w;
    if (host) __hip_atomic_store(host, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Route mode 4 (world-1 stateless Sends on a directory of up to kPresMax ids): the
// directory's rank bytes folded into 2 bits per id for this rank -- 1 here, 2 probe the
// hash table (a rank past 253), 0 anything else -- so a sort block stages the whole map
// in LDS (32 KB for 131072 ids) and resolves each message with an LDS read instead of a
// scattered global gather: 64 lanes gathering from 64 lines kept the sort's address unit
// stalled by the texture cache half its busy time (profiles/r6_pmc_head.txt).
constexpr uint32_t kPresMax = 1u << 18;  // ids (64 KB of map)
__host__ __device__ constexpr uint32_t pres_words(uint32_t n_dir) { return ((n_dir + 15) / 16 + 3) & ~3u; }
template <int = 0>
__global__ __launch_bounds__(256) void mbx_presence_kernel(const uint8_t* __restrict__ dirr, uint32_t n_dir,
                                                           int rank_self, uint32_t* __restrict__ pres) {
  const uint32_t wi = blockIdx.x * 256u + threadIdx.x;
  if (wi >= pres_words(n_dir)) return;
  alignas(16) uint8_t b[16];
  if (wi * 16 + 16 <= n_dir) {  // (the table is a whole allocation: 16-B aligned)
    *reinterpret_cast<uint4*>(b) = *reinterpret_cast<const uint4*>(dirr + (size_t)wi * 16);
  } else {
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) b[j] = wi * 16 + j < n_dir ? dirr[wi * 16 + j] : kRankMissing;
  }
  uint32_t w = 0;
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const uint32_t st = b[j] == (uint8_t)rank_self ? 1u : b[j] == kRankFallback ? 2u : 0u;
    w |= st << (2 * j);
  }
  pres[wi] = w;
}
__device__ __forceinline__ void stage_pres(const SortIn& in, uint32_t* lpres) {
  const uint32_t nw = pres_words(in.n_dir);
  for (uint32_t w = threadIdx.x * 4; w < nw; w += blockDim.x * 4)
    *reinterpret_cast<uint4*>(lpres + w) = *reinterpret_cast<const uint4*>(in.pres + w);
}
template <int SK>
__device__ __forceinline__ void resolve_pres(const SortIn& in, const uint32_t* lpres, const uint32_t (&a)[SK],
                                             int (&r)[SK], uint32_t (&mb)[SK]) {
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    mb[k] = a[k];
    if (a[k] < in.n_dir) {
      const uint32_t st = (lpres[a[k] >> 4] >> ((a[k] & 15) * 2)) & 3u;
      r[k] = st == 1 ? in.rank_self : -1;
      if (st == 2) lookup_entry(in.table, in.mask, actor_key(a[k]), r[k], mb[k]);
    } else if (a[k] != 0xffffffffu) {
      lookup_entry(in.table, in.mask, actor_key(a[k]), r[k], mb[k]);
    } else {
      r[k] = -1;
    }
  }
}

// One tile of the one-pass sort (the block claims it); returns its index.
//
// reserve (stateless batches): no look-back.  A stateless record runs on its
// own, so a ring need not hold its messages in message order -- only each
// tile's run in message order (the drains read a tile's runs through tinfo).
// The tile is the block's index and each shard's run is reserved with ONE
// atomicAdd on the shard's epoch counter (gsum row 0, which then holds the
// epoch's total): 16 device-scope atomics per tile, ~2048 per counter at 8 Mi
// messages -- against a look-back whose walk grows with the tiles in flight
// (each hop a memory-side round trip).
template <int MODE, bool A2, bool MC, int SK = kSK>
__device__ __forceinline__ uint32_t onesweep_tile(const SortIn& in, const MboxView& mv, unsigned long long* __restrict__ desc,
                                                  unsigned* __restrict__ tctr, uint32_t* __restrict__ gsum,
                                                  uint32_t* __restrict__ sidx, uint32_t* __restrict__ tinfo,
                                                  uint32_t* __restrict__ rw, const ReplyView& rv, bool spill,
                                                  bool all_sidx, unsigned char* smem_os, bool reserve = false) {
  const uint32_t S = 1u << mv.log_s;
  unsigned long long* base = reinterpret_cast<unsigned long long*>(smem_os);  // ring position of this tile's run (tail + prefix)
  uint32_t* room = reinterpret_cast<uint32_t*>(base + S);                     // offset limit past the tail
  uint32_t* pre = room + S;                                                   // the tile's prefix per shard
  uint32_t* wcnt_all = pre + S;                                               // [kST / kWave][S]
  auto wcnt = [&](unsigned ww, uint32_t sh) -> uint32_t& { return wcnt_all[ww * S + sh]; };
  __shared__ uint32_t tile_s;
  __shared__ uint32_t tmax[3];  // (in.rec8) the tile's field bit lengths
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  if (threadIdx.x < 3) tmax[threadIdx.x] = 0;  // (ordered before use by the tile's first barrier)
  // this Send's epoch tag, 1..0xffffff (the drain advances tctr[1]; the modulus keeps the tag inside the
  // descriptor's 24-bit field across the counter's wrap -- tag 0 is reserved for never-published words)
  const uint32_t tag = epoch_tag(tctr[1]);
  if (threadIdx.x == 0 && !reserve) {
    const uint32_t t = atomicAdd(&tctr[0], 1u);
    if (t == in.tiles - 1) atomicExch(&tctr[0], 0u);  // every block has claimed: ready for the next Send
    tile_s = t;
  }
  for (uint32_t s = lane; s < S; s += kWave) wcnt(w, s) = 0;
  uint32_t* lpres = reinterpret_cast<uint32_t*>(smem_os + ((onesweep_lds_bytes(S) + 15) & ~(size_t)15));
  if constexpr (MODE == 4) stage_pres(in, lpres);  // (the map, behind the barrier below)
  __syncthreads();
  // (reserve: tiles dealt XCD by XCD, as the ring drain deals them -- its reads of a tile's runs then
  // meet the lines in the L2 that took the sort's stores)
  const uint32_t t = reserve ? virt_block(blockIdx.x, gridDim.x) : tile_s;
  // the tile's columns: actors, then the arguments in flight across the gathers and the ranking
  uint32_t a[SK], mb[SK], meth[SK];
  int64_t v0[SK], v1[SK], v2[SK];
  int r[SK];
  load_actors<SK>(in, t, a);
  load_cols<A2, MC, SK>(in, t, v0, v1, v2, meth);
  if constexpr (MODE == 4) resolve_pres<SK>(in, lpres, a, r, mb);
  else resolve_k<MODE, SK>(in, a, r, mb);
  uint32_t wr[SK];
  // (an ordered batch in 8-B records, !spill: a message whose fields do not fit takes its
  // ring position like any other and is written as an escape record below -- FIFO kept)
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const bool ok = tile_index<SK>(t, k) < in.M && r[k] == in.rank_self && mb[k] < kMaxMbox;
    if (!ok) mb[k] = kNoSlot;
    const uint32_t sh = mb[k] & (S - 1);
    const uint64_t peers = match_bits(sh, mv.log_s, __ballot(ok));
    const unsigned below = mbcnt64(peers);
    const int leader = peers ? __builtin_ctzll(peers) : 0;
    unsigned old = 0;
    if (ok && below == 0) {
      old = wcnt(w, sh);
      wcnt(w, sh) = old + (unsigned)__popcll(peers);
    }
    wr[k] = (unsigned)__shfl((int)old, leader) + below;
  }
  __syncthreads();
  // per shard: wave offsets within the tile, publish the tile's count, look back for its prefix
  const uint64_t Q = 1ull << mv.log_q;
  unsigned long long timeouts = 0;
  int sp = 0;
  for (uint32_t s = threadIdx.x; s < S; s += kST) {
    uint32_t c = 0;
    uint64_t excl = 0;
    unsigned long long* d = desc + (size_t)t * S + s;
#pragma unroll
    for (int ww = 0; ww < kST / kWave; ++ww) {
      const uint32_t x = wcnt(ww, s);
      wcnt(ww, s) = c;
      c += x;
    }
    if (reserve) {
      excl = c ? atomicAdd(&mv.resv[s * kResvStride], c) : 0u;  // this tile's run of shard s
    } else if (t == 0) {
      __hip_atomic_exchange(d, desc_word(tag, kDescP, c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_exchange(d, desc_word(tag, kDescA, c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      excl = lookback(desc + s, S, (int64_t)t - 1, tag, timeouts);
      __hip_atomic_exchange(d, desc_word(tag, kDescP, excl + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!reserve && t == in.tiles - 1) gsum[s] = (uint32_t)(excl + c);  // the epoch's total of shard s
    const uint64_t tl = *ctr_tail(mv, s), hd = *ctr_head(mv, s);
    const uint64_t free = hd + Q > tl ? hd + Q - tl : 0;
    const uint32_t rm = (uint32_t)(free < 0xffffffffull ? free : 0xffffffffull);
    base[s] = tl;
    room[s] = rm;
    pre[s] = (uint32_t)excl;
    sp |= excl + c > rm;
    if (tinfo) {
      const uint32_t cc = excl >= rm ? 0u : (uint32_t)min((uint64_t)c, rm - excl);
      tinfo[(size_t)t * 2 * S + s] = (uint32_t)(tl + excl) + shard_rot(mv, s);
      tinfo[(size_t)t * 2 * S + S + s] = cc | (excl + c > rm ? kRunSpilled : 0u);
    }
  }
  // (in.rec8) the messages whose fields do not fit an 8-B record -- they spill -- and
  // the tile's fields OR-ed (their bit lengths size the next Send's records)
  uint32_t escm = 0;
  const uint32_t w8 = in.rec8 ? *in.r8w : 0u;  // this Send's 8-B field widths (recw: none, nothing escapes)
  uint64_t or_m = 0, or_0 = 0, or_1 = 0;
  const bool maxima = in.rec8 || in.recw;  // (wide pure records keep the maxima: back to 8 B once they fit)
  if (maxima) {
    const uint32_t wm = w8 & 0xffu, w0 = (w8 >> 8) & 0xffu, w1 = (w8 >> 16) & 0xffu;
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      if (mb[k] == kNoSlot) continue;
      const uint64_t z0 = ((uint64_t)v0[k] << 1) ^ (uint64_t)(v0[k] >> 63);
      const uint64_t z1 = ((uint64_t)v1[k] << 1) ^ (uint64_t)(v1[k] >> 63);
      or_m |= mb[k], or_0 |= z0, or_1 |= z1;
      if (in.rec8 && ((mb[k] >> wm) != 0 || (z0 >> w0) != 0 || (z1 >> w1) != 0)) escm |= 1u << k;
    }
  }
  sp |= escm != 0;
  if (maxima) {  // the tile's field bit lengths (read by thread 0 past the spill barrier)
    const uint32_t bm = wave_max_u32(bitlen64(or_m)), b0 = wave_max_u32(bitlen64(or_0)),
                   b1 = wave_max_u32(bitlen64(or_1));
    if (lane == 0) {
      atomicMax(&tmax[0], bm);
      atomicMax(&tmax[1], b0);
      atomicMax(&tmax[2], b1);
    }
  }
  bool tile_spill = false;
  if (spill) tile_spill = __syncthreads_or(sp) != 0;
  else __syncthreads();
  // a tile spilled by its records' widths (no run overran its ring): flag one of its
  // runs, so the drains take the tile in message order through the slot indices
  // (the thread that wrote shard 0's count word: program order)
  if (tile_spill && tinfo && threadIdx.x == 0) tinfo[(size_t)t * 2 * S + S] |= kRunSpilled;
  const bool wsidx = all_sidx || tile_spill;
  unsigned long long n_enq = 0, n_ovf = 0, n_miss = 0, n_spill = 0;
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int64_t i = tile_index<SK>(t, k);
    if (i >= in.M) continue;
    const uint32_t origin = in.origin_base + (uint32_t)i;
    if (mb[k] == kNoSlot) {
      ++n_miss;
      if (wsidx) sidx[i] = kNoSlot;
      write_status(rv, origin, kStatusNoActor);
      continue;
    }
    const uint32_t sh = mb[k] & (S - 1);
    const uint32_t off = pre[sh] + wcnt(w, sh) + wr[k];
    const bool esc = (escm >> k) & 1u;  // the record would not fit 8 B
    if (off >= room[sh] || (esc && spill)) {  // the ring is full (or a stateless record spills)
      if (spill) {  // the drain runs it from the batch: its route word is all it needs from here
        ++n_spill;
        sidx[i] = kSpillSlot;
        rw[i] = mb[k];
        continue;
      }
      ++n_ovf;
      if (wsidx) sidx[i] = kNoSlot;
      write_status(rv, origin, kStatusOverflow);
      continue;
    }
    const uint64_t slot = slot_at(mv, sh, base[sh] + off);
    if (wsidx) sidx[i] = (uint32_t)slot;
    const uint32_t mt = meth[k];
    if (in.recw) {  // wide pure record: {a0, a1} whole, the place in the tile beside it
      *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
          u32x4{(uint32_t)v0[k], (uint32_t)((uint64_t)v0[k] >> 32), (uint32_t)v1[k], (uint32_t)((uint64_t)v1[k] >> 32)};
      rec_place(mv)[slot] = (uint16_t)(i & ((kST * SK) - 1));
    } else if (in.rec8 && esc) {  // (ordered) escape: the place in the tile + bit 63, the fields aside
      reinterpret_cast<uint64_t*>(mv.rec)[slot] = (uint64_t)(i & ((kST * SK) - 1)) | (1ull << 63);
      *reinterpret_cast<u32x4*>(in.r8esc + 2 * slot) =
          u32x4{(uint32_t)v0[k], (uint32_t)((uint64_t)v0[k] >> 32), mb[k], 0u};
    } else if (in.rec8) {  // 8-B record (uniform method; stateless records that do not fit spilled above)
      const uint32_t wm = w8 & 0xffu, w0 = (w8 >> 8) & 0xffu;
      const uint64_t z0 = ((uint64_t)v0[k] << 1) ^ (uint64_t)(v0[k] >> 63);
      const uint64_t z1 = ((uint64_t)v1[k] << 1) ^ (uint64_t)(v1[k] >> 63);
      reinterpret_cast<uint64_t*>(mv.rec)[slot] =
          (uint64_t)(i & ((kST * SK) - 1)) | ((uint64_t)mb[k] << 12) | (z0 << (12 + wm)) | (z1 << (12 + wm + w0));
    } else if (mt < 128u && fits_i32(v0[k]) && fits_i32(v1[k]) && v2[k] == 0) {
      *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
          u32x4{origin | kCompactMark, mb[k] | (mt << 24), (uint32_t)v0[k], (uint32_t)v1[k]};
    } else {
      const uint32_t fl = v2[k] != 0 ? (uint32_t)kFlagA2 : 0u;
      *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
          u32x4{origin | kCompactMark, mb[k] | kCompactLong, (mt & 0xffffu) | (fl << 16), 0u};
      *reinterpret_cast<u32x4*>(rec_b(mv, slot)) =
          u32x4{(uint32_t)v0[k], (uint32_t)((uint64_t)v0[k] >> 32), (uint32_t)v1[k], (uint32_t)((uint64_t)v1[k] >> 32)};
      if (fl) mv.a2[slot] = v2[k];
    }
    ++n_enq;
  }
  // the tile's field bit lengths, for the next Send's widths (rec8_next): a memory-side write
  // (the fused kernel's last block reads it within the launch: its ticket follows a vmcnt(0) wait)
  if (maxima && threadIdx.x == 0) (void)atomicExch(&in.r8max[t], tmax[0] | (tmax[1] << 8) | (tmax[2] << 16));
  block_add_stats(mv.stats, n_enq, kMbEnqueued, n_ovf, kMbOverflow, n_miss, kMbNoActor);
  __syncthreads();  // block_add_stats' LDS partials are reused
  block_add_stats(mv.stats, n_spill, kMbSpilled, timeouts, kMbLookback, 0, -1);
  return t;
}

template <int MODE, bool A2, bool MC>
__global__ __launch_bounds__(kST) void mbx_onesweep_kernel(SortIn in, MboxView mv, unsigned long long* __restrict__ desc,
                                                           unsigned* __restrict__ tctr, uint32_t* __restrict__ gsum,
                                                           uint32_t* __restrict__ sidx, uint32_t* __restrict__ tinfo,
                                                           uint32_t* __restrict__ rw, ReplyView rv, bool spill,
                                                           bool all_sidx, bool reserve) {
  extern __shared__ __align__(16) unsigned char smem_os[];
  (void)onesweep_tile<MODE, A2, MC>(in, mv, desc, tctr, gsum, sidx, tinfo, rw, rv, spill, all_sidx, smem_os, reserve);
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

// An 8-B record (in.rec8) of the tile whose first message is `tile_origin`.
template <bool FRESH, int SK = kSK>
__device__ __forceinline__ SortRec decode_rec8(uint64_t r, const SortIn& in, uint32_t w8, uint32_t tile_origin) {
  const uint32_t wm = w8 & 0xffu, w0 = (w8 >> 8) & 0xffu, w1 = (w8 >> 16) & 0xffu;
  const uint64_t m0 = (1ull << w0) - 1;
  SortRec x;
  x.valid = true;
  x.origin = tile_origin + (uint32_t)(r & ((kST * SK) - 1));
  x.mb = (uint32_t)((r >> 12) & ((1ull << wm) - 1));
  x.method = in.method_uniform;
  x.flags = 0;
  x.a2 = 0;
  const uint64_t z0 = (r >> (12 + wm)) & m0, z1 = (r >> (12 + wm + w0)) & ((1ull << w1) - 1);
  x.a0 = (int64_t)(z0 >> 1) ^ -(int64_t)(z0 & 1);
  x.a1 = (int64_t)(z1 >> 1) ^ -(int64_t)(z1 & 1);
  return x;
}

// A wide pure record (in.recw): no mailbox -- its method reads none.
__device__ __forceinline__ SortRec decode_wide(const u32x4& h, const SortIn& in, uint32_t origin) {
  SortRec x;
  x.valid = true;
  x.origin = origin;
  x.mb = 0;
  x.method = in.method_uniform;
  x.flags = 0;
  x.a0 = (int64_t)(((uint64_t)h.y << 32) | h.x);
  x.a1 = (int64_t)(((uint64_t)h.w << 32) | h.z);
  x.a2 = 0;
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

// The epoch's total of shard s, cleared for the next Send: the reservation counter of
// a one-pass stateless Send (memory-side, as its tiles added to it), else the group sums.
__device__ __forceinline__ uint32_t epoch_sum(const MboxView& mv, uint32_t* gsum, uint32_t ngroups, uint32_t S,
                                              uint32_t s) {
  return mv.resv ? atomicExch(&mv.resv[s * kResvStride], 0u) : epoch_total(gsum, ngroups, S, s, true);
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
// Batches without ordered methods: every record runs on its own.
//
// Ring-order form (default): one block per tile.  The tile's records sit in S
// runs (the scatter's tinfo); the block reads them in RING order -- consecutive
// lanes take consecutive ring slots, so the loads are whole-line runs -- runs
// each handler, stages the reply in LDS at the message's place in the tile
// (origin), and writes the tile's replies out coalesced.  Replaces the
// message-order form's slot-index read (4 B per message) and its 16-B gather per
// message (one line per lane).
//
// Message-order form (tune mbox_drain_msg=1, and any tile with a spilled
// message): each message's record is taken from the ring slot the scatter
// recorded, replies coalesced; a spilled message runs straight from the batch.
//
// The last block commits every shard (and clears the group sums).
// RF: the record form -- 0 compact / long (16 / 32 B), 1 the 8-B record, 2 the wide
// pure record (16 B {a0, a1} + the u16 place)
template <int FIXED, bool FRESH = false, int RF = 0, int SK = kSK>
__device__ __forceinline__ void drain_tile_msg(MboxView mv, SortIn in, uint32_t t,
                                               const uint32_t* __restrict__ sidx, const uint32_t* __restrict__ rw,
                                               int64_t* __restrict__ state, uint32_t n_state, uint64_t delay_ticks,
                                               OutboxView ob, ReplyView rv, unsigned long long& done,
                                               unsigned long long& failed, unsigned long long& holes) {
  uint32_t sl[SK];
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int64_t i = tile_index<SK>(t, k);
    sl[k] = i < in.M ? __builtin_nontemporal_load(sidx + i) : kNoSlot;
  }
  using RecT = typename std::conditional<RF == 1, uint64_t, u32x4>::type;  // the ring record as loaded
  const uint32_t w8 = RF == 1 ? *in.r8w : 0u;  // the 8-B field widths this Send's sort used
  RecT ha[SK];
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    if constexpr (RF == 1) {
      const uint64_t* rp = reinterpret_cast<const uint64_t*>(mv.rec) + (sl[k] < kSpillSlot ? sl[k] : 0);
      ha[k] = sl[k] < kSpillSlot ? (FRESH ? __builtin_nontemporal_load(rp) : *rp) : 0ull;
    } else {
      const u32x4* rp = reinterpret_cast<const u32x4*>(rec_a(mv, sl[k] < kSpillSlot ? sl[k] : 0));
      ha[k] = sl[k] < kSpillSlot ? (FRESH ? __builtin_nontemporal_load(rp) : *rp) : u32x4{0u, 0u, 0u, 0u};
    }
  }
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    if (sl[k] == kNoSlot) continue;  // answered by the scatter (no actor / ring full)
    SortRec x;
    if (sl[k] == kSpillSlot) {  // its ring was full: the message runs straight from the batch
      const int64_t i = tile_index<SK>(t, k);
      x.valid = true;
      x.mb = rw[i];
      x.method = in.mcol ? (uint32_t)in.mcol[i] : in.method_uniform;
      x.flags = 0;
      x.a0 = in.a0[i];
      x.a1 = in.a1 ? in.a1[i] : 0;
      x.a2 = in.a2 ? in.a2[i] : 0;
    } else if constexpr (RF == 1) {
      x = decode_rec8<FRESH, SK>(ha[k], in, w8, in.origin_base + t * (kST * SK));
    } else if constexpr (RF == 2) {
      x = decode_wide(ha[k], in, 0u);
    } else {
      u32x4 hb = {0u, 0u, 0u, 0u};
      int64_t a2v = 0;
      if (rec_is_long(ha[k])) {
        const u32x4* bp = reinterpret_cast<const u32x4*>(rec_b(mv, sl[k]));
        hb = FRESH ? __builtin_nontemporal_load(bp) : *bp;
        if (((ha[k].z >> 16) & kFlagA2) && mv.a2) a2v = FRESH ? __builtin_nontemporal_load(mv.a2 + sl[k]) : mv.a2[sl[k]];
      }
      x = decode_sorted(ha[k], hb, a2v);
    }
    const uint32_t origin = in.origin_base + (uint32_t)tile_index<SK>(t, k);
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

template <int FIXED>
__global__ __launch_bounds__(kST) void mbx_drain_msg_kernel(MboxView mv, SortIn in, const uint32_t* __restrict__ sidx,
                                                            const uint32_t* __restrict__ rw,
                                                            int64_t* __restrict__ state, uint32_t n_state,
                                                            uint64_t delay_ticks, OutboxView ob, ReplyView rv,
                                                            uint32_t* __restrict__ gsum, uint32_t ngroups,
                                                            unsigned* __restrict__ ticket, unsigned* __restrict__ tctr) {
  // the scatter's block -> tile ranges: a tile's records sit in ~S short runs that
  // this block's waves read whole (line reuse in L1 / L2), not one record per block
  unsigned long long done = 0, failed = 0, holes = 0;
  const uint32_t v = virt_block(blockIdx.x, in.G);
  const uint32_t t0 = v * in.tpb, t1 = min(t0 + in.tpb, in.tiles);
  for (uint32_t t = t0; t < t1; ++t)
    drain_tile_msg<FIXED>(mv, in, t, sidx, rw, state, n_state, delay_ticks, ob, rv, done, failed, holes);
  block_add_stats(mv.stats, done, kMbProcessed, failed, kMbFailed, holes, kMbHoles);
  __shared__ bool last;
  if (threadIdx.x == 0) last = last_block_ticket(ticket);
  __syncthreads();
  if (last) {  // every block's records are read: the rings are consumed
    const uint32_t S = 1u << mv.log_s;
    for (uint32_t s = threadIdx.x; s < S; s += kST) epoch_commit(mv, s, epoch_sum(mv, gsum, ngroups, S, s));
    if (threadIdx.x == 0) tctr[1] += 1u;  // the next Send's one-pass epoch tag
  }
}

// Tile t's runs in LDS: per shard the slot bias (ring slot of run entry j =
// shard base | ((bias + j) & (Q - 1))) and an owner table (run entry j of the
// tile -> its shard), j in [0, total).  Entries past a shard's free room (an
// ordered batch's overflow: never written) are left out (the scatter clamped the
// counts).  Returns the total; `spill` is set when a run overflowed the room (a
// stateless tile's spill).
template <typename OwnT>
struct RunLds {
  uint32_t* bias;  // [S]
  uint32_t* excl;  // [S] exclusive prefix of the (clamped) counts
  OwnT* owner;     // [kSTile]: u8 for up to 256 shards, else u16
};

template <typename OwnT>
__device__ __forceinline__ uint32_t load_tile_runs(const MboxView& mv, const uint32_t* __restrict__ tinfo, uint32_t t,
                                                   const RunLds<OwnT>& L, int& spill) {
  __shared__ uint32_t wsum[kST / kWave];
  __shared__ uint32_t total_s;
  const uint32_t S = 1u << mv.log_s;
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  // thread j owns the shards [j * per, (j + 1) * per): a contiguous scan
  const uint32_t per = (S + kST - 1) / kST, s0 = threadIdx.x * per, s1 = min(S, s0 + per);
  uint32_t cnt[2] = {0u, 0u};  // per <= 2 (S <= 1024)
  uint32_t mine = 0;
  int sp = 0;
  for (uint32_t s = s0, q = 0; s < s1; ++s, ++q) {
    const uint32_t cw = tinfo[(size_t)t * 2 * S + S + s];
    sp |= (cw & kRunSpilled) != 0;
    cnt[q] = cw & ~kRunSpilled;
    mine += cnt[q];
    L.bias[s] = tinfo[(size_t)t * 2 * S + s];
  }
  const uint32_t incl = wave_incl_scan(mine);
  if (lane == kWave - 1) wsum[w] = incl;
  spill = __syncthreads_or(sp);
  uint32_t acc = incl - mine;
  for (unsigned ww = 0; ww < w; ++ww) acc += wsum[ww];
  if (threadIdx.x == kST - 1) total_s = acc + mine;
  for (uint32_t s = s0, q = 0; s < s1; ++s, ++q) {
    L.excl[s] = acc;
    L.bias[s] -= acc;
    for (uint32_t j = acc; j < acc + cnt[q]; ++j) L.owner[j] = (OwnT)s;
    acc += cnt[q];
  }
  __syncthreads();
  return total_s;
}

constexpr uint8_t kAbsent = 0xff;  // staged status: no record of this message in the tile's runs
// NARROW (S <= 256): a 1-B owner table whose bytes are reused for the staged
// statuses once the records are loaded -- 36 KB of LDS instead of 46 KB, four
// blocks per CU (with at most 64 VGPRs: launch bounds 8 waves per SIMD)
__host__ __device__ constexpr size_t ring_drain_lds_bytes(uint32_t S, size_t tile = kSTile) {
  return S <= 256 ? tile * (8 + 1) + (size_t)S * 8 : tile * (8 + 2 + 1) + (size_t)S * 8;
}

// Tile t's records, read in RING order from its runs (tinfo), each through the
// handler table; replies staged in LDS at their place in the tile and written
// out coalesced.  FRESH: the records were written by other waves of THIS block
// in this kernel (the fused sort + drain) -- loaded non-temporal (L1 bypassed:
// served by the XCD's L2, which holds the stores; a line another block of the
// CU cached earlier would be stale in L1).
struct DrainCounts {
  unsigned long long done = 0, failed = 0, holes = 0;
};

// (views and counts by value: references to a kernel's locals or arguments put
// them in scratch)
template <int FIXED, bool NARROW, bool FRESH, int RF = 0, int SK = kSK>
__device__ __forceinline__ DrainCounts drain_ring_tile(MboxView mv, SortIn in, uint32_t t,
                                                       const uint32_t* __restrict__ tinfo,
                                                       const uint32_t* __restrict__ sidx,
                                                       const uint32_t* __restrict__ rw, int64_t* __restrict__ state,
                                                       uint32_t n_state, uint64_t delay_ticks, OutboxView ob,
                                                       ReplyView rv, unsigned char* smem_rd) {
  unsigned long long done = 0, failed = 0, holes = 0;
  using OwnT = typename std::conditional<NARROW, uint8_t, uint16_t>::type;
  const uint32_t S = 1u << mv.log_s;
  int64_t* sval = reinterpret_cast<int64_t*>(smem_rd);  // [(kST * SK)] reply values by place in the tile
  RunLds<OwnT> L;
  L.bias = reinterpret_cast<uint32_t*>(sval + (kST * SK));
  L.excl = L.bias + S;
  L.owner = reinterpret_cast<OwnT*>(L.excl + S);
  // [(kST * SK)] statuses, kAbsent = none (NARROW: the owner table's bytes, once the records are loaded)
  uint8_t* sst = NARROW ? reinterpret_cast<uint8_t*>(L.owner) : reinterpret_cast<uint8_t*>(L.owner + (kST * SK));
  const uint64_t i0 = (uint64_t)t * (kST * SK);
  const uint32_t n_t = (uint32_t)min((uint64_t)(kST * SK), (uint64_t)in.M - i0);
  if constexpr (!NARROW)
    for (uint32_t j = threadIdx.x; j < (kST * SK); j += kST) sst[j] = kAbsent;
  int spill = 0;
  const uint32_t T = load_tile_runs(mv, tinfo, t, L, spill);
  if (spill) {  // some message of the tile spilled: the scatter left the tile's slot indices
    drain_tile_msg<FIXED, FRESH, RF, SK>(mv, in, t, sidx, rw, state, n_state, delay_ticks, ob, rv, done, failed, holes);
    return DrainCounts{done, failed, holes};
  }
  const uint64_t sbase_mask = (1ull << mv.log_q) - 1;
  using RecT = typename std::conditional<RF == 1, uint64_t, u32x4>::type;  // the ring record as loaded
  const uint32_t w8 = RF == 1 ? *in.r8w : 0u;  // the 8-B field widths this Send's sort used
  RecT ha[SK];
  uint32_t sl[SK];
  uint16_t pl[SK];  // (RF 2) the places in the tile
#pragma unroll
  for (int k = 0; k < SK; ++k) {  // ring order: lane-consecutive entries of the runs
    const uint32_t j = (uint32_t)k * kST + threadIdx.x;
    sl[k] = kNoSlot;
    if (j < T) {
      const uint32_t s = L.owner[j];
      sl[k] = (uint32_t)(((uint64_t)s << mv.log_q) | ((L.bias[s] + j) & sbase_mask));
      if constexpr (RF == 1) {
        const uint64_t* rp = reinterpret_cast<const uint64_t*>(mv.rec) + sl[k];
        ha[k] = FRESH ? __builtin_nontemporal_load(rp) : *rp;
      } else {
        const u32x4* rp = reinterpret_cast<const u32x4*>(rec_a(mv, sl[k]));
        ha[k] = FRESH ? __builtin_nontemporal_load(rp) : *rp;
        if constexpr (RF == 2) {
          const uint16_t* pp = rec_place(mv) + sl[k];
          pl[k] = FRESH ? __builtin_nontemporal_load(pp) : *pp;
        }
      }
    }
  }
  if constexpr (NARROW) {  // every owner entry is read: its bytes become the status stage
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < (kST * SK); j += kST) sst[j] = kAbsent;
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    if (sl[k] == kNoSlot) continue;
    SortRec x;
    if constexpr (RF == 1) {
      x = decode_rec8<FRESH, SK>(ha[k], in, w8, in.origin_base + (uint32_t)i0);
    } else if constexpr (RF == 2) {
      x = decode_wide(ha[k], in, in.origin_base + (uint32_t)i0 + pl[k]);
    } else {
      u32x4 hb = {0u, 0u, 0u, 0u};
      int64_t a2v = 0;
      if (rec_is_long(ha[k])) {
        const u32x4* bp = reinterpret_cast<const u32x4*>(rec_b(mv, sl[k]));
        hb = FRESH ? __builtin_nontemporal_load(bp) : *bp;
        if (((ha[k].z >> 16) & kFlagA2) && mv.a2) a2v = FRESH ? __builtin_nontemporal_load(mv.a2 + sl[k]) : mv.a2[sl[k]];
      }
      x = decode_sorted(ha[k], hb, a2v);
    }
    const uint32_t local = x.origin - in.origin_base - (uint32_t)i0;
    if (!x.valid || local >= n_t) {  // never written this epoch (cannot happen on a spill-free tile)
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
    sval[local] = rr.value;
    sst[local] = (uint8_t)rr.status;
    ++done;
  }
  __syncthreads();
  // (non-temporal: 56.4-58.8 vs 54.1-55.7 G on the headline step, one box, alternated; the
  // same stores measured flat-to-slower in the arrival, SeqFold and N > 1 completions,
  // which keep plain stores -- profiles/r6_small_sends.md)
#pragma unroll
  for (int k = 0; k < SK; ++k) {  // the tile's replies, coalesced (misses were answered by the scatter)
    const uint32_t j = (uint32_t)k * kST + threadIdx.x;
    if (j < n_t && sst[j] != kAbsent) put_reply_nt(rv, in.origin_base + (uint32_t)(i0 + j), sval[j], sst[j]);
  }
  return DrainCounts{done, failed, holes};
}

template <int FIXED, bool NARROW, int RF, int SK = kSK>
__global__ __launch_bounds__(kST, (NARROW && FIXED) ? 8 : 1) void mbx_drain_ring_kernel(MboxView mv, SortIn in, const uint32_t* __restrict__ tinfo,
                                                             const uint32_t* __restrict__ sidx,
                                                             const uint32_t* __restrict__ rw,
                                                             int64_t* __restrict__ state, uint32_t n_state,
                                                             uint64_t delay_ticks, OutboxView ob, ReplyView rv,
                                                             uint32_t* __restrict__ gsum, uint32_t ngroups,
                                                             unsigned* __restrict__ ticket, unsigned* __restrict__ tctr,
                                                             uint32_t* __restrict__ r8host) {
  extern __shared__ __align__(16) unsigned char smem_rd[];
  const uint32_t S = 1u << mv.log_s;
  DrainCounts dc;
  // tiles dealt XCD by XCD like the scatter's blocks (whose writes the XCD's L2 may still hold)
  const uint32_t t = virt_block(blockIdx.x, gridDim.x);
  if (t < in.tiles)
    dc = drain_ring_tile<FIXED, NARROW, false, RF, SK>(mv, in, t, tinfo, sidx, rw, state, n_state, delay_ticks, ob,
                                                       rv, smem_rd);
  block_add_stats(mv.stats, dc.done, kMbProcessed, dc.failed, kMbFailed, dc.holes, kMbHoles);
  __shared__ bool last;
  if (threadIdx.x == 0) last = last_block_ticket(ticket);
  __syncthreads();
  if (last) {  // every block's records are read: the rings are consumed
    for (uint32_t s = threadIdx.x; s < S; s += kST) epoch_commit(mv, s, epoch_sum(mv, gsum, ngroups, S, s));
    if (threadIdx.x == 0) tctr[1] += 1u;  // the next Send's one-pass epoch tag
    if constexpr (RF != 0) rec8_next(in, const_cast<uint32_t*>(in.r8w), r8host, in.tiles);
  }
}

// ---------------------------------------------------------------- fused one-pass sort + ring-order drain
// Batches of stateless methods (the parallel drain): the block that sorts tile t
// into the rings drains tile t's runs right after -- the runs of a tile are
// exactly the records it wrote, so no other block's progress is needed, only a
// barrier between the block's stores and its ring-order reads (FRESH loads).
// The records still go through the rings (written, then read back in ring
// order by other lanes than wrote them), but the Send is one launch instead of
// two, the drain's reads are L2 hits of lines the sort just wrote, and no block
// waits at a kernel boundary for the slowest tile.  The last block to finish
// commits every shard's epoch (tail = head = tail + total) and advances the
// look-back tag.  Tune mbox_fused=0: the separate kernels.
template <int MODE, bool A2, bool MC, int FIXED, int RF, int SK = kSK>
__global__ __launch_bounds__(kST) void mbx_sortdrain_kernel(SortIn in, MboxView mv, unsigned long long* __restrict__ desc,
                                                            unsigned* __restrict__ tctr, uint32_t* __restrict__ gsum,
                                                            uint32_t* __restrict__ sidx, uint32_t* __restrict__ tinfo,
                                                            uint32_t* __restrict__ rw, ReplyView rv,
                                                            int64_t* __restrict__ state, uint32_t n_state,
                                                            uint64_t delay_ticks, OutboxView ob,
                                                            unsigned* __restrict__ ticket, bool reserve,
                                                            uint32_t* __restrict__ r8host) {
  extern __shared__ __align__(16) unsigned char smem_sd[];
  const uint32_t S = 1u << mv.log_s;
  const uint32_t t = onesweep_tile<MODE, A2, MC, SK>(in, mv, desc, tctr, gsum, sidx, tinfo, rw, rv, true, false,
                                                     smem_sd, reserve);
  // every wave's ring stores are out before any wave reads the tile's runs
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const DrainCounts dc = drain_ring_tile<FIXED, true, true, RF, SK>(mv, in, t, tinfo, sidx, rw, state, n_state,
                                                                    delay_ticks, ob, rv, smem_sd);
  block_add_stats(mv.stats, dc.done, kMbProcessed, dc.failed, kMbFailed, dc.holes, kMbHoles);
  __shared__ bool last;
  if (threadIdx.x == 0) {
    // the last tile's block wrote the epoch totals (gsum): release them before its ticket
    if (t == in.tiles - 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    last = last_block_ticket(ticket);
    if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  if (last) {  // every block's records are read: the rings are consumed
    // (reserve: the totals were built by memory-side atomics in this launch -- read and
    // cleared the same way, not through this XCD's L2)
    for (uint32_t s = threadIdx.x; s < S; s += kST)
      epoch_commit(mv, s, epoch_sum(mv, gsum, 1, S, s));
    if (threadIdx.x == 0) tctr[1] += 1u;  // the next Send's one-pass epoch tag
    if constexpr (RF != 0) rec8_next(in, const_cast<uint32_t*>(in.r8w), r8host, in.tiles);
  }
}

// ---------------------------------------------------------------- arrival rings (fixed positions)
// Arrival sharding (batches without ordered methods): tile t's messages go to
// shard t & (S - 1), at ring offsets (t >> log S) * kSTile + (place in the
// tile) past the epoch's tail -- FIXED positions, so there is no count pass and
// no slot index: one enqueue pass resolves each message and writes its record
// (a tile is one contiguous 64 KB run of its ring: whole-line stores), and the
// drain reads the same positions in message order (whole-line loads, replies
// coalesced).  A message with no actor here leaves a zero record (its status is
// written by the enqueue); a tile whose run does not fit the ring's free room
// spills whole -- the drain runs it straight from the batch, re-resolving each
// message -- and tiles spill only as a suffix of a shard's sequence.
__device__ __forceinline__ bool arrival_fits(const MboxView& mv, const SortIn& in, uint32_t t, uint64_t& pos0,
                                             uint32_t tile = kSTile) {
  const uint32_t s = t & ((1u << mv.log_s) - 1);
  const uint64_t Q = 1ull << mv.log_q;
  const uint64_t tl = *ctr_tail(mv, s), hd = *ctr_head(mv, s);
  const uint64_t room = hd + Q > tl ? hd + Q - tl : 0;
  const uint64_t off = (uint64_t)(t >> mv.log_s) * tile;
  const uint64_t n_t = min((uint64_t)tile, (uint64_t)in.M - (uint64_t)t * tile);
  pos0 = tl + off;
  return off + n_t <= room;
}

template <int MODE, bool A2, bool MC>
__global__ __launch_bounds__(kST) void mbx_arrival_enqueue_kernel(SortIn in, MboxView mv, ReplyView rv) {
  unsigned long long n_enq = 0, n_miss = 0, n_spill = 0;
  const uint32_t t = virt_block(blockIdx.x, gridDim.x);
  if (t < in.tiles) {
    uint64_t pos0 = 0;
    const bool fits = arrival_fits(mv, in, t, pos0);
    const uint32_t s = t & ((1u << mv.log_s) - 1);
    uint32_t a[kSK], mb[kSK], meth[kSK];
    int64_t x0[kSK], x1[kSK], x2[kSK];
    int r[kSK];
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const int64_t i = tile_index(t, k);
      const bool ok = i < in.M;
      a[k] = ok ? __builtin_nontemporal_load(in.actor + i) : 0xffffffffu;
      x0[k] = ok ? __builtin_nontemporal_load(in.a0 + i) : 0;
      x1[k] = ok && in.a1 ? __builtin_nontemporal_load(in.a1 + i) : 0;
      x2[k] = 0;
      if constexpr (A2) x2[k] = ok ? __builtin_nontemporal_load(in.a2 + i) : 0;
      meth[k] = in.method_uniform;
      if constexpr (MC) meth[k] = ok ? (uint32_t)in.mcol[i] : 0u;
    }
    resolve_k<MODE>(in, a, r, mb);
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const int64_t i = tile_index(t, k);
      if (i >= in.M) continue;
      const uint32_t origin = in.origin_base + (uint32_t)i;
      const bool ok = r[k] == in.rank_self && mb[k] < kMaxMbox;
      const uint64_t slot = slot_at(mv, s, pos0 + (uint64_t)(i - (int64_t)t * kSTile));
      if (!ok) {
        ++n_miss;
        write_status(rv, origin, kStatusNoActor);
        if (fits) *reinterpret_cast<u32x4*>(rec_a(mv, slot)) = u32x4{0u, 0u, 0u, 0u};
        continue;
      }
      if (!fits) {
        ++n_spill;
        continue;
      }
      const uint32_t mt = meth[k];
      if (mt < 128u && fits_i32(x0[k]) && fits_i32(x1[k]) && x2[k] == 0) {
        *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
            u32x4{origin | kCompactMark, mb[k] | (mt << 24), (uint32_t)x0[k], (uint32_t)x1[k]};
      } else {
        const uint32_t fl = x2[k] != 0 ? (uint32_t)kFlagA2 : 0u;
        *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
            u32x4{origin | kCompactMark, mb[k] | kCompactLong, (mt & 0xffffu) | (fl << 16), 0u};
        *reinterpret_cast<u32x4*>(rec_b(mv, slot)) = u32x4{(uint32_t)x0[k], (uint32_t)((uint64_t)x0[k] >> 32),
                                                           (uint32_t)x1[k], (uint32_t)((uint64_t)x1[k] >> 32)};
        if (fl) mv.a2[slot] = x2[k];
      }
      ++n_enq;
    }
  }
  block_add_stats(mv.stats, n_enq, kMbEnqueued, n_miss, kMbNoActor, n_spill, kMbSpilled);
}

template <int FIXED, int MODE>
__global__ __launch_bounds__(kST) void mbx_arrival_drain_kernel(MboxView mv, SortIn in, int64_t* __restrict__ state,
                                                                uint32_t n_state, uint64_t delay_ticks, OutboxView ob,
                                                                ReplyView rv, unsigned* __restrict__ ticket) {
  unsigned long long done = 0, failed = 0;
  const uint32_t S = 1u << mv.log_s;
  const uint32_t t = virt_block(blockIdx.x, gridDim.x);
  if (t < in.tiles) {
    uint64_t pos0 = 0;
    const bool fits = arrival_fits(mv, in, t, pos0);
    const uint32_t s = t & (S - 1);
    SortRec x[kSK];
    if (fits) {
      u32x4 ha[kSK];
#pragma unroll
      for (int k = 0; k < kSK; ++k) {
        const int64_t i = tile_index(t, k);
        ha[k] = i < in.M ? *reinterpret_cast<const u32x4*>(rec_a(mv, slot_at(mv, s, pos0 + (uint64_t)(i - (int64_t)t * kSTile))))
                         : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int k = 0; k < kSK; ++k) {
        u32x4 hb = {0u, 0u, 0u, 0u};
        int64_t a2v = 0;
        if ((ha[k].x & kCompactMark) && rec_is_long(ha[k])) {
          const uint64_t slot = slot_at(mv, s, pos0 + (uint64_t)(tile_index(t, k) - (int64_t)t * kSTile));
          hb = *reinterpret_cast<const u32x4*>(rec_b(mv, slot));
          if (((ha[k].z >> 16) & kFlagA2) && mv.a2) a2v = mv.a2[slot];
        }
        x[k] = decode_sorted(ha[k], hb, a2v);  // a zero record (no actor): not valid
      }
    } else {  // the tile spilled: run it from the batch
      uint32_t a[kSK], mb[kSK];
      int r[kSK];
#pragma unroll
      for (int k = 0; k < kSK; ++k) {
        const int64_t i = tile_index(t, k);
        a[k] = i < in.M ? in.actor[i] : 0xffffffffu;
      }
      resolve_k<MODE>(in, a, r, mb);
#pragma unroll
      for (int k = 0; k < kSK; ++k) {
        const int64_t i = tile_index(t, k);
        x[k].valid = i < in.M && r[k] == in.rank_self && mb[k] < kMaxMbox;
        if (!x[k].valid) continue;
        x[k].mb = mb[k];
        x[k].method = in.mcol ? (uint32_t)in.mcol[i] : in.method_uniform;
        x[k].flags = 0;
        x[k].a0 = in.a0[i];
        x[k].a1 = in.a1 ? in.a1[i] : 0;
        x[k].a2 = in.a2 ? in.a2[i] : 0;
      }
    }
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      if (!x[k].valid) continue;  // no actor: answered by the enqueue
      MsgRecord m;
      m.actor = x[k].mb;
      m.method = (uint16_t)(FIXED ? FIXED : x[k].method);
      m.flags = (uint16_t)x[k].flags;
      m.a0 = x[k].a0, m.a1 = x[k].a1, m.a2 = x[k].a2;
      const ReplyRecord rr = run_handler(m, state, n_state, delay_ticks, ob);
      failed += rr.status != kStatusOk;
      write_reply(rv, in.origin_base + (uint32_t)tile_index(t, k), rr);
      ++done;
    }
  }
  block_add_stats(mv.stats, done, kMbProcessed, failed, kMbFailed, 0, -1);
  __shared__ bool last;
  if (threadIdx.x == 0) last = last_block_ticket(ticket);
  __syncthreads();
  if (last) {  // every tile is read: each shard consumed the positions of its tiles that fit
    for (uint32_t s = threadIdx.x; s < S; s += kST) {
      uint64_t used = 0;
      for (uint32_t tt = s; tt < in.tiles; tt += S) {
        uint64_t pos0 = 0;
        if (!arrival_fits(mv, in, tt, pos0)) break;  // the spilled suffix
        used += min((uint64_t)kSTile, (uint64_t)in.M - (uint64_t)tt * kSTile);
      }
      epoch_commit(mv, s, (uint32_t)used);
    }
  }
}

// Arrival rings, enqueue and drain in ONE launch.  Block t writes tile t's records
// into its run of ring t & (S - 1) (the positions mbx_arrival_enqueue_kernel uses) and,
// after a block barrier, drains that run: wave w consumes the records wave w ^ 4 wrote
// -- read back from the ring, decoded, its handler run -- so the ring is the hand-off
// between the block's waves, as it is between the two kernels of the general form (no
// grid-wide phase is needed: an arrival run belongs to one tile).  Uniform batches of at
// most two arguments; MODE 3 (rank byte routes, stateless methods) carries actor ids.
//
// Record format per WAVE (its producer decides with one ballot and tells its consumer
// through LDS, across the barrier the hand-off needs anyway; allow8 -- batches past 512
// tiles, the rule of the sort's 8-B records): 8 B {mailbox 24 | zigzag
// a0 20 | zigzag a1 20} when every message of the wave fits, in the first half of the
// wave's own 512 slots (message j in half j & 1 of slot j / 2 of that range: formats
// never overlap), else the 16-B compact form (32-B long form for a value past 32 bits).
constexpr int kArr8Mb = 24, kArr8Arg = 20;
constexpr uint64_t kArr8Null = ~0ull;  // a slot of no actor (mailbox 2^24 - 1 never fits the 8-B form)
__device__ __forceinline__ bool arr8_fits(uint32_t mb, int64_t x0, int64_t x1) {
  const uint64_t z0 = ((uint64_t)x0 << 1) ^ (uint64_t)(x0 >> 63), z1 = ((uint64_t)x1 << 1) ^ (uint64_t)(x1 >> 63);
  return mb < (1u << kArr8Mb) - 1u && (z0 >> kArr8Arg) == 0 && (z1 >> kArr8Arg) == 0;
}
template <int SK>
__device__ __forceinline__ uint64_t arr8_cell(const MboxView& mv, uint32_t s, uint64_t pos0, uint32_t j) {
  constexpr uint32_t run = SK * kWave;  // a wave's run of the tile
  return 2 * slot_at(mv, s, pos0 + (j & ~(run - 1)) + ((j & (run - 1)) >> 1)) + (j & 1);
}
// SK messages per thread: kSK (4096-message tiles), or 2 (1024) for batches of up to 512
// 4096-message tiles -- one 8-wave block per CU at 1 Mi messages hid too little latency
template <int MODE, int FIXED, int SK = kSK>
__global__ __launch_bounds__(kST) void mbx_arrival_fused_kernel(SortIn in, MboxView mv, int64_t* __restrict__ state,
                                                                uint32_t n_state, uint64_t delay_ticks, OutboxView ob,
                                                                ReplyView rv, unsigned* __restrict__ ticket,
                                                                bool allow8) {
  __shared__ uint32_t wave_rec8[kST / kWave];
  extern __shared__ __align__(16) unsigned char smem_af[];  // MODE 4: the presence map
  uint32_t* lpres = reinterpret_cast<uint32_t*>(smem_af);
  if constexpr (MODE == 4) {
    stage_pres(in, lpres);
    __syncthreads();
  }
  unsigned long long n_enq = 0, n_miss = 0, n_spill = 0, done = 0, failed = 0;
  const uint32_t S = 1u << mv.log_s;
  const uint32_t t = virt_block(blockIdx.x, gridDim.x);
  const unsigned w = threadIdx.x / kWave;
  if (t < in.tiles) {
    uint64_t pos0 = 0;
    constexpr uint32_t kTile = kST * SK;
    const bool fits = arrival_fits(mv, in, t, pos0, kTile);
    const uint32_t s = t & (S - 1);
    uint32_t a[SK], mb[SK];
    int64_t x0[SK], x1[SK];
    int r[SK];
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      const int64_t i = tile_index<SK>(t, k);
      const bool ok = i < in.M;
      a[k] = ok ? __builtin_nontemporal_load(in.actor + i) : 0xffffffffu;
      x0[k] = ok ? __builtin_nontemporal_load(in.a0 + i) : 0;
      x1[k] = ok && in.a1 ? __builtin_nontemporal_load(in.a1 + i) : 0;
    }
    if constexpr (MODE == 4) resolve_pres<SK>(in, lpres, a, r, mb);
    else resolve_k<MODE, SK>(in, a, r, mb);
    bool live[SK];
    bool narrow = allow8 && mv.planar != 0;
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      live[k] = tile_index<SK>(t, k) < in.M && r[k] == in.rank_self && mb[k] < kMaxMbox;
      if (live[k] && !arr8_fits(mb[k], x0[k], x1[k])) narrow = false;
    }
    const bool rec8 = __ballot(!narrow) == 0;  // (wave-uniform)
    if (lane_id() == 0) wave_rec8[w] = rec8;
    uint64_t* cells = reinterpret_cast<uint64_t*>(mv.rec);
#pragma unroll
    for (int k = 0; k < SK; ++k) {  // enqueue: the tile's records at their fixed ring positions
      const int64_t i = tile_index<SK>(t, k);
      if (i >= in.M) continue;
      const uint32_t origin = in.origin_base + (uint32_t)i;
      const uint32_t j = (uint32_t)(i - (int64_t)t * kTile);
      const uint64_t slot = slot_at(mv, s, pos0 + j);
      if (!live[k]) {
        ++n_miss;
        write_status(rv, origin, kStatusNoActor);
        if (fits && rec8) cells[arr8_cell<SK>(mv, s, pos0, j)] = kArr8Null;
        else if (fits) *reinterpret_cast<u32x4*>(rec_a(mv, slot)) = u32x4{0u, 0u, 0u, 0u};
        continue;
      }
      if (!fits) {  // the tile spilled: its messages run from the registers below
        ++n_spill;
        continue;
      }
      const uint32_t mt = in.method_uniform;
      if (rec8) {
        const uint64_t z0 = ((uint64_t)x0[k] << 1) ^ (uint64_t)(x0[k] >> 63);
        const uint64_t z1 = ((uint64_t)x1[k] << 1) ^ (uint64_t)(x1[k] >> 63);
        cells[arr8_cell<SK>(mv, s, pos0, j)] = (uint64_t)mb[k] | (z0 << kArr8Mb) | (z1 << (kArr8Mb + kArr8Arg));
      } else if (mt < 128u && fits_i32(x0[k]) && fits_i32(x1[k])) {
        *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
            u32x4{origin | kCompactMark, mb[k] | (mt << 24), (uint32_t)x0[k], (uint32_t)x1[k]};
      } else {
        *reinterpret_cast<u32x4*>(rec_a(mv, slot)) =
            u32x4{origin | kCompactMark, mb[k] | kCompactLong, mt & 0xffffu, 0u};
        *reinterpret_cast<u32x4*>(rec_b(mv, slot)) = u32x4{(uint32_t)x0[k], (uint32_t)((uint64_t)x0[k] >> 32),
                                                           (uint32_t)x1[k], (uint32_t)((uint64_t)x1[k] >> 32)};
      }
      ++n_enq;
    }
    __syncthreads();  // the run is in the ring: drain it
    const uint32_t w2 = w ^ 4u;  // (the wave whose records this one consumes)
    const bool rec8_2 = wave_rec8[w2] != 0;
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      SortRec x;
      int64_t i;
      if (fits) {  // wave w2's k-th record of this lane
        const uint32_t j = w2 * (SK * kWave) + (uint32_t)k * kWave + lane_id();
        i = (int64_t)t * kTile + j;
        if (i >= in.M) continue;
        if (rec8_2) {
          const uint64_t c = cells[arr8_cell<SK>(mv, s, pos0, j)];
          if (c == kArr8Null) continue;  // no actor: answered by the enqueue
          x.valid = true, x.method = in.method_uniform, x.flags = 0, x.a2 = 0;
          x.mb = (uint32_t)(c & ((1u << kArr8Mb) - 1));
          const uint64_t z0 = (c >> kArr8Mb) & ((1ull << kArr8Arg) - 1), z1 = c >> (kArr8Mb + kArr8Arg);
          x.a0 = (int64_t)(z0 >> 1) ^ -(int64_t)(z0 & 1);
          x.a1 = (int64_t)(z1 >> 1) ^ -(int64_t)(z1 & 1);
        } else {
          const uint64_t slot = slot_at(mv, s, pos0 + j);
          const u32x4 ha = *reinterpret_cast<const u32x4*>(rec_a(mv, slot));
          const u32x4 hb = rec_is_long(ha) ? *reinterpret_cast<const u32x4*>(rec_b(mv, slot)) : u32x4{0u, 0u, 0u, 0u};
          x = decode_sorted(ha, hb, 0);  // a zero record (no actor): not valid
          if (!x.valid) continue;
        }
      } else {  // a spilled tile: this thread's own messages, from its registers
        if (!live[k]) continue;  // (no actor: answered above)
        i = tile_index<SK>(t, k);
        x.valid = true, x.mb = mb[k], x.method = in.method_uniform, x.flags = 0;
        x.a0 = x0[k], x.a1 = x1[k], x.a2 = 0;
      }
      MsgRecord m;
      m.actor = x.mb;
      m.method = (uint16_t)(FIXED ? FIXED : x.method);
      m.flags = (uint16_t)x.flags;
      m.a0 = x.a0, m.a1 = x.a1, m.a2 = 0;
      const ReplyRecord rr = run_handler(m, state, n_state, delay_ticks, ob);
      failed += rr.status != kStatusOk;
      write_reply(rv, in.origin_base + (uint32_t)i, rr);
      ++done;
    }
  }
  block_add_stats(mv.stats, n_enq, kMbEnqueued, n_miss, kMbNoActor, n_spill, kMbSpilled);
  __syncthreads();  // block_add_stats' LDS partials are reused
  block_add_stats(mv.stats, done, kMbProcessed, failed, kMbFailed, 0, -1);
  __shared__ bool last;
  if (threadIdx.x == 0) last = last_block_ticket(ticket);
  __syncthreads();
  if (last) {  // every tile is read: each shard consumed the positions of its tiles that fit
    for (uint32_t sh = threadIdx.x; sh < S; sh += kST) {
      uint64_t used = 0;
      for (uint32_t tt = sh; tt < in.tiles; tt += S) {
        uint64_t p0 = 0;
        if (!arrival_fits(mv, in, tt, p0, kST * SK)) break;  // the spilled suffix
        used += min((uint64_t)(kST * SK), (uint64_t)in.M - (uint64_t)tt * (kST * SK));
      }
      epoch_commit(mv, sh, (uint32_t)used);
    }
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
// A12: the batch carries a second / third argument column.  Without them (a
// one-argument ordered method, e.g. SeqFold) the window's a1 / a2 arrays are not
// allocated: 68 instead of 100 KB of LDS, so two drain blocks fit a CU.
template <bool A12, int OK = kOrdK>
struct OrdLds {
  static constexpr int kWin = kOrdThreads * OK;
  uint32_t wcnt[kOrdWaves][kOrdThreads];  // per-wave bin counts -> offsets
  uint32_t bstart[kOrdThreads];
  uint32_t bcount[kOrdThreads];
  uint32_t wsum[kOrdWaves];
  uint32_t slot[kWin];
  uint32_t act[kWin];  // actor index for the handler (LDS-local or global mailbox)
  uint32_t meth[kWin];  // method | flags << 16
  uint32_t orig[kWin];  // origin: the completion's place for the reply
  int64_t a0[kWin], a1[A12 ? kWin : 2], a2[A12 ? kWin : 2];
};

// OK: records per thread per window (window = 512 * OK records: OK = 8 for one-argument batches).
// FIXED = kSeqFold: a uniform SeqFold batch.  With every actor of the shard in its
// own bin (at most kOrdThreads of them, state staged), thread b IS actor b's
// consumer for the whole Send: its state stays in a register and each record is
// one fold (reply = the state before, state = state * kFoldMul + a0) -- no handler
// switch, no LDS state round trip per message.
// R8: the sort wrote 8-B records (a uniform one-argument batch): each carries its
// place in its tile (12 bits), the mailbox and the zigzag argument at the widths
// *r8w; mbx_rec8_next_kernel derives the next Send's widths after the drain.
struct R8Args {
  const uint32_t* r8w = nullptr;  // this Send's widths (the sort's)
  uint32_t method = 0;            // the batch's uniform method
  const int64_t* esc = nullptr;   // escape records' {a0, mailbox}, by ring slot (SortIn::r8esc)
};
__device__ __forceinline__ SortRec decode_rec8_ord(uint64_t r, uint32_t w8, uint32_t method, const int64_t* esc,
                                                   uint64_t slot) {
  const uint32_t wm = w8 & 0xffu, w0 = (w8 >> 8) & 0xffu, w1 = (w8 >> 16) & 0xffu;
  SortRec x;
  x.valid = true;
  x.origin = (uint32_t)(r & (kSTile - 1));  // the place in the tile
  x.method = method;
  x.flags = 0;
  x.a2 = 0;
  if (r >> 63) {  // escape record (one-argument batches leave the top bit of a record zero)
    const u32x4 e = *reinterpret_cast<const u32x4*>(esc + 2 * slot);
    x.a0 = (int64_t)(((uint64_t)e.y << 32) | e.x);
    x.mb = e.z;
    x.a1 = 0;
    return x;
  }
  x.mb = (uint32_t)((r >> 12) & ((1ull << wm) - 1));
  const uint64_t z0 = (r >> (12 + wm)) & ((1ull << w0) - 1), z1 = (r >> (12 + wm + w0)) & ((1ull << w1) - 1);
  x.a0 = (int64_t)(z0 >> 1) ^ -(int64_t)(z0 & 1);
  x.a1 = (int64_t)(z1 >> 1) ^ -(int64_t)(z1 & 1);
  return x;
}

// A window's records (their first 16 B; R8: the 8-B record), wave w's positions.
template <bool R8, int OK>
__device__ __forceinline__ void ord_load_win(const MboxView& mv, uint64_t wa, uint64_t n_end, uint64_t sbase,
                                             uint64_t rot, uint64_t qmask, unsigned w, unsigned lane,
                                             typename std::conditional<R8, uint64_t, u32x4>::type (&h)[OK]) {
#pragma unroll
  for (int k = 0; k < OK; ++k) {
    const uint64_t q = wa + (uint64_t)w * (kWave * OK) + (uint64_t)k * kWave + lane;
    const uint64_t sl = sbase | ((q + rot) & qmask);
    const bool in = q < n_end && q < wa + (kOrdThreads * OK);
    if constexpr (R8) h[k] = in ? reinterpret_cast<const uint64_t*>(mv.rec)[sl] : 0ull;
    else h[k] = in ? *reinterpret_cast<const u32x4*>(rec_a(mv, sl)) : u32x4{0u, 0u, 0u, 0u};
  }
}

// (one block per CU whatever its registers -- the window's LDS -- so the register
// budget is that of 2 waves per SIMD: no spill for the prefetched window)
template <bool A12, int OK = kOrdK, int FIXED = 0, bool PF = false, bool R8 = false>
__global__ __launch_bounds__(kOrdThreads) __attribute__((amdgpu_waves_per_eu(1, 2))) void mbx_drain_ordered_kernel(MboxView mv, uint32_t* __restrict__ gsum,
                                                                        uint32_t ngroups, int64_t* __restrict__ state,
                                                                        uint32_t n_state, uint64_t delay_ticks,
                                                                        OutboxView ob, u32x4* __restrict__ srep,
                                                                        uint32_t origin_base, R8Args r8) {
  extern __shared__ __align__(16) unsigned char smem_ord[];
  OrdLds<A12, OK>& L = *reinterpret_cast<OrdLds<A12, OK>*>(smem_ord);
  int64_t* st_lds = reinterpret_cast<int64_t*>(smem_ord + sizeof(OrdLds<A12, OK>));
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
  const bool reg = FIXED == kSeqFold && in_lds && n_loc <= (uint32_t)kOrdThreads;  // actor b's state in thread b
  uint64_t sreg = reg && threadIdx.x < n_loc ? (uint64_t)st_lds[threadIdx.x] : 0ull;
  const uint32_t tot = tot_s;
  const uint64_t n = tot < free ? tot : free;
  const uint64_t sbase = (uint64_t)s << mv.log_q, qmask = Q - 1, rot = shard_rot(mv, s);  // slot_at, hoisted
  unsigned long long done = 0, failed = 0, holes = 0, serial = 0;
  // PF (the fold: the next window's records (their first 16 B) are loaded
  // while this one is binned and run -- one block per CU (the LDS), so the registers are
  // there.  (Round 3, with the handler switch's register file: measured no faster, 188 ->
  // 200 us, and spilled to scratch.)
  const uint64_t n_end = lo + n;
  using RawT = typename std::conditional<R8, uint64_t, u32x4>::type;  // a record's first (R8: only) word
  const uint32_t w8 = R8 ? *r8.r8w : 0u;
  RawT cur[PF ? OK : 1];
  if constexpr (PF) {
    if (lo < n_end) ord_load_win<R8, OK>(mv, lo, n_end, sbase, rot, qmask, w, lane, cur);
  }
  for (uint64_t w0 = lo; w0 < lo + n; w0 += (kOrdThreads * OK)) {
    const uint64_t w1 = lo + n < w0 + (kOrdThreads * OK) ? lo + n : w0 + (kOrdThreads * OK);
    for (uint32_t b = lane; b < kOrdThreads; b += kWave) L.wcnt[w][b] = 0;
    SortRec x[OK];
    uint32_t bin[OK], wr[OK];
    uint64_t slot[OK];
    RawT nxt[PF ? OK : 1];
    if constexpr (PF) {
      if (w0 + (kOrdThreads * OK) < n_end)
        ord_load_win<R8, OK>(mv, w0 + (kOrdThreads * OK), n_end, sbase, rot, qmask, w, lane, nxt);
    }
#pragma unroll
    for (int k = 0; k < OK; ++k) {  // wave w owns window positions [w * 64K, (w+1) * 64K)
      const uint64_t q = w0 + (uint64_t)w * (kWave * OK) + (uint64_t)k * kWave + lane;
      slot[k] = sbase | ((q + rot) & qmask);
      if (q < w1) {
        if constexpr (R8) {
          x[k] = decode_rec8_ord(PF ? (uint64_t)cur[k] : reinterpret_cast<const uint64_t*>(mv.rec)[slot[k]], w8,
                                 r8.method, r8.esc, slot[k]);
        } else if constexpr (PF) {
          u32x4 hb = {0u, 0u, 0u, 0u};
          int64_t a2v = 0;
          if (rec_is_long(cur[k])) {
            hb = *reinterpret_cast<const u32x4*>(rec_b(mv, slot[k]));
            if (((cur[k].z >> 16) & kFlagA2) && mv.a2) a2v = mv.a2[slot[k]];
          }
          x[k] = decode_sorted(cur[k], hb, a2v);
        } else {
          x[k] = load_sorted(mv, slot[k]);
        }
        if (!x[k].valid) ++holes;
      } else {
        x[k].valid = false;
      }
    }
    if constexpr (PF) {
#pragma unroll
      for (int k = 0; k < OK; ++k) cur[k] = nxt[k];
    }
#pragma unroll
    for (int k = 0; k < OK; ++k) {
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
    for (int k = 0; k < OK; ++k) {
      if (!x[k].valid) continue;
      const unsigned d = L.bstart[bin[k]] + L.wcnt[w][bin[k]] + wr[k];
      L.slot[d] = (uint32_t)slot[k];
      L.act[d] = in_lds ? (x[k].mb >> mv.log_s) : x[k].mb;
      if (!reg) L.meth[d] = x[k].method | (x[k].flags << 16);
      // the message's place in its tile (the completion reads the tile's runs)
      L.orig[d] = R8 ? x[k].origin : ((x[k].origin - origin_base) & (uint32_t)(kSTile - 1));
      L.a0[d] = x[k].a0;
      if constexpr (A12) {
        L.a1[d] = x[k].a1;
        L.a2[d] = x[k].a2;
      }
    }
    __syncthreads();
    if (reg) {  // uniform SeqFold, one actor per bin: the folds in a register
      const unsigned b = threadIdx.x, e = L.bstart[b] + L.bcount[b];
      if (L.bcount[b] > 1) serial += L.bcount[b] - 1;
      for (unsigned d = L.bstart[b]; d < e; ++d) {
        const uint64_t prev = sreg;
        uint32_t st = kStatusOk;
        if (L.act[d] == b && b < n_loc) {
          sreg = prev * kFoldMul + (uint64_t)L.a0[d];
        } else {  // a mailbox past the state (routed here by a stale registry entry)
          st = kStatusNoActor;
          ++failed;
        }
        const uint64_t v = st == kStatusOk ? prev : 0ull;
        srep[L.slot[d]] = u32x4{(uint32_t)v, (uint32_t)(v >> 32), st, L.orig[d]};
        ++done;
      }
    } else {  // this thread's bin, serially in ring order
      const unsigned b = threadIdx.x, e = L.bstart[b] + L.bcount[b];
      if (L.bcount[b] > 1) serial += L.bcount[b] - 1;  // records that waited behind their bin's earlier ones
      int64_t* st = in_lds ? st_lds : state;
      const uint32_t nst = in_lds ? n_loc : n_state;
      for (unsigned d = L.bstart[b]; d < e; ++d) {
        MsgRecord m;
        m.actor = L.act[d];
        m.method = (uint16_t)(L.meth[d] & 0xffffu);
        m.flags = (uint16_t)(L.meth[d] >> 16);
        m.a0 = L.a0[d];
        m.a1 = A12 ? L.a1[d] : 0;
        m.a2 = A12 ? L.a2[d] : 0;
        const ReplyRecord rr = run_handler(m, st, nst, delay_ticks, ob, true);
        failed += rr.status != kStatusOk;
        srep[L.slot[d]] = u32x4{(uint32_t)rr.value, (uint32_t)((uint64_t)rr.value >> 32), (uint32_t)rr.status, L.orig[d]};
        ++done;
        if (!in_lds) vm_drain();  // global state: this store lands before the bin's next load
      }
    }
    __syncthreads();  // the window's LDS is reused
  }
  if (reg && threadIdx.x < n_loc) st_lds[threadIdx.x] = (int64_t)sreg;
  if (reg) __syncthreads();
  if (in_lds)
    for (uint32_t j = threadIdx.x; j < n_loc; j += kOrdThreads) state[s + (uint64_t)j * S] = st_lds[j];
  block_add_stats(mv.stats, done, kMbProcessed, failed, kMbFailed, holes, kMbHoles);
  __syncthreads();  // block_add_stats' LDS partials are reused
  block_add_stats(mv.stats, serial, kMbSerial, 0, -1, 0, -1);
  if (threadIdx.x == 0) epoch_commit(mv, s, tot);
}

// The next Send's 8-B field widths after an ordered 8-B-record Send (one block, launched
// after the ordered drain: every block of it has decoded with this Send's widths).
template <int = 0>  // (a template: the header is compiled into every launcher TU that uses it)
__global__ __launch_bounds__(256) void mbx_rec8_next_kernel(const uint32_t* __restrict__ r8max,
                                                            uint32_t* __restrict__ r8w, uint32_t* __restrict__ host,
                                                            uint32_t tiles) {
  rec8_next_from(r8max, r8w, host, tiles);
}

template <int = 0>
__global__ __launch_bounds__(kST) void mbx_complete_ring_kernel(SortIn in, MboxView mv,
                                                                const uint32_t* __restrict__ tinfo,
                                                                const u32x4* __restrict__ srep, ReplyView rv,
                                                                unsigned* __restrict__ tctr) {
  extern __shared__ __align__(16) unsigned char smem_cr[];
  if (blockIdx.x == 0 && threadIdx.x == 0) tctr[1] += 1u;  // the next Send's one-pass epoch tag (the sort is done)
  const uint32_t S = 1u << mv.log_s;
  int64_t* sval = reinterpret_cast<int64_t*>(smem_cr);
  RunLds<uint16_t> L;
  L.bias = reinterpret_cast<uint32_t*>(sval + kSTile);
  L.excl = L.bias + S;
  L.owner = reinterpret_cast<uint16_t*>(L.excl + S);
  uint8_t* sst = reinterpret_cast<uint8_t*>(L.owner + kSTile);
  const uint32_t t = virt_block(blockIdx.x, gridDim.x);
  if (t >= in.tiles) return;
  const uint64_t i0 = (uint64_t)t * kSTile;
  const uint32_t n_t = (uint32_t)min((uint64_t)kSTile, (uint64_t)in.M - i0);
  for (uint32_t j = threadIdx.x; j < kSTile; j += kST) sst[j] = kAbsent;
  int spill = 0;
  const uint32_t T = load_tile_runs(mv, tinfo, t, L, spill);
  const uint64_t qmask = (1ull << mv.log_q) - 1;
  u32x4 r[kSK];
#pragma unroll
  for (int k = 0; k < kSK; ++k) {
    const uint32_t j = (uint32_t)k * kST + threadIdx.x;
    if (j < T) {
      const uint32_t s = L.owner[j];
      // (read once: non-temporal -- SeqFold 25.64-25.87 vs 25.22-25.57 G and 25.74-25.85 vs
      // 25.35-25.52 G in two sessions, alternated; profiles/r6_small_sends.md)
      r[k] = __builtin_nontemporal_load(srep + (((uint64_t)s << mv.log_q) | ((L.bias[s] + j) & qmask)));
    } else {
      r[k] = u32x4{0u, 0u, 0u, 0xffffffffu};
    }
  }
#pragma unroll
  for (int k = 0; k < kSK; ++k) {
    const uint32_t local = r[k].w;  // the place in the tile (the drains write it; 0xffffffff: none)
    if (local < n_t) {
      sval[local] = (int64_t)(((uint64_t)r[k].y << 32) | r[k].x);
      sst[local] = (uint8_t)r[k].z;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kSK; ++k) {
    const uint32_t j = (uint32_t)k * kST + threadIdx.x;
    if (j < n_t && sst[j] != kAbsent) put_reply(rv, in.origin_base + (uint32_t)(i0 + j), sval[j], sst[j]);
  }
}

// ---------------------------------------------------------------- host
// The fused sort + drain kernel: slower than the two kernels for large batches once the sort
// reserves its runs (8 Mi: 149 vs 95 + 39 us; its register file halves the drain's occupancy),
// faster for small ones, where a launch and a kernel boundary weigh more (1 Mi bench step: 5-7 %
// in three sessions).  Fused up to 512 tiles (2 Mi messages); tune mbox_fused=1 / 0 forces it.

// ---------------------------------------------------------------- out-of-TU launchers
// The fused one-pass sort + ring-order drain of a stateless Send (mailbox_sort_fused.hip).
struct MbxFusedLaunch {
  SortIn in;
  MboxView mv;
  unsigned long long* desc;
  unsigned* tctr;
  uint32_t *gsum, *sidx, *tinfo, *rw;
  ReplyView rv;
  int64_t* state;
  uint32_t n_state;
  uint64_t delay_ticks;
  OutboxView ob;
  unsigned* ticket;
  bool reserve;
  uint32_t* r8host;
  size_t lds;
  hipStream_t st;
  int rf, mode;
  bool fixed_mul, rank_route, a2, mcol;
};
void mbx_launch_fused(const MbxFusedLaunch& f);
void mbx_launch_fused_dir(const MbxFusedLaunch& f);    // route modes 1, 3
void mbx_launch_fused_other(const MbxFusedLaunch& f);  // route modes 0, 2

// The ordered drain + the ring-order completion of an ordered Send (mailbox_sort_ordered.hip).
struct MbxOrderedLaunch {
  SortIn in;
  MboxView mv;
  uint32_t* gsum;
  uint32_t ngroups;
  int64_t* state;
  uint32_t n_state;
  uint64_t delay_ticks;
  OutboxView ob;
  u32x4* stage_rep;
  uint32_t origin_base;
  uint32_t Sv;
  bool r8_on, a12, fold;
  R8Args r8a;
  uint32_t *r8max, *r8w, *r8host;
  uint32_t* tinfo;
  ReplyView rv;
  unsigned* tctr;
  uint32_t tile_grid;
  hipStream_t st;
};
void mbx_launch_ordered(const MbxOrderedLaunch& o);

}  // namespace ptype
