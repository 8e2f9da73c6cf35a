// Sorted exchange (design: exchange_sorted.hpp).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>

#include "exchange_sorted.hpp"
#include "mailbox.hpp"
#include "mailbox_dev.hpp"
#include "sort_common.hpp"
#include "tune.hpp"

namespace ptype {

namespace {
constexpr int kXOrdThreads = 512;  // receiver ordered drain: one block per wire shard, one bin per thread
constexpr int kXOrdK = 4;
constexpr int kXOrdWin = kXOrdThreads * kXOrdK;
constexpr int kXOrdWaves = kXOrdThreads / kWave;
constexpr uint32_t kXOrdStateMax = 4096;
constexpr int kXDispU = 4;
constexpr int kXMaxBuckets = kSxMaxRanks * kSxShards;
}  // namespace

// ---------------------------------------------------------------- layout
PackedLayout sx_layout(const uint64_t* meta) {
  uint64_t m[kMetaWords];
  std::copy(meta, meta + kMetaWords, m);
  // every value of the widest mailbox (or actor id) seen fits, plus one: all-ones is
  // the null record.  Sized by the bit length, not the value: under skewed load the
  // largest id a batch happens to carry changes from Send to Send, and a batch
  // whose max is 2^b - 1 after an agreement that saw 2^b - 2 must not overflow.
  {
    const uint64_t v = meta[kMetaMbox];
    const int b = v ? 64 - __builtin_clzll(v) : 0;
    m[kMetaMbox] = (b >= 63 ? ~0ull >> 1 : (1ull << b) - 1) + 1;
  }
  return packed_layout(m);
}

static int sx_round_S(int S) { return S <= 4 ? S : S <= 6 ? 6 : 8; }

// A field fits the layout in force (the mailbox all-ones value is reserved).
// reject_ordered: the agreement in force saw no ordered method, so no rank
// sorts by actor shard this Send and the receivers skip their ordered drain --
// an ordered message overflows (re-sent once the agreement carries its method).
__device__ __forceinline__ bool sx_fits(const PackedLayout& L, uint32_t meth, uint32_t hdr_method, uint32_t mb,
                                        uint64_t z0, uint64_t z1, uint64_t z2, bool reject_ordered) {
  auto fits = [&](int q, uint64_t v) { return L.w[q] >= 64 || (v >> L.w[q]) == 0; };
  if (reject_ordered && method_ordered(meth)) return false;
  if (L.w[0] ? !fits(0, meth) : meth != hdr_method) return false;
  if (L.w[1] == 0 || (uint64_t)mb >= low_mask(L.w[1])) return false;
  return fits(2, z0) && fits(3, z1) && fits(4, z2);
}

// A received region sorted by actor shard (its sender's batch may carry ordered
// methods): served by the ordered drain; every other region by the parallel one.
__device__ __forceinline__ bool sx_sharded(const uint32_t* region) {
  const uint32_t hw = region[3];
  return ((hw >> 16) & kFlagValid) && ((hw >> 16) & kFlagSharded) && region[0];
}
__device__ __forceinline__ bool sx_any_sharded(const uint32_t* recv, int64_t req_stride, int R) {
  for (int p = 0; p < R; ++p)
    if (sx_sharded(recv + (int64_t)p * req_stride)) return true;
  return false;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t t = (uint32_t)__shfl_xor((int)v, off);
    v = t > v ? t : v;
  }
  return v;
}

// ---------------------------------------------------------------- sender: count
// Registry modes 0/1 (hash probe / directory gather) also leave each message's
// resolved route word ((mailbox << 8) | rank, kDirMissing when unroutable) in
// rw[] -- the chunk's perm column, overwritten by the scatter -- so the scatter
// reads it coalesced instead of repeating the random gather (affine mode 2
// computes its routes and passes rw = null).
template <int MODE>
__global__ __launch_bounds__(kST) void sx_count_kernel(SortIn in, int R, uint32_t K, uint32_t* __restrict__ hist,
                                                       unsigned long long* __restrict__ meta,
                                                       uint32_t* __restrict__ rw) {
  __shared__ uint32_t cnt[kXMaxBuckets];
  __shared__ uint32_t mbmax_s;
  const uint32_t B = (uint32_t)R * K;
  const uint32_t v = virt_block(blockIdx.x, in.G);
  for (uint32_t b = threadIdx.x; b < B; b += kST) cnt[b] = 0;
  if (threadIdx.x == 0) mbmax_s = 0;
  __syncthreads();
  uint32_t mbmax = 0;
  const uint32_t t0 = v * in.tpb, t1 = min(t0 + in.tpb, in.tiles);
  uint32_t a[kSK];
  if (t0 < t1) load_actors(in, t0, a);
  for (uint32_t t = t0; t < t1; ++t) {
    int r[kSK];
    uint32_t mb[kSK];
    resolve_k<MODE>(in, a, r, mb);
    if (t + 1 < t1) load_actors(in, t + 1, a);
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const bool ok = r[k] >= 0 && r[k] < R && mb[k] < kMaxMbox;
      if constexpr (MODE != 2) {
        const int64_t i = tile_index(t, k);
        if (i < in.M) rw[i] = ok ? (mb[k] << 8) | (uint32_t)r[k] : kDirMissing;
      }
      if (ok) {
        atomicAdd(&cnt[(uint32_t)r[k] * K + (mb[k] & (K - 1))], 1u);
        mbmax = mb[k] > mbmax ? mb[k] : mbmax;
      }
    }
  }
  mbmax = wave_max(mbmax);
  if (lane_id() == 0 && mbmax) atomicMax(&mbmax_s, mbmax);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < B; b += kST) hist[(size_t)v * B + b] = cnt[b];
  if (threadIdx.x == 0 && mbmax_s) meta_max(meta + kMetaMbox, mbmax_s);
}

// ---------------------------------------------------------------- sender: scan + region tables
// Block d owns region d's K bucket columns of hist [G][R * K] (K = 64 actor
// shards when the sender's batch may carry ordered methods, else 1): exclusive
// prefix over blocks (in place), the buckets' offsets within the region, its
// shard table (clamped to C) and header, and the region total into meta[kMetaCap].
__global__ __launch_bounds__(1024) void sx_scan_kernel(uint32_t* __restrict__ hist, uint32_t G, int R, uint32_t K,
                                                       uint32_t* __restrict__ sendbuf, int64_t req_stride,
                                                       SxCaps caps, uint32_t method_uniform,
                                                       uint32_t hdr_flags, int rank_self,
                                                       unsigned long long* __restrict__ meta,
                                                       uint32_t* __restrict__ boff) {
  __shared__ uint32_t part[16][64];
  __shared__ uint32_t wsum[16];
  const uint32_t B = (uint32_t)R * K;
  const uint32_t d = blockIdx.x;
  const uint32_t C = caps.c[d];  // this destination's capacity
  constexpr int64_t tab_off = 4;
  uint32_t* region = sendbuf + (int64_t)d * req_stride;
  unsigned long long* pair = meta + kSxMetaPair + rank_self * R + d;
  if (K == 1) {  // one column: every thread a row (G <= 1024), a block-wide scan
    const uint32_t r = threadIdx.x, w = r / kWave, lane = lane_id();
    const uint32_t x = r < G ? hist[(size_t)r * B + d] : 0u;
    const uint32_t inc = wave_incl_scan(x);
    if (lane == kWave - 1) wsum[w] = inc;
    __syncthreads();
    uint32_t off = inc - x;
    for (uint32_t j = 0; j < w; ++j) off += wsum[j];
    if (r < G) hist[(size_t)r * B + d] = off;
    if (r == blockDim.x - 1) {
      const uint32_t all = off + x;
      const uint32_t n = all < C ? all : C;
      boff[d] = 0;
      region[tab_off] = 0;
      for (int s = 1; s <= kSxShards; ++s) region[tab_off + s] = n;
      *reinterpret_cast<uint4*>(region) = make_uint4(n, all, (uint32_t)rank_self, (hdr_flags << 16) | method_uniform);
      if (all) {
        meta_max(meta + kMetaCap, all);
        meta_max(pair, all);
      }
    }
    return;
  }
  const uint32_t lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const uint32_t c = d * K + lane;
  const uint32_t rows = (G + 15) / 16, r0 = min(G, g * rows), r1 = min(G, r0 + rows);
  uint32_t sum = 0;
  {
    uint32_t r = r0;
    for (; r + 8 <= r1; r += 8) {
      uint32_t x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = hist[(size_t)(r + j) * B + c];
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += x[j];
    }
    for (; r < r1; ++r) sum += hist[(size_t)r * B + c];
  }
  part[g][lane] = sum;
  __syncthreads();
  uint32_t run = 0, total = 0;
  for (uint32_t j = 0; j < 16; ++j) {
    if (j < g) run += part[j][lane];
    total += part[j][lane];
  }
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t x = hist[(size_t)r * B + c];
    hist[(size_t)r * B + c] = run;
    run += x;
  }
  if (g == 0) {
    const uint32_t inc = wave_incl_scan(total);
    const uint32_t off = inc - total;
    const uint32_t all = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    boff[c] = off;
    region[tab_off + lane] = off < C ? off : C;
    if (lane == 0) {
      const uint32_t n = all < C ? all : C;
      region[tab_off + kSxShards] = n;
      *reinterpret_cast<uint4*>(region) = make_uint4(n, all, (uint32_t)rank_self, (hdr_flags << 16) | method_uniform);
      if (all) {
        meta_max(meta + kMetaCap, all);
        meta_max(pair, all);
      }
    }
  }
}

// This block's overflow answers into meta[kMetaOverflow] (a count per rank; the
// agreement's MAX then says whether ANY rank must re-send -- send_all reads it
// from the agreement's pinned copy, no count pass and no extra collective).
__device__ __forceinline__ void fold_overflow(uint32_t n, unsigned long long* meta) {
  for (int off = 32; off > 0; off >>= 1) n += __shfl_xor(n, off);
  if (lane_id() == 0 && n) atomicAdd(meta + kMetaOverflow, (unsigned long long)n);
}

// ---------------------------------------------------------------- sender: scatter
template <int MODE, int S>
__global__ __launch_bounds__(kST) void sx_scatter_kernel(SortIn in, int R, uint32_t K, const uint32_t* __restrict__ hist,
                                                         const uint32_t* __restrict__ boff,
                                                         uint32_t* __restrict__ sendbuf, int64_t req_stride,
                                                         uint32_t C, SxCaps caps, PackedLayout L,
                                                         int32_t* __restrict__ perm,
                                                         unsigned long long* __restrict__ meta, bool reject_ordered,
                                                         uint32_t* __restrict__ first_ovf, uint32_t lo) {
  // C: the region stride in records (positions are encoded rk * C + pos);
  // caps: each destination's capacity (<= C) -- a message past it overflows.
  // first_ovf (sharded Sends): per bucket, the smallest Send-wide message index
  // that overflowed (word kXMaxBuckets: zero once any did) -- sx_fifo_fixup_kernel
  // then overflows every later message of that bucket, so each (sender, actor)
  // pair runs a message-order PREFIX and send_all re-sends the suffix in order.
  __shared__ uint32_t cap_s[kSxMaxRanks];
  __shared__ uint32_t run[kXMaxBuckets];
  __shared__ uint32_t bo[kXMaxBuckets];
  __shared__ uint32_t wcnt[kST / kWave][kXMaxBuckets];
  const uint32_t B = (uint32_t)R * K;
  const uint32_t bbits = B > 1 ? 32 - __builtin_clz(B - 1) : 0;  // bucket index bits
  const uint32_t v = virt_block(blockIdx.x, in.G);
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  for (uint32_t b = threadIdx.x; b < B; b += kST) {
    run[b] = hist[(size_t)v * B + b];
    bo[b] = boff[b];
  }
  if (threadIdx.x < (unsigned)kSxMaxRanks) cap_s[threadIdx.x] = caps.c[threadIdx.x];
  MetaAcc acc;
  uint32_t n_ovf = 0;  // messages answered kStatusOverflow (folded into the agreement: send_all's re-send test)
  const uint32_t t0 = v * in.tpb, t1 = min(t0 + in.tpb, in.tiles);
  for (uint32_t t = t0; t < t1; ++t) {
    for (uint32_t b = lane; b < B; b += kWave) wcnt[w][b] = 0;
    // phase 1: routes and ranks only (a small register file: occupancy hides the loads)
    int r[kSK];
    uint32_t mb[kSK];
    if constexpr (MODE == 2) {
      uint32_t a[kSK];
      load_actors(in, t, a);
      resolve_k<MODE>(in, a, r, mb);
    } else {  // the count pass's route words (see sx_count_kernel)
      uint32_t rw[kSK];
#pragma unroll
      for (int k = 0; k < kSK; ++k) {
        const int64_t i = tile_index(t, k);
        rw[k] = i < in.M ? (uint32_t)perm[i] : kDirMissing;
      }
#pragma unroll
      for (int k = 0; k < kSK; ++k) {
        r[k] = rw[k] == kDirMissing ? -1 : (int)(rw[k] & 0xffu);
        mb[k] = rw[k] >> 8;
      }
    }
    // one register per item into phase 2: (rank within the wave's run << 8) | rank
    // (0xff: no such actor) -- the bucket is recomputed from (rank, mailbox)
    uint32_t pr[kSK];
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const bool ok = r[k] >= 0 && r[k] < R && mb[k] < kMaxMbox;
      const uint32_t bk = ok ? (uint32_t)r[k] * K + (mb[k] & (K - 1)) : 0u;
      const uint64_t peers = match_bits(bk, bbits, __ballot(ok));
      const unsigned below = mbcnt64(peers);
      const int leader = peers ? __builtin_ctzll(peers) : 0;
      unsigned old = 0;
      if (ok && below == 0) {
        old = wcnt[w][bk];
        wcnt[w][bk] = old + (unsigned)__popcll(peers);
      }
      pr[k] = ok ? (((unsigned)__shfl((int)old, leader) + below) << 8) | (uint32_t)r[k] : 0xffu;
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < B; b += kST) {
      uint32_t rr = run[b];
#pragma unroll
      for (int ww = 0; ww < kST / kWave; ++ww) {
        const uint32_t c = wcnt[ww][b];
        wcnt[ww][b] = rr;
        rr += c;
      }
      run[b] = rr;
    }
    __syncthreads();
    // phase 2: each message's arguments, packed at its position
#pragma unroll
    for (int k = 0; k < kSK; ++k) {
      const int64_t i = tile_index(t, k);
      if (i >= in.M) continue;
      const uint32_t rk = pr[k] & 0xffu;
      if (rk == 0xffu) {
        perm[i] = -2;  // no such actor: the completion answers kStatusNoActor
        continue;
      }
      const uint32_t bk = rk * K + (mb[k] & (K - 1));
      const uint32_t pos = bo[bk] + wcnt[w][bk] + (pr[k] >> 8);
      if (pos >= cap_s[rk]) {  // past the capacity in force: answered kStatusOverflow, re-sent by send_all
        perm[i] = -1;
        ++n_ovf;
        if (first_ovf) {
          atomicMin(first_ovf + bk, lo + (uint32_t)i);
          atomicMin(first_ovf + kXMaxBuckets, 0u);
        }
        continue;
      }
      const int64_t x0 = __builtin_nontemporal_load(in.a0 + i);
      const int64_t x1 = in.a1 ? __builtin_nontemporal_load(in.a1 + i) : 0;
      const int64_t x2 = in.a2 ? __builtin_nontemporal_load(in.a2 + i) : 0;
      const uint32_t meth = in.mcol ? (uint32_t)in.mcol[i] : in.method_uniform;
      const uint64_t z0 = zz_enc(x0), z1 = zz_enc(x1), z2 = in.a2 ? zz_enc(x2) : 0ull;
      acc.z0 = z0 > acc.z0 ? z0 : acc.z0;
      acc.z1 = z1 > acc.z1 ? z1 : acc.z1;
      if (in.a2) acc.z2 = z2 > acc.z2 ? z2 : acc.z2;
      if (in.mcol) {  // a uniform method is flagged once per batch (meta_publish)
        acc.mm = meth > acc.mm ? meth : acc.mm;
        acc.flags |= 1u << (meth < 7 ? meth : 7);
      }
      uint64_t f[5];
      const bool fit = sx_fits(L, meth, in.method_uniform, mb[k], z0, z1, z2, reject_ordered);
      if (fit) {
        f[0] = meth, f[1] = mb[k], f[2] = z0, f[3] = z1, f[4] = z2;
        perm[i] = (int32_t)(rk * C + pos);
      } else {  // wider than the layout in force: a null record holds the slot
        f[0] = 0, f[1] = low_mask(L.w[1]), f[2] = 0, f[3] = 0, f[4] = 0;
        perm[i] = -1;
        ++n_ovf;
        if (first_ovf) {
          atomicMin(first_ovf + bk, lo + (uint32_t)i);
          atomicMin(first_ovf + kXMaxBuckets, 0u);
        }
      }
      uint32_t rec[S];
      packed_pack<S>(L, f, rec);
      store_words<S>(sendbuf + (int64_t)rk * req_stride + kSxRecOff + (int64_t)pos * S, rec);
    }
    __syncthreads();
  }
  acc.mb = 0;  // the count pass folds the mailboxes
  meta_publish(acc, in.mcol != nullptr, in.method_uniform, in.M, meta);
  fold_overflow(n_ovf, meta);
}

// ---------------------------------------------------------------- sender: FIFO fix-up (sharded Sends)
// After a sharded chunk's scatter: when any message of this Send overflowed
// (first_ovf[kXMaxBuckets] == 0), every PLACED message of this chunk whose
// bucket (destination rank, actor shard) overflowed at an earlier message index
// -- an earlier chunk's capacity, or a field wider than the layout in force --
// becomes a null record and answers kStatusOverflow too.  A record's bucket is
// read back from its region's shard table.  No overflow: one load, exit.
template <int S>
__global__ __launch_bounds__(256) void sx_fifo_fixup_kernel(uint32_t* __restrict__ sendbuf, int64_t req_stride, int R,
                                                            uint32_t C, PackedLayout L, int32_t* __restrict__ perm,
                                                            int64_t m, uint32_t lo,
                                                            const uint32_t* __restrict__ first_ovf,
                                                            unsigned long long* __restrict__ meta) {
  if (__hip_atomic_load(first_ovf + kXMaxBuckets, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
  __shared__ uint32_t tab[kSxMaxRanks][kSxShards + 1];
  __shared__ uint32_t fo[kXMaxBuckets];
  for (uint32_t j = threadIdx.x; j < (uint32_t)R * (kSxShards + 1); j += blockDim.x) {
    const uint32_t q = j / (kSxShards + 1), s = j % (kSxShards + 1);
    tab[q][s] = sendbuf[(int64_t)q * req_stride + 4 + s];
  }
  for (uint32_t b = threadIdx.x; b < (uint32_t)R * kSxShards; b += blockDim.x)
    fo[b] = __hip_atomic_load(first_ovf + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  uint32_t n_ovf = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t p = perm[i];
    if (p < 0) continue;
    const uint32_t rk = (uint32_t)p / C, pos = (uint32_t)p % C;
    uint32_t s = 0;  // the shard whose run holds pos: the last s with tab[rk][s] <= pos
#pragma unroll
    for (uint32_t step = kSxShards / 2; step; step >>= 1)
      if (tab[rk][s + step] <= pos) s += step;
    if (fo[rk * kSxShards + s] < lo + (uint32_t)i) {
      uint64_t f[5] = {0, low_mask(L.w[1]), 0, 0, 0};
      uint32_t rec[S];
      packed_pack<S>(L, f, rec);
      store_words<S>(sendbuf + (int64_t)rk * req_stride + kSxRecOff + (int64_t)pos * S, rec);
      perm[i] = -1;
      ++n_ovf;
    }
  }
  fold_overflow(n_ovf, meta);
}

// ---------------------------------------------------------------- sender: one pass (rank-only batches)
// count + scan + scatter as ONE kernel when the sender sorts by rank alone
// (K = 1: a region is one message-ordered run, so a message's position is its
// tile's prefix within the region plus its rank in the tile -- no region-wide
// totals are needed before writing).  Each block claims the next tile in launch
// order, resolves its messages (the directory gather, once), ranks them per
// destination, publishes the tile's per-destination counts and looks back over
// earlier tiles' descriptors for its prefix (decoupled look-back, as in the
// mailbox sort: mailbox_sort.hip mbx_onesweep_kernel; u64 descriptors {tag 24 |
// status 2 | value 38} through memory-side atomics), then packs and stores its
// records.  The last tile writes the region headers and shard tables, the
// last block to finish advances the epoch tag (every block has read it by then).
//
// reserve (the default for rank-only batches): no look-back.  A rank-only
// region is a queue of stateless records that the receiver runs in parallel,
// so a region need not hold this sender's messages in message order: each
// tile reserves its run in every destination's region with ONE atomicAdd on
// that region's counter (rcnt), and the last block to finish writes the
// headers from the totals (and clears the counters for the next chunk).

// (2048-message tiles and the argument columns loaded with the actors measured no
// faster: removed, profiles/r5_mailbox_ab.md)
template <int MODE, int S, int SK>
__device__ __forceinline__ void sx_onesweep_body(SortIn in, int R, unsigned long long* __restrict__ desc,
                                                 unsigned* __restrict__ tctr, unsigned* __restrict__ ticket,
                                                 uint32_t* __restrict__ sendbuf, int64_t req_stride,
                                                 uint32_t C, SxCaps caps, uint32_t hdr_word3,
                                                 int rank_self, PackedLayout L, int32_t* __restrict__ perm,
                                                 unsigned long long* __restrict__ meta,
                                                 unsigned long long* __restrict__ stats,
                                                 uint32_t* __restrict__ rcnt, bool reserve,
                                                 bool reject_ordered) {
  __shared__ uint32_t wcnt[kST / kWave][kSxMaxRanks];
  __shared__ uint32_t pre[kSxMaxRanks];
  __shared__ uint32_t cap_s[kSxMaxRanks];  // per-destination capacities (C: the region stride in records)
  __shared__ uint32_t tile_s, tag_s, mbmax_s;
  constexpr int64_t tab_off = 4;
  if (threadIdx.x < (unsigned)kSxMaxRanks) cap_s[threadIdx.x] = caps.c[threadIdx.x];
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  if (threadIdx.x == 0) {
    tag_s = epoch_tag(tctr[1]);  // 1..0xffffff across the counter's wrap
    if (!reserve) {
      const uint32_t t = atomicAdd(&tctr[0], 1u);
      if (t == in.tiles - 1) atomicExch(&tctr[0], 0u);  // every block has claimed
      tile_s = t;
    } else {
      tile_s = virt_block(blockIdx.x, gridDim.x);  // (tiles dealt XCD by XCD)
    }
    mbmax_s = 0;
  }
  if (lane < kSxMaxRanks) wcnt[w][lane] = 0;
  __syncthreads();
  const uint32_t t = tile_s, tag = tag_s;
  const uint32_t rbits = R > 1 ? 32 - __builtin_clz((uint32_t)R - 1) : 0;
  // phase 1: routes and ranks (a small register file: occupancy hides the gathers)
  uint32_t pr[SK], mb[SK];
  uint32_t mbmax = 0;
  {
    uint32_t a[SK];
    int r[SK];
    load_actors<SK>(in, t, a);
    resolve_k<MODE, SK>(in, a, r, mb);
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      const bool ok = tile_index<SK>(t, k) < in.M && r[k] >= 0 && r[k] < R && mb[k] < kMaxMbox;
      if (ok) mbmax = mb[k] > mbmax ? mb[k] : mbmax;
      const uint32_t bk = ok ? (uint32_t)r[k] : 0u;
      const uint64_t peers = match_bits(bk, rbits, __ballot(ok));
      const unsigned below = mbcnt64(peers);
      const int leader = peers ? __builtin_ctzll(peers) : 0;
      unsigned old = 0;
      if (ok && below == 0) {
        old = wcnt[w][bk];
        wcnt[w][bk] = old + (unsigned)__popcll(peers);
      }
      pr[k] = ok ? (((unsigned)__shfl((int)old, leader) + below) << 8) | bk : 0xffu;
    }
  }
  mbmax = wave_max(mbmax);
  if (lane == 0 && mbmax) atomicMax(&mbmax_s, mbmax);
  __syncthreads();
  if (threadIdx.x < (unsigned)R) {  // destination d: wave offsets, publish, look back
    const uint32_t d = threadIdx.x;
    uint32_t c = 0;
#pragma unroll
    for (int ww = 0; ww < kST / kWave; ++ww) {
      const uint32_t x = wcnt[ww][d];
      wcnt[ww][d] = c;
      c += x;
    }
    unsigned long long* dp = desc + (size_t)t * R + d;
    uint64_t excl = 0;
    unsigned long long timeouts = 0;
    if (reserve) {
      excl = c ? atomicAdd(&rcnt[d], c) : 0u;  // this tile's run of region d (headers: the last block)
    } else if (t == 0) {
      __hip_atomic_exchange(dp, desc_word(tag, kDescP, c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_exchange(dp, desc_word(tag, kDescA, c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      excl = lookback(desc + d, (uint32_t)R, (int64_t)t - 1, tag, timeouts);
      __hip_atomic_exchange(dp, desc_word(tag, kDescP, excl + c), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
      if (timeouts) atomicAdd(&stats[2], timeouts);
    }
    pre[d] = (uint32_t)excl;
    if (!reserve && t == in.tiles - 1) {  // region d's header and (single-run) shard table
      const uint32_t all = (uint32_t)(excl + c), n = all < cap_s[d] ? all : cap_s[d];
      uint32_t* region = sendbuf + (int64_t)d * req_stride;
      region[tab_off] = 0;
      for (int s2 = 1; s2 <= kSxShards; ++s2) region[tab_off + s2] = n;
      *reinterpret_cast<uint4*>(region) = make_uint4(n, all, (uint32_t)rank_self, hdr_word3);
      if (all) {
        meta_max(meta + kMetaCap, all);
        meta_max(meta + kSxMetaPair + rank_self * R + d, all);
      }
    }
  }
  __syncthreads();
  // phase 2: each message's arguments, packed at its position
  MetaAcc acc;
  uint32_t n_ovf = 0;
#pragma unroll
  for (int k = 0; k < SK; ++k) {
    const int64_t i = tile_index<SK>(t, k);
    if (i >= in.M) continue;
    const uint32_t rk = pr[k] & 0xffu;
    if (rk == 0xffu) {
      perm[i] = -2;  // no such actor: the completion answers kStatusNoActor
      continue;
    }
    const uint32_t pos = pre[rk] + wcnt[w][rk] + (pr[k] >> 8);
    if (pos >= cap_s[rk]) {  // past the capacity in force: answered kStatusOverflow, re-sent by send_all
      perm[i] = -1;
      ++n_ovf;
      continue;
    }
    const int64_t x0 = __builtin_nontemporal_load(in.a0 + i);
    const int64_t x1 = in.a1 ? __builtin_nontemporal_load(in.a1 + i) : 0;
    const int64_t x2 = in.a2 ? __builtin_nontemporal_load(in.a2 + i) : 0;
    const uint32_t meth = in.mcol ? (uint32_t)in.mcol[i] : in.method_uniform;
    const uint64_t z0 = zz_enc(x0), z1 = zz_enc(x1), z2 = in.a2 ? zz_enc(x2) : 0ull;
    acc.z0 = z0 > acc.z0 ? z0 : acc.z0;
    acc.z1 = z1 > acc.z1 ? z1 : acc.z1;
    if (in.a2) acc.z2 = z2 > acc.z2 ? z2 : acc.z2;
    if (in.mcol) {
      acc.mm = meth > acc.mm ? meth : acc.mm;
      acc.flags |= 1u << (meth < 7 ? meth : 7);
    }
    uint64_t f[5];
    const bool fit = sx_fits(L, meth, in.method_uniform, mb[k], z0, z1, z2, reject_ordered);
    if (fit) {
      f[0] = meth, f[1] = mb[k], f[2] = z0, f[3] = z1, f[4] = z2;
      perm[i] = (int32_t)(rk * C + pos);
    } else {  // wider than the layout in force: a null record holds the slot
      f[0] = 0, f[1] = low_mask(L.w[1]), f[2] = 0, f[3] = 0, f[4] = 0;
      perm[i] = -1;
      ++n_ovf;
    }
    uint32_t rec[S];
    packed_pack<S>(L, f, rec);
    store_words<S>(sendbuf + (int64_t)rk * req_stride + kSxRecOff + (int64_t)pos * S, rec);
  }
  acc.mb = mbmax_s;  // (the mailbox maximum of this tile: every lane sees the block's)
  meta_publish(acc, in.mcol != nullptr, in.method_uniform, in.M, meta);
  fold_overflow(n_ovf, meta);
  __shared__ bool last;
  if (threadIdx.x == 0) last = last_block_ticket(ticket);
  __syncthreads();
  if (last && threadIdx.x == 0) tctr[1] += 1u;  // every block has read this launch's tag: the next one's
  if (last && reserve && threadIdx.x < (unsigned)R) {  // every tile has reserved: the regions' headers
    const uint32_t d = threadIdx.x;
    const uint32_t all = atomicExch(&rcnt[d], 0u), n = all < cap_s[d] ? all : cap_s[d];  // (memory-side)
    uint32_t* region = sendbuf + (int64_t)d * req_stride;
    region[tab_off] = 0;
    for (int s2 = 1; s2 <= kSxShards; ++s2) region[tab_off + s2] = n;
    *reinterpret_cast<uint4*>(region) = make_uint4(n, all, (uint32_t)rank_self, hdr_word3);
    if (all) {
      meta_max(meta + kMetaCap, all);
      meta_max(meta + kSxMetaPair + rank_self * R + d, all);
    }
  }
}

#define PT_SX_OS_PARAMS                                                                                        \
  SortIn in, int R, unsigned long long *__restrict__ desc, unsigned *__restrict__ tctr,                          \
      unsigned *__restrict__ ticket, uint32_t *__restrict__ sendbuf, int64_t req_stride, uint32_t C, SxCaps caps, \
      uint32_t hdr_word3, int rank_self, PackedLayout L, int32_t *__restrict__ perm,                             \
      unsigned long long *__restrict__ meta, unsigned long long *__restrict__ stats, uint32_t *__restrict__ rcnt, \
      bool reserve, bool reject_ordered
#define PT_SX_OS_ARGS \
  in, R, desc, tctr, ticket, sendbuf, req_stride, C, caps, hdr_word3, rank_self, L, perm, meta, stats, rcnt, reserve, reject_ordered
// SK messages per thread: kSK (4096-message tiles), or 2 (1024) for a small chunk -- a
// 512 Ki chunk is 128 tiles of 4096, a grid that leaves half the CUs idle
template <int MODE, int S, int SK = kSK>
__global__ __launch_bounds__(kST) void sx_onesweep_kernel(PT_SX_OS_PARAMS) {
  sx_onesweep_body<MODE, S, SK>(PT_SX_OS_ARGS);
}
#undef PT_SX_OS_PARAMS
#undef PT_SX_OS_ARGS

// ---------------------------------------------------------------- receiver: parallel drain
// grid (X, R): block (x, p) strides over source p's region in 64-record groups
// per wave; a reply lands at its request's position (one ok-bitmap word per group).
template <int S, int FIXED>
__device__ __forceinline__ unsigned long long sx_drain_range(const uint32_t* rq, int64_t count, uint32_t hm,
                                                             const PackedLayout& L, uint8_t* vals,
                                                             unsigned long long* okmap, int64_t* state,
                                                             uint32_t n_state, uint64_t delay_ticks,
                                                             unsigned long long& toowide) {
  unsigned long long failed = 0;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const unsigned lane = lane_id();
  const uint64_t null_mb = low_mask(L.w[1]);
  for (int64_t base = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~(kWave - 1)); base < count;
       base += step * kXDispU) {
    uint32_t wv[kXDispU][S];
#pragma unroll
    for (int u = 0; u < kXDispU; ++u) {
      const int64_t s = base + u * step + lane;
      if (s < count) load_words<S>(rq + kSxRecOff + s * S, wv[u]);
    }
#pragma unroll
    for (int u = 0; u < kXDispU; ++u) {
      const int64_t gb = base + u * step;
      if (gb >= count) break;
      const int64_t s = gb + lane;
      const bool in = s < count;
      ReplyRecord rr;
      rr.value = 0;
      rr.status = kStatusOk;
      bool null = false;
      if (in) {
        const uint64_t mbf = packed_field<S>(L, 1, wv[u]);
        null = mbf == null_mb;
        if (!null) {
          MsgRecord m;
          m.actor = (uint32_t)mbf;
          m.method = (uint16_t)(FIXED ? FIXED : (L.w[0] ? (uint32_t)packed_field<S>(L, 0, wv[u]) : hm));
          m.flags = kFlagValid | kFlagRouted;
          m.a0 = zz_dec(packed_field<S>(L, 2, wv[u]));
          m.a1 = zz_dec(packed_field<S>(L, 3, wv[u]));
          m.a2 = zz_dec(packed_field<S>(L, 4, wv[u]));
          rr = run_handler(m, state, n_state, delay_ticks);
        } else {
          rr.status = kStatusOverflow;  // nobody reads it: the sender answered this one itself
        }
      }
      bool ok = rr.status == kStatusOk;
      uint64_t code = ok ? (L.vb == 8 ? (uint64_t)rr.value : zz_enc(rr.value)) : (uint64_t)rr.status;
      if (ok && L.vb < 8 && (code >> (8 * L.vb))) {  // impossible under the agreed bounds: fail loudly
        ok = false;
        code = kStatusFailed;
        toowide += in;
      }
      failed += in && !ok && !null;
      const unsigned long long bits = __ballot(in && ok);
      if (in) {
        switch (L.vb) {
          case 1: vals[s] = (uint8_t)code; break;
          case 2: reinterpret_cast<uint16_t*>(vals)[s] = (uint16_t)code; break;
          case 4: reinterpret_cast<uint32_t*>(vals)[s] = (uint32_t)code; break;
          default: reinterpret_cast<uint64_t*>(vals)[s] = code;
        }
      }
      if (lane == 0) okmap[gb / kWave] = bits;
    }
  }
  return failed;
}

template <int S>
__global__ __launch_bounds__(256) void sx_drain_par_kernel(const uint32_t* __restrict__ recv, int64_t req_stride,
                                                           int64_t C, PackedLayout L, int R, bool may_order,
                                                           uint32_t* __restrict__ reply, int64_t rep_stride,
                                                           int64_t* __restrict__ state, uint32_t n_state,
                                                           uint64_t delay_ticks, unsigned long long* __restrict__ stats) {
  const int p = blockIdx.y;
  const uint32_t* rq = recv + (int64_t)p * req_stride;
  if (may_order && sx_sharded(rq)) {  // the ordered drain (launched next) serves this region:
    if (blockIdx.x == 0) {            // its reply header and zeroed ok bitmap first (it sets bits one record at a time)
      const uint4 h = *reinterpret_cast<const uint4*>(rq);
      const int64_t count = ((h.w >> 16) & kFlagValid) ? (int64_t)(h.x < C ? h.x : C) : 0;
      uint32_t* rp = reply + (int64_t)p * rep_stride;
      if (threadIdx.x == 0) *reinterpret_cast<uint4*>(rp) = make_uint4((uint32_t)count, 0u, 0u, 0u);
      for (int64_t j = threadIdx.x; j < packed_ok_words(count); j += blockDim.x) rp[4 + j] = 0u;
    }
    return;
  }
  const uint4 h = *reinterpret_cast<const uint4*>(rq);
  const int64_t count = ((h.w >> 16) & kFlagValid) ? (int64_t)(h.x < C ? h.x : C) : 0;
  const uint32_t hm = h.w & 0xffffu;
  uint32_t* rp = reply + (int64_t)p * rep_stride;
  unsigned long long* okmap = reinterpret_cast<unsigned long long*>(rp + 4);
  uint8_t* vals = reinterpret_cast<uint8_t*>(rp + 4 + packed_ok_words(count));
  if (blockIdx.x == 0 && threadIdx.x == 0) *reinterpret_cast<uint4*>(rp) = make_uint4((uint32_t)count, 0u, 0u, 0u);
  unsigned long long toowide = 0, failed;
  if (!L.w[0] && hm == kCalculatorMultiply)
    failed = sx_drain_range<S, kCalculatorMultiply>(rq, count, hm, L, vals, okmap, state, n_state, delay_ticks, toowide);
  else
    failed = sx_drain_range<S, 0>(rq, count, hm, L, vals, okmap, state, n_state, delay_ticks, toowide);
  for (int off = 32; off > 0; off >>= 1) {
    failed += __shfl_xor(failed, off);
    toowide += __shfl_xor(toowide, off);
  }
  if (lane_id() == 0 && failed) atomicAdd(&stats[0], failed);
  if (lane_id() == 0 && toowide) atomicAdd(&stats[1], toowide);
}

// ---------------------------------------------------------------- receiver: ordered drain
// Launched after the parallel drain, which wrote the sharded regions' reply
// headers and zeroed their ok bitmaps (one launch less per chunk than a
// separate init kernel).  grid: one block per actor shard.
struct SxOrdLds {
  uint32_t wcnt[kXOrdWaves][kXOrdThreads];
  uint32_t bstart[kXOrdThreads];
  uint32_t bcount[kXOrdThreads];
  uint32_t wsum[kXOrdWaves];
  uint32_t pos[kXOrdWin];
  uint32_t act[kXOrdWin];
  uint32_t meth[kXOrdWin];
  int64_t a0[kXOrdWin], a1[kXOrdWin], a2[kXOrdWin];
};

template <int S>
__global__ __launch_bounds__(kXOrdThreads) void sx_drain_ord_kernel(const uint32_t* __restrict__ recv,
                                                                    int64_t req_stride, int64_t tab_off, int64_t C,
                                                                    PackedLayout L, int R,
                                                                    uint32_t* __restrict__ reply, int64_t rep_stride,
                                                                    int64_t* __restrict__ state, uint32_t n_state,
                                                                    uint64_t delay_ticks,
                                                                    unsigned long long* __restrict__ stats) {
  if (!sx_any_sharded(recv, req_stride, R)) return;
  extern __shared__ __align__(16) unsigned char smem_sx[];
  SxOrdLds& Ls = *reinterpret_cast<SxOrdLds*>(smem_sx);
  int64_t* st_lds = reinterpret_cast<int64_t*>(smem_sx + sizeof(SxOrdLds));
  const uint32_t s = blockIdx.x;
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  const uint32_t n_loc = (state && s < n_state) ? (n_state - 1 - s) / kSxShards + 1 : 0;
  const bool in_lds = state && n_loc <= kXOrdStateMax;
  if (in_lds)
    for (uint32_t j = threadIdx.x; j < n_loc; j += kXOrdThreads) st_lds[j] = state[s + (uint64_t)j * kSxShards];
  __syncthreads();
  const uint64_t null_mb = low_mask(L.w[1]);
  unsigned long long failed = 0;
  for (int p = 0; p < R; ++p) {  // source-rank order: every (sender, actor) pair stays FIFO
    const uint32_t* rq = recv + (int64_t)p * req_stride;
    if (!sx_sharded(rq)) continue;  // (a region of a batch without ordered methods: the parallel drain's)
    const uint4 h = *reinterpret_cast<const uint4*>(rq);
    const int64_t count = (int64_t)(h.x < C ? h.x : C);
    const uint32_t hm = h.w & 0xffffu;
    const uint32_t lo = min((int64_t)rq[tab_off + s], count), hi = min((int64_t)rq[tab_off + s + 1], count);
    uint32_t* rp = reply + (int64_t)p * rep_stride;
    unsigned long long* okmap = reinterpret_cast<unsigned long long*>(rp + 4);
    uint8_t* vals = reinterpret_cast<uint8_t*>(rp + 4 + packed_ok_words(count));
    for (uint32_t w0 = lo; w0 < hi; w0 += kXOrdWin) {
      for (uint32_t b = lane; b < kXOrdThreads; b += kWave) Ls.wcnt[w][b] = 0;
      uint32_t q[kXOrdK], bin[kXOrdK], wr[kXOrdK], mbv[kXOrdK], mv[kXOrdK];
      int64_t x0[kXOrdK], x1[kXOrdK], x2[kXOrdK];
      bool valid[kXOrdK];
#pragma unroll
      for (int k = 0; k < kXOrdK; ++k) {  // wave w owns window positions [w * 64K, (w+1) * 64K)
        q[k] = w0 + w * (kWave * kXOrdK) + k * kWave + lane;
        valid[k] = q[k] < hi;
        uint32_t rec[S];
        if (valid[k]) {
          load_words<S>(rq + kSxRecOff + (int64_t)q[k] * S, rec);
          const uint64_t mbf = packed_field<S>(L, 1, rec);
          valid[k] = mbf != null_mb;
          mbv[k] = (uint32_t)mbf;
          mv[k] = L.w[0] ? (uint32_t)packed_field<S>(L, 0, rec) : hm;
          x0[k] = zz_dec(packed_field<S>(L, 2, rec));
          x1[k] = zz_dec(packed_field<S>(L, 3, rec));
          x2[k] = zz_dec(packed_field<S>(L, 4, rec));
        }
      }
#pragma unroll
      for (int k = 0; k < kXOrdK; ++k) {
        bin[k] = valid[k] ? (mbv[k] >> kSxShardBits) & (kXOrdThreads - 1) : 0u;
        const uint64_t peers = match_bits(bin[k], 9, __ballot(valid[k]));
        const unsigned below = mbcnt64(peers);
        const int leader = peers ? __builtin_ctzll(peers) : 0;
        unsigned old = 0;
        if (valid[k] && below == 0) {
          old = Ls.wcnt[w][bin[k]];
          Ls.wcnt[w][bin[k]] = old + (unsigned)__popcll(peers);
        }
        wr[k] = (unsigned)__shfl((int)old, leader) + below;
      }
      __syncthreads();
      {
        const unsigned b = threadIdx.x;
        unsigned r = 0;
#pragma unroll
        for (int ww = 0; ww < kXOrdWaves; ++ww) {
          const unsigned c = Ls.wcnt[ww][b];
          Ls.wcnt[ww][b] = r;
          r += c;
        }
        Ls.bcount[b] = r;
        const unsigned inc = wave_incl_scan(r);
        if (lane == kWave - 1) Ls.wsum[w] = inc;
        __syncthreads();
        unsigned off = inc - r;
        for (unsigned ww = 0; ww < w; ++ww) off += Ls.wsum[ww];
        Ls.bstart[b] = off;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kXOrdK; ++k) {
        if (!valid[k]) continue;
        const unsigned d = Ls.bstart[bin[k]] + Ls.wcnt[w][bin[k]] + wr[k];
        Ls.pos[d] = q[k];
        Ls.act[d] = in_lds ? (mbv[k] >> kSxShardBits) : mbv[k];
        Ls.meth[d] = mv[k];
        Ls.a0[d] = x0[k];
        Ls.a1[d] = x1[k];
        Ls.a2[d] = x2[k];
      }
      __syncthreads();
      if (in_lds && n_loc <= (uint32_t)kXOrdThreads && !L.w[0] && hm == kSeqFold) {
        // a uniform SeqFold region with one actor per bin: thread b folds actor b's
        // messages with the state in a register (mailbox_sort.hip, the same fold)
        const unsigned b = threadIdx.x, e = Ls.bstart[b] + Ls.bcount[b];
        uint64_t sreg = b < n_loc ? (uint64_t)st_lds[b] : 0ull;
        for (unsigned d = Ls.bstart[b]; d < e; ++d) {
          const bool mine = Ls.act[d] == b && b < n_loc;
          const uint64_t prev = sreg;
          if (mine) sreg = prev * kFoldMul + (uint64_t)Ls.a0[d];
          bool ok = mine;
          uint64_t code = ok ? (L.vb == 8 ? prev : zz_enc((int64_t)prev)) : (uint64_t)kStatusNoActor;
          if (ok && L.vb < 8 && (code >> (8 * L.vb))) {
            ok = false;
            code = kStatusFailed;
          }
          failed += !ok;
          const uint32_t qq = Ls.pos[d];
          switch (L.vb) {
            case 1: vals[qq] = (uint8_t)code; break;
            case 2: reinterpret_cast<uint16_t*>(vals)[qq] = (uint16_t)code; break;
            case 4: reinterpret_cast<uint32_t*>(vals)[qq] = (uint32_t)code; break;
            default: reinterpret_cast<uint64_t*>(vals)[qq] = code;
          }
          if (ok) atomicOr(&okmap[qq / kWave], 1ull << (qq % kWave));
        }
        if (b < n_loc) st_lds[b] = (int64_t)sreg;
      } else {
        const unsigned b = threadIdx.x, e = Ls.bstart[b] + Ls.bcount[b];
        int64_t* st = in_lds ? st_lds : state;
        const uint32_t nst = in_lds ? n_loc : n_state;
        for (unsigned d = Ls.bstart[b]; d < e; ++d) {
          MsgRecord m;
          m.actor = Ls.act[d];
          m.method = (uint16_t)Ls.meth[d];
          m.flags = kFlagValid | kFlagRouted;
          m.a0 = Ls.a0[d], m.a1 = Ls.a1[d], m.a2 = Ls.a2[d];
          const ReplyRecord rr = run_handler(m, st, nst, delay_ticks, OutboxView(), true);
          bool ok = rr.status == kStatusOk;
          uint64_t code = ok ? (L.vb == 8 ? (uint64_t)rr.value : zz_enc(rr.value)) : (uint64_t)rr.status;
          if (ok && L.vb < 8 && (code >> (8 * L.vb))) {
            ok = false;
            code = kStatusFailed;
          }
          failed += !ok;
          const uint32_t qq = Ls.pos[d];
          switch (L.vb) {
            case 1: vals[qq] = (uint8_t)code; break;
            case 2: reinterpret_cast<uint16_t*>(vals)[qq] = (uint16_t)code; break;
            case 4: reinterpret_cast<uint32_t*>(vals)[qq] = (uint32_t)code; break;
            default: reinterpret_cast<uint64_t*>(vals)[qq] = code;
          }
          if (ok) atomicOr(&okmap[qq / kWave], 1ull << (qq % kWave));
          if (!in_lds) vm_drain();
        }
      }
      __syncthreads();
    }
  }
  if (in_lds)
    for (uint32_t j = threadIdx.x; j < n_loc; j += kXOrdThreads) state[s + (uint64_t)j * kSxShards] = st_lds[j];
  for (int off = 32; off > 0; off >>= 1) failed += __shfl_xor(failed, off);
  if (lane_id() == 0 && failed) atomicAdd(&stats[0], failed);
}

// ---------------------------------------------------------------- host
SortedExchange::SortedExchange(int device, uintptr_t comm, int R, int rank, int64_t max_chunk, int chunks,
                               int64_t C_alloc, int64_t C0, std::shared_ptr<HostComm> fake)
    : device_(device), cell_(reinterpret_cast<CommCell*>(comm)), fake_(std::move(fake)), R_(R), rank_(rank), chunks_(chunks),
      max_chunk_(max_chunk), C_alloc_(C_alloc) {
  if (R < 1 || R > kSxMaxRanks) throw std::invalid_argument("SortedExchange: 1 <= ranks <= 16");
  if (chunks < 1 || chunks > kSxMaxChunks) throw std::invalid_argument("SortedExchange: 1 <= chunks <= 4");
  if (max_chunk < 1 || C_alloc < 64 || C0 < 1 || C0 > C_alloc) throw std::invalid_argument("SortedExchange: geometry");
  if (C_alloc > 0x7fffffff / R) throw std::invalid_argument("SortedExchange: R * C must fit an int32 position");
  if (fake_ && (cell_ || fake_->size() != R || rank < 0 || rank >= R))
    throw std::invalid_argument("SortedExchange: fake communicator must match R and replace comm");
  if (!fake_ && !cell_) throw std::invalid_argument("SortedExchange: needs a communicator (RCCL or FakeComm)");
  if (cell_ && (!rccl().alltoall || !rccl().allreduce))
    throw std::runtime_error("SortedExchange: RCCL entry points not found in the process");
  PT_HIP_CHECK(hipSetDevice(device_));
  int lo = 0, hi = 0;
  PT_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  PT_HIP_CHECK(hipStreamCreateWithPriority(&comm_stream_, hipStreamNonBlocking, hi));
  const int64_t rq = sx_req_words(C_alloc, 8), rp = packed_rep_words(C_alloc, 8);
  for (int i = 0; i < chunks_; ++i) {
    Bufs& b = bufs_[i];
    PT_HIP_CHECK(hipMalloc(&b.send, (size_t)R * rq * 4));
    PT_HIP_CHECK(hipMalloc(&b.recv, (size_t)R * rq * 4));
    PT_HIP_CHECK(hipMalloc(&b.reply, (size_t)R * rp * 4));
    PT_HIP_CHECK(hipMalloc(&b.back, (size_t)R * rp * 4));
    PT_HIP_CHECK(hipMalloc(&b.perm, (size_t)max_chunk * 4));
    // The compute -> comm-stream hand-offs (routed, served) publish the request and
    // reply regions to a reader on this device: RCCL's own send kernel here (it
    // stages them through its FIFO; no peer reads a user buffer) or the loopback
    // copy.  The comm -> compute hand-offs (req_in, rep_in) publish what RCCL's
    // receive kernel (or the loopback copy) wrote here.  Their events drop the
    // system-scope fence (-3.5 % of the loopback-8 step for the first pair,
    // profiles/r5_mailbox_ab.md).  IpcComm's peers read and write the regions in
    // place from their own processes, so a device-side comm keeps it.
    const bool sys_fence = fake_ && fake_->device_side();
    const unsigned flags = hipEventDisableTiming | (sys_fence ? 0u : hipEventDisableSystemFence);
    const unsigned out_flags = flags, in_flags = flags;
    for (hipEvent_t* e : {&ev_routed_[i], &ev_served_[i]}) PT_HIP_CHECK(hipEventCreateWithFlags(e, out_flags));
    for (hipEvent_t* e : {&ev_req_in_[i], &ev_rep_in_[i]}) PT_HIP_CHECK(hipEventCreateWithFlags(e, in_flags));
  }
  PT_HIP_CHECK(hipMalloc(&hist_, (size_t)kMboxSortHistWords * 4));
  PT_HIP_CHECK(hipMalloc(&boff_, (size_t)kXMaxBuckets * 4));
  const int64_t max_tiles = (max_chunk + kSTile - 1) / kSTile;
  PT_HIP_CHECK(hipMalloc(&desc_, (size_t)std::max<int64_t>(max_tiles, 1) * R * 8));
  PT_HIP_CHECK(hipMemset(desc_, 0, (size_t)std::max<int64_t>(max_tiles, 1) * R * 8));  // tag 0: never a live tag
  PT_HIP_CHECK(hipMalloc(&tctr_, 2 * sizeof(unsigned)));
  PT_HIP_CHECK(hipMemset(tctr_, 0, 2 * sizeof(unsigned)));
  PT_HIP_CHECK(hipMalloc(&ticket_, kTicketWords * sizeof(unsigned)));
  PT_HIP_CHECK(hipMemset(ticket_, 0, kTicketWords * sizeof(unsigned)));
  PT_HIP_CHECK(hipMalloc(&first_ovf_, (kXMaxBuckets + 1) * sizeof(uint32_t)));
  PT_HIP_CHECK(hipMalloc(&rcnt_, kSxMaxChunks * kSxMaxRanks * sizeof(uint32_t)));
  PT_HIP_CHECK(hipMemset(rcnt_, 0, kSxMaxChunks * kSxMaxRanks * sizeof(uint32_t)));
  PT_HIP_CHECK(hipMalloc(&meta_dev_, 2 * kSxMetaWords * sizeof(uint64_t)));
  PT_HIP_CHECK(hipMemset(meta_dev_, 0, 2 * kSxMetaWords * sizeof(uint64_t)));
  PT_HIP_CHECK(hipMalloc(&stats_, 3 * sizeof(unsigned long long)));
  PT_HIP_CHECK(hipMemset(stats_, 0, 3 * sizeof(unsigned long long)));
  PT_HIP_CHECK(hipHostMalloc(&meta_host_, 2 * kSxMetaWords * sizeof(uint64_t), hipHostMallocDefault));
  memset(meta_host_, 0, 2 * kSxMetaWords * sizeof(uint64_t));
  for (auto& e : ev_meta_) PT_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  PT_HIP_CHECK(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
  // start-up layout: every column at full width (8-dword records, 8-byte replies)
  uint64_t wide[kMetaWords] = {};
  wide[kMetaMbox] = (kMaxMbox >> 1) - 1;  // (sx_layout: 24-bit field, every mailbox below kMaxMbox - 1)
  for (int j = 0; j < 3; ++j) wide[kMetaArg0 + j] = ~0ull;
  wide[kMetaMethod] = 0xffff;
  wide[kMetaMcol] = 1;
  for (int m = 0; m < 8; ++m) wide[kMetaFlags + m] = 1;
  L_ = sx_layout(wide);
  C_ = C0;
  for (auto& c : cap_) c = (uint32_t)C0;
}

SortedExchange::~SortedExchange() {
  (void)hipSetDevice(device_);
  // RCCL: no synchronisation (a collective stuck on a dead peer must not hang the
  // owner).  A device-side comm's waits end at its timeout: drain them, so no
  // kernel of this engine still reads buffers freed below.
  if (fake_ && fake_->device_side()) (void)hipStreamSynchronize(comm_stream_);
  for (int i = 0; i < chunks_; ++i) {
    Bufs& b = bufs_[i];
    for (void* p : {(void*)b.send, (void*)b.recv, (void*)b.reply, (void*)b.back, (void*)b.perm}) (void)hipFree(p);
    for (hipEvent_t e : {ev_routed_[i], ev_req_in_[i], ev_served_[i], ev_rep_in_[i]}) (void)hipEventDestroy(e);
  }
  for (hipEvent_t e : ev_meta_) (void)hipEventDestroy(e);
  (void)hipEventDestroy(ev_join_);
  (void)hipFree(hist_);
  (void)hipFree(boff_);
  (void)hipFree(desc_);
  (void)hipFree(tctr_);
  (void)hipFree(ticket_);
  (void)hipFree(rcnt_);
  (void)hipFree(first_ovf_);
  (void)hipFree(meta_dev_);
  (void)hipFree(stats_);
  (void)hipHostFree(meta_host_);
  (void)hipStreamDestroy(comm_stream_);
}

std::vector<uint64_t> SortedExchange::stats() const {
  unsigned long long h[3] = {0, 0, 0};
  PT_HIP_CHECK(hipMemcpy(h, stats_, sizeof h, hipMemcpyDeviceToHost));
  return {h[0], h[1], h[2]};
}

void SortedExchange::set_epoch_counter(uint32_t v) {
  PT_HIP_CHECK(hipSetDevice(device_));
  PT_HIP_CHECK(hipDeviceSynchronize());
  PT_HIP_CHECK(hipMemcpy(tctr_ + 1, &v, sizeof v, hipMemcpyHostToDevice));
}

uint32_t SortedExchange::epoch_counter() const {
  uint32_t v = 0;
  PT_HIP_CHECK(hipSetDevice(device_));
  PT_HIP_CHECK(hipMemcpy(&v, tctr_ + 1, sizeof v, hipMemcpyDeviceToHost));
  return v;
}

static uint64_t sx_now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// A host wait on this engine's event that a retired generation ends: RCCL kernels
// return once the DataPlane aborted the communicator, and the poll sees the cell's
// poison first (no host wait outlives a peer failure the watchdog caught).
void SortedExchange::wait_event(hipEvent_t e) const {
  for (int spin = 0;; ++spin) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) PT_HIP_CHECK(q);
    if (cell_ && cell_->failed()) throw std::runtime_error("ncclRemoteError: the data-plane generation was aborted");
    if (spin > 256) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

uint64_t SortedExchange::last_overflow() const { return sends_ > 0 ? overflow_of(sends_ - 1) : 0; }

uint64_t SortedExchange::overflow_of(int64_t k) const {
  if (k < 0 || k >= sends_) return 0;
  const int j = (int)(k & 1);
  if (meta_send_[j] != k) throw std::runtime_error("SortedExchange: no agreement of that Send (captured, or reused)");
  const uint64_t t0 = sx_now_ns();
  wait_event(ev_meta_[j]);
  prof_.overflow_waits += 1;
  prof_.overflow_wait_ns += sx_now_ns() - t0;
  return meta_host_[j * kSxMetaWords + kMetaOverflow];
}

void SortedExchange::adopt(const uint64_t* meta, int64_t from) {
  L_ = sx_layout(meta);
  // the busiest bucket of the last kNeedWindow agreements: a small Send (send_all's
  // re-send of a few overflowed messages) must not shrink the capacity of the full
  // Sends after it.  Every rank sees the same agreements, so all derive the same C.
  const int h = need_n_++ % kNeedWindow;
  need_hist_[h] = meta[kMetaCap];
  const int RR = R_ * R_;
  std::copy(meta + kSxMetaPair, meta + kSxMetaPair + RR, pair_hist_[h]);
  // the busiest bucket two Sends ago plus 1 % and 8 sigma: uniform traffic then
  // overflows with probability ~1e-15 per bucket, and skewed traffic that is
  // stable over a few Sends fits as well
  auto capacity = [&](uint64_t need) {
    int64_t c = (int64_t)((double)need * 1.01 + 8.0 * sqrt((double)need) + 64.0);
    c = ((c + 63) / 64) * 64;
    return std::max<int64_t>(64, std::min<int64_t>(c, C_alloc_));
  };
  uint64_t busiest = 0;
  for (int j = 0; j < kNeedWindow && j < need_n_; ++j) busiest = std::max(busiest, need_hist_[j]);
  C_ = capacity(busiest);
  // per pair (sender p -> destination q): the same rule over that pair's totals.
  // Under skew (one hot destination) the uniform C moves every pair at the hot
  // pair's size; prefixes of per-pair capacities move what the traffic needs.
  // Worth it only when the bytes saved are real: every rank evaluates the same
  // matrix, so all take the same decision.
  int64_t sum_pairs = 0;
  for (int k = 0; k < RR; ++k) {
    uint64_t need = 0;
    for (int j = 0; j < kNeedWindow && j < need_n_; ++j) need = std::max(need, pair_hist_[j][k]);
    cap_[k] = (uint32_t)std::min<int64_t>(capacity(need), C_);
    sum_pairs += cap_[k];
  }
  // (loopback: one rank stands for a symmetric node and only its own row is filled -- the
  // decision is taken on that row)
  if (fake_ && fake_->loopback()) {
    sum_pairs = 0;
    for (int q = 0; q < R_; ++q) sum_pairs += (int64_t)R_ * cap_[rank_ * R_ + q];
  }
  pairs_ = R_ > 1 && (double)sum_pairs < 0.85 * (double)C_ * RR;
  if (!pairs_)
    for (int k = 0; k < RR; ++k) cap_[k] = (uint32_t)C_;
  agreed_ = true;
  spec_from_ = from;
  std::copy(meta, meta + kMetaWords, spec_meta_);
}

void SortedExchange::pick_spec(hipStream_t cs) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(cs, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone) return;
  // Send k uses the agreement of Send k - 2 (a fixed lag: every rank derives
  // the same geometry); it has normally completed long ago
  const int64_t want = sends_ - 2;
  if (want < 0) return;
  const int j = (int)(want & 1);
  if (meta_send_[j] != want) return;  // recorded under a graph capture: keep the layout in force
  const uint64_t t0 = sx_now_ns();
  wait_event(ev_meta_[j]);
  prof_.spec_wait_ns += sx_now_ns() - t0;
  adopt(meta_host_ + j * kSxMetaWords, want);
}

void SortedExchange::a2a(const void* src, void* dst, size_t stride, const size_t* send, const size_t* recv,
                         bool grouped_p2p) {
  if (fake_) {
    if (send) fake_->alltoallv(rank_, src, dst, stride, send, recv, cur_comm_);
    else fake_->alltoall(rank_, src, dst, stride, cur_comm_);
    return;
  }
  // tune sx_self_copy: at world 1 the all-to-all is a device copy.  RCCL
  // collectives issued on this engine's comm stream crash hipGraph
  // instantiation on this stack (ncclAllToAll and grouped send / recv alike,
  // tools/rccl_capture_probe.py, profiles/r3_rccl_capture_probe.txt), so the
  // capture test validates the captured pipeline with the copy in their place.
  if (self_copy_ && R_ == 1) {
    PT_HIP_CHECK(hipMemcpyAsync(dst, src, recv ? recv[0] : stride, hipMemcpyDeviceToDevice, cur_comm_));
    return;
  }
  auto check = [](int rc, const char* what) {
    if (rc != 0)
      throw std::runtime_error(std::string(what) + " failed: " + (rccl().errstr ? rccl().errstr(rc) : std::to_string(rc)));
  };
  CellUse u(cell_);
  if ((grouped_p2p || send) && rccl().p2p()) {
    // per-pair prefixes (send / recv sizes), or under a hipGraph capture:
    // ncclAllToAll's captured form crashed graph instantiation here (RCCL 2.26;
    // tools/rccl_capture_probe.py) while grouped ncclSend / ncclRecv -- what
    // torch captures -- instantiate and replay
    check(rccl().group_start(), "ncclGroupStart");
    for (int q = 0; q < R_; ++q) {
      check(rccl().send((const char*)src + (size_t)q * stride, send ? send[q] : stride, kNcclInt8, q, u.comm,
                        cur_comm_), "ncclSend");
      check(rccl().recv((char*)dst + (size_t)q * stride, recv ? recv[q] : stride, kNcclInt8, q, u.comm, cur_comm_),
            "ncclRecv");
    }
    check(rccl().group_end(), "ncclGroupEnd");
    return;
  }
  if (send) throw std::runtime_error("SortedExchange: per-pair sizes need RCCL's grouped send / recv");
  check(rccl().alltoall(src, dst, stride, kNcclInt8, u.comm, cur_comm_), "ncclAllToAll");
}

void SortedExchange::allreduce_meta(uint64_t* dev, hipStream_t s) {
  if (fake_) {
    fake_->allreduce_max(rank_, dev, kSxMetaPair + R_ * R_, s);
    return;
  }
  CellUse u(cell_);
  const int rc = rccl().allreduce(dev, dev, kSxMetaPair + R_ * R_, kNcclUint64, kNcclMax, u.comm, s);
  if (rc != 0)
    throw std::runtime_error(std::string("ncclAllReduce failed: ") + (rccl().errstr ? rccl().errstr(rc) : std::to_string(rc)));
}

void SortedExchange::send(const SxSend& a) {
  const uint64_t t_enter = sx_now_ns();
  struct Tally {  // every return path counts the call
    HostProfile& p;
    uint64_t t0;
    ~Tally() {
      p.sends += 1;
      p.total_ns += sx_now_ns() - t0;
    }
  } tally{prof_, t_enter};
  if (a.M < 0 || a.M > max_chunk_ * chunks_) throw std::invalid_argument("SortedExchange: batch exceeds max_batch");
  if (a.M > 0 && (!a.actor || !a.a0)) throw std::invalid_argument("SortedExchange: actor and a0 columns required");
  if (a.cap == 0 || (a.cap & (a.cap - 1))) throw std::invalid_argument("table capacity must be a power of two");
  PT_HIP_CHECK(hipSetDevice(device_));
  if (fake_) fake_->check();  // an earlier collective's failure surfaces here (IpcComm: a peer missed one)
  const hipStream_t cs = as_stream(a.stream);
  // Under a hipGraph capture the collectives go on the capturing stream itself: RCCL calls on a
  // stream forked into the capture crash graph instantiation on this stack, issued on the
  // capture stream they instantiate and replay correctly (tools/rccl_capture_probe.py sx1cs,
  // profiles/r3_rccl_capture_probe.txt) -- the captured Send then runs its chunks' collectives in
  // order with their compute instead of beside it.
  const Tune tn = tune();
  // Small Sends put their collectives on the caller's stream: a Send of up to
  // kSxSmallSend messages is bound by its ~26 HIP calls (~90 us of host time, eight
  // of them cross-stream event hand-offs), not by its bytes -- on one stream it
  // issues 15 calls (~31 us) and its GPU side loses the hand-off gaps (loopback-8,
  // 256 Ki / 1 Mi msgs per rank: 0.120 -> 0.089 / 0.130 -> 0.103 ms per step,
  // profiles/r6_small_sends.md).  Larger Sends keep the comm stream, whose
  // all-to-alls overlap the other chunk's kernels.  A per-rank choice: RCCL matches
  // collectives by their order on the communicator, not by stream (the switch from
  // the comm stream joins it first, below).
  // tune sx_comm_cs: -1 auto (the rule above), 0 never, 1 always (a graph-capture probe:
  // tools/rccl_capture_probe.py sx1cs)
  const bool comm_on_cs = tn.sx_comm_cs > 0 || (tn.sx_comm_cs < 0 && a.M <= kSxSmallSend);
  self_copy_ = tn.sx_self_copy != 0;
  hipStreamCaptureStatus capst = hipStreamCaptureStatusNone;
  const bool capturing = hipStreamIsCapturing(cs, &capst) == hipSuccess && capst != hipStreamCaptureStatusNone;
  cur_comm_ = (comm_on_cs || (capturing && cell_)) ? cs : comm_stream_;
  if (cur_comm_ == cs && last_comm_ == comm_stream_ && !capturing) {
    // the comm stream's last collectives (the previous Send's agreement) ahead of this
    // Send's on the caller's stream: one communicator, one order of execution
    PT_HIP_CHECK(hipEventRecord(ev_join_, comm_stream_));
    PT_HIP_CHECK(hipStreamWaitEvent(cs, ev_join_, 0));
  }
  if (!capturing) last_comm_ = cur_comm_ == cs ? nullptr : comm_stream_;
  pick_spec(cs);
  const PackedLayout L = L_;
  const int S = sx_round_S(L.S);
  const int64_t C = C_;
  constexpr int64_t tab_off = 4;  // the shard table follows the header
  const int64_t rq = sx_req_words(C, S), rp = packed_rep_words(C, L.vb);
  // per-pair capacities: this rank's requests to q fit cap_out[q], p's to this
  // rank cap_in[p]; with pairs_ only those prefixes move (grouped send / recv).
  // Loopback (one rank standing for all): what "arrives" from q is what this
  // rank sent to q, so the inbound capacities are the outbound ones.
  const bool loop = fake_ && fake_->loopback();
  SxCaps caps_out{}, caps_in{};
  size_t rq_send[kSxMaxRanks], rq_recv[kSxMaxRanks], rp_send[kSxMaxRanks], rp_recv[kSxMaxRanks];
  int64_t req_moved = 0, rep_moved = 0;
  for (int q = 0; q < R_; ++q) {
    caps_out.c[q] = pairs_ ? cap_[rank_ * R_ + q] : (uint32_t)C;
    caps_in.c[q] = pairs_ ? (loop ? caps_out.c[q] : cap_[q * R_ + rank_]) : (uint32_t)C;
    rq_send[q] = 4 * (size_t)sx_req_words(caps_out.c[q], S);
    rq_recv[q] = 4 * (size_t)sx_req_words(caps_in.c[q], S);
    rp_send[q] = 4 * (size_t)packed_rep_words(caps_in.c[q], L.vb);   // replies to q answer q's requests
    rp_recv[q] = 4 * (size_t)packed_rep_words(caps_out.c[q], L.vb);
    req_moved += (int64_t)rq_send[q] / 4;
    rep_moved += (int64_t)rp_send[q] / 4;
  }
  const bool pairs = pairs_;
  wire_ = SxWire();
  wire_.L = L;
  wire_.S = S;
  wire_.C = C;
  wire_.req_words = rq;
  wire_.rep_words = rp;
  wire_.agreed = agreed_;
  wire_.spec_from = spec_from_;
  std::copy(spec_meta_, spec_meta_ + kMetaWords, wire_.meta);
  wire_.req_moved = req_moved;
  wire_.rep_moved = rep_moved;
  wire_.pairs = pairs;
  std::copy(caps_out.c, caps_out.c + kSxMaxRanks, wire_.cap_out);
  std::copy(caps_in.c, caps_in.c + kSxMaxRanks, wire_.cap_in);
  const int cur = (int)(sends_ & 1);
  uint64_t* meta = meta_dev_ + cur * kSxMetaWords;
  // the previous Send's first completion cleared this buffer (it runs after that
  // Send's reply all-to-all, so after the agreement copy of Send - 2 on the comm
  // stream); a captured Send clears it itself
  if (!meta_zeroed_[cur] || capturing) PT_HIP_CHECK(hipMemsetAsync(meta, 0, kSxMetaWords * sizeof(uint64_t), cs));
  meta_zeroed_[cur] = false;
  // Sharded (ordered) regions only while the agreement in force saw an ordered
  // method on some rank (or before the first agreement): every rank derives the
  // same answer, so when it is no, no region is sharded anywhere and the
  // receivers launch no ordered drain at all.  A rank whose batch carries ordered
  // methods meanwhile answers them OVERFLOW (send_all re-sends them) and folds
  // their method flags into this Send's agreement, which permits them two Sends on.
  bool shard_ok = !agreed_;
  for (int m = 0; m < 7 && !shard_ok; ++m)
    if (method_ordered((uint32_t)m) && spec_meta_[kMetaFlags + m]) shard_ok = true;
  if (spec_meta_[kMetaFlags + 7]) shard_ok = true;  // method ids >= 7: may be ordered
  const bool may_order = a.ordered && shard_ok;
  const bool wants_order = a.ordered && (a.method_col != 0 || method_ordered((uint32_t)a.method_uniform));
  const bool reject_ordered = wants_order && !shard_ok;
  // sort by actor shard only when this rank's batch may carry ordered methods;
  // otherwise by rank alone (a region is then one FIFO queue of this sender)
  const bool sharded = may_order && wants_order;
  // rank byte gathers (MODE 3) for a rank-only sort of a stateless uniform method:
  // a message needs only its destination rank (1 B per id: a 1 M-actor table is
  // 1 MB, L2-resident, against the 4 MB directory), and carries its actor id
  const bool stateless = a.method_col == 0 && method_stateless((uint32_t)a.method_uniform);
  int mode = (a.affine_w && a.n_dir) ? 2 : (a.dir && a.n_dir) ? 1 : 0;
  if (mode == 1 && a.dir_rank && stateless && !sharded && a.n_dir <= kMaxMbox) mode = 3;
  wire_.shard_ok = shard_ok;
  wire_.route_mode = mode;
  const uint32_t K = sharded ? (uint32_t)kSxShards : 1u;
  // a sharded Send's per-bucket first overflow (sx_fifo_fixup_kernel): none yet
  if (sharded) PT_HIP_CHECK(hipMemsetAsync(first_ovf_, 0xff, (kXMaxBuckets + 1) * sizeof(uint32_t), cs));
  const uint32_t B = (uint32_t)R_ * K;
  auto chunk_in = [&](int i, int64_t& lo, int64_t& m) {
    lo = std::min<int64_t>((int64_t)i * max_chunk_, a.M);
    m = std::min<int64_t>(a.M, lo + max_chunk_) - lo;
    SortIn in{};
    auto off = [](uintptr_t p, int64_t e, int64_t sz) { return p ? p + (uintptr_t)(e * sz) : (uintptr_t)0; };
    in.actor = (const uint32_t*)off(a.actor, lo, 4);
    in.a0 = (const int64_t*)off(a.a0, lo, 8);
    in.a1 = (const int64_t*)off(a.a1, lo, 8);
    in.a2 = (const int64_t*)off(a.a2, lo, 8);
    in.mcol = (const uint16_t*)off(a.method_col, lo, 2);
    in.method_uniform = (uint32_t)a.method_uniform;
    in.M = m;
    in.table = (const TableEntry*)a.table;
    in.mask = a.cap - 1;
    in.dir = (const uint32_t*)a.dir;
    in.dirr = (const uint8_t*)a.dir_rank;
    in.n_dir = a.n_dir;
    in.aw = a.affine_w;
    in.aw_shift = (a.affine_w && (a.affine_w & (a.affine_w - 1)) == 0) ? __builtin_ctz(a.affine_w) : -1;
    in.rank_self = rank_;
    const int64_t tiles = (m + kSTile - 1) / kSTile;
    int64_t G = std::min<int64_t>({std::max<int64_t>(tiles, 1), (int64_t)(kMboxSortHistWords / B), 1024});
    if (G >= 8) G -= G % 8;
    in.G = (uint32_t)std::max<int64_t>(G, 1);
    in.tiles = (uint32_t)tiles;
    in.tpb = (uint32_t)((tiles + in.G - 1) / in.G);
    return in;
  };
  // (one stream for both sides: stream order is the hand-off, no events)
  const bool split = cur_comm_ != cs;
  auto serve = [&](int i) {
    Bufs& b = bufs_[i];
    if (split) PT_HIP_CHECK(hipStreamWaitEvent(cs, ev_req_in_[i], 0));
    // ~2048 blocks over the R regions (at least one per region)
    const int64_t per = std::max<int64_t>(1, max_chunk_ / R_);
    constexpr int drain_blocks = 2048, drain_per = 1024;
    const unsigned X = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>((per + drain_per - 1) / drain_per, std::max(1, drain_blocks / R_)));
#define PT_SX_PAR(SV)                                                                                         \
  hipLaunchKernelGGL((sx_drain_par_kernel<SV>), dim3(X, R_), dim3(256), 0, cs, (const uint32_t*)b.recv, rq, C, L, \
                     R_, may_order, b.reply, rp, (int64_t*)a.state, a.n_state, a.delay_ticks, stats_)
    switch (S) {
      case 1: PT_SX_PAR(1); break;
      case 2: PT_SX_PAR(2); break;
      case 3: PT_SX_PAR(3); break;
      case 4: PT_SX_PAR(4); break;
      case 6: PT_SX_PAR(6); break;
      default: PT_SX_PAR(8); break;
    }
#undef PT_SX_PAR
    if (may_order) {  // after the parallel drain (it initialised the sharded regions' replies)
      const size_t lds = sizeof(SxOrdLds) + (size_t)kXOrdStateMax * sizeof(int64_t);
#define PT_SX_ORD(SV)                                                                                            \
  do {                                                                                                           \
    static bool attr = false;                                                                                    \
    if (!attr) {                                                                                                 \
      PT_HIP_CHECK(hipFuncSetAttribute((const void*)sx_drain_ord_kernel<SV>,                                     \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                   \
      attr = true;                                                                                               \
    }                                                                                                            \
    hipLaunchKernelGGL((sx_drain_ord_kernel<SV>), dim3(kSxShards), dim3(kXOrdThreads), lds, cs,                 \
                       (const uint32_t*)b.recv, rq, tab_off, C, L, R_, b.reply, rp, (int64_t*)a.state, a.n_state, \
                       a.delay_ticks, stats_);                                                                   \
  } while (0)
      switch (S) {
        case 1: PT_SX_ORD(1); break;
        case 2: PT_SX_ORD(2); break;
        case 3: PT_SX_ORD(3); break;
        case 4: PT_SX_ORD(4); break;
        case 6: PT_SX_ORD(6); break;
        default: PT_SX_ORD(8); break;
      }
#undef PT_SX_ORD
    }
    PT_HIP_CHECK(hipGetLastError());
    if (split) {
      PT_HIP_CHECK(hipEventRecord(ev_served_[i], cs));
      PT_HIP_CHECK(hipStreamWaitEvent(cur_comm_, ev_served_[i], 0));
    }
    a2a(b.reply, b.back, (size_t)rp * 4, pairs ? rp_send : nullptr, pairs ? rp_recv : nullptr, capturing);
    if (split) PT_HIP_CHECK(hipEventRecord(ev_rep_in_[i], cur_comm_));
  };
  for (int i = 0; i < chunks_; ++i) {
    Bufs& b = bufs_[i];
    int64_t lo, m;
    const SortIn in = chunk_in(i, lo, m);
#define PT_SX_MODE(KERNEL, ...)                                      \
  do {                                                               \
    if (mode == 2) hipLaunchKernelGGL((KERNEL<2>), __VA_ARGS__);     \
    else if (mode == 1) hipLaunchKernelGGL((KERNEL<1>), __VA_ARGS__); \
    else hipLaunchKernelGGL((KERNEL<0>), __VA_ARGS__);               \
  } while (0)
    // rank-only batches: one pass with per-tile run reservation (the default; no look-back),
    // tune sx_sort=1: the look-back form (measured slower at R = 8, 4 Mi msgs per chunk: 90 us
    // vs 34 + 6.5 + 44 for count + scan + scatter -- its memory-side atomic round trips),
    // sx_sort=2: count + scan + scatter
    const int sx_mode = tn.sx_sort;
    const bool reserve = sx_mode == 0;
    if (!sharded && in.tiles > 0 && (sx_mode != 2 || mode == 3)) {
      const uint32_t hdr3 =
          ((uint32_t)(kFlagValid | (mode == 3 ? kFlagActorIds : 0)) << 16) | (uint32_t)a.method_uniform;
#define PT_SX_OS(MO, SV)                                                                                     \
  hipLaunchKernelGGL((sx_onesweep_kernel<MO, SV>), dim3(in.tiles), dim3(kST), 0, cs, in, R_, desc_, tctr_,  \
                     ticket_, b.send, rq, (uint32_t)C, caps_out, hdr3, rank_, L, b.perm, (unsigned long long*)meta, \
                     stats_, rcnt_ + i * kSxMaxRanks, reserve, reject_ordered)
#define PT_SX_OS_S(MO)              \
  switch (S) {                      \
    case 1: PT_SX_OS(MO, 1); break; \
    case 2: PT_SX_OS(MO, 2); break; \
    case 3: PT_SX_OS(MO, 3); break; \
    case 4: PT_SX_OS(MO, 4); break; \
    case 6: PT_SX_OS(MO, 6); break; \
    default: PT_SX_OS(MO, 8); break; \
  }
      // a chunk of under 512 tiles: 1024-message tiles (8-B records of the directory routes)
      const bool small_tiles = reserve && S <= 2 && (mode == 3 || mode == 1) && in.tiles < 512;
      if (small_tiles) {
        SortIn in1 = in;
        in1.tiles = (uint32_t)((m + kST * 2 - 1) / (kST * 2));
#define PT_SX_OS1(MO, SV)                                                                                        \
  hipLaunchKernelGGL((sx_onesweep_kernel<MO, SV, 2>), dim3(in1.tiles), dim3(kST), 0, cs, in1, R_, desc_, tctr_,   \
                     ticket_, b.send, rq, (uint32_t)C, caps_out, hdr3, rank_, L, b.perm,                  \
                     (unsigned long long*)meta, stats_, rcnt_ + i * kSxMaxRanks, reserve, reject_ordered)
        if (mode == 3) {
          if (S == 1) PT_SX_OS1(3, 1); else PT_SX_OS1(3, 2);
        } else {
          if (S == 1) PT_SX_OS1(1, 1); else PT_SX_OS1(1, 2);
        }
#undef PT_SX_OS1
      } else if (mode == 3) {
        PT_SX_OS_S(3)
      } else if (mode == 2) {
        PT_SX_OS_S(2)
      } else if (mode == 1) {
        PT_SX_OS_S(1)
      } else {
        PT_SX_OS_S(0)
      }
#undef PT_SX_OS_S
#undef PT_SX_OS
      PT_HIP_CHECK(hipGetLastError());
      if (split) {
        PT_HIP_CHECK(hipEventRecord(ev_routed_[i], cs));
        PT_HIP_CHECK(hipStreamWaitEvent(cur_comm_, ev_routed_[i], 0));
      }
      a2a(b.send, b.recv, (size_t)rq * 4, pairs ? rq_send : nullptr, pairs ? rq_recv : nullptr, capturing);
      if (split) PT_HIP_CHECK(hipEventRecord(ev_req_in_[i], cur_comm_));
      if (i > 0) serve(i - 1);
      continue;
    }
    PT_SX_MODE(sx_count_kernel, dim3(in.G), dim3(kST), 0, cs, in, R_, K, hist_, (unsigned long long*)meta,
               mode == 2 ? nullptr : (uint32_t*)b.perm);
    hipLaunchKernelGGL(sx_scan_kernel, dim3(R_), dim3(1024), 0, cs, hist_, in.G, R_, K, b.send, rq, caps_out,
                       (uint32_t)a.method_uniform,
                       (uint32_t)(kFlagValid | (sharded ? kFlagSharded : 0)), rank_, (unsigned long long*)meta, boff_);
#undef PT_SX_MODE
#define PT_SX_SCAT(MO, SV)                                                                                       \
  hipLaunchKernelGGL((sx_scatter_kernel<MO, SV>), dim3(in.G), dim3(kST), 0, cs, in, R_, K, (const uint32_t*)hist_, \
                     (const uint32_t*)boff_, b.send, rq, (uint32_t)C, caps_out, L, b.perm, (unsigned long long*)meta, \
                     reject_ordered, sharded ? first_ovf_ : nullptr, (uint32_t)lo)
#define PT_SX_SCAT_S(MO)            \
  switch (S) {                      \
    case 1: PT_SX_SCAT(MO, 1); break; \
    case 2: PT_SX_SCAT(MO, 2); break; \
    case 3: PT_SX_SCAT(MO, 3); break; \
    case 4: PT_SX_SCAT(MO, 4); break; \
    case 6: PT_SX_SCAT(MO, 6); break; \
    default: PT_SX_SCAT(MO, 8); break; \
  }
    if (mode == 2) {
      PT_SX_SCAT_S(2)
    } else if (mode == 1) {
      PT_SX_SCAT_S(1)
    } else {
      PT_SX_SCAT_S(0)
    }
#undef PT_SX_SCAT_S
#undef PT_SX_SCAT
    if (sharded && m > 0) {
      const unsigned fx = (unsigned)std::min<int64_t>((m + 2047) / 2048, 1024);
#define PT_SX_FIX(SV)                                                                                         \
  hipLaunchKernelGGL((sx_fifo_fixup_kernel<SV>), dim3(fx), dim3(256), 0, cs, b.send, rq, R_, (uint32_t)C, L, \
                     b.perm, m, (uint32_t)lo, (const uint32_t*)first_ovf_, (unsigned long long*)meta)
      switch (S) {
        case 1: PT_SX_FIX(1); break;
        case 2: PT_SX_FIX(2); break;
        case 3: PT_SX_FIX(3); break;
        case 4: PT_SX_FIX(4); break;
        case 6: PT_SX_FIX(6); break;
        default: PT_SX_FIX(8); break;
      }
#undef PT_SX_FIX
    }
    PT_HIP_CHECK(hipGetLastError());
    if (split) {
      PT_HIP_CHECK(hipEventRecord(ev_routed_[i], cs));
      PT_HIP_CHECK(hipStreamWaitEvent(cur_comm_, ev_routed_[i], 0));
    }
    a2a(b.send, b.recv, (size_t)rq * 4, pairs ? rq_send : nullptr, pairs ? rq_recv : nullptr, capturing);
    if (split) PT_HIP_CHECK(hipEventRecord(ev_req_in_[i], cur_comm_));
    if (i > 0) serve(i - 1);
  }
  serve(chunks_ - 1);
  // this Send's agreement, for Send + 2 (the comm stream is past every chunk's
  // scatter).  A captured Send keeps the layout in force (a replay runs no host
  // code to adopt a new one), so it records no agreement.
  if (!capturing) {
    allreduce_meta(meta, cur_comm_);
    PT_HIP_CHECK(hipMemcpyAsync(meta_host_ + cur * kSxMetaWords, meta, (kSxMetaPair + R_ * R_) * sizeof(uint64_t),
                                hipMemcpyDeviceToHost, cur_comm_));
    PT_HIP_CHECK(hipEventRecord(ev_meta_[cur], cur_comm_));
    meta_send_[cur] = sends_;
    // a device-side comm (IpcComm) can fail inside the agreement too: joined back
    // into the caller's stream, every op of this Send (and its failure word) is
    // behind the caller's next sync, and no wait kernel of it outlives the engine
    if (fake_ && fake_->device_side() && cur_comm_ != cs) {
      PT_HIP_CHECK(hipEventRecord(ev_join_, cur_comm_));
      PT_HIP_CHECK(hipStreamWaitEvent(cs, ev_join_, 0));
    }
  } else {
    meta_send_[cur] = -1;
  }
  for (int i = 0; i < chunks_; ++i) {
    int64_t lo, m;
    (void)chunk_in(i, lo, m);
    if (split) PT_HIP_CHECK(hipStreamWaitEvent(cs, ev_rep_in_[i], 0));
    if (m > 0) {
      // the first completion also clears the agreement buffer of Send + 1 (that of
      // Send - 1, whose copy to the host precedes this Send's reply all-to-alls)
      const bool zero = !capturing && !meta_zeroed_[cur ^ 1];
      launch_complete_sx((uintptr_t)bufs_[i].back, C, R_, L.vb, (uintptr_t)bufs_[i].perm, m,
                         a.out_val + (uintptr_t)(lo * 8), a.out_st + (uintptr_t)(lo * 4), (uintptr_t)cs,
                         fake_ ? (uintptr_t)fake_->device_failed() : 0,
                         zero ? (uintptr_t)(meta_dev_ + (cur ^ 1) * kSxMetaWords) : 0, zero ? kSxMetaWords : 0);
      if (zero) meta_zeroed_[cur ^ 1] = true;
    }
  }
  ++sends_;
}

}  // namespace ptype
