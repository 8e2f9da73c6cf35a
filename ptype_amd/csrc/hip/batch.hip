// Batch data path of the actor runtime: the device-native `Send` pipeline.
//
//   gen_requests   synthetic client load (SoA columns)
//   route_*        K1: GPU-registry lookup -> destination rank -> stable
//                  bucketing into per-rank epoch slots in HBM (send buffer)
//   <RCCL all-to-all of the epoch slots over xGMI>
//   dispatch       K3: per received record, switch on method id into the
//                  compiled-in handler, write the reply in place
//   <RCCL all-to-all of the reply slots back to the senders>
//   complete       K8: scatter replies back to the caller's message order
//
// Reference behaviour replaced: Client.Go fan-out + net/rpc round trip per call
// (cluster/rpc.go:69-105, :176-183) and the server's goroutine-per-request
// dispatch (stdlib, wired at example/calculator/server/server.go:16-20).
//
// Client batches are SoA (GPU-native): actor u32[M], a0/a1/a2 int64[M] (a1/a2
// optional), method either a column or one uniform id.
//
// Routing is deterministic and needs no inter-block synchronisation inside a
// streaming kernel:
//   route_prep     one coalesced pass: route directory / registry lookup ->
//                  route word (rank | mbox << 8) per message + block histogram
//   route_scan     one block: exclusive scan of the histograms per destination,
//                  slot headers, overflow / no-actor statistics
//   route_scatter  same block ranges again, stable in-order placement (wave
//                  ballots + a small LDS prefix per tile), SoA -> packed records
// Destination slots hold messages in the senders' message order, so the GPU
// output is bit-identical to the CPU reference.
//
// Wire format v2 (everything in u32 words; every region starts 16-B aligned):
//   request region per destination d, REQ = round4(4 + C * stride) words:
//     header  {delivered, raw count, sender rank, kFlagValid << 16 | method}
//     records [C] x stride words: mbox, [method if method column], a0 lo/hi,
//             [a1 lo/hi], [a2 lo/hi]   -> stride = 1 + mc + 2 * nargs
//   a calculator call (uniform method, two args) is 20 B on the wire, not 32.
//   reply region per destination, REP = round4(4 + 2C + ceil(C / 4)) words:
//     header {count, 0, 0, 0}; values int64[C]; statuses u8[C]
//   i.e. 9 B per reply instead of a 16-B record.  The reverse all-to-all brings
//   every reply back to the slot its request left from; `perm[i]` remembers it
//   as d * C + pos (-1 overflow, -2 no actor).
#include <algorithm>
#include <vector>

#include "common.hpp"
#include "handlers.hpp"
#include "packed.hpp"
#include "route_common.hpp"

namespace ptype {

// `seed_ptr` (optional) lets a captured graph draw a new batch per replay.
// (Advancing the seed inside this kernel, last block out, was measured slower than
// the separate one-element add it replaces: 8192 blocks ending on a ticket round
// trip cost more than the ~4 us launch; fewer, longer blocks stream slower.)
// h % n without a 64-bit divide (gfx950 has no integer divider: `%` expands to a
// long dependent sequence): q = mulhi(h, floor((2^64 - 1) / n)) undershoots
// floor(h / n) by at most 2, so at most two corrections make it exact.
__device__ __forceinline__ uint32_t mod_u64_u32(uint64_t h, uint32_t n, uint64_t magic) {
  const uint64_t q = __umul64hi(h, magic);
  uint64_t r = h - q * n;
  r = r >= n ? r - n : r;
  r = r >= n ? r - n : r;
  return (uint32_t)r;
}

// WIDE: full-range int64 arguments (two more hashes per message) -- values no
// narrow record holds, for the wide-argument figures (16-B ring records).
// NT: non-temporal stores -- for batches of up to 1 Mi messages (28.8 vs 27.8 G on the 1 Mi
// step, one box, alternated); an 8 Mi batch keeps plain stores (57.1-57.9 vs 53.6-54.8 G
// with NT) -- profiles/r6_small_sends.md
template <bool WIDE, bool NT = false>
__global__ __launch_bounds__(256) void gen_requests_kernel(uint32_t* __restrict__ actor, int64_t* __restrict__ a0,
                                                           int64_t* __restrict__ a1, int64_t M, uint32_t n_actors,
                                                           uint64_t seed, const uint64_t* __restrict__ seed_ptr,
                                                           uint64_t magic) {
  if (seed_ptr) seed = *seed_ptr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix64(seed ^ (uint64_t)i * 0x9e3779b97f4a7c15ull);
    const uint32_t ac = magic ? mod_u64_u32(h, n_actors, magic) : (uint32_t)(h % n_actors);
    int64_t x0, x1;
    if constexpr (WIDE) {
      x0 = (int64_t)mix64(h ^ 0xa0761d6478bd642full);
      x1 = (int64_t)mix64(h ^ 0xe7037ed1a0b428dbull);
    } else {
      x0 = (int64_t)((h >> 20) & 0xffff) - 0x8000;
      x1 = (int64_t)((h >> 40) & 0xffff);
    }
    if constexpr (NT) {
      __builtin_nontemporal_store(ac, actor + i);
      __builtin_nontemporal_store(x0, a0 + i);
      if (a1) __builtin_nontemporal_store(x1, a1 + i);
    } else {
      actor[i] = ac;
      a0[i] = x0;
      if (a1) a1[i] = x1;  // (null: a one-argument batch)
    }
  }
}

// Replica routing (SURVEY 2.4 "service replication"): a replicated stateless
// service is hosted on several ranks, each holding the same logical actors
// [0, n) at its mailboxes [0, n) -- global actor id a * W + rank in the strided
// id space of the group (so the route directory's affine rule applies).  The
// client picks the replica per message with the reference client's rules: the
// selected replicas (all of them in mesh mode, else FNV-1a picks -- host side,
// ConnectionBalancer::select_nodes) taken round robin, the first call to index 1
// (cluster/rpc.go:176-183, 246-270): message i of a Send whose counter starts at
// seq0 goes to sel[(seq0 + 1 + i) % n_sel].  Ids >= n map to -1 (no actor).
constexpr int kMaxReplicaSel = 64;
struct ReplicaSel {
  uint8_t rank[kMaxReplicaSel];
  uint32_t n;
};

__global__ __launch_bounds__(256) void replica_route_kernel(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                            int64_t M, ReplicaSel sel, uint64_t first, uint32_t W,
                                                            uint32_t n_logical) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += step) {
    const uint32_t a = (uint32_t)in[i];
    const uint32_t j = (uint32_t)((first + (uint64_t)i) % sel.n);
    out[i] = a < n_logical ? (int32_t)(a * W + sel.rank[j]) : -1;
  }
}

// Pass 1: lookup + histogram.  Block b owns messages [b*P, min(M,(b+1)*P)).
// Each thread resolves K messages per tile (coalesced, item-major), with their
// lookups overlapped.  With a route directory (DIR) an actor id below n_dir costs
// one 4-B read; the hash table is probed only for ids outside it (or fallbacks).
// MODE 0: hash probe; 1: route directory; 2: affine placement (ids below n_dir
// verified to sit at rank id % W, mailbox id / W -- route words computed, no
// gathers; W a power of two uses shifts).
//
// META: the v3 width pass rides along (the batch's argument columns are read in
// the same tiles, column maxima published per block into mc.meta), so a packed
// Send reads its batch once before the agreement instead of twice.
template <int K, int MODE, bool META = false, bool PIPE = false>
__global__ __launch_bounds__(kRouteThreads) void route_prep_kernel(const uint32_t* __restrict__ actor, int64_t M,
                                                                   int64_t P, const TableEntry* __restrict__ table,
                                                                   uint64_t mask, const uint32_t* __restrict__ dir,
                                                                   uint32_t n_dir, uint32_t aw, int aw_shift, int R,
                                                                   uint32_t* __restrict__ route,
                                                                   uint32_t* __restrict__ hist, MetaCols mc = {},
                                                                   CapFold cf = {}) {
  constexpr bool DIR = MODE == 1;
  __shared__ unsigned h[kMaxRanks + 1];
  for (int d = threadIdx.x; d <= R; d += blockDim.x) h[d] = 0;
  __syncthreads();
  const int64_t lo = blockIdx.x * P, hi = lo + P < M ? lo + P : M;
  const unsigned lane = lane_id();
  // lane l owns destination l's count for this wave (registers, not LDS atomics:
  // with 8 destinations, 4 waves' leaders hammering 9 LDS words made the pass
  // LDS-atomic bound -- SQ_WAIT_INST_LDS 50x the single-destination case)
  unsigned hc = 0;
  MetaAcc macc;
  // PIPE: the next tile's actor ids are loaded before this tile's directory
  // gathers, so a wave's HBM latency overlaps its gather latency
  uint32_t an[K];
  if constexpr (PIPE) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = lo + k * kRouteThreads + threadIdx.x;
      an[k] = i < hi ? __builtin_nontemporal_load(actor + i) : 0u;
    }
  }
  for (int64_t base = lo; base < hi; base += K * kRouteThreads) {
    uint32_t a[K];
    int r[K];
    uint32_t mb[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = base + k * kRouteThreads + threadIdx.x;
      // streaming column: non-temporal, so it does not evict the route directory from L2
      if constexpr (PIPE) {
        a[k] = an[k];
        const int64_t j = i + K * kRouteThreads;
        an[k] = j < hi ? __builtin_nontemporal_load(actor + j) : 0u;
      } else {
        a[k] = i < hi ? __builtin_nontemporal_load(actor + i) : 0u;
      }
    }
    if constexpr (META) {
      int64_t v0[K], v1[K], v2[K];
      uint32_t me[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int64_t i = base + k * kRouteThreads + threadIdx.x;
        const bool in = i < hi;
        v0[k] = in ? __builtin_nontemporal_load(mc.a0 + i) : 0;
        v1[k] = in && mc.a1 ? __builtin_nontemporal_load(mc.a1 + i) : 0;
        v2[k] = in && mc.a2 ? __builtin_nontemporal_load(mc.a2 + i) : 0;
        me[k] = in && mc.mcol ? (uint32_t)mc.mcol[i] : 0u;
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int64_t i = base + k * kRouteThreads + threadIdx.x;
        if (i < hi) macc.take(a[k], v0[k], v1[k], v2[k], me[k], mc.n_dir, mc.aw);
      }
    }
    if constexpr (MODE == 2) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (a[k] < n_dir) {
          r[k] = aw_shift >= 0 ? (int)(a[k] & (aw - 1)) : (int)(a[k] % aw);
          mb[k] = aw_shift >= 0 ? a[k] >> aw_shift : a[k] / aw;
        } else {
          lookup_entry(table, mask, actor_key(a[k]), r[k], mb[k]);
        }
      }
    } else if constexpr (DIR) {
      uint32_t w[K];
#pragma unroll
      for (int k = 0; k < K; ++k) w[k] = a[k] < n_dir ? dir[a[k]] : kDirFallback;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (w[k] == kDirFallback) {
          lookup_entry(table, mask, actor_key(a[k]), r[k], mb[k]);
        } else {
          r[k] = w[k] == kDirMissing ? -1 : (int)(w[k] & 0xff);
          mb[k] = w[k] >> 8;
        }
      }
    } else {
      uint64_t key[K];
#pragma unroll
      for (int k = 0; k < K; ++k) key[k] = actor_key(a[k]);
      lookup_many<K>(table, mask, key, r, mb);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = base + k * kRouteThreads + threadIdx.x;
      int d = -1;  // -1: no message in this lane
      if (i < hi) {
        const bool ok = r[k] >= 0 && r[k] < R && mb[k] < kMaxMbox;
        d = ok ? r[k] : R;  // column R counts registry misses
        __builtin_nontemporal_store(ok ? ((uint32_t)r[k] | (mb[k] << 8)) : kRouteNoActor, route + i);
      }
      // wave histogram: one ballot per destination present in the wave
      uint64_t active = __ballot(d >= 0);
      while (active) {
        const int leader = __builtin_ctzll(active);
        const int dl = __builtin_amdgcn_readlane(d, leader);
        const uint64_t m = __ballot(d == dl);
        if (dl < kWave) {
          if (lane == (unsigned)dl) hc += (unsigned)__popcll(m);
        } else if (lane == (unsigned)leader) {  // the miss column of a 64-rank world
          atomicAdd(&h[dl], (unsigned)__popcll(m));
        }
        active &= ~m;
      }
    }
  }
  if (hc) atomicAdd(&h[lane], hc);  // lane <= R here: only owned columns are non-zero
  __syncthreads();
  // column-major [R + 1][G]: the scan reads each destination's column contiguously
  for (int d = threadIdx.x; d <= R; d += blockDim.x) hist[(int64_t)d * gridDim.x + blockIdx.x] = h[d];
  if constexpr (META) meta_publish(macc, mc.mcol != nullptr, mc.method_uniform, M, mc.meta);
  if (cf.tot) {  // adaptive capacity (CapFold): column totals, then the last block takes the max
    __shared__ unsigned s_last;
    const unsigned tid = threadIdx.x;
    unsigned* tot = cf.tot + (blockIdx.x % kCapCopies) * kMaxCapCols;  // spread: same-address atomics serialise
    if (tid <= (unsigned)R && h[tid]) {
      // device-scope atomics complete at the memory side (coherent across XCDs); the
      // returned value is consumed so the add has landed before the barrier below
      const unsigned old = atomicAdd(&tot[tid], h[tid]);
      if (old == 0xffffffffu) h[tid] = 0;
    }
    __syncthreads();
    if (tid == 0) s_last = last_block_ticket(cf.ticket);
    __syncthreads();
    if (s_last && tid <= (unsigned)R) {
      unsigned t = 0;
      for (unsigned c = 0; c < kCapCopies; ++c)  // memory-side read + reset for the next launch
        t += atomicExch(&cf.tot[c * kMaxCapCols + tid], 0u);
      if (tid < (unsigned)R && t) atomicMax(&cf.meta[kMetaCap], (unsigned long long)t);
      if (cf.counts && tid < (unsigned)R) cf.counts[(size_t)tid * cf.count_stride] = t;
    }
  }
}

// Slot headers + overflow / no-actor statistics from the column totals (block-level;
// after the barrier that publishes `tot`).
__device__ __forceinline__ void scan_headers(const unsigned* tot, int R, int64_t C, uint32_t* __restrict__ sendbuf,
                                             int64_t req_words, uint32_t method_uniform,
                                             unsigned long long* __restrict__ stats, int rank_self) {
  const bool identity = R == 1 && tot[1] == 0 && (int64_t)tot[0] <= C;
  for (int d = threadIdx.x; d < R; d += blockDim.x) {
    const unsigned total = tot[d];
    uint4* h4 = reinterpret_cast<uint4*>(sendbuf + (int64_t)d * req_words);
    const unsigned delivered = total < C ? total : (unsigned)C;
    const uint32_t flags = kFlagValid | (identity ? kFlagIdentity : 0);
    h4[0] = make_uint4(delivered, total, (unsigned)rank_self, (flags << 16) | (method_uniform & 0xffffu));
    if (total > C) atomicAdd(&stats[1], (unsigned long long)(total - C));
  }
  if (threadIdx.x == 0 && tot[R]) stats[0] += tot[R];
}

// Pass 2 (one block): per-destination exclusive scan over the blocks' histograms
// -> per-block bases, slot headers, statistics.  Up to 16 ranks (RC = R + 1
// columns held in registers): every thread loads its ~G/1024 rows whole (all
// loads in flight at once), each column is scanned by wave shuffles, and ONE
// block barrier exchanges the wave totals -- the columns no longer go one after
// another (the column-serial scan took 28 us at 8 ranks: half the route).
// Headers are written after all columns so the no-actor total is known: a batch
// that maps whole and gap-free onto a single slot (R = 1, no unknown actor, no
// overflow) is flagged kFlagIdentity -- slot position == message index, which
// lets direct completion skip the inverse index.
template <int RC>
__global__ __launch_bounds__(1024) void route_scan_kernel(uint32_t* __restrict__ hist, int G, int R, int64_t C,
                                                          uint32_t* __restrict__ sendbuf, int64_t req_words,
                                                          uint32_t method_uniform,
                                                          unsigned long long* __restrict__ stats, int rank_self) {
  constexpr int kRows = 2;  // rows per thread held in registers (G <= 2048: route_grid's target)
  __shared__ unsigned wsum[1024 / kWave][RC];
  __shared__ unsigned tot[kMaxRanks + 1];
  const unsigned lane = lane_id(), w = threadIdx.x / kWave, nw = blockDim.x / kWave;
  const int per = (G + (int)blockDim.x - 1) / (int)blockDim.x;
  const int b0 = threadIdx.x * per, b1 = b0 + per < G ? b0 + per : G;
  const int cols = R + 1;
  const bool fast = per <= kRows;
  unsigned cell[kRows][RC], sum[RC], v[RC];
#pragma unroll
  for (int d = 0; d < RC; ++d) sum[d] = 0;
  if (fast) {  // every load of the thread issued before any is used
#pragma unroll
    for (int r = 0; r < kRows; ++r)
#pragma unroll
      for (int d = 0; d < RC; ++d) {
        cell[r][d] = (b0 + r < b1 && d < cols) ? hist[(int64_t)d * G + b0 + r] : 0u;
        sum[d] += cell[r][d];
      }
  } else {
    for (int b = b0; b < b1; ++b)
#pragma unroll
      for (int d = 0; d < RC; ++d) sum[d] += d < cols ? hist[(int64_t)d * G + b] : 0u;
  }
#pragma unroll
  for (int d = 0; d < RC; ++d) {  // inclusive scan of each column across the wave (DPP)
    v[d] = wave_incl_scan(sum[d]);
    if (lane == kWave - 1) wsum[w][d] = v[d];
  }
  __syncthreads();
  if (w == 0) {  // exclusive scan of the wave totals, per column (lanes = waves)
#pragma unroll
    for (int d = 0; d < RC; ++d) {
      const unsigned x = lane < nw ? wsum[lane][d] : 0u;
      const unsigned y = wave_incl_scan(x);
      if (lane < nw) wsum[lane][d] = y - x;
      if (lane == nw - 1 && d < cols) tot[d] = y;
    }
  }
  __syncthreads();
#pragma unroll
  for (int d = 0; d < RC; ++d) {
    if (d >= cols) continue;
    unsigned run = wsum[w][d] + v[d] - sum[d];  // exclusive prefix of this thread's first block
    if (fast) {
#pragma unroll
      for (int r = 0; r < kRows; ++r)
        if (b0 + r < b1) {
          hist[(int64_t)d * G + b0 + r] = run;  // hist becomes the per-block base
          run += cell[r][d];
        }
    } else {
      for (int b = b0; b < b1; ++b) {
        uint32_t* c = hist + (int64_t)d * G + b;
        const unsigned x = *c;
        *c = run;
        run += x;
      }
    }
  }
  scan_headers(tot, R, C, sendbuf, req_words, method_uniform, stats, rank_self);
}

// Pass 2, any R (R + 1 > 17 columns): the columns one after another.
// Wave-level scans (shuffles) + one LDS exchange of wave totals: 3 barriers per
// column instead of a 1024-wide Hillis-Steele.  Headers are written after all
// columns so the no-actor total is known: a batch that maps whole and gap-free
// onto a single slot (R = 1, no unknown actor, no overflow) is flagged
// kFlagIdentity -- slot position == message index, which lets direct completion
// skip the inverse index.
__global__ __launch_bounds__(1024) void route_scan_wide_kernel(uint32_t* __restrict__ hist, int G, int R, int64_t C,
                                                          uint32_t* __restrict__ sendbuf, int64_t req_words,
                                                          uint32_t method_uniform,
                                                          unsigned long long* __restrict__ stats, int rank_self) {
  __shared__ unsigned wsum[1024 / kWave];
  __shared__ unsigned tot[kMaxRanks + 1];
  const unsigned lane = lane_id(), w = threadIdx.x / kWave, nw = blockDim.x / kWave;
  const int per = (G + blockDim.x - 1) / blockDim.x;
  const int b0 = threadIdx.x * per, b1 = b0 + per < G ? b0 + per : G;
  for (int d = 0; d <= R; ++d) {
    unsigned s = 0;
    for (int b = b0; b < b1; ++b) s += hist[(int64_t)d * G + b];
    unsigned v = s;  // inclusive scan within the wave
    for (int off = 1; off < kWave; off <<= 1) {
      const unsigned t = __shfl_up(v, off);
      if (lane >= (unsigned)off) v += t;
    }
    if (lane == kWave - 1) wsum[w] = v;
    __syncthreads();
    if (w == 0) {  // scan of the wave totals
      unsigned x = lane < nw ? wsum[lane] : 0u;
      for (int off = 1; off < kWave; off <<= 1) {
        const unsigned t = __shfl_up(x, off);
        if (lane >= (unsigned)off) x += t;
      }
      if (lane < nw) wsum[lane] = x;
    }
    __syncthreads();
    unsigned run = (w ? wsum[w - 1] : 0u) + v - s;  // exclusive prefix of this thread's first block
    for (int b = b0; b < b1; ++b) {                   // hist becomes the per-block base
      const unsigned c = hist[(int64_t)d * G + b];
      hist[(int64_t)d * G + b] = run;
      run += c;
    }
    if (threadIdx.x == 0) tot[d] = wsum[nw - 1];
    __syncthreads();
  }
  scan_headers(tot, R, C, sendbuf, req_words, method_uniform, stats, rank_self);
}

// Pass 3: stable placement + SoA -> packed wire records (format <NARGS, MC>).
template <int NARGS, bool MC>
__global__ __launch_bounds__(kRouteThreads) void route_scatter_kernel(
    const uint32_t* __restrict__ route, const int64_t* __restrict__ a0, const int64_t* __restrict__ a1,
    const int64_t* __restrict__ a2, const uint16_t* __restrict__ method_col, uint32_t method_uniform, int64_t M,
    int64_t P, int R, int64_t C, const uint32_t* __restrict__ base, uint32_t* __restrict__ sendbuf,
    int64_t req_words, int32_t* __restrict__ perm, DirectView dv) {
  __shared__ unsigned cnt[kScatterItems][kRouteThreads / kWave][kMaxRanks];
  __shared__ unsigned run[kMaxRanks];
  for (int d = threadIdx.x; d < R; d += blockDim.x) run[d] = base[(int64_t)d * gridDim.x + blockIdx.x];
  const int64_t lo = blockIdx.x * P, hi = lo + P < M ? lo + P : M;
  if (dv.src)  // the scan flagged a gap-free single slot: positions are message indices
    dv.identity = ((sendbuf[(int64_t)dv.self * req_words + 3] >> 16) & kFlagIdentity) != 0;
  __syncthreads();
  auto route_at = [route](int64_t i) { return route[i]; };
  for (int64_t tile = lo; tile < hi; tile += kScatterTile)
    scatter_tile<NARGS, MC>(tile, hi, route_at, a0, a1, a2, method_col, method_uniform, R, C,
                            V2Emit<NARGS, MC>{sendbuf, req_words},
                            perm, cnt, run, dv);
}

// K3 (batch form).  grid.y = source rank, grid.x tiles the delivered range.
// FIXED != 0: the slot's method is known (uniform per source slot, no method
// column), so the handler switch constant-folds and the loop body is just that
// handler; FIXED == 0 switches per message.
template <int NARGS, bool MC, int FIXED>
__device__ __forceinline__ unsigned long long dispatch_range(const uint32_t* __restrict__ rq, int64_t count,
                                                             uint32_t hdr_method, int64_t* __restrict__ vals,
                                                             uint8_t* __restrict__ sts, int64_t* __restrict__ state,
                                                             uint32_t n_state, uint64_t delay_ticks,
                                                             OutboxView ob, DirectView dv, bool direct,
                                                             bool ident) {
  constexpr int kStride = 1 + (MC ? 1 : 0) + 2 * NARGS;
  unsigned long long failed = 0;
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < count; s += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t* r = rq + 4 + s * kStride;
    uint32_t wv[kStride];
    load_words<kStride>(r, wv);
    MsgRecord m;
    m.actor = wv[0];
    m.method = (uint16_t)(FIXED ? FIXED : (MC ? (wv[1] & 0xffffu) : hdr_method));
    m.flags = kFlagValid | kFlagRouted;
    constexpr int o = 1 + (MC ? 1 : 0);
    m.a0 = (int64_t)(((uint64_t)wv[o + 1] << 32) | wv[o]);
    m.a1 = 0;
    m.a2 = 0;
    if constexpr (NARGS > 1) m.a1 = (int64_t)(((uint64_t)wv[o + 3] << 32) | wv[o + 2]);
    if constexpr (NARGS > 2) m.a2 = (int64_t)(((uint64_t)wv[o + 5] << 32) | wv[o + 4]);
    const ReplyRecord rr = run_handler(m, state, n_state, delay_ticks, ob);
    failed += rr.status != kStatusOk;
    if (direct) {  // own slot: straight into the caller's outputs
      const int64_t i = ident ? s : (int64_t)dv.src[s];
      dv.out_val[i] = rr.value;
      dv.out_st[i] = rr.status;
    } else {
      vals[s] = rr.value;
      sts[s] = (uint8_t)rr.status;
    }
  }
  return failed;
}

template <int NARGS, bool MC>
__global__ __launch_bounds__(256) void dispatch_kernel(const uint32_t* __restrict__ recv, int64_t req_words,
                                                       int64_t C, uint32_t* __restrict__ reply, int64_t rep_words,
                                                       int64_t* __restrict__ state, uint32_t n_state,
                                                       uint64_t delay_ticks, unsigned long long* __restrict__ stats,
                                                       OutboxView ob, DirectView dv, unsigned stage_cap) {
  extern __shared__ __align__(16) unsigned char smem[];
  if (stage_cap) {  // handlers' outbox sends staged in LDS, published once per block (handlers.hpp)
    ob.stg = outbox_stage(smem, stage_cap);
    __syncthreads();
  }
  const int d = blockIdx.y;
  const bool direct = dv.src != nullptr && d == dv.self;
  const uint32_t* rq = recv + (int64_t)d * req_words;
  const uint4 h = *reinterpret_cast<const uint4*>(rq);
  const bool valid = (h.w >> 16) & kFlagValid;
  const int64_t count = valid ? (int64_t)(h.x < C ? h.x : C) : 0;
  uint32_t* rp = reply + (int64_t)d * rep_words;
  int64_t* vals = reinterpret_cast<int64_t*>(rp + 4);
  uint8_t* sts = reinterpret_cast<uint8_t*>(rp + 4 + 2 * C);
  if (blockIdx.x == 0 && threadIdx.x == 0)  // reply header: delivered count (sender audits it)
    *reinterpret_cast<uint4*>(rp) = make_uint4((uint32_t)count, 0u, 0u, 0u);
  const OutboxView obp = ob;
  const uint32_t hm = h.w & 0xffffu;
  const bool ident = direct && ((h.w >> 16) & kFlagIdentity);
  unsigned long long failed;
  if constexpr (!MC) {
    switch (hm) {  // uniform per slot: one specialised loop per hot method
      case kCalculatorMultiply:
        failed = dispatch_range<NARGS, MC, kCalculatorMultiply>(rq, count, hm, vals, sts, state, n_state,
                                                                delay_ticks, obp, dv, direct, ident);
        break;
      case kPrimeCheck:
        failed = dispatch_range<NARGS, MC, kPrimeCheck>(rq, count, hm, vals, sts, state, n_state, delay_ticks, obp, dv, direct, ident);
        break;
      case kCounterAdd:
        failed = dispatch_range<NARGS, MC, kCounterAdd>(rq, count, hm, vals, sts, state, n_state, delay_ticks, obp, dv, direct, ident);
        break;
      default:
        failed = dispatch_range<NARGS, MC, 0>(rq, count, hm, vals, sts, state, n_state, delay_ticks, obp, dv, direct, ident);
    }
  } else {
    failed = dispatch_range<NARGS, MC, 0>(rq, count, hm, vals, sts, state, n_state, delay_ticks, obp, dv, direct, ident);
  }
  if (stage_cap) outbox_flush(ob);  // every thread of the block reaches here
  for (int off = 32; off > 0; off >>= 1) failed += __shfl_xor(failed, off);
  if (lane_id() == 0 && failed) atomicAdd(&stats[2], failed);
}

// World 1, no collectives: the local Send.  With one destination there is
// nothing to bucket, so resolution and dispatch fuse into one streaming pass:
// each message is resolved against the registry mirror (affine directory /
// route directory / hash probe, exactly as route_prep), handed to its
// mailbox's handler, and its reply written into the caller's outputs.  No
// epoch slot, no histogram, no scan: 20 B in and 12 B out per calculator call.
// MODE as route_prep; FIXED != 0: uniform method known at launch (the handler
// switch constant-folds).
//
// K messages per thread per tile (item-major, so every column access stays
// coalesced), with ALL of a tile's streaming loads issued before the first
// registry read is used: with one message per iteration the chain was
// actor load -> directory gather -> (branch) -> argument loads, three
// dependent memory latencies per message, and the random-placement step ran
// the pass at 59 us vs 38 us for the gather-free affine rule (profiles/README.md).
template <int MODE, int FIXED, int K = 4>
__global__ __launch_bounds__(256) void local_send_kernel(
    const uint32_t* __restrict__ actor, const int64_t* __restrict__ a0, const int64_t* __restrict__ a1,
    const int64_t* __restrict__ a2, const uint16_t* __restrict__ mcol, uint32_t method_uniform, int64_t M,
    const TableEntry* __restrict__ table, uint64_t mask, const uint32_t* __restrict__ dir, uint32_t n_dir,
    uint32_t aw, int aw_shift, int64_t* __restrict__ state, uint32_t n_state, uint64_t delay_ticks, OutboxView ob,
    int64_t* __restrict__ out_val, int32_t* __restrict__ out_st, unsigned long long* __restrict__ stats,
    unsigned long long* __restrict__ checksum, unsigned stage_cap, const unsigned long long* __restrict__ m_dev) {
  if (m_dev) {  // device-counted batch (an outbox bank): M is its capacity, the count says how many
    const unsigned long long n = *m_dev;
    if ((int64_t)n < M) M = (int64_t)n;
  }
  unsigned long long nomatch = 0, failed = 0, sum = 0;
  const int64_t tile = (int64_t)K * blockDim.x;
  extern __shared__ __align__(16) unsigned char smem[];
  if (stage_cap) {  // handlers' outbox sends staged per tile (one reservation per block, handlers.hpp)
    ob.stg = outbox_stage(smem, stage_cap);
    __syncthreads();
  }
  for (int64_t base = blockIdx.x * tile; base < M; base += (int64_t)gridDim.x * tile) {
    uint32_t a[K];
    int64_t x0[K], x1[K], x2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = base + k * (int64_t)blockDim.x + threadIdx.x;
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
      for (int k = 0; k < K; ++k) w[k] = a[k] < n_dir ? dir[a[k]] : kDirFallback;  // K gathers in flight
#pragma unroll
      for (int k = 0; k < K; ++k) {
        r[k] = w[k] == kDirMissing ? -1 : (int)(w[k] & 0xff);
        mb[k] = w[k] >> 8;
      }
#pragma unroll
      for (int k = 0; k < K; ++k)  // (a tail lane's id 0xffffffff resolves to nothing: no probe)
        if (w[k] == kDirFallback && a[k] != 0xffffffffu) lookup_entry(table, mask, actor_key(a[k]), r[k], mb[k]);
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
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = base + k * (int64_t)blockDim.x + threadIdx.x;
      if (i >= M) continue;
      ReplyRecord rr;
      if (r[k] == 0 && mb[k] < kMaxMbox) {
        MsgRecord m;
        m.actor = mb[k];
        m.method = (uint16_t)(FIXED ? FIXED : (mcol ? (uint32_t)mcol[i] : method_uniform));
        m.flags = kFlagValid | kFlagRouted;
        m.a0 = x0[k];
        m.a1 = x1[k];
        m.a2 = x2[k];
        rr = run_handler(m, state, n_state, delay_ticks, ob);
        failed += rr.status != kStatusOk;
      } else {
        rr.value = 0;
        rr.status = kStatusNoActor;
        ++nomatch;
      }
      __builtin_nontemporal_store(rr.value, out_val + i);
      __builtin_nontemporal_store((int32_t)rr.status, out_st + i);
      sum += (unsigned long long)rr.value;
    }
    if (stage_cap) {  // publish when the stage could not take another tile, and at the end
      const bool last = base + (int64_t)gridDim.x * tile >= M;  // block-uniform
      __syncthreads();  // this tile's emits have landed in LDS
      const unsigned staged = *ob.stg.n;
      __syncthreads();  // every thread read it before the next tile's emits move it
      if (last || staged + (unsigned)tile > stage_cap) outbox_flush(ob);
    }
  }
  // counters as the slot path keeps them (ws stats: 0 no-actor, 2 handler-failed),
  // one atomic per block and only when non-zero
  __shared__ unsigned long long part[3][256 / kWave];
  for (int off = 32; off > 0; off >>= 1) {
    nomatch += __shfl_xor(nomatch, off);
    failed += __shfl_xor(failed, off);
    sum += __shfl_xor(sum, off);
  }
  const int w = threadIdx.x / kWave;
  if (lane_id() == 0) part[0][w] = nomatch, part[1][w] = failed, part[2][w] = sum;
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned long long v = 0;
    for (int k = 0; k < 256 / kWave; ++k) v += part[threadIdx.x][k];
    if (threadIdx.x == 0 && v) atomicAdd(&stats[0], v);
    if (threadIdx.x == 1 && v) atomicAdd(&stats[2], v);
    if (threadIdx.x == 2 && checksum) atomicAdd(checksum, v);
  }
}

// K8: replies back to message order (SoA outputs).
// direct: negative perm entries were completed by the scatter / own-slot dispatch.
__global__ __launch_bounds__(256) void complete_kernel(const uint32_t* __restrict__ rep, int64_t rep_words,
                                                       uint32_t C, const int32_t* __restrict__ perm, int64_t M,
                                                       int64_t* __restrict__ out_val, int32_t* __restrict__ out_st,
                                                       unsigned long long* __restrict__ checksum, bool direct,
                                                       const uint64_t* __restrict__ failed) {
  unsigned long long sum = 0;
  // a failed collective wrote no reply slots (see complete_packed_kernel)
  const bool lost = failed && __hip_atomic_load(failed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t p = perm[i];
    if (lost && (p >= 0 || p == -3)) {
      out_val[i] = 0;
      out_st[i] = kStatusNotDelivered;
      continue;
    }
    if (direct && p < 0) {
      if (checksum) sum += (unsigned long long)out_val[i];
      continue;
    }
    int64_t v = 0;
    int32_t st;
    if (p >= 0) {
      const uint32_t d = (uint32_t)p / C, pos = (uint32_t)p - d * C;
      const uint32_t* rb = rep + (int64_t)d * rep_words;
      v = reinterpret_cast<const int64_t*>(rb + 4)[pos];
      st = reinterpret_cast<const uint8_t*>(rb + 4 + 2 * (int64_t)C)[pos];
    } else {
      st = p == -1 ? kStatusOverflow : kStatusNoActor;
    }
    out_val[i] = v;
    out_st[i] = st;
    sum += (unsigned long long)v;
  }
  if (checksum) {  // block-reduce first: one atomic per block, not per wave
    __shared__ unsigned long long part[4];
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
    if (lane_id() == 0) part[threadIdx.x / kWave] = sum;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(checksum, part[0] + part[1] + part[2] + part[3]);
  }
}

static inline unsigned grid_cap(int64_t work, int per, unsigned cap) {
  int64_t g = (work + per - 1) / per;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

void launch_replica_route(uintptr_t in, uintptr_t out, int64_t M, const std::vector<int>& ranks, uint64_t seq0,
                          uint32_t W, uint32_t n_logical, uintptr_t stream) {
  if (M <= 0) return;
  if (ranks.empty() || ranks.size() > (size_t)kMaxReplicaSel)
    throw std::invalid_argument("replica_route: 1.." + std::to_string(kMaxReplicaSel) + " selected replicas");
  if ((uint64_t)n_logical * W > 0x7fffffffull) throw std::invalid_argument("replica_route: ids exceed int32");
  ReplicaSel sel{};
  for (size_t k = 0; k < ranks.size(); ++k) {
    if (ranks[k] < 0 || (uint32_t)ranks[k] >= W) throw std::invalid_argument("replica_route: rank out of range");
    sel.rank[k] = (uint8_t)ranks[k];
  }
  sel.n = (uint32_t)ranks.size();
  hipLaunchKernelGGL(replica_route_kernel, dim3(grid_cap(M, 256, 2048)), dim3(256), 0, as_stream(stream),
                     (const int32_t*)in, (int32_t*)out, M, sel, (seq0 + 1) % sel.n, W, n_logical);
  PT_HIP_CHECK(hipGetLastError());
}

int replica_sel_max() { return kMaxReplicaSel; }

void launch_gen_requests(uintptr_t actor, uintptr_t a0, uintptr_t a1, int64_t M, uint32_t n_actors, uint64_t seed,
                         uintptr_t seed_ptr, uintptr_t stream, bool wide) {
  if (M <= 0) return;
  if (n_actors == 0) throw std::invalid_argument("n_actors must be > 0");
  // (measured: four messages per thread with 16-B stores, non-temporal stores, plain `%`
  // and grids from 512 to 8192 blocks were no faster -- removed, tools/gen_sweep.py)
  const uint64_t magic = ~0ull / n_actors;
  const dim3 g(grid_cap(M, 256, 8192u));
  const bool nt = M <= (1 << 20);
#define PT_GEN(W, N)                                                                                       \
  hipLaunchKernelGGL((gen_requests_kernel<W, N>), g, dim3(256), 0, as_stream(stream), (uint32_t*)actor,   \
                     (int64_t*)a0, (int64_t*)a1, M, n_actors, seed, (const uint64_t*)seed_ptr, magic)
  if (wide) {
    if (nt) PT_GEN(true, true);
    else PT_GEN(true, false);
  } else {
    if (nt) PT_GEN(false, true);
    else PT_GEN(false, false);
  }
#undef PT_GEN
  PT_HIP_CHECK(hipGetLastError());
}

// Route blocks: G = ceil(M / P); the scan kernel handles up to 1024 * 64 blocks.
int64_t route_grid(int64_t M, int64_t* P_out) {
  // ~2048 blocks whatever the batch size (8 per CU): a pipelined chunk of 2 Mi
  // messages at P = 4096 was only 512 blocks, and the prep / scatter passes --
  // barrier-separated tiles, latency-bound -- ran at a quarter of the machine.
  // P is a whole number of scatter tiles (512 messages), at least one.
  constexpr int64_t target = 2048;
  int64_t P = (M + target - 1) / target;
  P = ((P + kScatterTile - 1) / kScatterTile) * kScatterTile;
  if (P < kScatterTile) P = kScatterTile;
  int64_t G = (M + P - 1) / P;
  if (G < 1) G = 1;
  *P_out = P;
  return G;
}

// Tuning knobs: items per thread of the 3-pass route_prep (0 = default) and the
// route algorithm (0 = 3-pass prep/scan/scatter, 1 = single-pass look-back).
// Measured on MI355X (profiles/README.md): the single-pass kernel saves the route
// word round trip and the scan launch but its inclusive-prefix frontier crosses
// ~2048 blocks at ~64 blocks per cross-XCD status round trip (~1.5-2 us), so it
// loses (189 vs 139 us at 8 Mi messages); the 3-pass route is the default.
static int g_prep_items = 0;
static int g_route_mode = 0;
static int g_prep_pipe = 0;  // directory path: >= 0 next tile's ids loaded ahead (default), -1 off
void set_route_tuning(int prep_items, int mode, int prep_pipe) {
  g_prep_items = prep_items;
  g_route_mode = mode;
  g_prep_pipe = prep_pipe;
}

void launch_route_fused(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                        int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir,
                        int R, int64_t C, int nargs, bool mc, int64_t req_words, uintptr_t sendbuf, uintptr_t perm,
                        uintptr_t lb, uintptr_t stats, int rank_self, DirectView dv, uintptr_t stream);

template <int K, int MODE, bool PIPE = false>
static void launch_prep(dim3 g, hipStream_t s, uintptr_t actor, int64_t M, int64_t P, uintptr_t table, uint64_t cap,
                        uintptr_t dir, uint32_t n_dir, int R, uintptr_t route, uintptr_t hist, uint32_t aw = 0,
                        const MetaCols* mc = nullptr, const CapFold* cf = nullptr) {
  const int aw_shift = (aw && (aw & (aw - 1)) == 0) ? __builtin_ctz(aw) : -1;
  const CapFold fold = cf ? *cf : CapFold{};
  if (mc)
    hipLaunchKernelGGL((route_prep_kernel<K, MODE, true, PIPE>), g, dim3(kRouteThreads), 0, s, (const uint32_t*)actor,
                       M, P, (const TableEntry*)table, cap - 1, (const uint32_t*)dir, n_dir, aw, aw_shift, R,
                       (uint32_t*)route, (uint32_t*)hist, *mc, fold);
  else
    hipLaunchKernelGGL((route_prep_kernel<K, MODE, false, PIPE>), g, dim3(kRouteThreads), 0, s, (const uint32_t*)actor,
                       M, P, (const TableEntry*)table, cap - 1, (const uint32_t*)dir, n_dir, aw, aw_shift, R,
                       (uint32_t*)route, (uint32_t*)hist, MetaCols{}, fold);
}

// Region sizes of wire format v2 (u32 words; see the header comment).
int64_t wire_req_words(int64_t C, int nargs, bool mc) {
  const int64_t w = 4 + C * (1 + (mc ? 1 : 0) + 2 * nargs);
  return (w + 3) & ~3ll;
}
int64_t wire_rep_words(int64_t C) {
  const int64_t w = 4 + 2 * C + (C + 3) / 4;
  return (w + 3) & ~3ll;
}

static void check_format(int nargs, int64_t C, int R) {
  if (nargs < 1 || nargs > 3) throw std::invalid_argument("wire format: 1 <= nargs <= 3");
  if (R < 1 || R > kMaxRanks) throw std::invalid_argument("route: 1 <= R <= 64");
  if (C < 1 || C >= (1ll << 31) / R) throw std::invalid_argument("route: bad capacity");
}

#define PT_FORMAT_SWITCH(nargs, mc, F) \
  switch ((nargs) * 2 + ((mc) ? 1 : 0)) { \
    case 2: F(1, false); break;          \
    case 3: F(1, true); break;           \
    case 4: F(2, false); break;          \
    case 5: F(2, true); break;           \
    case 6: F(3, false); break;          \
    default: F(3, true); break;          \
  }

static DirectView make_direct(const std::vector<uintptr_t>& direct, int self) {
  DirectView dv;
  if (!direct.empty()) {
    if (direct.size() != 3) throw std::invalid_argument("direct: [src, out_val, out_status]");
    dv.src = (int32_t*)direct[0];
    dv.out_val = (int64_t*)direct[1];
    dv.out_st = (int32_t*)direct[2];
    dv.self = self;
  }
  return dv;
}

int64_t route_prep_scan(uintptr_t actor, int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir,
                        uint32_t n_dir, int R, int64_t C, int64_t req_words, uintptr_t sendbuf, uintptr_t route,
                        uintptr_t hist, uintptr_t stats, int rank_self, uint32_t affine_w, uintptr_t stream,
                        int64_t* P_out);

void launch_route(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                  int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir, int R,
                  int64_t C, int nargs, bool mc, uintptr_t sendbuf, uintptr_t perm, uintptr_t route, uintptr_t hist,
                  uintptr_t lb, uintptr_t stats, int rank_self, const std::vector<uintptr_t>& direct,
                  uint32_t affine_w, uintptr_t stream) {
  const DirectView dv = make_direct(direct, rank_self);
  check_format(nargs, C, R);
  if (cap == 0 || (cap & (cap - 1))) throw std::invalid_argument("table capacity must be a power of two");
  if (method_col && !mc) throw std::invalid_argument("route: method column needs a method-column wire format");
  const int64_t req_words = wire_req_words(C, nargs, mc);
  if (g_route_mode == 1 && lb) {
    launch_route_fused(actor, a0, a1, a2, method_col, method_uniform, M, table, cap, dir, n_dir, R, C, nargs, mc,
                       req_words, sendbuf, perm, lb, stats, rank_self, dv, stream);
    return;
  }
  int64_t P;
  const int64_t G = route_prep_scan(actor, method_uniform, M, table, cap, dir, n_dir, R, C, req_words, sendbuf, route,
                                    hist, stats, rank_self, affine_w, stream, &P);
  hipStream_t s = as_stream(stream);
  if (M > 0) {
#define PT_SCATTER(NA, MCV)                                                                                         \
  hipLaunchKernelGGL((route_scatter_kernel<NA, MCV>), dim3((unsigned)G), dim3(kRouteThreads), 0, s,                  \
                     (const uint32_t*)route, (const int64_t*)a0, (const int64_t*)a1, (const int64_t*)a2,             \
                     (const uint16_t*)method_col, (uint32_t)method_uniform, M, P, R, C, (const uint32_t*)hist,      \
                     (uint32_t*)sendbuf, req_words, (int32_t*)perm, dv)
    PT_FORMAT_SWITCH(nargs, mc, PT_SCATTER)
#undef PT_SCATTER
  }
  PT_HIP_CHECK(hipGetLastError());
}

// Pass 1 of the 3-pass route (shared by wire formats v2 and v3): route words +
// block histograms.  Independent of the wire layout, so the v3 engine runs it
// while the host waits for the layout agreement.  Returns G; *P_out = P.
int64_t route_prep(uintptr_t actor, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir, int R,
                   uintptr_t route, uintptr_t hist, uint32_t affine_w, uintptr_t stream, int64_t* P_out,
                   const MetaCols* mc, const CapFold* cf) {
  if (cf && R + 1 > kMaxCapCols) throw std::invalid_argument("route_prep: capacity fold needs R <= 64");
  int64_t P;
  const int64_t G = route_grid(M, &P);
  *P_out = P;
  hipStream_t s = as_stream(stream);
  if (M > 0) {
    const dim3 g((unsigned)G);
    const int k = g_prep_items;
    if (affine_w && n_dir) {
      launch_prep<4, 2>(g, s, actor, M, P, table, cap, 0, n_dir, R, route, hist, affine_w, mc, cf);
    } else if (dir && n_dir) {
      // measured (tools/prep_sweep.py, 4 Mi messages, 1M-actor directory, R = 8): prep
      // 33.3 us at 2 items, 30.3 at 4 items with the next tile's ids loaded ahead
      // (profiles/r2_prep_sweep.txt) -- the gathers into a directory that does not
      // fit one XCD's L2 next to the streams bound it, not the id-load latency
      if (g_prep_pipe >= 0) {
        if (k == 4) launch_prep<4, 1, true>(g, s, actor, M, P, table, cap, dir, n_dir, R, route, hist, 0, mc, cf);
        else if (k == 8) launch_prep<8, 1, true>(g, s, actor, M, P, table, cap, dir, n_dir, R, route, hist, 0, mc, cf);
        else if (k == 2) launch_prep<2, 1, true>(g, s, actor, M, P, table, cap, dir, n_dir, R, route, hist, 0, mc, cf);
        else launch_prep<4, 1, true>(g, s, actor, M, P, table, cap, dir, n_dir, R, route, hist, 0, mc, cf);
      } else if (k == 1) launch_prep<1, 1>(g, s, actor, M, P, table, cap, dir, n_dir, R, route, hist, 0, mc, cf);
      else if (k == 4) launch_prep<4, 1>(g, s, actor, M, P, table, cap, dir, n_dir, R, route, hist, 0, mc, cf);
      else if (k == 8) launch_prep<8, 1>(g, s, actor, M, P, table, cap, dir, n_dir, R, route, hist, 0, mc, cf);
      else launch_prep<2, 1>(g, s, actor, M, P, table, cap, dir, n_dir, R, route, hist, 0, mc, cf);
    } else {
      // probe path: 2 lookups in flight per thread is best; 4 costs occupancy (98 VGPRs)
      if (k == 1) launch_prep<1, 0>(g, s, actor, M, P, table, cap, 0, 0, R, route, hist, 0, mc, cf);
      else if (k == 4) launch_prep<4, 0>(g, s, actor, M, P, table, cap, 0, 0, R, route, hist, 0, mc, cf);
      else launch_prep<2, 0>(g, s, actor, M, P, table, cap, 0, 0, R, route, hist, 0, mc, cf);
    }
  } else {
    PT_HIP_CHECK(hipMemsetAsync((void*)hist, 0, sizeof(uint32_t) * (R + 1) * G, s));
  }
  PT_HIP_CHECK(hipGetLastError());
  return G;
}

// Pass 2: per-destination bases and slot headers in regions of `req_words`.
void route_scan(int64_t G, int R, int64_t C, int64_t req_words, uintptr_t sendbuf, uintptr_t hist,
                int method_uniform, uintptr_t stats, int rank_self, uintptr_t stream) {
#define PT_SCAN(K)                                                                                              \
  hipLaunchKernelGGL(K, dim3(1), dim3(1024), 0, as_stream(stream), (uint32_t*)hist, (int)G, R, C, (uint32_t*)sendbuf, \
                     req_words, (uint32_t)method_uniform, (unsigned long long*)stats, rank_self)
  if (R + 1 <= 2) PT_SCAN(route_scan_kernel<2>);
  else if (R + 1 <= 5) PT_SCAN(route_scan_kernel<5>);
  else if (R + 1 <= 9) PT_SCAN(route_scan_kernel<9>);
  else if (R + 1 <= 17) PT_SCAN(route_scan_kernel<17>);
  else PT_SCAN(route_scan_wide_kernel);
#undef PT_SCAN
  PT_HIP_CHECK(hipGetLastError());
}

int64_t route_prep_scan(uintptr_t actor, int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir,
                        uint32_t n_dir, int R, int64_t C, int64_t req_words, uintptr_t sendbuf, uintptr_t route,
                        uintptr_t hist, uintptr_t stats, int rank_self, uint32_t affine_w, uintptr_t stream,
                        int64_t* P_out) {
  const int64_t G = route_prep(actor, M, table, cap, dir, n_dir, R, route, hist, affine_w, stream, P_out, nullptr, nullptr);
  route_scan(G, R, C, req_words, sendbuf, hist, method_uniform, stats, rank_self, stream);
  return G;
}

void launch_dispatch(uintptr_t recv, int R, int64_t C, int nargs, bool mc, uintptr_t reply, uintptr_t state,
                     uint32_t n_state, uint64_t delay_ticks, uintptr_t stats, int64_t expected_per_rank,
                     const std::vector<uintptr_t>& outbox, uint64_t outbox_cap, const std::vector<uintptr_t>& direct,
                     int self, uintptr_t stream) {
  const DirectView dv = make_direct(direct, self);
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
  check_format(nargs, C, R);
  const int64_t per = expected_per_rank > 0 ? expected_per_rank : C;
  const unsigned gx = grid_cap(per, 256, (unsigned)(4096 / R > 0 ? 4096 / R : 1));
  const int64_t req_words = wire_req_words(C, nargs, mc), rep_words = wire_rep_words(C);
  const unsigned stage_cap = outbox_cap ? kOutboxStage : 0;  // LDS stage only where handlers can send
  const size_t smem = stage_cap ? outbox_stage_bytes(stage_cap) : 0;
#define PT_DISPATCH(NA, MCV)                                                                                    \
  hipLaunchKernelGGL((dispatch_kernel<NA, MCV>), dim3(gx, R), dim3(256), smem, as_stream(stream),               \
                     (const uint32_t*)recv, req_words, C, (uint32_t*)reply, rep_words, (int64_t*)state, n_state, \
                     delay_ticks, (unsigned long long*)stats, ob, dv, stage_cap)
  PT_FORMAT_SWITCH(nargs, mc, PT_DISPATCH)
#undef PT_DISPATCH
  PT_HIP_CHECK(hipGetLastError());
}

void launch_complete(uintptr_t rep, int64_t C, uintptr_t perm, int64_t M, uintptr_t out_val, uintptr_t out_st,
                     uintptr_t checksum, bool direct, uintptr_t stream, uintptr_t failed) {
  if (M <= 0) return;
  if (C < 1 || C > 0x7fffffff) throw std::invalid_argument("complete: bad capacity");
  hipLaunchKernelGGL(complete_kernel, dim3(grid_cap(M, 256, checksum ? 1024 : 8192)), dim3(256), 0,
                     as_stream(stream), (const uint32_t*)rep, wire_rep_words(C), (uint32_t)C, (const int32_t*)perm, M,
                     (int64_t*)out_val, (int32_t*)out_st, (unsigned long long*)checksum, direct,
                     (const uint64_t*)failed);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_local_send(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                       int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir,
                       uint32_t affine_w, uintptr_t state, uint32_t n_state, uint64_t delay_ticks,
                       const std::vector<uintptr_t>& outbox, uint64_t outbox_cap, uintptr_t out_val, uintptr_t out_st,
                       uintptr_t stats, uintptr_t checksum, uintptr_t stream, uintptr_t m_dev) {
  if (M <= 0) return;
  if (cap == 0 || (cap & (cap - 1))) throw std::invalid_argument("table capacity must be a power of two");
  if (!actor || !a0 || !out_val || !out_st || !stats) throw std::invalid_argument("local send: missing column");
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
  const int aw_shift = (affine_w && (affine_w & (affine_w - 1)) == 0) ? __builtin_ctz(affine_w) : -1;
  const int mode = (affine_w && n_dir) ? 2 : (dir && n_dir) ? 1 : 0;
  const bool fixed = !method_col && method_uniform == kCalculatorMultiply;
  constexpr unsigned max_blocks = 16384u;
  // The calculator on the directory path (the gather-bound hot path): one tile per
  // block, 8-16 K blocks -- measured (profiles/r2_local_items_sweep.txt) 2 Mi msgs:
  // 1 item x 8192 blocks 67.4 G msg/s vs 4 x 2048 59.1; 8 Mi: 2 x 16384 101.1 vs
  // 4 x 8192 94.8.  The gather-free affine path and outbox-sending handlers keep
  // 4 items x <= 8192 blocks (8 Mi affine: 122 vs 112; token-ring tells: 14.8 vs
  // 11.3 G msg/s -- smaller tiles mean more outbox reservations).
  const bool hot = fixed && mode == 1;
  const int kk = !hot ? 4 : M <= 256ll * 8192 ? 1 : M <= 2ll * 256 * 16384 ? 2 : 4;
  // outbox sends staged in LDS (the hot calculator method never sends), published
  // with one reservation per 2 tiles: every reservation is a returning atomic on the
  // outbox count, and same-address atomics serialise (token-ring tells: 1 -> 14.6,
  // 2 -> 15.5, 4 -> 15.2 G msg/s)
  constexpr unsigned ot = 2;
  const bool sends = outbox_cap && !fixed;
  const dim3 g(grid_cap(M, 256 * kk * (sends ? ot : 1u), hot ? max_blocks : 8192u));
  const unsigned stage_cap = sends ? 256u * kk * ot : 0;
  const size_t smem = stage_cap ? outbox_stage_bytes(stage_cap) : 0;
#define PT_LOCAL_K(MO, FX, KK)                                                                                        \
  hipLaunchKernelGGL((local_send_kernel<MO, FX, KK>), g, dim3(256), smem, as_stream(stream), (const uint32_t*)actor, \
                     (const int64_t*)a0, (const int64_t*)a1, (const int64_t*)a2, (const uint16_t*)method_col,       \
                     (uint32_t)method_uniform, M, (const TableEntry*)table, cap - 1, (const uint32_t*)dir, n_dir,     \
                     affine_w, aw_shift, (int64_t*)state, n_state, delay_ticks, ob, (int64_t*)out_val,              \
                     (int32_t*)out_st, (unsigned long long*)stats, (unsigned long long*)checksum, stage_cap,       \
                     (const unsigned long long*)m_dev)
#define PT_LOCAL(MO, FX)                  \
  switch (kk) {                           \
    case 1: PT_LOCAL_K(MO, FX, 1); break; \
    case 2: PT_LOCAL_K(MO, FX, 2); break; \
    default: PT_LOCAL_K(MO, FX, 4);       \
  }
  if (mode == 2) {
    if (fixed) PT_LOCAL(2, kCalculatorMultiply) else PT_LOCAL(2, 0)
  } else if (mode == 1) {
    if (fixed) PT_LOCAL(1, kCalculatorMultiply) else PT_LOCAL(1, 0)
  } else {
    if (fixed) PT_LOCAL(0, kCalculatorMultiply) else PT_LOCAL(0, 0)
  }
#undef PT_LOCAL_K
#undef PT_LOCAL
  PT_HIP_CHECK(hipGetLastError());
}

// Device-driven pump epochs (ActorExchange.pump at world 1): the consumed outbox
// bank's count becomes the epoch's record and is reset for the bank's next turn.
__global__ void outbox_advance_kernel(unsigned long long* __restrict__ count, uint64_t cap,
                                      long long* __restrict__ epoch_m, int64_t j) {
  const unsigned long long n = count[0];
  epoch_m[j] = (long long)(n < cap ? n : cap);
  count[0] = 0;
}

// Multi-rank device-counted epochs route a bank's FULL capacity (the route and
// all-to-all passes take host sizes); the slots past the bank's device count
// become no-actor messages (answered locally, never on the wire).
__global__ __launch_bounds__(256) void outbox_seal_kernel(uint32_t* __restrict__ actor, uint64_t cap,
                                                          const unsigned long long* __restrict__ count) {
  const unsigned long long n0 = count[0];
  const uint64_t n = n0 < cap ? n0 : cap;
  for (uint64_t i = n + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x)
    actor[i] = 0xffffffffu;
}

void launch_outbox_seal(uintptr_t actor, uint64_t cap, uintptr_t count, uintptr_t stream) {
  if (!actor || !count) throw std::invalid_argument("outbox_seal: null buffer");
  if (cap == 0) return;
  hipLaunchKernelGGL(outbox_seal_kernel, dim3(grid_cap((int64_t)cap, 256, 1024)), dim3(256), 0, as_stream(stream),
                     (uint32_t*)actor, cap, (const unsigned long long*)count);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_outbox_advance(uintptr_t count, uint64_t cap, uintptr_t epoch_m, int64_t j, uintptr_t stream) {
  if (!count || !epoch_m || j < 0) throw std::invalid_argument("outbox_advance: null buffer or negative index");
  hipLaunchKernelGGL(outbox_advance_kernel, dim3(1), dim3(1), 0, as_stream(stream), (unsigned long long*)count, cap,
                     (long long*)epoch_m, j);
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
