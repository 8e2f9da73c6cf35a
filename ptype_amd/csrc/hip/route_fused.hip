// K1 in one pass: registry lookup + stable bucketing + wire packing with a
// decoupled look-back across blocks (the single-pass scan of Merrill & Garland,
// per destination column).
//
// The 3-pass route (batch.hip) writes every message's route word to HBM, scans
// the block histograms in a separate one-block kernel and reads the route words
// back.  Here each block keeps its P route words in LDS:
//   phase 1  coalesced actor loads, directory / hash lookups (K in flight per
//            thread), route words -> LDS, block histogram (wave ballots)
//   phase 2  per column (R destinations + the no-actor column), one wave
//            publishes the block's aggregate, walks back over predecessor
//            blocks' 64-bit status words 64 at a time (one per lane) until an
//            inclusive prefix, publishes its own inclusive prefix; the last
//            block also writes the slot headers and the overflow / no-actor
//            statistics
//   phase 3  the same tile placement as the 3-pass scatter (route_common.hpp),
//            reading route words from LDS
// Output is bit-identical to the 3-pass route and the CPU reference.
//
// Status: opt-in (set_route_tuning(mode=1)).  Measured on MI355X it is slower
// than the 3-pass route: status words must be read at agent scope, which on
// gfx950 means a cross-XCD round trip (~1.5-2 us) per window, and the prefix
// frontier advances ~64 blocks per round trip across ~2048 blocks.
//
// Forward progress: blocks take their position from a dynamic ticket, so every
// predecessor of a waiting block has started and none of them waits on a later
// block.  Status words are {epoch:32, flag:2, value:30}; the epoch lives in the
// high half of the ticket word and advances when the last ticket is handed out,
// so no memset is needed between launches -- and a captured hipGraph replays
// correctly because the epoch is read from device memory, not baked into the
// kernel arguments.
#include "route_common.hpp"

namespace ptype {

constexpr uint64_t kLbNotReady = 0, kLbAggregate = 1, kLbPrefix = 2;
constexpr uint64_t kLbValueMask = (1ull << 30) - 1;

__device__ __forceinline__ uint64_t lb_pack(uint32_t epoch, uint64_t flag, uint64_t value) {
  return ((uint64_t)epoch << 32) | (flag << 30) | (value & kLbValueMask);
}

template <int NARGS, bool MC, bool DIR>
__global__ __launch_bounds__(kRouteThreads) void route_fused_kernel(
    const uint32_t* __restrict__ actor, const int64_t* __restrict__ a0, const int64_t* __restrict__ a1,
    const int64_t* __restrict__ a2, const uint16_t* __restrict__ method_col, uint32_t method_uniform, int64_t M,
    int64_t P, const TableEntry* __restrict__ table, uint64_t mask, const uint32_t* __restrict__ dir, uint32_t n_dir,
    int R, int64_t C, uint32_t* __restrict__ sendbuf, int64_t req_words, int32_t* __restrict__ perm,
    unsigned long long* __restrict__ ctrl, uint64_t* __restrict__ status, int G,
    unsigned long long* __restrict__ stats, int rank_self, DirectView dv) {
  extern __shared__ uint32_t lds_route[];  // P route words of this block
  __shared__ unsigned h[kMaxRanks + 1];
  __shared__ unsigned run[kMaxRanks];
  __shared__ unsigned cnt[kScatterItems][kRouteThreads / kWave][kMaxRanks];
  __shared__ unsigned long long s_ticket;
  __shared__ unsigned s_tot[kMaxRanks + 1];
  const unsigned tid = threadIdx.x, lane = lane_id();
  if (tid == 0) {
    const unsigned long long t = atomicAdd(ctrl, 1ull);
    s_ticket = t;
    if ((int)(t & 0xffffffffu) == G - 1)  // last ticket: open the next epoch for the next launch
      atomicExch(ctrl, ((t >> 32) + 1) << 32);
  }
  for (int d = tid; d <= R; d += blockDim.x) h[d] = 0;
  __syncthreads();
  const int b = (int)(s_ticket & 0xffffffffu);
  const uint32_t epoch = (uint32_t)(s_ticket >> 32);
  const int64_t lo = (int64_t)b * P, hi = lo + P < M ? lo + P : M;

  // ---- phase 1: route words -> LDS, block histogram
  constexpr int K = DIR ? 4 : 2;
  for (int64_t base = lo; base < hi; base += K * kRouteThreads) {
    uint32_t a[K];
    int r[K];
    uint32_t mb[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t i = base + k * kRouteThreads + tid;
      a[k] = i < hi ? actor[i] : 0u;
    }
    if constexpr (DIR) {
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
      const int64_t i = base + k * kRouteThreads + tid;
      int d = -1;
      if (i < hi) {
        const bool ok = r[k] >= 0 && r[k] < R && mb[k] < kMaxMbox;
        d = ok ? r[k] : R;
        lds_route[i - lo] = ok ? ((uint32_t)r[k] | (mb[k] << 8)) : kRouteNoActor;
      }
      uint64_t active = __ballot(d >= 0);
      while (active) {
        const int leader = __builtin_ctzll(active);
        const int dl = __shfl(d, leader);
        const uint64_t m = __ballot(d == dl);
        if (lane == (unsigned)leader) atomicAdd(&h[dl], (unsigned)__popcll(m));
        active &= ~m;
      }
    }
  }
  __syncthreads();

  // ---- phase 2: decoupled look-back, one column (R destinations + the no-actor
  // column) per wave at a time; each step reads a window of 64 predecessors' status
  // words at once (one per lane).  The words are self-contained, so relaxed
  // agent-scope atomics suffice -- no acquire/release cache maintenance per probe.
  {
    const unsigned w = tid / kWave;
    for (int c = (int)w; c <= R; c += kRouteThreads / kWave) {
      const uint64_t agg = h[c];
      uint64_t* mine = status + (int64_t)b * (R + 1) + c;
      uint64_t excl = 0;
      if (lane == 0)
        __hip_atomic_store(mine, lb_pack(epoch, b == 0 ? kLbPrefix : kLbAggregate, agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      uint64_t spins = 0;
      for (int jb = b - 1; jb >= 0;) {
        const int j = jb - (int)lane;
        uint64_t wd = lb_pack(epoch, kLbPrefix, 0);  // before block 0: an empty inclusive prefix
        if (j >= 0)
          wd = __hip_atomic_load(status + (int64_t)j * (R + 1) + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t flag = (wd >> 30) & 3;
        const bool ready = (uint32_t)(wd >> 32) == epoch && flag != kLbNotReady;
        if (__ballot(!ready)) {  // some predecessor in the window has not published yet
          if (++spins > (1ull << 24)) {  // never hang the GPU on a bug: flag it, let the host raise
            if (lane == 0) atomicOr(&stats[3], 1ull);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        const uint64_t pmask = __ballot(flag == kLbPrefix);
        // closest inclusive prefix in the window (lowest lane = nearest predecessor)
        const unsigned stop = pmask ? (unsigned)__builtin_ctzll(pmask) : 63u;
        uint64_t v = lane <= stop ? (wd & kLbValueMask) : 0;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        excl += v;
        if (pmask) break;
        jb -= kWave;
      }
      if (lane == 0) {
        if (b != 0)
          __hip_atomic_store(mine, lb_pack(epoch, kLbPrefix, excl + agg), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        if (c < R) run[c] = (unsigned)excl;
        if (b == G - 1) s_tot[c] = (unsigned)(excl + agg);
      }
    }
  }
  __syncthreads();
  if (b == G - 1) {  // totals: slot headers (+ identity flag, as the 3-pass scan) and statistics
    const bool identity = R == 1 && s_tot[1] == 0 && (int64_t)s_tot[0] <= C;
    for (int c = tid; c <= R; c += blockDim.x) {
      const uint64_t total = s_tot[c];
      if (c < R) {
        uint4* h4 = reinterpret_cast<uint4*>(sendbuf + (int64_t)c * req_words);
        const unsigned delivered = total < (uint64_t)C ? (unsigned)total : (unsigned)C;
        const uint32_t flags = kFlagValid | (identity ? kFlagIdentity : 0);
        h4[0] = make_uint4(delivered, (unsigned)total, (unsigned)rank_self, (flags << 16) | (method_uniform & 0xffffu));
        if (total > (uint64_t)C) atomicAdd(&stats[1], (unsigned long long)(total - C));
      } else if (total) {
        atomicAdd(&stats[0], (unsigned long long)total);
      }
    }
  }
  __syncthreads();

  // ---- phase 3: stable placement from the LDS route words
  auto route_at = [lo](int64_t i) { return lds_route[i - lo]; };
  for (int64_t tile = lo; tile < hi; tile += kScatterTile)
    scatter_tile<NARGS, MC>(tile, hi, route_at, a0, a1, a2, method_col, method_uniform, R, C,
                            V2Emit<NARGS, MC>{sendbuf, req_words},
                            perm, cnt, run, dv);
}

// Messages per block: 4096 (16 KB of LDS route words); larger for huge batches
// so the status array stays small.  Returns G; *P_out = P.
int64_t route_fused_grid(int64_t M, int64_t* P_out) {
  int64_t P = 4096;
  while ((M + P - 1) / P > 65536 && P < 16384) P *= 2;
  int64_t G = (M + P - 1) / P;
  if (G < 1) G = 1;
  *P_out = P;
  return G;
}

template <int NA, bool MCV, bool D>
static void launch_fused_t(int64_t G, int64_t P, hipStream_t s, uintptr_t actor, uintptr_t a0, uintptr_t a1,
                           uintptr_t a2, uintptr_t method_col, int method_uniform, int64_t M, uintptr_t table,
                           uint64_t cap, uintptr_t dir, uint32_t n_dir, int R, int64_t C, uintptr_t sendbuf,
                           int64_t req_words, uintptr_t perm, uintptr_t lb, uintptr_t stats, int rank_self,
                           DirectView dv) {
  unsigned long long* ctrl = (unsigned long long*)lb;
  uint64_t* status = (uint64_t*)lb + 1;
  hipLaunchKernelGGL((route_fused_kernel<NA, MCV, D>), dim3((unsigned)G), dim3(kRouteThreads),
                     (size_t)P * sizeof(uint32_t), s, (const uint32_t*)actor, (const int64_t*)a0, (const int64_t*)a1,
                     (const int64_t*)a2, (const uint16_t*)method_col, (uint32_t)method_uniform, M, P,
                     (const TableEntry*)table, cap - 1, (const uint32_t*)dir, n_dir, R, C, (uint32_t*)sendbuf,
                     req_words, (int32_t*)perm, ctrl, status, (int)G, (unsigned long long*)stats, rank_self, dv);
}

// `lb` = workspace of 1 + G * (R + 1) u64 words, zeroed once at allocation.
void launch_route_fused(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                        int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir,
                        int R, int64_t C, int nargs, bool mc, int64_t req_words, uintptr_t sendbuf, uintptr_t perm,
                        uintptr_t lb, uintptr_t stats, int rank_self, DirectView dv, uintptr_t stream) {
  if (M >= (1ll << 30)) throw std::invalid_argument("route: at most 2^30 messages per epoch");
  int64_t P;
  const int64_t G = route_fused_grid(M, &P);
  hipStream_t s = as_stream(stream);
  const bool d = dir && n_dir;
#define PT_FUSED(NA, MCV)                                                                                      \
  (d ? launch_fused_t<NA, MCV, true>(G, P, s, actor, a0, a1, a2, method_col, method_uniform, M, table, cap, dir, \
                                     n_dir, R, C, sendbuf, req_words, perm, lb, stats, rank_self, dv)            \
     : launch_fused_t<NA, MCV, false>(G, P, s, actor, a0, a1, a2, method_col, method_uniform, M, table, cap, 0, 0, \
                                      R, C, sendbuf, req_words, perm, lb, stats, rank_self, dv))
  switch (nargs * 2 + (mc ? 1 : 0)) {
    case 2: PT_FUSED(1, false); break;
    case 3: PT_FUSED(1, true); break;
    case 4: PT_FUSED(2, false); break;
    case 5: PT_FUSED(2, true); break;
    case 6: PT_FUSED(3, false); break;
    default: PT_FUSED(3, true); break;
  }
#undef PT_FUSED
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
