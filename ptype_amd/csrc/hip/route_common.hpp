// Route kernels' shared device code: registry lookups (hash probe / route
// directory) and the stable in-order placement of one tile of messages into the
// epoch slots (wire format v2, see batch.hip).  Used by the 3-pass route
// (batch.hip) and the single-pass look-back route (route_fused.hip).
#pragma once
#include "common.hpp"

namespace ptype {

constexpr int kMaxRanks = 64;
constexpr int kRouteThreads = 256;
constexpr int kScatterItems = 2;
constexpr int kScatterTile = kRouteThreads * kScatterItems;
constexpr uint32_t kRouteNoActor = 0xffu;  // route word rank byte for a registry miss
constexpr uint32_t kMaxMbox = 1u << 24;

// Resolve `key` against one probe group held in registers.  Written with named
// registers and selects, not an indexed array + early return: that form made
// hipcc spill the group to scratch and serialise every lookup on vmcnt(0).
__device__ __forceinline__ void check_entry(const uint4& e, uint64_t key, int& rank, uint32_t& mbox, bool& done) {
  const uint64_t k = ((uint64_t)e.y << 32) | e.x;
  const bool hit = !done && k == key;
  const bool miss = !done && k == kKeyEmpty;
  rank = hit ? (int)e.z : rank;
  mbox = hit ? e.w : mbox;
  done = done || hit || miss;
}

// Linear group probing from group `g` on (the first `skip` slots already checked).
__device__ __forceinline__ void lookup_from(const TableEntry* __restrict__ t, uint64_t mask, uint64_t key, uint64_t g,
                                            uint64_t skip, int& rank, uint32_t& mbox, bool& done) {
  for (uint64_t step = skip; step <= mask && !done; step += kGroup, g = (g + kGroup) & mask) {
    const uint4* p = reinterpret_cast<const uint4*>(t + g);
    const uint4 e0 = p[0], e1 = p[1], e2 = p[2], e3 = p[3];  // one 64-B line, four loads in flight
    check_entry(e0, key, rank, mbox, done);
    check_entry(e1, key, rank, mbox, done);
    check_entry(e2, key, rank, mbox, done);
    check_entry(e3, key, rank, mbox, done);
  }
}

__device__ __forceinline__ void lookup_entry(const TableEntry* __restrict__ t, uint64_t mask, uint64_t key,
                                             int& rank, uint32_t& mbox) {
  rank = -1;
  mbox = 0;
  bool done = false;
  lookup_from(t, mask, key, probe_start(key, mask), 0, rank, mbox, done);
}

// K independent lookups with all K first-group lines in flight at once (the
// registry is L2/MALL resident, so a lookup is latency- not bandwidth-bound:
// memory-level parallelism per thread is what hides it).  Keys that miss their
// first group (rare at load factor <= 0.5) continue one at a time.
template <int K>
__device__ __forceinline__ void lookup_many(const TableEntry* __restrict__ t, uint64_t mask, const uint64_t (&key)[K],
                                            int (&rank)[K], uint32_t (&mbox)[K]) {
  uint4 e[K][kGroup];
  uint64_t g[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    g[k] = probe_start(key[k], mask);
    const uint4* p = reinterpret_cast<const uint4*>(t + g[k]);
#pragma unroll
    for (int j = 0; j < kGroup; ++j) e[k][j] = p[j];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    bool done = false;
    rank[k] = -1;
    mbox[k] = 0;
#pragma unroll
    for (int j = 0; j < kGroup; ++j) check_entry(e[k][j], key[k], rank[k], mbox[k], done);
    if (!done) lookup_from(t, mask, key[k], (g[k] + kGroup) & mask, kGroup, rank[k], mbox[k], done);
  }
}

// Records are packed at a stride of 5/6/7/8 dwords, so they are only dword
// aligned; gfx950 global memory takes dword-aligned multi-dword accesses, so
// move them as x4/x2/x1 chunks (declared 4-B aligned) instead of one u32 per op.
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));

template <int K>
__device__ __forceinline__ void store_words(uint32_t* p, const uint32_t (&w)[K]) {
  int j = 0;
#pragma unroll
  for (; j + 4 <= K; j += 4) *reinterpret_cast<u32x4a*>(p + j) = u32x4a{w[j], w[j + 1], w[j + 2], w[j + 3]};
  if constexpr (K % 4 >= 2) {
    *reinterpret_cast<u32x2a*>(p + j) = u32x2a{w[j], w[j + 1]};
    j += 2;
  }
  if constexpr (K % 2 == 1) p[K - 1] = w[K - 1];
}

template <int K>
__device__ __forceinline__ void load_words(const uint32_t* p, uint32_t (&w)[K]) {
  int j = 0;
#pragma unroll
  for (; j + 4 <= K; j += 4) {
    const u32x4a v = *reinterpret_cast<const u32x4a*>(p + j);
    w[j] = v.x, w[j + 1] = v.y, w[j + 2] = v.z, w[j + 3] = v.w;
  }
  if constexpr (K % 4 >= 2) {
    const u32x2a v = *reinterpret_cast<const u32x2a*>(p + j);
    w[j] = v.x, w[j + 1] = v.y;
    j += 2;
  }
  if constexpr (K % 2 == 1) w[K - 1] = p[K - 1];
}

// Direct completion of self-directed messages: the scatter records, for every
// message routed to this rank's own slot, the message index at its slot position
// (`src`), and writes the no-actor / overflow statuses straight into the caller's
// outputs; the dispatch of the own slot then writes each reply into the caller's
// arrays, so no reply staging and no completion pass are needed for them (all of
// them at N = 1).  Passed BY VALUE (never take the address of a kernel argument).
struct DirectView {
  int32_t* src = nullptr;  // [C]: slot position -> message index (self slot)
  int64_t* out_val = nullptr;
  int32_t* out_st = nullptr;
  int self = -1;
  bool identity = false;  // positions ARE message indices: src is not written
};

// One scatter tile's inputs, loaded ahead of its placement (scatter_load), so a
// block can have the next tile's loads in flight across this tile's barriers.
struct ScatterIn {
  uint32_t rw[kScatterItems];
  uint32_t meth[kScatterItems];
  int64_t v[kScatterItems][3];
};

template <int NARGS, bool MC, class RouteAt>
__device__ __forceinline__ void scatter_load(int64_t tile, int64_t hi, RouteAt route_at,
                                             const int64_t* __restrict__ a0, const int64_t* __restrict__ a1,
                                             const int64_t* __restrict__ a2,
                                             const uint16_t* __restrict__ method_col, uint32_t method_uniform,
                                             ScatterIn& x) {
#pragma unroll
  for (int k = 0; k < kScatterItems; ++k) {
    const int64_t i = tile + k * kRouteThreads + threadIdx.x;
    const bool in = i < hi;
    x.rw[k] = in ? route_at(i) : kRouteNoActor;
    x.v[k][0] = in ? a0[i] : 0;
    x.v[k][1] = NARGS > 1 && in && a1 ? a1[i] : 0;
    x.v[k][2] = NARGS > 2 && in && a2 ? a2[i] : 0;
    x.meth[k] = MC ? (in && method_col ? (uint32_t)method_col[i] : method_uniform) : 0u;
  }
}

// Place the tile [tile, min(tile + kScatterTile, hi)) in message order.
// `perm` may be null only with direct completion at world 1 (nothing comes back).
// `run[d]` is the next free slot position of destination d for this block and
// is advanced past the tile.  Block-level: every thread of the block must call
// it (two barriers inside).
template <class Emit>
__device__ __forceinline__ void scatter_place(int64_t tile, int64_t hi, const ScatterIn& x, int R, int64_t C,
                                              Emit emit, int32_t* __restrict__ perm,
                                              unsigned (&cnt)[kScatterItems][kRouteThreads / kWave][kMaxRanks],
                                              unsigned* run, DirectView dv) {
  const unsigned tid = threadIdx.x, w = tid / kWave, lane = lane_id();
  int d[kScatterItems];
  unsigned rk[kScatterItems];
#pragma unroll
  for (int k = 0; k < kScatterItems; ++k) {
    const int64_t i = tile + k * kRouteThreads + tid;
    d[k] = (i < hi && (x.rw[k] & 0xff) != kRouteNoActor) ? (int)(x.rw[k] & 0xff) : -1;
    rk[k] = 0;
  }
  // rank within (item k, wave w, destination): ballots, peeled per present destination
#pragma unroll
  for (int k = 0; k < kScatterItems; ++k) {
    unsigned c = 0;  // lane l counts destination l (R <= 64): one LDS store per lane, not one per destination
    uint64_t active = __ballot(d[k] >= 0);
    while (active) {
      const int leader = __builtin_ctzll(active);
      const int dl = __builtin_amdgcn_readlane(d[k], leader);
      const uint64_t m = __ballot(d[k] == dl);
      if (d[k] == dl) rk[k] = mbcnt64(m);
      if (lane == (unsigned)dl) c = (unsigned)__popcll(m);
      active &= ~m;
    }
    if (lane < (unsigned)R) cnt[k][w][lane] = c;
  }
  __syncthreads();
  // per destination: exclusive prefix in message order (k-major, then wave)
  for (int q = tid; q < R; q += blockDim.x) {
    unsigned r = run[q];
    for (int k = 0; k < kScatterItems; ++k)
      for (int ww = 0; ww < kRouteThreads / kWave; ++ww) {
        const unsigned c = cnt[k][ww][q];
        cnt[k][ww][q] = r;
        r += c;
      }
    run[q] = r;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kScatterItems; ++k) {
    const int64_t i = tile + k * kRouteThreads + tid;
    if (i >= hi) continue;
    if (d[k] < 0) {
      if (perm) perm[i] = -2;
      if (dv.src) {
        dv.out_val[i] = 0;
        dv.out_st[i] = kStatusNoActor;
      }
      continue;
    }
    const int64_t pos = (int64_t)cnt[k][w][d[k]] + rk[k];
    if (pos >= C) {
      if (perm) perm[i] = -1;
      if (dv.src) {
        dv.out_val[i] = 0;
        dv.out_st[i] = kStatusOverflow;
      }
      continue;
    }
    if (dv.src && d[k] == dv.self) {
      if (perm) perm[i] = -3;  // completed by the dispatch of the own slot
      if (!dv.identity) dv.src[pos] = (int32_t)i;
    } else {
      perm[i] = (int32_t)((int64_t)d[k] * C + pos);  // never null here: remote replies need it
    }
    emit(d[k], pos, x.rw[k] >> 8, x.v[k], x.meth[k]);
  }
  __syncthreads();
}


// Load + place in one call (callers without cross-tile prefetch).
template <int NARGS, bool MC, class RouteAt, class Emit>
__device__ __forceinline__ void scatter_tile(int64_t tile, int64_t hi, RouteAt route_at,
                                             const int64_t* __restrict__ a0, const int64_t* __restrict__ a1,
                                             const int64_t* __restrict__ a2,
                                             const uint16_t* __restrict__ method_col, uint32_t method_uniform,
                                             int R, int64_t C, Emit emit, int32_t* __restrict__ perm,
                                             unsigned (&cnt)[kScatterItems][kRouteThreads / kWave][kMaxRanks],
                                             unsigned* run, DirectView dv) {
  ScatterIn x;
  scatter_load<NARGS, MC>(tile, hi, route_at, a0, a1, a2, method_col, method_uniform, x);
  scatter_place(tile, hi, x, R, C, emit, perm, cnt, run, dv);
}

// Wire format v2 record writer for scatter_tile: mbox, [method], args as lo/hi
// dword pairs at a fixed stride of 1 + MC + 2 * NARGS dwords.
template <int NARGS, bool MC>
struct V2Emit {
  uint32_t* sendbuf;
  int64_t req_words;
  __device__ __forceinline__ void operator()(int d, int64_t pos, uint32_t mbox, const int64_t (&v)[3],
                                             uint32_t meth) const {
    constexpr int kStride = 1 + (MC ? 1 : 0) + 2 * NARGS;
    uint32_t* o = sendbuf + (int64_t)d * req_words + 4 + pos * kStride;
    uint32_t rec[kStride];
    rec[0] = mbox;  // local mailbox index at the destination
    if constexpr (MC) rec[1] = meth & 0xffffu;
#pragma unroll
    for (int j = 0; j < NARGS; ++j) {
      rec[1 + (MC ? 1 : 0) + 2 * j] = (uint32_t)v[j];
      rec[2 + (MC ? 1 : 0) + 2 * j] = (uint32_t)((uint64_t)v[j] >> 32);
    }
    store_words<kStride>(o, rec);
  }
};

}  // namespace ptype
