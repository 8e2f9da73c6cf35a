// Batch data path of the actor runtime: the device-native `Send` pipeline.
//
//   gen_requests   synthetic client load (one MsgRecord per message)
//   route_bucket   K1: GPU-registry lookup -> destination rank -> LDS-staged
//                  counting sort -> per-rank epoch slots in HBM (send buffer)
//   <RCCL all-to-all of the epoch slots over xGMI; skipped when R == 1>
//   dispatch       K3: per received record, switch on method id into the
//                  compiled-in handler, write the reply record in place
//   <RCCL all-to-all of the reply slots back to the senders>
//   complete       K8: scatter replies back to the caller's message order
//
// Reference behaviour replaced: Client.Go fan-out + net/rpc round trip per call
// (cluster/rpc.go:69-105, :176-183) and the server's goroutine-per-request
// dispatch (stdlib, wired at example/calculator/server/server.go:16-20).
//
// Epoch slot layout, per destination rank d: [C + 1] records, record 0 is a
// header {actor = delivered count, a0 = raw count incl. overflow, a1 = sender
// rank}; records 1..C are messages.  Replies use the same [R][C+1] geometry so
// the reverse all-to-all returns every reply to the slot its request left from;
// `perm[i]` remembers that slot for message i (or -1 overflow, -2 no actor).
#include "common.hpp"
#include "handlers.hpp"

namespace ptype {

constexpr int kRouteThreads = 256;
constexpr int kRouteItems = 4;
constexpr int kRouteTile = kRouteThreads * kRouteItems;  // 1024 records = 32 KiB of LDS
constexpr int kMaxRanks = 64;

__device__ __forceinline__ void lookup_entry(const TableEntry* __restrict__ t, uint64_t mask, uint64_t key,
                                             int& rank, uint32_t& mbox) {
  rank = -1;
  mbox = 0;
  uint64_t h = mix64(key) & mask;
  for (uint64_t probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
    const uint4 e = *reinterpret_cast<const uint4*>(&t[h]);
    const uint64_t k = ((uint64_t)e.y << 32) | e.x;
    if (k == key) {
      rank = (int)e.z;
      mbox = e.w;
      return;
    }
    if (k == kKeyEmpty) return;
  }
}

__global__ __launch_bounds__(256) void gen_requests_kernel(MsgRecord* __restrict__ out, int64_t M,
                                                           uint32_t n_actors, uint16_t method, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix64(seed ^ (uint64_t)i * 0x9e3779b97f4a7c15ull);
    uint4 lo, hi;
    lo.x = (uint32_t)(h % n_actors);
    lo.y = (uint32_t)method | ((uint32_t)kFlagValid << 16);
    const int64_t a0 = (int64_t)((h >> 20) & 0xffff) - 0x8000;
    const int64_t a1 = (int64_t)((h >> 40) & 0xffff);
    lo.z = (uint32_t)a0;
    lo.w = (uint32_t)((uint64_t)a0 >> 32);
    hi.x = (uint32_t)a1;
    hi.y = (uint32_t)((uint64_t)a1 >> 32);
    hi.z = 0;
    hi.w = 0;
    uint4* o = reinterpret_cast<uint4*>(out + i);
    o[0] = lo;
    o[1] = hi;
  }
}

__global__ __launch_bounds__(kRouteThreads) void route_bucket_kernel(
    const MsgRecord* __restrict__ in, int64_t M, const TableEntry* __restrict__ table, uint64_t mask, int R,
    int64_t C, MsgRecord* __restrict__ sendbuf, int32_t* __restrict__ perm, unsigned* __restrict__ counts,
    unsigned* __restrict__ ticket, unsigned long long* __restrict__ stats, int rank_self) {
  __shared__ uint4 stage[kRouteTile * 2];        // 32 KiB: the tile, sorted by destination
  __shared__ unsigned wcnt[kRouteThreads / kWave][kMaxRanks];
  __shared__ unsigned doff[kMaxRanks + 1];       // exclusive prefix of the block's per-dest counts
  __shared__ unsigned gbase[kMaxRanks];          // reserved global base per dest
  const unsigned tid = threadIdx.x, w = tid / kWave, lane = lane_id();
  const uint4* in4 = reinterpret_cast<const uint4*>(in);
  uint4* out4 = reinterpret_cast<uint4*>(sendbuf);
  unsigned long long nomatch = 0, overflow = 0;

  for (int64_t tile = blockIdx.x * (int64_t)kRouteTile; tile < M; tile += (int64_t)gridDim.x * kRouteTile) {
    uint4 lo[kRouteItems], hi[kRouteItems];
    int dest[kRouteItems];
    unsigned lrank[kRouteItems];
#pragma unroll
    for (int k = 0; k < kRouteItems; ++k) {
      const int64_t idx = tile + k * kRouteThreads + tid;
      dest[k] = -2;  // -2: no message in this lane
      if (idx < M) {
        lo[k] = in4[idx * 2];
        hi[k] = in4[idx * 2 + 1];
      }
    }
#pragma unroll
    for (int k = 0; k < kRouteItems; ++k) {
      const int64_t idx = tile + k * kRouteThreads + tid;
      if (idx < M) {
        int r;
        uint32_t mb;
        lookup_entry(table, mask, actor_key(lo[k].x), r, mb);
        if (r >= 0 && r < R) {
          dest[k] = r;
          lo[k].x = mb;  // route: the receiver indexes its mailbox directly
          lo[k].y |= (uint32_t)kFlagRouted << 16;
        } else {
          dest[k] = -1;
          perm[idx] = -2;
          ++nomatch;
        }
      }
    }
    // wave-level ranking per destination: ballot + mbcnt, no LDS atomics
    for (int d = 0; d < R; ++d) {
      unsigned c = 0;
#pragma unroll
      for (int k = 0; k < kRouteItems; ++k) {
        const uint64_t m = __ballot(dest[k] == d);
        if (dest[k] == d) lrank[k] = c + mbcnt64(m);
        c += (unsigned)__popcll(m);
      }
      if (lane == 0) wcnt[w][d] = c;
    }
    __syncthreads();
    if (tid < (unsigned)R) {
      unsigned tot = 0;
      for (unsigned x = 0; x < kRouteThreads / kWave; ++x) tot += wcnt[x][tid];
      gbase[tid] = tot ? atomicAdd(&counts[tid], tot) : 0u;
      doff[tid + 1] = tot;
    }
    __syncthreads();
    if (tid == 0) {
      doff[0] = 0;
      for (int d = 0; d < R; ++d) doff[d + 1] += doff[d];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRouteItems; ++k) {
      const int d = dest[k];
      if (d < 0) continue;
      unsigned woff = 0;
      for (unsigned x = 0; x < w; ++x) woff += wcnt[x][d];
      const unsigned pin = woff + lrank[k];
      const unsigned lp = doff[d] + pin;
      stage[lp * 2] = lo[k];
      stage[lp * 2 + 1] = hi[k];
      const int64_t idx = tile + k * kRouteThreads + tid;
      const int64_t slot = (int64_t)gbase[d] + pin;
      if (slot < C) {
        perm[idx] = (int32_t)((int64_t)d * (C + 1) + 1 + slot);
      } else {
        perm[idx] = -1;
        ++overflow;
      }
    }
    __syncthreads();
    // write-out: consecutive lanes write consecutive 16-B halves of the sorted tile
    const unsigned nb = doff[R];
    for (unsigned q = tid; q < nb * 2; q += kRouteThreads) {
      const unsigned p = q >> 1;
      int d = 0;
      while (d + 1 < R && doff[d + 1] <= p) ++d;
      const int64_t slot = (int64_t)gbase[d] + (p - doff[d]);
      if (slot < C) out4[((int64_t)d * (C + 1) + 1 + slot) * 2 + (q & 1)] = stage[q];
    }
    __syncthreads();
  }

  for (int off = 32; off > 0; off >>= 1) {
    nomatch += __shfl_xor(nomatch, off);
    overflow += __shfl_xor(overflow, off);
  }
  if (lane == 0 && (nomatch | overflow)) {
    atomicAdd(&stats[0], nomatch);
    atomicAdd(&stats[1], overflow);
  }
  // last-arriving block publishes the per-destination headers
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(ticket, 1u);
    if (prev == gridDim.x - 1) {
      for (int d = 0; d < R; ++d) {
        const unsigned raw = atomicAdd(&counts[d], 0u);
        uint4 h0, h1;
        h0.x = raw < C ? raw : (unsigned)C;
        h0.y = (uint32_t)kFlagValid << 16;
        h0.z = raw;
        h0.w = 0;
        h1.x = (unsigned)rank_self;
        h1.y = 0;
        h1.z = 0;
        h1.w = 0;
        out4[(int64_t)d * (C + 1) * 2] = h0;
        out4[(int64_t)d * (C + 1) * 2 + 1] = h1;
      }
    }
  }
}

// K3 (batch form).  grid.y = source rank, grid.x tiles the slot range.
__global__ __launch_bounds__(256) void dispatch_kernel(const MsgRecord* __restrict__ recv, int64_t C,
                                                       ReplyRecord* __restrict__ reply, int64_t* __restrict__ state,
                                                       uint32_t n_state, uint64_t delay_ticks,
                                                       unsigned long long* __restrict__ stats) {
  const int d = blockIdx.y;
  const uint4* r4 = reinterpret_cast<const uint4*>(recv + (int64_t)d * (C + 1));
  const uint4 h = r4[0];
  const bool valid = (h.y >> 16) & kFlagValid;
  const int64_t count = valid ? (int64_t)(h.x < C ? h.x : C) : 0;
  ReplyRecord* rp = reply + (int64_t)d * (C + 1);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ReplyRecord hr;
    hr.value = count;
    hr.status = kStatusOk;
    hr.actor = (uint32_t)count;
    rp[0] = hr;
  }
  unsigned long long failed = 0;
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < count; s += (int64_t)gridDim.x * blockDim.x) {
    const uint4 lo = r4[(1 + s) * 2], hi = r4[(1 + s) * 2 + 1];
    MsgRecord m;
    m.actor = lo.x;
    m.method = (uint16_t)(lo.y & 0xffff);
    m.flags = (uint16_t)(lo.y >> 16);
    m.a0 = (int64_t)(((uint64_t)lo.w << 32) | lo.z);
    m.a1 = (int64_t)(((uint64_t)hi.y << 32) | hi.x);
    m.a2 = (int64_t)(((uint64_t)hi.w << 32) | hi.z);
    const ReplyRecord r = run_handler(m, state, n_state, delay_ticks);
    failed += r.status != kStatusOk;
    rp[1 + s] = r;
  }
  for (int off = 32; off > 0; off >>= 1) failed += __shfl_xor(failed, off);
  if (lane_id() == 0 && failed) atomicAdd(&stats[2], failed);
}

// K8: replies back to message order.
__global__ __launch_bounds__(256) void complete_kernel(const ReplyRecord* __restrict__ rep,
                                                       const int32_t* __restrict__ perm, int64_t M,
                                                       int64_t* __restrict__ out_val, int32_t* __restrict__ out_st,
                                                       unsigned long long* __restrict__ checksum) {
  unsigned long long sum = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t p = perm[i];
    int64_t v = 0;
    int32_t st;
    if (p >= 0) {
      const uint4 r = *reinterpret_cast<const uint4*>(rep + p);
      v = (int64_t)(((uint64_t)r.y << 32) | r.x);
      st = (int32_t)r.z;
    } else {
      st = p == -1 ? kStatusOverflow : kStatusNoActor;
    }
    out_val[i] = v;
    out_st[i] = st;
    sum += (unsigned long long)v;
  }
  if (checksum) {
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
    if (lane_id() == 0) atomicAdd(checksum, sum);
  }
}

static inline unsigned grid_cap(int64_t work, int per, unsigned cap) {
  int64_t g = (work + per - 1) / per;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

void launch_gen_requests(uintptr_t out, int64_t M, uint32_t n_actors, int method, uint64_t seed, uintptr_t stream) {
  if (M <= 0) return;
  if (n_actors == 0) throw std::invalid_argument("n_actors must be > 0");
  hipLaunchKernelGGL(gen_requests_kernel, dim3(grid_cap(M, 256, 8192)), dim3(256), 0, as_stream(stream),
                     (MsgRecord*)out, M, n_actors, (uint16_t)method, seed);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_route_bucket(uintptr_t in, int64_t M, uintptr_t table, uint64_t cap, int R, int64_t C,
                         uintptr_t sendbuf, uintptr_t perm, uintptr_t counts, uintptr_t ticket, uintptr_t stats,
                         int rank_self, uintptr_t stream) {
  if (R < 1 || R > kMaxRanks) throw std::invalid_argument("route_bucket: 1 <= R <= 64");
  if (C < 1 || C >= (1ll << 31) / R) throw std::invalid_argument("route_bucket: bad capacity");
  if (cap == 0 || (cap & (cap - 1))) throw std::invalid_argument("table capacity must be a power of two");
  // >= 1 block even for M == 0 so the last arriver still writes the headers
  const unsigned g = grid_cap(M, kRouteTile, 2048);
  hipLaunchKernelGGL(route_bucket_kernel, dim3(g), dim3(kRouteThreads), 0, as_stream(stream), (const MsgRecord*)in,
                     M, (const TableEntry*)table, cap - 1, R, C, (MsgRecord*)sendbuf, (int32_t*)perm,
                     (unsigned*)counts, (unsigned*)ticket, (unsigned long long*)stats, rank_self);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_dispatch(uintptr_t recv, int R, int64_t C, uintptr_t reply, uintptr_t state, uint32_t n_state,
                     uint64_t delay_ticks, uintptr_t stats, int64_t expected_per_rank, uintptr_t stream) {
  if (R < 1) throw std::invalid_argument("dispatch: R >= 1");
  // size the grid for the expected fill, not the capacity, so padding costs no blocks
  int64_t per = expected_per_rank > 0 ? expected_per_rank : C;
  const unsigned gx = grid_cap(per, 256, (unsigned)(4096 / R > 0 ? 4096 / R : 1));
  hipLaunchKernelGGL(dispatch_kernel, dim3(gx, R), dim3(256), 0, as_stream(stream), (const MsgRecord*)recv, C,
                     (ReplyRecord*)reply, (int64_t*)state, n_state, delay_ticks, (unsigned long long*)stats);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_complete(uintptr_t rep, uintptr_t perm, int64_t M, uintptr_t out_val, uintptr_t out_st,
                     uintptr_t checksum, uintptr_t stream) {
  if (M <= 0) return;
  hipLaunchKernelGGL(complete_kernel, dim3(grid_cap(M, 256, 8192)), dim3(256), 0, as_stream(stream),
                     (const ReplyRecord*)rep, (const int32_t*)perm, M, (int64_t*)out_val, (int32_t*)out_st,
                     (unsigned long long*)checksum);
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
