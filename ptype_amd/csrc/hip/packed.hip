// Wire format v3 kernels (see packed.hpp): the width pass that feeds the
// per-Send agreement, the packing scatter, the unpacking dispatch with a
// value-plane + ok-bitmap reply, and the completion that decodes it.
//
// Route passes 1 + 2 (route words, histograms, bases, slot headers) are the
// v2 kernels (batch.hip: route_prep_scan) run with v3 region sizes; only the
// record writer of the scatter differs (PackedEmit).
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "handlers.hpp"
#include "packed.hpp"
#include "route_common.hpp"

namespace ptype {

int64_t route_prep(uintptr_t actor, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir, int R,
                   uintptr_t route, uintptr_t hist, uint32_t affine_w, uintptr_t stream, int64_t* P_out,
                   const MetaCols* mc = nullptr, const CapFold* cf = nullptr);
void route_scan(int64_t G, int R, int64_t C, int64_t req_words, uintptr_t sendbuf, uintptr_t hist,
                int method_uniform, uintptr_t stats, int rank_self, uintptr_t stream);
int64_t route_grid(int64_t M, int64_t* P_out);
int64_t wire_rep_words(int64_t C);

constexpr int kStatTooWide = 4;  // workspace stat word: replies that did not fit vb (never, by construction)

// ---- width pass: column maxima of one batch -> meta[kMetaWords] (atomic max)
__global__ __launch_bounds__(256) void packed_meta_kernel(const uint32_t* __restrict__ actor,
                                                          const int64_t* __restrict__ a0,
                                                          const int64_t* __restrict__ a1,
                                                          const int64_t* __restrict__ a2,
                                                          const uint16_t* __restrict__ mcol, uint32_t method_uniform,
                                                          int64_t M, uint32_t n_dir, uint32_t aw,
                                                          unsigned long long* __restrict__ meta) {
  MetaAcc acc;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  // without an affine directory the mailbox bound does not depend on the actor
  // id (MetaAcc::take), so the actor column is not read at all (4 of 20 B/msg)
  const bool need_actor = aw != 0;
  // 4 elements per iteration, every load issued before any is used: the pass is
  // one streaming read of the batch and needs the memory-level parallelism
  for (; i + 3 * stride < M; i += 4 * stride) {
    uint32_t a[4] = {0, 0, 0, 0}, me[4] = {0, 0, 0, 0};
    int64_t v0[4], v1[4] = {0, 0, 0, 0}, v2[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (need_actor) a[k] = __builtin_nontemporal_load(actor + i + k * stride);
      v0[k] = __builtin_nontemporal_load(a0 + i + k * stride);
      if (a1) v1[k] = __builtin_nontemporal_load(a1 + i + k * stride);
      if (a2) v2[k] = __builtin_nontemporal_load(a2 + i + k * stride);
      if (mcol) me[k] = mcol[i + k * stride];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc.take(a[k], v0[k], v1[k], v2[k], me[k], n_dir, aw);
  }
  for (; i < M; i += stride)
    acc.take(need_actor ? actor[i] : 0u, a0[i], a1 ? a1[i] : 0, a2 ? a2[i] : 0, mcol ? (uint32_t)mcol[i] : 0u, n_dir,
             aw);
  meta_publish(acc, mcol != nullptr, method_uniform, M, meta);
}

// ---- scatter: v3 record writer for scatter_tile
template <int S>
struct PackedEmit {
  uint32_t* sendbuf;
  int64_t req_words;
  PackedLayout L;
  __device__ __forceinline__ void operator()(int d, int64_t pos, uint32_t mbox, const int64_t (&v)[3],
                                             uint32_t meth) const {
    const uint64_t f[5] = {meth, mbox, zz_enc(v[0]), zz_enc(v[1]), zz_enc(v[2])};
    uint32_t rec[S];
    packed_pack<S>(L, f, rec);
    store_words<S>(sendbuf + (int64_t)d * req_words + 4 + pos * S, rec);
  }
};

template <int S>
__global__ __launch_bounds__(kRouteThreads) void route_scatter_packed_kernel(
    const uint32_t* __restrict__ route, const int64_t* __restrict__ a0, const int64_t* __restrict__ a1,
    const int64_t* __restrict__ a2, const uint16_t* __restrict__ method_col, uint32_t method_uniform, int64_t M,
    int64_t P, int R, int64_t C, const uint32_t* __restrict__ base, uint32_t* __restrict__ sendbuf,
    int64_t req_words, PackedLayout L, int32_t* __restrict__ perm, DirectView dv, bool pipe) {
  __shared__ unsigned cnt[kScatterItems][kRouteThreads / kWave][kMaxRanks];
  __shared__ unsigned run[kMaxRanks];
  for (int d = threadIdx.x; d < R; d += blockDim.x) run[d] = base[(int64_t)d * gridDim.x + blockIdx.x];
  const int64_t lo = blockIdx.x * P, hi = lo + P < M ? lo + P : M;
  if (dv.src) dv.identity = ((sendbuf[(int64_t)dv.self * req_words + 3] >> 16) & kFlagIdentity) != 0;
  __syncthreads();
  auto route_at = [route](int64_t i) { return route[i]; };
  const PackedEmit<S> emit{sendbuf, req_words, L};
  // every column is read when present (null-checked): the layout's widths say what is packed
  if (pipe) {  // the next tile's loads in flight across this tile's ranking barriers
    ScatterIn cur, nxt;
    if (lo < hi) scatter_load<3, true>(lo, hi, route_at, a0, a1, a2, method_col, method_uniform, cur);
    for (int64_t tile = lo; tile < hi; tile += kScatterTile) {
      if (tile + kScatterTile < hi)  // block-uniform
        scatter_load<3, true>(tile + kScatterTile, hi, route_at, a0, a1, a2, method_col, method_uniform, nxt);
      scatter_place(tile, hi, cur, R, C, emit, perm, cnt, run, dv);
      cur = nxt;
    }
    return;
  }
  for (int64_t tile = lo; tile < hi; tile += kScatterTile)
    scatter_tile<3, true>(tile, hi, route_at, a0, a1, a2, method_col, method_uniform, R, C, emit, perm, cnt, run, dv);
}

// ---- dispatch: unpack, run the handler, reply into the value plane + ok bitmap
// kDispU 64-slot groups per wave iteration (records loaded before any is used).
// 4 measured slower than 1 (bench --loopback 8: 25.3 vs 20.6 us per 4 Mi
// records): the pass was VALU-bound on field extraction, not latency-bound.
constexpr int kDispU = 1;

template <int S, int FIXED>
__device__ __forceinline__ unsigned long long dispatch_range_packed(
    const uint32_t* __restrict__ rq, int64_t count, uint32_t hdr_method, PackedLayout L, uint8_t* __restrict__ vals,
    unsigned long long* __restrict__ okmap, int64_t* __restrict__ state, uint32_t n_state, uint64_t delay_ticks,
    OutboxView ob, DirectView dv, bool direct, bool ident, unsigned long long& toowide) {
  unsigned long long failed = 0;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const unsigned lane = lane_id();
  // wave-uniform loop: each group covers 64 consecutive slots (base % 64 == 0),
  // so one lane writes the group's whole ok-bitmap word -- no atomics
  for (int64_t base = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~(kWave - 1)); base < count;
       base += step * kDispU) {
    uint32_t wv[kDispU][S];
#pragma unroll
    for (int u = 0; u < kDispU; ++u) {
      const int64_t s = base + u * step + lane;
      if (s < count) load_words<S>(rq + 4 + s * S, wv[u]);
    }
#pragma unroll
    for (int u = 0; u < kDispU; ++u) {
      const int64_t gb = base + u * step;  // wave-uniform
      if (gb >= count) break;
      const int64_t s = gb + lane;
      const bool in = s < count;
      ReplyRecord rr;
      rr.value = 0;
      rr.status = kStatusOk;
      if (in) {
        MsgRecord m;
        m.actor = (uint32_t)packed_field<S>(L, 1, wv[u]);
        m.method = (uint16_t)(FIXED ? FIXED : (L.w[0] ? (uint32_t)packed_field<S>(L, 0, wv[u]) : hdr_method));
        m.flags = kFlagValid | kFlagRouted;
        m.a0 = zz_dec(packed_field<S>(L, 2, wv[u]));
        m.a1 = zz_dec(packed_field<S>(L, 3, wv[u]));
        m.a2 = zz_dec(packed_field<S>(L, 4, wv[u]));
        rr = run_handler(m, state, n_state, delay_ticks, ob);
      }
      if (direct) {  // own slot: straight into the caller's outputs, no wire, no width limit
        failed += in && rr.status != kStatusOk;
        if (in) {
          const int64_t i = ident ? s : (int64_t)dv.src[s];
          dv.out_val[i] = rr.value;
          dv.out_st[i] = rr.status;
        }
        continue;
      }
      bool ok = rr.status == kStatusOk;
      uint64_t code = ok ? (L.vb == 8 ? (uint64_t)rr.value : zz_enc(rr.value)) : (uint64_t)rr.status;
      if (ok && L.vb < 8 && (code >> (8 * L.vb))) {  // impossible under the agreed bounds: fail loudly
        ok = false;
        code = kStatusFailed;
        toowide += in;
      }
      failed += in && !ok;
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
__global__ __launch_bounds__(256) void dispatch_packed_kernel(const uint32_t* __restrict__ recv, int64_t req_words,
                                                              int64_t C, PackedLayout L, uint32_t* __restrict__ reply,
                                                              int64_t rep_words, int64_t* __restrict__ state,
                                                              uint32_t n_state, uint64_t delay_ticks,
                                                              unsigned long long* __restrict__ stats, OutboxView ob,
                                                              DirectView dv, unsigned stage_cap) {
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
  unsigned long long* okmap = reinterpret_cast<unsigned long long*>(rp + 4);  // sized by the count (packed.hpp)
  uint8_t* vals = reinterpret_cast<uint8_t*>(rp + 4 + packed_ok_words(count));
  if (blockIdx.x == 0 && threadIdx.x == 0) *reinterpret_cast<uint4*>(rp) = make_uint4((uint32_t)count, 0u, 0u, 0u);
  const uint32_t hm = h.w & 0xffffu;
  const bool ident = direct && ((h.w >> 16) & kFlagIdentity);
  unsigned long long toowide = 0, failed;
  if (!L.w[0] && hm == kCalculatorMultiply)  // uniform hot method: the handler switch constant-folds
    failed = dispatch_range_packed<S, kCalculatorMultiply>(rq, count, hm, L, vals, okmap, state, n_state, delay_ticks,
                                                           ob, dv, direct, ident, toowide);
  else
    failed = dispatch_range_packed<S, 0>(rq, count, hm, L, vals, okmap, state, n_state, delay_ticks, ob, dv, direct,
                                         ident, toowide);
  if (stage_cap) outbox_flush(ob);  // every thread of the block reaches here
  for (int off = 32; off > 0; off >>= 1) {
    failed += __shfl_xor(failed, off);
    toowide += __shfl_xor(toowide, off);
  }
  if (lane_id() == 0 && failed) atomicAdd(&stats[2], failed);
  if (lane_id() == 0 && toowide) atomicAdd(&stats[kStatTooWide], toowide);
}

// ---- v2 reply regions -> v3 reply regions (mailbox delivery on receipt at N > 1:
// the drain answers in v2 geometry, in ring order; this pass writes what the
// reverse all-to-all moves).  grid (X, R), 64-slot groups per wave as dispatch.
__global__ __launch_bounds__(256) void pack_replies_kernel(const uint32_t* __restrict__ v2, int64_t v2_words,
                                                           int64_t C, uint32_t* __restrict__ reply, int64_t rep_words,
                                                           int vb, unsigned long long* __restrict__ stats) {
  const int d = blockIdx.y;
  const uint32_t* src = v2 + (int64_t)d * v2_words;
  const int64_t count = std::min<int64_t>(src[0], C);
  const int64_t* sval = reinterpret_cast<const int64_t*>(src + 4);
  const uint8_t* sst = reinterpret_cast<const uint8_t*>(src + 4 + 2 * C);
  uint32_t* rp = reply + (int64_t)d * rep_words;
  unsigned long long* okmap = reinterpret_cast<unsigned long long*>(rp + 4);
  uint8_t* vals = reinterpret_cast<uint8_t*>(rp + 4 + packed_ok_words(count));
  if (blockIdx.x == 0 && threadIdx.x == 0) *reinterpret_cast<uint4*>(rp) = make_uint4((uint32_t)count, 0u, 0u, 0u);
  const unsigned lane = lane_id();
  unsigned long long toowide = 0;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t gb = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~(kWave - 1)); gb < count; gb += step) {
    const int64_t s = gb + lane;
    const bool in = s < count;
    const int64_t value = in ? sval[s] : 0;
    const int32_t status = in ? (int32_t)sst[s] : kStatusOk;
    bool ok = status == kStatusOk;
    uint64_t code = ok ? (vb == 8 ? (uint64_t)value : zz_enc(value)) : (uint64_t)status;
    if (ok && vb < 8 && (code >> (8 * vb))) {  // impossible under the agreed bounds: fail loudly
      ok = false;
      code = kStatusFailed;
      toowide += in;
    }
    const unsigned long long bits = __ballot(in && ok);
    if (in) {
      switch (vb) {
        case 1: vals[s] = (uint8_t)code; break;
        case 2: reinterpret_cast<uint16_t*>(vals)[s] = (uint16_t)code; break;
        case 4: reinterpret_cast<uint32_t*>(vals)[s] = (uint32_t)code; break;
        default: reinterpret_cast<uint64_t*>(vals)[s] = code;
      }
    }
    if (lane == 0) okmap[gb / kWave] = bits;
  }
  for (int off = 32; off > 0; off >>= 1) toowide += __shfl_xor(toowide, off);
  if (lane == 0 && toowide) atomicAdd(&stats[kStatTooWide], toowide);
}

// ---- K8 for v3 replies: a gather per message (coalesced outputs); kCompU
// messages per thread per trip, all perm reads, then all reply reads, in flight
// (4 messages per thread per trip: 2 and 8 measured no faster, nor non-temporal stores)
constexpr int32_t kPastBatch = INT32_MIN;  // (perm codes: >= 0 slot position, -1 overflow, -2 no actor, -3 direct)

template <int kCompU>
__global__ __launch_bounds__(256) void complete_packed_kernel(const uint32_t* __restrict__ rep, int64_t rep_words,
                                                              uint32_t C, int R, int vb,
                                                              const int32_t* __restrict__ perm, int64_t M,
                                                              int64_t* __restrict__ out_val,
                                                              int32_t* __restrict__ out_st,
                                                              unsigned long long* __restrict__ checksum, bool direct,
                                                              const uint64_t* __restrict__ failed,
                                                              uint64_t* __restrict__ zero, int64_t zero_words) {
  // (an optional word range cleared on the way: the sorted exchange's next-Send
  // agreement vector, instead of a separate fill launch on the critical path)
  if (zero)
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < zero_words; w += (int64_t)gridDim.x * blockDim.x)
      zero[w] = 0;
  // each source region's value plane starts past its count-sized ok bitmap: the
  // offsets once per block in LDS, not a dependent header load per message
  __shared__ uint32_t voff[kMaxRanks];
  // a failed collective (IpcComm: a peer missed it) wrote no reply regions: every
  // message that went through one answers kStatusNotDelivered (direct completion
  // included -- its own-slot dispatch saw an empty region)
  const bool lost = failed && __hip_atomic_load(failed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  // (the count clamped to the region: a region no peer wrote this time -- a failed
  // collective -- holds whatever the buffer held, and must not move the plane out)
  for (int d = threadIdx.x; d < R; d += blockDim.x)
    voff[d] = 4 + (uint32_t)packed_ok_words(std::min<int64_t>(rep[(int64_t)d * rep_words], (int64_t)C));
  __syncthreads();
  unsigned long long sum = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < M; i0 += stride * kCompU) {
    int32_t p[kCompU];
#pragma unroll
    for (int u = 0; u < kCompU; ++u) {
      const int64_t i = i0 + u * stride;
      p[u] = i < M ? perm[i] : kPastBatch;
    }
    uint64_t code[kCompU];
    unsigned long long okw[kCompU];
#pragma unroll
    for (int u = 0; u < kCompU; ++u) {
      code[u] = 0;
      okw[u] = 0;
      if (p[u] >= 0) {
        const uint32_t d = (uint32_t)p[u] / C, pos = (uint32_t)p[u] - d * C;
        const uint32_t* rb = rep + (int64_t)d * rep_words;
        // [header][ok bitmap sized by the region's count][values]
        const uint8_t* vals = reinterpret_cast<const uint8_t*>(rb + voff[d]);
        okw[u] = reinterpret_cast<const unsigned long long*>(rb + 4)[pos / kWave] >> (pos % kWave);
        switch (vb) {
          case 1: code[u] = vals[pos]; break;
          case 2: code[u] = reinterpret_cast<const uint16_t*>(vals)[pos]; break;
          case 4: code[u] = reinterpret_cast<const uint32_t*>(vals)[pos]; break;
          default: code[u] = reinterpret_cast<const uint64_t*>(vals)[pos];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kCompU; ++u) {
      const int64_t i = i0 + u * stride;
      if (p[u] == kPastBatch) continue;
      if (lost && (p[u] >= 0 || p[u] == -3)) {
        out_val[i] = 0;
        out_st[i] = kStatusNotDelivered;
        continue;
      }
      if (direct && p[u] < 0) {
        if (checksum) sum += (unsigned long long)out_val[i];
        continue;
      }
      int64_t v = 0;
      int32_t st;
      if (p[u] >= 0) {
        if (okw[u] & 1) {
          v = vb == 8 ? (int64_t)code[u] : zz_dec(code[u]);
          st = kStatusOk;
        } else {
          st = (int32_t)code[u];
        }
      } else {
        st = p[u] == -1 ? kStatusOverflow : kStatusNoActor;
      }
      out_val[i] = v;
      out_st[i] = st;
      sum += (unsigned long long)v;
    }
  }
  if (checksum) {
    __shared__ unsigned long long part[4];
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
    if (lane_id() == 0) part[threadIdx.x / kWave] = sum;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(checksum, part[0] + part[1] + part[2] + part[3]);
  }
}

// The sorted exchange's completion (no checksum, no direct slots): the same gather as
// complete_packed_kernel with the value width a template parameter -- a third fewer
// VGPRs, so more waves hide the perm -> reply-gather chain (the kernel waits on memory
// 77 % of its wave cycles, profiles/r6_pmc_l8.txt).
template <int VB, int U>
__global__ __launch_bounds__(256) void complete_sx_kernel(const uint32_t* __restrict__ rep, int64_t rep_words,
                                                          uint32_t C, int R, const int32_t* __restrict__ perm,
                                                          int64_t M, int64_t* __restrict__ out_val,
                                                          int32_t* __restrict__ out_st,
                                                          const uint64_t* __restrict__ failed,
                                                          uint64_t* __restrict__ zero, int64_t zero_words) {
  if (zero)
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < zero_words; w += (int64_t)gridDim.x * blockDim.x)
      zero[w] = 0;
  __shared__ uint32_t voff[kMaxRanks];
  const bool lost = failed && __hip_atomic_load(failed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  for (int d = threadIdx.x; d < R; d += blockDim.x)
    voff[d] = 4 + (uint32_t)packed_ok_words(std::min<int64_t>(rep[(int64_t)d * rep_words], (int64_t)C));
  __syncthreads();
  using VT = typename std::conditional<VB == 1, uint8_t,
             typename std::conditional<VB == 2, uint16_t,
             typename std::conditional<VB == 4, uint32_t, uint64_t>::type>::type>::type;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < M; i0 += stride * U) {
    int32_t p[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      p[u] = i < M ? perm[i] : kPastBatch;
    }
    uint64_t code[U];
    uint32_t ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      code[u] = 0;
      ok[u] = 0;
      if (p[u] >= 0) {
        const uint32_t d = (uint32_t)p[u] / C, pos = (uint32_t)p[u] - d * C;
        const uint32_t* rb = rep + (int64_t)d * rep_words;
        ok[u] = (uint32_t)(reinterpret_cast<const unsigned long long*>(rb + 4)[pos / kWave] >> (pos % kWave)) & 1u;
        code[u] = reinterpret_cast<const VT*>(rb + voff[d])[pos];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (p[u] == kPastBatch) continue;
      int64_t v = 0;
      int32_t st;
      if (lost && p[u] >= 0) {
        st = kStatusNotDelivered;
      } else if (p[u] >= 0) {
        if (ok[u]) {
          v = VB == 8 ? (int64_t)code[u] : zz_dec(code[u]);
          st = kStatusOk;
        } else {
          st = (int32_t)code[u];
        }
      } else {
        st = p[u] == -1 ? kStatusOverflow : kStatusNoActor;
      }
      out_val[i] = v;
      out_st[i] = st;
    }
  }
}

void launch_complete_sx(uintptr_t rep, int64_t C, int R, int vb, uintptr_t perm, int64_t M, uintptr_t out_val,
                        uintptr_t out_st, uintptr_t stream, uintptr_t failed, uintptr_t zero, int64_t zero_words) {
  if (M <= 0) return;
  if (C < 1 || C > 0x7fffffff) throw std::invalid_argument("complete: bad capacity");
  if (R < 1 || R > kMaxRanks) throw std::invalid_argument("complete: 1 <= R <= 64");
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((M + 256 * 4 - 1) / (256 * 4), 8192));
#define PT_CSX(VBV)                                                                                                  \
  hipLaunchKernelGGL((complete_sx_kernel<VBV, 4>), dim3(g), dim3(256), 0, as_stream(stream), (const uint32_t*)rep,   \
                     packed_rep_words(C, VBV), (uint32_t)C, R, (const int32_t*)perm, M, (int64_t*)out_val,          \
                     (int32_t*)out_st, (const uint64_t*)failed, (uint64_t*)zero, zero_words)
  switch (vb) {
    case 1: PT_CSX(1); break;
    case 2: PT_CSX(2); break;
    case 4: PT_CSX(4); break;
    case 8: PT_CSX(8); break;
    default: throw std::invalid_argument("complete: vb in {1,2,4,8}");
  }
#undef PT_CSX
  PT_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- launchers
static unsigned grid_for(int64_t work, int per, unsigned cap) {
  const int64_t g = (work + per - 1) / per;
  return (unsigned)(g < 1 ? 1 : g > cap ? cap : g);
}

static DirectView direct_of(const std::vector<uintptr_t>& direct, int self) {
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

void check_packed_layout(const PackedLayout& L, int R, int64_t C) {
  if (L.S < 1 || L.S > 8) throw std::invalid_argument("packed layout: 1 <= S <= 8 dwords");
  if (L.vb != 1 && L.vb != 2 && L.vb != 4 && L.vb != 8) throw std::invalid_argument("packed layout: vb in {1,2,4,8}");
  int end = 0;
  for (int q = 0; q < 5; ++q) {
    if (L.w[q] > 64) throw std::invalid_argument("packed layout: field wider than 64 bits");
    end = std::max(end, L.off[q] + L.w[q]);
  }
  if (end > 32 * L.S) throw std::invalid_argument("packed layout: fields exceed the record");
  if (R < 1 || R > kMaxRanks) throw std::invalid_argument("route: 1 <= R <= 64");
  if (C < 1 || C >= (1ll << 31) / R) throw std::invalid_argument("route: bad capacity");
}

void launch_packed_meta(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                        int method_uniform, int64_t M, uint32_t n_dir, uint32_t affine_w, uintptr_t meta,
                        uintptr_t stream) {
  hipStream_t s = as_stream(stream);
  PT_HIP_CHECK(hipMemsetAsync((void*)meta, 0, kMetaWords * sizeof(uint64_t), s));
  if (M > 0 && (!a0 || !actor)) throw std::invalid_argument("packed meta: actor and a0 columns required");
  constexpr unsigned cap = 1024u;  // blocks: measured best on MI355X (profiles/r1_meta_sweep.jsonl)
  hipLaunchKernelGGL(packed_meta_kernel, dim3(grid_for(M, 256 * 8, cap)), dim3(256), 0, s, (const uint32_t*)actor,
                     (const int64_t*)a0, (const int64_t*)a1, (const int64_t*)a2, (const uint16_t*)method_col,
                     (uint32_t)method_uniform, M, n_dir, affine_w, (unsigned long long*)meta);
  PT_HIP_CHECK(hipGetLastError());
}

#define PT_S_SWITCH(S_, F) \
  switch (S_) {            \
    case 1: F(1); break;   \
    case 2: F(2); break;   \
    case 3: F(3); break;   \
    case 4: F(4); break;   \
    case 5: F(5); break;   \
    case 6: F(6); break;   \
    case 7: F(7); break;   \
    default: F(8); break;  \
  }

void launch_route_packed(uintptr_t actor, uintptr_t a0, uintptr_t a1, uintptr_t a2, uintptr_t method_col,
                         int method_uniform, int64_t M, uintptr_t table, uint64_t cap, uintptr_t dir, uint32_t n_dir,
                         int R, int64_t C, const PackedLayout& L, uintptr_t sendbuf, uintptr_t perm, uintptr_t route,
                         uintptr_t hist, uintptr_t stats, int rank_self, const std::vector<uintptr_t>& direct,
                         uint32_t affine_w, uintptr_t stream, bool prepped) {
  check_packed_layout(L, R, C);
  if (cap == 0 || (cap & (cap - 1))) throw std::invalid_argument("table capacity must be a power of two");
  if (method_col && !L.w[0]) throw std::invalid_argument("route: method column needs a method field in the layout");
  const DirectView dv = direct_of(direct, rank_self);
  const int64_t req_words = packed_req_words(C, L.S);
  int64_t P;
  // `prepped`: pass 1 already ran on this stream (route_prep before the agreement wait)
  const int64_t G = prepped ? route_grid(M, &P)
                            : route_prep(actor, M, table, cap, dir, n_dir, R, route, hist, affine_w, stream, &P);
  route_scan(G, R, C, req_words, sendbuf, hist, method_uniform, stats, rank_self, stream);
  constexpr bool scatter_pipe = true;  // (tiles loaded one ahead of their placement)
  if (M > 0) {
#define PT_SCATTER_P(SV)                                                                                             \
  hipLaunchKernelGGL((route_scatter_packed_kernel<SV>), dim3((unsigned)G), dim3(kRouteThreads), 0, as_stream(stream), \
                     (const uint32_t*)route, (const int64_t*)a0, (const int64_t*)a1, (const int64_t*)a2,              \
                     (const uint16_t*)method_col, (uint32_t)method_uniform, M, P, R, C, (const uint32_t*)hist,       \
                     (uint32_t*)sendbuf, req_words, L, (int32_t*)perm, dv, scatter_pipe)
    PT_S_SWITCH(L.S, PT_SCATTER_P)
#undef PT_SCATTER_P
  }
  PT_HIP_CHECK(hipGetLastError());
}

void launch_dispatch_packed(uintptr_t recv, int R, int64_t C, const PackedLayout& L, uintptr_t reply, uintptr_t state,
                            uint32_t n_state, uint64_t delay_ticks, uintptr_t stats, int64_t expected_per_rank,
                            const std::vector<uintptr_t>& outbox, uint64_t outbox_cap,
                            const std::vector<uintptr_t>& direct, int self, uintptr_t stream) {
  check_packed_layout(L, R, C);
  const DirectView dv = direct_of(direct, self);
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
  const int64_t per = expected_per_rank > 0 ? expected_per_rank : C;
  constexpr unsigned target = 4096u;  // blocks over all sources
  const unsigned gx = grid_for(per, 256, (unsigned)(target / R > 0 ? target / R : 1));
  const int64_t req_words = packed_req_words(C, L.S), rep_words = packed_rep_words(C, L.vb);
  const unsigned stage_cap = outbox_cap ? kOutboxStage : 0;  // LDS stage only where handlers can send
  const size_t smem = stage_cap ? outbox_stage_bytes(stage_cap) : 0;
#define PT_DISPATCH_P(SV)                                                                                          \
  hipLaunchKernelGGL((dispatch_packed_kernel<SV>), dim3(gx, R), dim3(256), smem, as_stream(stream),                 \
                     (const uint32_t*)recv, req_words, C, L, (uint32_t*)reply, rep_words, (int64_t*)state, n_state, \
                     delay_ticks, (unsigned long long*)stats, ob, dv, stage_cap)
  PT_S_SWITCH(L.S, PT_DISPATCH_P)
#undef PT_DISPATCH_P
  PT_HIP_CHECK(hipGetLastError());
}

void launch_complete_packed(uintptr_t rep, int64_t C, int R, int vb, uintptr_t perm, int64_t M, uintptr_t out_val,
                            uintptr_t out_st, uintptr_t checksum, bool direct, uintptr_t stream, uintptr_t failed,
                            uintptr_t zero, int64_t zero_words) {
  if (M <= 0) return;
  if (C < 1 || C > 0x7fffffff) throw std::invalid_argument("complete: bad capacity");
  if (R < 1 || R > kMaxRanks) throw std::invalid_argument("complete: 1 <= R <= 64");
  if (vb != 1 && vb != 2 && vb != 4 && vb != 8) throw std::invalid_argument("complete: vb in {1,2,4,8}");
  hipLaunchKernelGGL(complete_packed_kernel<4>, dim3(grid_for(M, 256 * 4, checksum ? 1024 : 8192)), dim3(256), 0,
                     as_stream(stream), (const uint32_t*)rep, packed_rep_words(C, vb), (uint32_t)C, R, vb,
                     (const int32_t*)perm, M, (int64_t*)out_val, (int32_t*)out_st, (unsigned long long*)checksum,
                     direct, (const uint64_t*)failed, (uint64_t*)zero, zero_words);
  PT_HIP_CHECK(hipGetLastError());
}
void launch_pack_replies(uintptr_t v2, int R, int64_t C, uintptr_t reply, int vb, uintptr_t stats,
                         int64_t expected_per_rank, uintptr_t stream) {
  if (R < 1 || C < 1 || !v2 || !reply || !stats) throw std::invalid_argument("pack_replies: geometry");
  if (vb != 1 && vb != 2 && vb != 4 && vb != 8) throw std::invalid_argument("pack_replies: vb in {1, 2, 4, 8}");
  const int64_t per = expected_per_rank > 0 ? expected_per_rank : C;
  const unsigned gx = grid_for(per, 256, (unsigned)(4096 / R > 0 ? 4096 / R : 1));
  hipLaunchKernelGGL(pack_replies_kernel, dim3(gx, R), dim3(256), 0, as_stream(stream), (const uint32_t*)v2,
                     wire_rep_words(C), C, (uint32_t*)reply, packed_rep_words(C, vb), vb,
                     (unsigned long long*)stats);
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
