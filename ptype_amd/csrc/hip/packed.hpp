// Wire format v3 ("packed"): width-adaptive bit-packed epoch records for the
// multi-GPU exchange, where xGMI bytes -- not kernels -- bound a Send.
//
// The reference's wire is gob (encoding/gob behind stdlib net/rpc, used at
// cluster/rpc.go:65 and :88), which writes every integer as a variable-length
// value: Args{A: 7, B: 8} costs a few bytes, not two machine words.  A GPU
// epoch cannot give each record its own length (receivers index records by
// slot position, and the all-to-all is equal-split), so v3 applies the same
// idea per *exchange*: before an epoch every rank reduces its batch to column
// maxima (mailbox bound, zigzag magnitude of each argument, methods present),
// one 16-word ncclAllReduce(MAX) agrees them across the node, and every record
// of the Send is packed into the fewest dwords that hold
//
//     [method : wm] [mailbox : wx] [a0 : w0] [a1 : w1] [a2 : w2]     (LSB first)
//
// with zigzag-encoded arguments (gob's signed-int encoding).  Replies carry a
// value plane of vb in {1, 2, 4, 8} bytes per record, sized from the methods
// present and the argument bounds (e.g. Multiply: |A*B| <= |A|max * |B|max), plus
// an ok-bitmap; a non-OK reply carries its status code in the value field.
//
// Calculator.Multiply on the headline bench (A in [-2^15, 2^15), B in
// [0, 2^16), 131072 mailboxes per rank): 17 + 16 + 17 = 50 bits -> 8 B per
// request and 4 B + 1 bit per reply, against 20 B + 9 B in v2 -- 2.4x fewer
// bytes on every all-to-all.  Values that do not fit are impossible by
// construction (the widths are global maxima); the dispatcher still checks
// every reply against vb and fails it loudly rather than truncating.
//
// Region sizes (u32 words, every region 16-B aligned, like v2):
//   request per destination: round4(4 + C * S)           header as in v2
//   reply per destination:   round4(4 + V + 2 * ceil(C / 64))
//                            header {count,0,0,0}; value plane V = 2 * ceil(C * vb / 8)
//                            words; ok bitmap as u64 words (bit s = record s ok)
#pragma once
#include <stdint.h>

#include <algorithm>
#include <stdexcept>

#include "records.hpp"
#ifdef __HIPCC__
#include "route_common.hpp"  // kMaxMbox (the width pass bounds unresolved mailboxes by it)
#endif

namespace ptype {

// Meta vector reduced per Send (u64 words; ncclAllReduce MAX across ranks).
enum PackedMeta : int {
  kMetaMbox = 0,    // largest local mailbox index any record may carry
  kMetaArg0 = 1,    // largest zigzag(a_j), j = 0..2 -> words 1..3
  kMetaMethod = 4,  // largest method id sent
  kMetaMcol = 5,    // 1 if any rank sends a per-record method column (then every record carries one)
  kMetaCap = 6,     // largest per-destination bucket of any chunk on any rank (adaptive slot capacity)
  kMetaOverflow = 7,  // sorted exchange: messages a rank answered STATUS_OVERFLOW this Send (MAX: any rank's)
  kMetaFlags = 8,   // words 8..15: 1 if method id (word - 8) occurs; word 15: ids >= 7
  kMetaWords = 16,
};

struct PackedLayout {  // passed BY VALUE to kernels (lands in SGPRs)
  uint8_t off[5];  // bit offsets: 0 method, 1 mailbox, 2..4 args
  uint8_t w[5];    // bit widths (0 = field absent / all zero)
  uint8_t S;       // dwords per request record (1..8)
  uint8_t vb;      // reply value bytes (1, 2, 4, 8)
};

__host__ __device__ __forceinline__ uint64_t zz_enc(int64_t v) { return ((uint64_t)v << 1) ^ (uint64_t)(v >> 63); }
__host__ __device__ __forceinline__ int64_t zz_dec(uint64_t z) { return (int64_t)(z >> 1) ^ -(int64_t)(z & 1); }
__host__ __device__ __forceinline__ uint64_t low_mask(int w) { return w >= 64 ? ~0ull : ((1ull << w) - 1); }

inline int bit_len(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

// Region sizes in u32 words.  A request region of n records: [header 4][n * S];
// a reply region of n replies: [header 4][ok bitmap 2 * ceil(n / 64)][values
// n * vb bytes, 8-B padded].  The ok bitmap comes FIRST and both parts are sized
// by the count, so the used part of a region is a prefix whose length both ends
// know from the count alone -- what the exact-size exchange (grouped
// ncclSend / ncclRecv, engine.hpp) moves.  Allocation size: the same with n = C.
__host__ __device__ inline int64_t packed_req_words(int64_t n, int S) { return (4 + n * S + 3) & ~3ll; }
__host__ __device__ inline int64_t packed_val_words(int64_t n, int vb) { return 2 * ((n * vb + 7) / 8); }
__host__ __device__ inline int64_t packed_ok_words(int64_t n) { return 2 * ((n + 63) / 64); }
__host__ __device__ inline int64_t packed_rep_words(int64_t n, int vb) {
  return (4 + packed_ok_words(n) + packed_val_words(n, vb) + 3) & ~3ll;
}

// Reply value bits for the methods present (flags) under argument bounds.
// Every bound holds for any int64 inputs within the maxima, so a handler's
// reply never exceeds it (the dispatcher checks again on the device).
inline int packed_reply_bits(const uint64_t* meta) {
  auto flag = [&](int m) { return meta[kMetaFlags + m] != 0; };
  const uint64_t z0 = meta[kMetaArg0], z1 = meta[kMetaArg0 + 1], z2 = meta[kMetaArg0 + 2];
  auto mag = [](uint64_t z) { return (unsigned __int128)(z / 2 + (z & 1)); };  // |v| <= mag(zz(v))
  int bits = 0;
  if (flag(kCalculatorMultiply)) {  // zz(a * b) <= 2 |a| |b|
    const unsigned __int128 p = 2 * mag(z0) * mag(z1);
    bits = std::max(bits, (p >> 64) ? 64 : bit_len((uint64_t)p));
  }
  if (flag(kEcho)) bits = std::max(bits, bit_len(z0));
  if (flag(kPrimeCheck)) {  // the target or a divisor in [a0, min(a1, a2)): |reply| <= max |a_j|
    const uint64_t z = std::max(z0, std::max(z1, z2));
    bits = std::max(bits, z == ~0ull ? 64 : bit_len(z + 1));
  }
  // stateful / forwarding / unknown handlers: state-dependent replies are full width
  if (flag(kRetryTest) || flag(kCounterAdd) || flag(kForward) || meta[kMetaFlags + 7] != 0) bits = 64;
  return std::max(bits, 8);  // a non-OK reply carries its status code in the value field
}

// Layout from the agreed meta vector alone, so every rank derives the same one
// whatever columns its own batch has (a missing column contributes zeros).
inline PackedLayout packed_layout(const uint64_t* meta) {
  PackedLayout L{};
  int off = 0;
  auto put = [&](int q, int w) {
    L.off[q] = (uint8_t)off;
    L.w[q] = (uint8_t)w;
    off += w;
  };
  put(0, meta[kMetaMcol] ? std::max(1, bit_len(meta[kMetaMethod])) : 0);
  put(1, bit_len(meta[kMetaMbox]));
  for (int j = 0; j < 3; ++j) put(2 + j, bit_len(meta[kMetaArg0 + j]));
  L.S = (uint8_t)std::max(1, (off + 31) / 32);
  if (L.S > 8) throw std::logic_error("packed layout: record exceeds 8 dwords");
  const int vbits = packed_reply_bits(meta);
  L.vb = (uint8_t)(vbits <= 8 ? 1 : vbits <= 16 ? 2 : vbits <= 32 ? 4 : 8);
  return L;
}

#ifdef __HIPCC__
// Dword j of a record from compile-time S and runtime field offsets: every
// (dword, field) pair is a pair of selects over shifts, never an indexed
// register array (indexed arrays are what made hipcc spill to scratch before).
//
// Records of up to 64 bits (S <= 2, the calculator's 50-bit record) are built
// and read as one u64: a field is one 64-bit shift + mask, not a select chain
// per (dword, field) -- the unpacking dispatch was VALU-bound on those chains.
template <int S>
__device__ __forceinline__ void packed_pack(const PackedLayout L, const uint64_t (&f)[5], uint32_t (&rec)[S]) {
  if constexpr (S <= 2) {
    uint64_t v = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q)
      if (L.w[q]) v |= (f[q] & low_mask(L.w[q])) << L.off[q];  // off + w <= 64 here
    rec[0] = (uint32_t)v;
    if constexpr (S == 2) rec[1] = (uint32_t)(v >> 32);
    return;
  }
#pragma unroll
  for (int j = 0; j < S; ++j) {
    uint32_t x = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int sh = (int)L.off[q] - 32 * j;
      const uint64_t v = f[q] & low_mask(L.w[q]);
      if (L.w[q] && sh >= 0 && sh < 32) x |= (uint32_t)(v << sh);
      else if (L.w[q] && sh < 0 && sh > -64) x |= (uint32_t)(v >> -sh);
    }
    rec[j] = x;
  }
}

// Width-pass accumulator: column maxima of the records one thread saw.
struct MetaAcc {
  uint64_t mb = 0, z0 = 0, z1 = 0, z2 = 0, mm = 0;
  uint32_t flags = 0;
  __device__ __forceinline__ void take(uint32_t a, int64_t v0, int64_t v1, int64_t v2, uint32_t meth, uint32_t n_dir,
                                       uint32_t aw) {
    // affine directory: the route is (a % aw, a / aw); otherwise any mailbox below kMaxMbox
    const uint64_t m = (aw && a < n_dir) ? a / aw : (uint64_t)(kMaxMbox - 1);
    mb = m > mb ? m : mb;
    const uint64_t x0 = zz_enc(v0), x1 = zz_enc(v1), x2 = zz_enc(v2);
    z0 = x0 > z0 ? x0 : z0;
    z1 = x1 > z1 ? x1 : z1;
    z2 = x2 > z2 ? x2 : z2;
    mm = meth > mm ? meth : mm;
    flags |= 1u << (meth < 7 ? meth : 7);
  }
};

// The width-pass columns, passed BY VALUE to route pass 1 when it also runs the
// width pass (the v3 engine fuses them: one read of the batch instead of two).
struct MetaCols {
  const int64_t* a0;
  const int64_t* a1;
  const int64_t* a2;
  const uint16_t* mcol;
  uint32_t method_uniform, n_dir, aw;
  unsigned long long* meta;
};

// Adaptive slot capacity folded into route pass 1 (replaces the one-block
// hist_cap pass: a launch and ~12 us per chunk).  Every block adds its column
// counts into `tot`; the last block out (ticket) takes the busiest destination
// column into meta[kMetaCap] (atomic max) and resets `tot` and the ticket, so the
// words are zero again for the next launch.  Passed BY VALUE.
struct CapFold {
  unsigned* tot = nullptr;     // [kCapCopies][kMaxCapCols], zero between launches
  unsigned* ticket = nullptr;  // [kTicketWords] (last_block_ticket), zero between launches
  unsigned long long* meta = nullptr;
  // optional: this launch's destination totals, counts[q * count_stride] for q < R
  // (this rank's row of the agreement's count matrix: the exact-size exchange's X1)
  unsigned long long* counts = nullptr;
  uint32_t count_stride = 1;
};
constexpr int kMaxCapCols = 65;   // R + 1 <= 64 + 1 (the registry-miss column)
constexpr unsigned kCapCopies = 16;  // block b adds into copy b % 16 (same-address atomics serialise)
constexpr size_t kCapFoldWords = kCapCopies * kMaxCapCols + kTicketWords;

// Block-wide reduction of every thread's accumulator into meta[] (atomic max).
// Every thread of the block (up to 1024 threads) must call it.  A block only issues the
// atomic when its value beats what meta[] already holds (a relaxed read, at worst
// stale-low, i.e. one unneeded atomic): thousands of blocks hitting the same 16
// words with atomics serialise at L2, and on random data the maxima settle after
// the first few blocks.
__device__ __forceinline__ void meta_max(unsigned long long* p, uint64_t v) {
  if (v > __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(p, (unsigned long long)v);
}
__device__ __forceinline__ void meta_publish(MetaAcc acc, bool has_mcol, uint32_t method_uniform, int64_t M,
                                             unsigned long long* __restrict__ meta) {
  if (!has_mcol) {  // uniform method: no column maxima (flagged once per batch below)
    acc.mm = 0;
    acc.flags = 0;
  }
  for (int off = 32; off > 0; off >>= 1) {
    uint64_t t;
    t = __shfl_xor(acc.mb, off), acc.mb = t > acc.mb ? t : acc.mb;
    t = __shfl_xor(acc.z0, off), acc.z0 = t > acc.z0 ? t : acc.z0;
    t = __shfl_xor(acc.z1, off), acc.z1 = t > acc.z1 ? t : acc.z1;
    t = __shfl_xor(acc.z2, off), acc.z2 = t > acc.z2 ? t : acc.z2;
    t = __shfl_xor(acc.mm, off), acc.mm = t > acc.mm ? t : acc.mm;
    acc.flags |= __shfl_xor(acc.flags, off);
  }
  __shared__ uint64_t part[1024 / 64][6];  // (sized for 256 threads once: 512-thread blocks overran it)
  const int w = threadIdx.x / 64, nw = (int)(blockDim.x / 64);
  if ((threadIdx.x & 63) == 0) {
    part[w][0] = acc.mb, part[w][1] = acc.z0, part[w][2] = acc.z1, part[w][3] = acc.z2, part[w][4] = acc.mm,
    part[w][5] = acc.flags;
  }
  __syncthreads();
  if (threadIdx.x < 5) {  // words 0..3 = mailbox, a0..a2; thread 4 -> kMetaMethod
    uint64_t v = 0;
    for (int k = 0; k < nw; ++k) v = part[k][threadIdx.x] > v ? part[k][threadIdx.x] : v;
    if (v) meta_max(meta + (threadIdx.x == 4 ? (int)kMetaMethod : (int)threadIdx.x), v);
  } else if (threadIdx.x == 5) {
    uint32_t f = 0;
    for (int k = 0; k < nw; ++k) f |= (uint32_t)part[k][5];
    if (M > 0 && blockIdx.x == 0) {
      if (has_mcol) {
        meta_max(meta + kMetaMcol, 1);
      } else {
        f |= 1u << (method_uniform < 7 ? method_uniform : 7);
        meta_max(meta + kMetaMethod, method_uniform);
      }
    }
    while (f) {
      const int b = __builtin_ctz(f);
      meta_max(meta + kMetaFlags + b, 1);
      f &= f - 1;
    }
  }
}

template <int S>
__device__ __forceinline__ uint64_t packed_field(const PackedLayout L, int q, const uint32_t (&rec)[S]) {
  if constexpr (S <= 2) {
    const uint64_t r = S == 2 ? ((uint64_t)rec[S - 1] << 32 | rec[0]) : (uint64_t)rec[0];
    return L.w[q] ? (r >> L.off[q]) & low_mask(L.w[q]) : 0ull;
  }
  uint64_t v = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const int sh = 32 * j - (int)L.off[q];
    if (sh >= 0 && sh < 64) v |= (uint64_t)rec[j] << sh;
    else if (sh < 0 && sh > -32) v |= (uint64_t)(rec[j] >> -sh);
  }
  return L.w[q] ? (v & low_mask(L.w[q])) : 0ull;
}
#endif

}  // namespace ptype
