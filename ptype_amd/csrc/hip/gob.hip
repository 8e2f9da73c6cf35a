// K4: encoding/gob value messages of fixed-schema structs, on the GPU (SURVEY
// §2.3 K4; the host codec is csrc/core/gob.cpp).
//
// The reference's net/rpc moves every call's arguments and reply as gob values
// (cluster/rpc.go:59-67 -> net/rpc's gob codec; the calculator's Args{A, B int},
// example/calculator/calculator.go:5-8).  For a batch of such values held as
// columns in HBM (one int64 column per struct field), these kernels produce and
// consume the exact bytes the host codec (and Go) uses for the VALUE messages of
// a registered type -- the type definition is sent once per stream by the host:
//
//   message  = uint(len) int(type id) struct
//   struct   = { uint(field delta) int(value) }  for every NON-ZERO field, then 0
//   uint(x)  = x < 128 ? byte(x) : byte(-n) + n big-endian bytes
//   int(i)   = uint(i < 0 ? ~i << 1 | 1 : i << 1)
//
// Encode is three passes (the route's prep / scan / scatter shape): per-block
// byte totals, one-block scan of the totals, then each lane writes its message at
// its prefix (one lane = one message).  Decode takes the message offsets (the
// framing layer that read the stream knows them) and parses one message per
// lane, with a status per message.  Outputs are bit-identical to the host codec
// (tests/test_gob_gpu.py).
#include <vector>

#include "common.hpp"

namespace ptype {

constexpr int kGobMaxFields = 8;  // => a message is at most 1 + 9 + 8 * 10 + 1 = 91 B: a 1-byte length
constexpr int kGobThreads = 256;
constexpr int kGobItems = 4;      // messages per thread per pass
constexpr int64_t kGobTile = (int64_t)kGobThreads * kGobItems;

enum GobStatus : int32_t { kGobOk = 0, kGobTruncated = 1, kGobWrongType = 2, kGobBadField = 3, kGobTrailing = 4 };

struct GobCols {  // by value
  int64_t* col[kGobMaxFields];
  int nf;
};

__device__ __forceinline__ uint64_t gob_zz(int64_t i) {
  return i < 0 ? ((uint64_t)(~i) << 1) | 1ull : (uint64_t)i << 1;
}
__device__ __forceinline__ int gob_uint_len(uint64_t x) {
  return x < 128 ? 1 : 1 + ((64 - __clzll((long long)x) + 7) >> 3);
}
__device__ __forceinline__ uint8_t* gob_put_uint(uint8_t* p, uint64_t x) {
  if (x < 128) {
    *p = (uint8_t)x;
    return p + 1;
  }
  const int n = (64 - __clzll((long long)x) + 7) >> 3;
  *p++ = (uint8_t)(256 - n);
  for (int k = n - 1; k >= 0; --k) *p++ = (uint8_t)(x >> (8 * k));
  return p;
}

// Length of row i's whole message (length byte included).
__device__ __forceinline__ int gob_msg_len(const GobCols& c, int64_t i, uint32_t type_id) {
  int body = 1;  // the struct's terminating 0
  int last = -1;
#pragma unroll
  for (int f = 0; f < kGobMaxFields; ++f) {
    if (f >= c.nf) break;
    const int64_t v = c.col[f][i];
    if (v == 0) continue;
    body += gob_uint_len((uint64_t)(f - last)) + gob_uint_len(gob_zz(v));
    last = f;
  }
  return 1 + gob_uint_len(gob_zz((int64_t)type_id)) + body;
}

// Block-wide exclusive scan of one value per thread (256 threads); returns the
// thread's prefix and writes the block total to *total.
__device__ __forceinline__ unsigned block_excl_scan(unsigned v, unsigned* total) {
  __shared__ unsigned wsum[kGobThreads / kWave];
  const unsigned w = threadIdx.x / kWave, lane = lane_id();
  const unsigned incl = wave_incl_scan(v);
  if (lane == kWave - 1) wsum[w] = incl;
  __syncthreads();
  unsigned base = 0, tot = 0;
#pragma unroll
  for (unsigned k = 0; k < kGobThreads / kWave; ++k) {
    base += k < w ? wsum[k] : 0u;
    tot += wsum[k];
  }
  __syncthreads();  // wsum reused by the next call
  *total = tot;
  return base + incl - v;
}

// Pass 1: bytes per block of kGobTile messages.
__global__ __launch_bounds__(kGobThreads) void gob_size_kernel(GobCols c, int64_t M, uint32_t type_id,
                                                               unsigned* __restrict__ block_bytes) {
  const int64_t lo = blockIdx.x * kGobTile;
  unsigned mine = 0;
#pragma unroll
  for (int k = 0; k < kGobItems; ++k) {
    const int64_t i = lo + (int64_t)k * kGobThreads + threadIdx.x;
    if (i < M) mine += (unsigned)gob_msg_len(c, i, type_id);
  }
  unsigned total;
  block_excl_scan(mine, &total);
  if (threadIdx.x == 0) block_bytes[blockIdx.x] = total;
}

// Pass 2 (one block): exclusive prefix of the block totals, in place as u64 bases.
__global__ __launch_bounds__(1024) void gob_scan_kernel(const unsigned* __restrict__ block_bytes, int G,
                                                        unsigned long long* __restrict__ base,
                                                        int64_t* __restrict__ offsets, int64_t M) {
  __shared__ unsigned long long carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int b0 = 0; b0 < G; b0 += 1024) {
    const int b = b0 + (int)threadIdx.x;
    const unsigned long long v = b < G ? block_bytes[b] : 0ull;
    // scan of 1024 u64 values: per wave, then across the 16 waves
    __shared__ unsigned long long ws[16];
    unsigned long long x = v;
    for (int off = 1; off < kWave; off <<= 1) {
      const unsigned long long y = __shfl_up(x, off);
      if (lane_id() >= (unsigned)off) x += y;
    }
    const unsigned w = threadIdx.x / kWave;
    if (lane_id() == kWave - 1) ws[w] = x;
    __syncthreads();
    unsigned long long pre = carry;
    for (unsigned k = 0; k < w; ++k) pre += ws[k];
    if (b < G) base[b] = pre + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = pre + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) offsets[M] = (int64_t)carry;  // total bytes
}

// Pass 3: every lane writes its message at its prefix; offsets[i] = its start.
__global__ __launch_bounds__(kGobThreads) void gob_write_kernel(GobCols c, int64_t M, uint32_t type_id,
                                                                const unsigned long long* __restrict__ base,
                                                                uint8_t* __restrict__ out,
                                                                int64_t* __restrict__ offsets) {
  const int64_t lo = blockIdx.x * kGobTile;
  int len[kGobItems];
#pragma unroll
  for (int k = 0; k < kGobItems; ++k) {
    const int64_t i = lo + (int64_t)k * kGobThreads + threadIdx.x;
    len[k] = i < M ? gob_msg_len(c, i, type_id) : 0;
  }
  // item-major message order inside the block: scan item by item
  unsigned long long at = base[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kGobItems; ++k) {
    unsigned total;
    const unsigned pre = block_excl_scan((unsigned)len[k], &total);
    const int64_t i = lo + (int64_t)k * kGobThreads + threadIdx.x;
    if (i < M) {
      const unsigned long long o = at + pre;
      offsets[i] = (int64_t)o;
      uint8_t* p = out + o;
      p = gob_put_uint(p, (uint64_t)(len[k] - 1));
      p = gob_put_uint(p, gob_zz((int64_t)type_id));
      int last = -1;
#pragma unroll
      for (int f = 0; f < kGobMaxFields; ++f) {
        if (f >= c.nf) break;
        const int64_t v = c.col[f][i];
        if (v == 0) continue;
        p = gob_put_uint(p, (uint64_t)(f - last));
        p = gob_put_uint(p, gob_zz(v));
        last = f;
      }
      *p = 0;
    }
    at += total;
  }
}

// ---- decode: one message per lane, [offsets[i], offsets[i + 1])
__device__ __forceinline__ bool gob_get_uint(const uint8_t*& p, const uint8_t* end, uint64_t* x) {
  if (p >= end) return false;
  const uint8_t c0 = *p++;
  if (c0 < 128) {
    *x = c0;
    return true;
  }
  const int n = 256 - (int)c0;
  if (n > 8 || end - p < n) return false;
  uint64_t v = 0;
  for (int k = 0; k < n; ++k) v = (v << 8) | *p++;
  *x = v;
  return true;
}
__device__ __forceinline__ int64_t gob_unzz(uint64_t u) {
  return (u & 1) ? (int64_t)~(u >> 1) : (int64_t)(u >> 1);
}

__global__ __launch_bounds__(256) void gob_decode_kernel(const uint8_t* __restrict__ buf,
                                                         const int64_t* __restrict__ offsets, int64_t M,
                                                         uint32_t type_id, GobCols c,
                                                         int32_t* __restrict__ status) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* p = buf + offsets[i];
    const uint8_t* end = buf + offsets[i + 1];
    int64_t v[kGobMaxFields];
#pragma unroll
    for (int f = 0; f < kGobMaxFields; ++f) v[f] = 0;
    int32_t st = kGobOk;
    uint64_t len = 0, tid = 0;
    if (!gob_get_uint(p, end, &len) || (uint64_t)(end - p) != len) {
      st = kGobTruncated;
    } else if (!gob_get_uint(p, end, &tid) || gob_unzz(tid) != (int64_t)type_id) {
      st = kGobWrongType;
    } else {
      int field = -1;
      for (;;) {
        uint64_t delta;
        if (!gob_get_uint(p, end, &delta)) {
          st = kGobTruncated;
          break;
        }
        if (delta == 0) break;
        field += (int)delta;
        uint64_t u;
        if (field >= c.nf || delta > (uint64_t)kGobMaxFields) {
          st = kGobBadField;
          break;
        }
        if (!gob_get_uint(p, end, &u)) {
          st = kGobTruncated;
          break;
        }
#pragma unroll
        for (int f = 0; f < kGobMaxFields; ++f)
          if (f == field) v[f] = gob_unzz(u);  // (named registers, no indexed array)
      }
      if (st == kGobOk && p != end) st = kGobTrailing;
    }
#pragma unroll
    for (int f = 0; f < kGobMaxFields; ++f)
      if (f < c.nf) c.col[f][i] = st == kGobOk ? v[f] : 0;
    status[i] = st;
  }
}

// ---------------------------------------------------------------- launchers
static GobCols gob_cols(const std::vector<uintptr_t>& cols) {
  if (cols.empty() || cols.size() > (size_t)kGobMaxFields) throw std::invalid_argument("gob: 1..8 int fields");
  GobCols c{};
  c.nf = (int)cols.size();
  for (size_t f = 0; f < cols.size(); ++f) {
    if (!cols[f]) throw std::invalid_argument("gob: null column");
    c.col[f] = (int64_t*)cols[f];
  }
  return c;
}

// Worst-case bytes of M messages with nf fields (the output buffer's size).
int64_t gob_max_bytes(int64_t M, int nf, uint32_t type_id) {
  (void)type_id;
  return M * (int64_t)(1 + 9 + nf * 10 + 1);
}

// Workspace words (u64) for M messages: block totals + bases.
int64_t gob_ws_words(int64_t M) {
  const int64_t G = (M + kGobTile - 1) / kGobTile;
  return 2 * (G > 0 ? G : 1);
}

void launch_gob_encode(const std::vector<uintptr_t>& cols, int64_t M, uint32_t type_id, uintptr_t out,
                       uintptr_t offsets, uintptr_t ws, uintptr_t stream) {
  const GobCols c = gob_cols(cols);
  hipStream_t s = as_stream(stream);
  if (M <= 0) {
    PT_HIP_CHECK(hipMemsetAsync((void*)offsets, 0, sizeof(int64_t), s));
    return;
  }
  if (M >= (1ll << 31)) throw std::invalid_argument("gob encode: at most 2^31 messages");
  const int64_t G = (M + kGobTile - 1) / kGobTile;
  unsigned* block_bytes = (unsigned*)ws;
  unsigned long long* base = (unsigned long long*)ws + G;
  hipLaunchKernelGGL(gob_size_kernel, dim3((unsigned)G), dim3(kGobThreads), 0, s, c, M, type_id, block_bytes);
  hipLaunchKernelGGL(gob_scan_kernel, dim3(1), dim3(1024), 0, s, block_bytes, (int)G, base, (int64_t*)offsets, M);
  hipLaunchKernelGGL(gob_write_kernel, dim3((unsigned)G), dim3(kGobThreads), 0, s, c, M, type_id,
                     (const unsigned long long*)base, (uint8_t*)out, (int64_t*)offsets);
  PT_HIP_CHECK(hipGetLastError());
}

void launch_gob_decode(uintptr_t buf, uintptr_t offsets, int64_t M, uint32_t type_id, const std::vector<uintptr_t>& cols,
                       uintptr_t status, uintptr_t stream) {
  const GobCols c = gob_cols(cols);
  if (M <= 0) return;
  int64_t g = (M + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(gob_decode_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), (const uint8_t*)buf,
                     (const int64_t*)offsets, M, type_id, c, (int32_t*)status);
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
