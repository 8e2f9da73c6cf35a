// AoS -> SoA conversion of 32-B request records (MsgBatch.from_records on the
// device): records arriving from rings / host clients become the SoA columns the
// route kernels stream.  Two implementations, measured against each other
// ("MFMA-packed batch copies" are only defensible as exact byte
// transposition, and only if they beat a plain dwordx4 copy):
//
//   copy   one lane per record: two dwordx4 loads, five coalesced column stores
//   mfma   v_mfma_i32_16x16x32_i8 with the record bytes as the B operand
//          (B[byte][record], 16 records x 32 bytes per wave tile, each lane
//          loading 8 bytes) and constant 0/1 selection matrices as A, so that
//          D[i][rec] = byte sel(i) of record rec -- exact in i32 (one non-zero
//          product per sum).  The output layout hands each lane 4 bytes of one
//          record per MFMA: lane group g gets bytes 4g..4g+3 and 16+4g..+3.
//
// The record layout is MsgRecord (records.hpp): actor u32 | method u16 | flags
// u16 | a0 i64 | a1 i64 | a2 i64.
#include "common.hpp"

namespace ptype {

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void records_to_soa_copy_kernel(const uint4* __restrict__ rec, int64_t M,
                                                                  uint32_t* __restrict__ actor,
                                                                  uint16_t* __restrict__ method,
                                                                  int64_t* __restrict__ a0, int64_t* __restrict__ a1,
                                                                  int64_t* __restrict__ a2) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < M; r += (int64_t)gridDim.x * blockDim.x) {
    const uint4 lo = rec[2 * r], hi = rec[2 * r + 1];
    actor[r] = lo.x;
    method[r] = (uint16_t)(lo.y & 0xffffu);
    a0[r] = (int64_t)(((uint64_t)lo.w << 32) | lo.z);
    a1[r] = (int64_t)(((uint64_t)hi.y << 32) | hi.x);
    a2[r] = (int64_t)(((uint64_t)hi.w << 32) | hi.z);
  }
}

// Selection operand (A, 16 x 32 i8): lane l holds row l % 16, bytes 8 * (l / 16) .. +7.
__device__ __forceinline__ long sel_operand(int first_byte) {
  const unsigned lane = lane_id();
  const int row = lane % 16, k0 = 8 * (lane / 16);
  const int b = first_byte + row - k0;  // column of the single 1 in this row, relative to the lane's 8
  return (b >= 0 && b < 8) ? (long)(1ull << (8 * b)) : 0l;
}

__device__ __forceinline__ uint32_t pack_bytes(const v4i& d) {
  return (uint32_t)(d.x & 0xff) | ((uint32_t)(d.y & 0xff) << 8) | ((uint32_t)(d.z & 0xff) << 16) |
         ((uint32_t)(d.w & 0xff) << 24);
}

__global__ __launch_bounds__(256) void records_to_soa_mfma_kernel(const uint64_t* __restrict__ rec, int64_t M,
                                                                  uint32_t* __restrict__ actor,
                                                                  uint16_t* __restrict__ method,
                                                                  uint32_t* __restrict__ a0w, uint32_t* __restrict__ a1w,
                                                                  uint32_t* __restrict__ a2w) {
  const unsigned lane = lane_id(), g = lane / 16;
  const long sel_lo = sel_operand(0), sel_hi = sel_operand(16);  // bytes 0..15 and 16..31
  const int64_t tiles = (M + 15) / 16;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t waves = (int64_t)gridDim.x * blockDim.x / kWave;
  for (int64_t t = wave; t < tiles; t += waves) {
    const int64_t r = t * 16 + lane % 16;  // this lane's record (B column) and output record
    const bool in = r < M;
    // B operand: 8 bytes of record r starting at byte 8 * g (one dwordx2 per lane)
    const long b = in ? (long)rec[r * 4 + g] : 0l;
    const v4i z = {0, 0, 0, 0};
    const v4i d_lo = __builtin_amdgcn_mfma_i32_16x16x32_i8(sel_lo, b, z, 0, 0, 0);  // bytes 4g..4g+3
    const v4i d_hi = __builtin_amdgcn_mfma_i32_16x16x32_i8(sel_hi, b, z, 0, 0, 0);  // bytes 16+4g..
    if (!in) continue;
    const uint32_t w_lo = pack_bytes(d_lo), w_hi = pack_bytes(d_hi);
    switch (g) {
      case 0: actor[r] = w_lo; a1w[2 * r] = w_hi; break;
      case 1: method[r] = (uint16_t)(w_lo & 0xffffu); a1w[2 * r + 1] = w_hi; break;
      case 2: a0w[2 * r] = w_lo; a2w[2 * r] = w_hi; break;
      default: a0w[2 * r + 1] = w_lo; a2w[2 * r + 1] = w_hi; break;
    }
  }
}

void launch_records_to_soa(uintptr_t rec, int64_t M, uintptr_t actor, uintptr_t method, uintptr_t a0, uintptr_t a1,
                           uintptr_t a2, bool mfma, uintptr_t stream) {
  if (M <= 0) return;
  hipStream_t s = as_stream(stream);
  if (mfma) {
    const int64_t tiles = (M + 15) / 16;
    int64_t blocks = (tiles + 3) / 4;  // 4 waves per block, one tile per wave per iteration
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(records_to_soa_mfma_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint64_t*)rec, M,
                       (uint32_t*)actor, (uint16_t*)method, (uint32_t*)a0, (uint32_t*)a1, (uint32_t*)a2);
  } else {
    int64_t blocks = (M + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(records_to_soa_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint4*)rec, M,
                       (uint32_t*)actor, (uint16_t*)method, (int64_t*)a0, (int64_t*)a1, (int64_t*)a2);
  }
  PT_HIP_CHECK(hipGetLastError());
}

}  // namespace ptype
