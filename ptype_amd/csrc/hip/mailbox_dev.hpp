// Device-side helpers shared by the mailbox kernels (mailbox.hip: tagged rings,
// live consumer; mailbox_sort.hip: sorted epoch mailboxes).  Layout and
// protocol: mailbox.hpp.
#pragma once
#include "mailbox.hpp"

namespace ptype {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Write-through (sc1) 16-B store: the record halves a concurrent consumer on
// another XCD reads (MI355X_MICROARCH.md, hand-off forms: sc1 payload stores
// drained before the signal).
__device__ __forceinline__ void st16_sc1(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// A read that cannot be served by a stale L2 line: the per-XCD L2s are not
// coherent with each other while a kernel runs, and a word another XCD keeps
// rewriting (a tail, a ring slot) can sit in this XCD's L2 from an earlier
// read.  A no-op atomic executes at the memory side and returns memory's value.
__device__ __forceinline__ unsigned long long ld_fresh(unsigned long long* p) {
  return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32x4 ld16_fresh(uint32_t* p) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  const unsigned long long lo = ld_fresh(q), hi = ld_fresh(q + 1);
  return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}
__device__ __forceinline__ uint64_t sys_ld64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ unsigned long long* ctr_tail(const MboxView& mv, uint32_t s) {
  return mv.ctr + (uint64_t)s * kMboxCtrStride;
}
__device__ __forceinline__ unsigned long long* ctr_done(const MboxView& mv, uint32_t s) {
  return mv.ctr + (uint64_t)s * kMboxCtrStride + 1;
}
__device__ __forceinline__ unsigned long long* ctr_head(const MboxView& mv, uint32_t s) {
  return mv.ctr + (uint64_t)s * kMboxCtrStride + 16;
}
// A record is two 16-B halves in two planes: plane A {tag, mailbox, origin,
// method | flags} at rec[slot], plane B {a0, a1} at rec[b_off + slot], so a
// wave's store of one half covers 64 consecutive 16-B cells -- whole lines.  As
// one 32-B record per slot (the removed interleaved form) each store instruction wrote
// every other 16 B of 64 records: the enqueue's DRAM writes were 419 MB for 268 MB
// of records (PMC WRITE_SIZE).  Bench mailbox step: 0.247 ms (32-B records) ->
// 0.215 ms (planes, de-aliased; see the pad in the Mailboxes constructor).
// Ring position -> slot.  Each shard's ring is ROTATED by a hashed offset: the
// shards' tails advance in step under uniform traffic, and with power-of-two
// ring strides their active lines would sit at the same offset of every ring --
// the same HBM channels (S = 256: drain 114 us vs 66 us at S = 64, the rings
// 2 MB apart).  The rotation spreads them over the channels; a slot stays a
// bijection of (shard, position mod Q).
__device__ __forceinline__ uint32_t shard_rot(const MboxView& mv, uint32_t s) {
  return mv.log_q ? (s * 0x9E3779B1u) >> (32 - mv.log_q) : 0u;
}
__device__ __forceinline__ uint64_t slot_at(const MboxView& mv, uint32_t s, uint64_t pos) {
  return ((uint64_t)s << mv.log_q) | ((pos + shard_rot(mv, s)) & ((1ull << mv.log_q) - 1));
}
__device__ __forceinline__ uint32_t* rec_a(const MboxView& mv, uint64_t slot) {
  return mv.rec + slot * (mv.planar ? 4 : 8);
}
__device__ __forceinline__ uint32_t* rec_b(const MboxView& mv, uint64_t slot) {
  return mv.planar ? mv.rec + mv.b_off + slot * 4 : mv.rec + slot * 8 + 4;
}
// (planar rings) a u16 per slot in plane B's memory: the wide pure records' places
__device__ __forceinline__ uint16_t* rec_place(const MboxView& mv) {
  return reinterpret_cast<uint16_t*>(mv.rec + mv.b_off);
}
__device__ __forceinline__ uint32_t* rec_at(const MboxView& mv, uint32_t s, uint64_t pos) {
  return rec_a(mv, slot_at(mv, s, pos));
}
__device__ __forceinline__ uint32_t lap_tag(const MboxView& mv, uint64_t pos) {
  return (uint32_t)(pos >> mv.log_q) + 1u;
}

// Block-reduced stats: three counters added once per block, striped by block so
// the grid's adds do not serialise on one word (readers sum the stripes).  Any
// block size up to 1024 threads.
__device__ __forceinline__ void block_add_stats(unsigned long long* stats, unsigned long long v0, int w0,
                                                unsigned long long v1, int w1, unsigned long long v2, int w2) {
  __shared__ unsigned long long part[3][16];
  for (int off = 32; off > 0; off >>= 1) {
    v0 += __shfl_xor(v0, off);
    v1 += __shfl_xor(v1, off);
    v2 += __shfl_xor(v2, off);
  }
  const int w = threadIdx.x / kWave;
  if (lane_id() == 0) part[0][w] = v0, part[1][w] = v1, part[2][w] = v2;
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned long long v = 0;
    for (int k = 0; k < (int)(blockDim.x / kWave); ++k) v += part[threadIdx.x][k];
    const int word = threadIdx.x == 0 ? w0 : threadIdx.x == 1 ? w1 : w2;
    // striped by block: one word for the whole grid serialised thousands of
    // same-address atomics (~9 ns each) at the kernel's end (readers sum stripes)
    const size_t stripe = (size_t)((blockIdx.x + blockIdx.y * gridDim.x) % kMbStripes) * kMbStatWords;
    if (v && word >= 0) atomicAdd(&stats[stripe + word], v);
  }
}

// ---------------------------------------------------------------- record decode + reply
struct MboxMsg {
  MsgRecord m;
  uint32_t origin;
  bool valid;
};

__device__ __forceinline__ MboxMsg decode(const u32x4& ha, const u32x4& hb, const int64_t* a2v) {
  MboxMsg x;
  x.m.actor = ha.y;
  x.origin = ha.z;
  x.m.method = (uint16_t)(ha.w & 0xffffu);
  x.m.flags = (uint16_t)(ha.w >> 16);
  x.m.a0 = (int64_t)(((uint64_t)hb.y << 32) | hb.x);
  x.m.a1 = (int64_t)(((uint64_t)hb.w << 32) | hb.z);
  x.m.a2 = (x.m.flags & kFlagA2) && a2v ? *a2v : 0;
  x.valid = true;
  return x;
}

__device__ __forceinline__ void put_reply(const ReplyView& rv, uint32_t origin, int64_t value, int32_t status) {
  if ((uint64_t)origin >= rv.n) return;
  if (rv.slots) {  // wire v2 reply regions: values int64[C] then statuses u8[C] per source rank
    const uint32_t d = origin / rv.C, pos = origin - d * rv.C;
    uint32_t* rb = rv.slots + (int64_t)d * rv.rep_words;
    reinterpret_cast<int64_t*>(rb + 4)[pos] = value;
    reinterpret_cast<uint8_t*>(rb + 4 + 2 * (int64_t)rv.C)[pos] = (uint8_t)status;
    return;
  }
  rv.val[origin] = value;
  rv.st[origin] = status;
}
// put_reply for a block's coalesced reply stores: the caller's outputs are not read
// again by this Send, so the stores stream (non-temporal) instead of filling the L2
__device__ __forceinline__ void put_reply_nt(const ReplyView& rv, uint32_t origin, int64_t value, int32_t status) {
  if (rv.slots || (uint64_t)origin >= rv.n) {
    put_reply(rv, origin, value, status);
    return;
  }
  __builtin_nontemporal_store(value, rv.val + origin);
  __builtin_nontemporal_store(status, rv.st + origin);
}
__device__ __forceinline__ void write_reply(const ReplyView& rv, uint32_t origin, const ReplyRecord& r) {
  put_reply(rv, origin, r.value, r.status);
}
__device__ __forceinline__ void write_status(const ReplyView& rv, uint32_t origin, int32_t status) {
  put_reply(rv, origin, 0, status);
}

}  // namespace ptype
