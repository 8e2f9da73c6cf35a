// Compiled-in device actor handlers: the method table that the dispatch kernels
// switch on.  This is the GPU-side replacement of stdlib net/rpc's reflective
// `service.call` (reference: server registration in
// example/calculator/server/server.go:16-20, handler bodies in
// example/calculator/calculator.go:9-12 and example/optimus/prime.go:15-25; the
// fault-injecting test actor in cluster/rpc_test.go:55-77).
#pragma once
#include "common.hpp"

namespace ptype {

// Device outbox: messages emitted by handlers -- actor-to-actor
// sends that never leave the GPU until the next exchange epoch routes them.
// SoA columns in HBM, like a client batch; slots are reserved with ONE atomic
// per wave (ballot over the emitting lanes, leader adds the popcount, lanes
// take base + rank).  A full outbox counts drops instead of overwriting.
//
// Block staging (OutboxStage, kernels that pass one): the lanes append to an LDS
// copy of the columns instead, and the block publishes the tile's records with
// ONE global reservation and coalesced copies (outbox_flush).  Every wave's
// reservation is an atomic on the same word, and same-address atomics serialise
// device-wide (~7 ns each): 16 K wave reservations per Mi emitted messages were
// the whole 113 us of a token-ring epoch.
struct OutboxStage {
  unsigned* n = nullptr;  // LDS: records staged (may pass cap: the excess went straight to HBM)
  unsigned long long* base = nullptr;  // LDS: the block's global reservation
  uint32_t* actor = nullptr;
  uint16_t* method = nullptr;
  int64_t* a0 = nullptr;
  int64_t* a1 = nullptr;
  int64_t* a2 = nullptr;
  unsigned cap = 0;
};

struct OutboxView {
  uint32_t* actor = nullptr;
  int64_t* a0 = nullptr;
  int64_t* a1 = nullptr;
  int64_t* a2 = nullptr;
  uint16_t* method = nullptr;
  unsigned long long* count = nullptr;  // [0] reserved slots, [1] dropped
  uint64_t cap = 0;
  OutboxStage stg;  // block staging in LDS (stg.n null: off)
};

// Records a block stages (one 1024-message tile of local_send; a dispatch block
// publishes at its end, anything past the stage goes straight to HBM): 30 KB.
constexpr unsigned kOutboxStage = 1024;

// LDS bytes of a stage of `cap` records (the layout outbox_stage() carves).
__host__ __device__ constexpr size_t outbox_stage_bytes(unsigned cap) {
  return 16 + (size_t)cap * (3 * sizeof(int64_t) + sizeof(uint32_t) + sizeof(uint16_t)) + 16;
}

// Carve a stage out of dynamic LDS (`smem`, 16-B aligned) and empty it; call
// before the first emit and follow with a barrier.
__device__ __forceinline__ OutboxStage outbox_stage(unsigned char* smem, unsigned cap) {
  OutboxStage s;
  s.base = reinterpret_cast<unsigned long long*>(smem);
  s.n = reinterpret_cast<unsigned*>(smem + 8);
  s.a0 = reinterpret_cast<int64_t*>(smem + 16);
  s.a1 = s.a0 + cap;
  s.a2 = s.a1 + cap;
  s.actor = reinterpret_cast<uint32_t*>(s.a2 + cap);
  s.method = reinterpret_cast<uint16_t*>(s.actor + cap);
  s.cap = cap;
  if (threadIdx.x == 0) *s.n = 0;
  return s;
}

// Block-wide (every thread, block-uniform control flow): one reservation for the
// staged records, coalesced copies to HBM, stage emptied for the next tile.
__device__ __forceinline__ void outbox_flush(OutboxView ob) {  // by value, like outbox_emit
  const OutboxStage s = ob.stg;
  __syncthreads();  // every emit of the tile has landed in LDS
  const unsigned n = *s.n < s.cap ? *s.n : s.cap;
  if (threadIdx.x == 0) *s.base = n ? atomicAdd(&ob.count[0], (unsigned long long)n) : 0ull;
  __syncthreads();
  const unsigned long long base = *s.base;
  unsigned long long drop = 0;
  for (unsigned j = threadIdx.x; j < n; j += blockDim.x) {
    const unsigned long long slot = base + j;
    if (slot < ob.cap) {
      ob.actor[slot] = s.actor[j];
      ob.method[slot] = s.method[j];
      ob.a0[slot] = s.a0[j];
      ob.a1[slot] = s.a1[j];
      ob.a2[slot] = s.a2[j];
    } else {
      ++drop;
    }
  }
  if (drop) atomicAdd(&ob.count[1], drop);
  __syncthreads();  // copies read the stage before it is reset
  if (threadIdx.x == 0) *s.n = 0;
  __syncthreads();
}

// Called by the lanes that emit, from inside a (possibly divergent) branch.  The
// view travels BY VALUE everywhere: taking the address of the kernel argument
// made hipcc copy it to scratch in every thread (64 B/lane of HBM writes).
__device__ __forceinline__ void outbox_emit(OutboxView ob, uint32_t actor, uint16_t method, int64_t a0,
                                            int64_t a1, int64_t a2) {
  if (ob.stg.n) {  // block staging: an LDS atomic per wave
    const uint64_t sm = __ballot(1);
    const int sl = __builtin_ctzll(sm);
    unsigned li = 0;
    if (lane_id() == (unsigned)sl) li = atomicAdd(ob.stg.n, (unsigned)__popcll(sm));
    li = __shfl(li, sl) + mbcnt64(sm);
    if (li < ob.stg.cap) {
      ob.stg.actor[li] = actor;
      ob.stg.method[li] = method;
      ob.stg.a0[li] = a0;
      ob.stg.a1[li] = a1;
      ob.stg.a2[li] = a2;
      return;
    }
    // stage full (a handler emitting more than one record per message): straight to HBM
  }
  const uint64_t m = __ballot(1);  // the lanes executing this emit
  const int leader = __builtin_ctzll(m);
  const unsigned rank = mbcnt64(m);
  unsigned long long base = 0;
  if (lane_id() == (unsigned)leader) base = atomicAdd(&ob.count[0], (unsigned long long)__popcll(m));
  base = __shfl(base, leader);
  const uint64_t slot = base + rank;
  if (slot < ob.cap) {
    ob.actor[slot] = actor;
    ob.method[slot] = method;
    ob.a0[slot] = a0;
    ob.a1[slot] = a1;
    ob.a2[slot] = a2;
  } else {
    atomicAdd(&ob.count[1], 1ull);
  }
}

// Runs one request against the actor state of the mailbox it was routed to.
// `state` holds one int64 per local mailbox (the reference's `type Calculator int`
// receiver is exactly one machine int of actor state).  `delay_ticks` is the
// per-candidate delay of Prime.Check in 100 MHz ticks (250 ms in the reference;
// 0 for throughput runs).
//
// `exclusive`: the caller owns the actor for this call (the mailbox consumer that
// owns its shard, runs ordered methods one at a time per actor, in mailbox order),
// so an ordered method is a plain read-modify-write.  Elsewhere (the parallel
// batch dispatch, the latency-path wave) an ordered method is a CAS loop: still
// linearizable -- no update is lost -- just not in any defined order.
__device__ __forceinline__ ReplyRecord run_handler(const MsgRecord& m, int64_t* __restrict__ state,
                                                   uint32_t n_state, uint64_t delay_ticks,
                                                   OutboxView ob = OutboxView(), bool exclusive = false) {
  ReplyRecord r;
  r.value = 0;
  r.status = kStatusOk;
  r.actor = m.actor;
  switch (m.method) {
    case kCalculatorMultiply:
      r.value = m.a0 * m.a1;
      break;
    case kPrimeCheck: {
      // for i in [Min, min(Max, Target)): if i != 0 && Target % i == 0 -> i ; else Target
      const int64_t lo = m.a0, hi = m.a1 < m.a2 ? m.a1 : m.a2, target = m.a2;
      r.value = target;
      if (lo >= 0 && target > 0 && target <= 0xffffffffll) {
        // 32-bit divisibility: a u32 remainder is a handful of VALU ops, a 64-bit
        // one a long emulated sequence -- the whole optimus workload lives here
        const uint32_t t32 = (uint32_t)target;
        for (int64_t i = lo; i < hi; ++i) {
          spin_ticks(delay_ticks);
          if (i != 0 && t32 % (uint32_t)i == 0) {
            r.value = i;
            break;
          }
        }
        break;
      }
      for (int64_t i = lo; i < hi; ++i) {
        spin_ticks(delay_ticks);
        if (i != 0 && target % i == 0) {
          r.value = i;
          break;
        }
      }
      break;
    }
    case kEcho:
      r.value = m.a0;
      break;
    case kRetryTest: {
      // called++ ; ok iff called >= callsBeforePass (a0); reply = called
      if (m.actor < n_state) {
        const int64_t c = atomicAdd(reinterpret_cast<unsigned long long*>(state + m.actor), 1ull) + 1;
        if (c >= m.a0) {
          r.value = c;
        } else {
          r.status = kStatusFailed;
        }
      } else {
        r.status = kStatusNoActor;
      }
      break;
    }
    case kCounterAdd:
      if (m.actor < n_state) {
        r.value = (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(state + m.actor),
                                     (unsigned long long)m.a0) + m.a0;
      } else {
        r.status = kStatusNoActor;
      }
      break;
    case kForward:
      // a hop of a message chain: count the visit, pass the token on (device-side send)
      if (m.actor < n_state) {
        r.value = (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(state + m.actor), 1ull) + 1;
        if (m.a1 > 0) {
          if (ob.cap) {
            const uint64_t stride = (uint64_t)m.a2 & 0xffffffffull, n = (uint64_t)m.a2 >> 32;
            const uint64_t next = n ? ((uint64_t)m.a0 + stride) % n : (uint64_t)m.a0;
            outbox_emit(ob, (uint32_t)m.a0, kForward, (int64_t)next, m.a1 - 1, m.a2);
          } else {
            r.status = kStatusFailed;  // no outbox bound: the send cannot happen
          }
        }
      } else {
        r.status = kStatusNoActor;
      }
      break;
    case kSeqFold:
      if (m.actor < n_state) {
        unsigned long long* p = reinterpret_cast<unsigned long long*>(state + m.actor);
        if (exclusive) {
          const uint64_t prev = *p;
          *p = prev * kFoldMul + (uint64_t)m.a0;
          r.value = (int64_t)prev;
        } else {
          unsigned long long prev = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          for (;;) {
            const unsigned long long next = prev * kFoldMul + (uint64_t)m.a0;
            if (__hip_atomic_compare_exchange_weak(p, &prev, next, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT))
              break;
          }
          r.value = (int64_t)prev;
        }
      } else {
        r.status = kStatusNoActor;
      }
      break;
    default:
      r.status = kStatusNoMethod;
  }
  return r;
}

}  // namespace ptype
