// Compiled-in device actor handlers: the method table that the dispatch kernels
// switch on.  This is the GPU-side replacement of stdlib net/rpc's reflective
// `service.call` (reference: server registration in
// example/calculator/server/server.go:16-20, handler bodies in
// example/calculator/calculator.go:9-12 and example/optimus/prime.go:15-25; the
// fault-injecting test actor in cluster/rpc_test.go:55-77).
#pragma once
#include "common.hpp"

namespace ptype {

// Runs one request against the actor state of the mailbox it was routed to.
// `state` holds one int64 per local mailbox (the reference's `type Calculator int`
// receiver is exactly one machine int of actor state).  `delay_ticks` is the
// per-candidate delay of Prime.Check in 100 MHz ticks (250 ms in the reference;
// 0 for throughput runs).
__device__ __forceinline__ ReplyRecord run_handler(const MsgRecord& m, int64_t* __restrict__ state,
                                                   uint32_t n_state, uint64_t delay_ticks) {
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
    default:
      r.status = kStatusNoMethod;
  }
  return r;
}

}  // namespace ptype
