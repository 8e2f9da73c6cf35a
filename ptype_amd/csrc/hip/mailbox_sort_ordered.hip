// The ordered drain of a mailbox Send and its ring-order completion (its own
// object: the variants build beside mailbox_sort.hip's).  Kernels:
// mailbox_sort_dev.hpp (mbx_drain_ordered_kernel, mbx_complete_ring_kernel);
// design: mailbox_sort.hip.
#include "mailbox_sort_dev.hpp"

namespace ptype {

void mbx_launch_ordered(const MbxOrderedLaunch& o) {
  const SortIn& in = o.in;
  const MboxView& mv = o.mv;
  const hipStream_t st = o.st;
  const uint32_t Sv = o.Sv;
  const bool r8_on = o.r8_on;
  // state staged per shard: what its actors need (mailboxes s, s + S, ...), not the cap
  const uint32_t n_loc = o.state && o.n_state ? std::min<uint32_t>((o.n_state + Sv - 1) / Sv, kOrdStateMax) : 0;
  const size_t st_lds = (size_t)n_loc * sizeof(int64_t);  // (covers every shard the kernel stages: n_loc <= cap)
  const bool a12 = o.a12;  // (a column given: staged; none: the handlers see zeros)
  const R8Args r8a = o.r8a;
#define PT_ORD5(A12, OKV, FXV, PFV, R8V)                                                                      \
do {                                                                                                        \
  const size_t lds = sizeof(OrdLds<A12, OKV>) + std::max<size_t>(st_lds, 16);                              \
  static bool attr = false;                                                                                 \
  if (!attr) { /* above the 64 KB default dynamic LDS */                                                    \
    PT_HIP_CHECK(hipFuncSetAttribute((const void*)mbx_drain_ordered_kernel<A12, OKV, FXV, PFV, R8V>,        \
                                     hipFuncAttributeMaxDynamicSharedMemorySize,                            \
                                     (int)(sizeof(OrdLds<A12, OKV>) + (size_t)kOrdStateMax * sizeof(int64_t)))); \
    attr = true;                                                                                            \
  }                                                                                                         \
  hipLaunchKernelGGL((mbx_drain_ordered_kernel<A12, OKV, FXV, PFV, R8V>), dim3(Sv), dim3(kOrdThreads), lds,  \
                     st, mv, o.gsum, o.ngroups, o.state, o.n_state, o.delay_ticks, o.ob, o.stage_rep,       \
                     o.origin_base, r8a);                                             \
} while (0)
  // one-argument batches: 4096-record windows, and a uniform SeqFold batch folds in
  // registers with the next window prefetched (0.341 vs 0.357 ms per 8 Mi SeqFold step,
  // round 5); two- and three-argument batches: 2048-record windows, the handler switch
  const bool fold = o.fold;
  if (r8_on) {  // (one-argument, 4096-record form)
    if (fold) PT_ORD5(false, 8, kSeqFold, true, true);
    else PT_ORD5(false, 8, 0, false, true);
  } else if (!a12) {
    if (fold) PT_ORD5(false, 8, kSeqFold, true, false);
    else PT_ORD5(false, 8, 0, false, false);
  } else {
    PT_ORD5(true, kOrdK, 0, false, false);
  }
#undef PT_ORD5
  if (r8_on)
    hipLaunchKernelGGL(mbx_rec8_next_kernel<>, dim3(1), dim3(256), 0, st, (const uint32_t*)o.r8max, o.r8w, o.r8host,
                       in.tiles);
  PT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(mbx_complete_ring_kernel<>, dim3(o.tile_grid), dim3(kST),
                     (size_t)kSTile * (8 + 2 + 1) + (size_t)Sv * 8, st, in, mv,
                     (const uint32_t*)o.tinfo, (const u32x4*)o.stage_rep, o.rv, o.tctr);
}

}  // namespace ptype
