// The fused one-pass sort + ring-order drain of a stateless mailbox Send, in two
// objects that build beside mailbox_sort.hip's: this one the directory routes
// (route modes 1 and 3, Join's default), mailbox_sort_fused_other.hip (which
// includes this file with PT_FUSED_OTHER_MODES) the hash-probe and affine ones.
// Kernels: mailbox_sort_dev.hpp (mbx_sortdrain_kernel); design: mailbox_sort.hip.
#include "mailbox_sort_dev.hpp"

namespace ptype {

#ifndef PT_FUSED_OTHER_MODES
void mbx_launch_fused_dir(const MbxFusedLaunch& f) {
#else
void mbx_launch_fused_other(const MbxFusedLaunch& f) {
#endif

  const SortIn& in = f.in;
  const MboxView& mv = f.mv;
  const hipStream_t st = f.st;
  const size_t lds = f.lds;
  const int rf = f.rf, mode = f.mode;
  const bool fixed_mul = f.fixed_mul, rank_route = f.rank_route;
  struct {
    bool a2, method_col;
  } a{f.a2, f.mcol};
  ReplyView rv = f.rv;
  OutboxView ob = f.ob;
#define PT_SD2(MO, A2, MC, FX)                                                                                    \
  do {                                                                                                            \
    if (!(A2) && !(MC) && rf == 1)                                                                                \
      hipLaunchKernelGGL((mbx_sortdrain_kernel<MO, false, false, FX, 1>), dim3(in.tiles), dim3(kST), lds, st, in,  \
                         mv, f.desc, f.tctr, f.gsum, f.sidx, f.tinfo, f.rw, rv,              \
                         f.state, f.n_state, f.delay_ticks, ob, f.ticket, f.reserve, f.r8host);          \
    else if (!(A2) && !(MC) && (MO) == 3 && rf == 2)                                                              \
      hipLaunchKernelGGL((mbx_sortdrain_kernel<3, false, false, FX, 2>), dim3(in.tiles), dim3(kST), lds, st, in,   \
                         mv, f.desc, f.tctr, f.gsum, f.sidx, f.tinfo, f.rw, rv,              \
                         f.state, f.n_state, f.delay_ticks, ob, f.ticket, f.reserve, f.r8host);          \
    else                                                                                                          \
      hipLaunchKernelGGL((mbx_sortdrain_kernel<MO, A2, MC, FX, 0>), dim3(in.tiles), dim3(kST), lds, st, in, mv, \
                         f.desc, f.tctr, f.gsum, f.sidx, f.tinfo, f.rw, rv,                  \
                         f.state, f.n_state, f.delay_ticks, ob, f.ticket, f.reserve, f.r8host);          \
  } while (0)
#define PT_SD(MO)                                                            \
  do {                                                                       \
    if (a.a2 && a.method_col) PT_SD2(MO, true, true, 0);                     \
    else if (a.method_col) PT_SD2(MO, false, true, 0);                       \
    else if (a.a2) {                                                         \
      if (fixed_mul) PT_SD2(MO, true, false, kCalculatorMultiply);           \
      else PT_SD2(MO, true, false, 0);                                       \
    } else {                                                                 \
      if (fixed_mul) PT_SD2(MO, false, false, kCalculatorMultiply);          \
      else PT_SD2(MO, false, false, 0);                                      \
    }                                                                        \
  } while (0)
#ifndef PT_FUSED_OTHER_MODES
    if (rank_route) {
      if (fixed_mul) PT_SD2(3, false, false, kCalculatorMultiply);
      else PT_SD2(3, false, false, 0);
    } else {
      PT_SD(1);
    }
#else
    if (mode == 2) PT_SD(2); else PT_SD(0);
#endif
#undef PT_SD
#undef PT_SD2
    PT_HIP_CHECK(hipGetLastError());
}

#ifndef PT_FUSED_OTHER_MODES
void mbx_launch_fused(const MbxFusedLaunch& f) {
  if (f.rank_route || f.mode == 1) mbx_launch_fused_dir(f);
  else mbx_launch_fused_other(f);
}
#endif

}  // namespace ptype
