// Row-layout build kernel launcher (the kernel: build_rows_kernel.h).
#include "build_rows_kernel.h"

// four-wave workgroups whose layout admits at most two waves per SIMD run the
// 256-register (WPE = 2) instantiation
#define ROWS_CASE(NS_, NY_, NU_, M_)                                                  \
  if (ns == NS_ && ny == NY_ && nu == NU_ && m == M_ && P.nd == 2 && P.nu_tot == 4) { \
    const int w_ = cmpc_rows_waves_per_group(P.rows);                                  \
    const bool two_ = w_ == 4 && cmpc_rows_resident_groups(P.rows, 4) * 4 <= 8;        \
    if (ring) {                                                                        \
      if (two_) return rows_launch<NS_, NY_, NU_, M_, 4, true, 2>(P, s);               \
      if (w_ == 4) return rows_launch<NS_, NY_, NU_, M_, 4, true>(P, s);               \
      if (w_ == 2) return rows_launch<NS_, NY_, NU_, M_, 2, true>(P, s);               \
    } else {                                                                           \
      if (two_) return rows_launch<NS_, NY_, NU_, M_, 4, false, 2>(P, s);              \
      if (w_ == 4) return rows_launch<NS_, NY_, NU_, M_, 4, false>(P, s);              \
      if (w_ == 2) return rows_launch<NS_, NY_, NU_, M_, 2, false>(P, s);              \
    }                                                                                  \
    return -1;                                                                         \
  }

int cmpc_launch_build_rows(const BuildParams& P, int ns, int ny, int nu, int m, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!P.rows.ok) return -1;
  bool ring = false;
  for (int c = 0; c < CMPC_MAX_INPUTS; ++c) ring = ring || P.rows.ring[c] > 0;
  if (!ring && P.rows.nseg > 2 * 2) return -1;  // the plain kernel unrolls over 2 ND bounds
  ROWS_CASE(11, 3, 2, 2)  // parallel coop        (ControlledOutputIndices <0,1,3>)
  ROWS_CASE(11, 2, 2, 2)  // parallel ncoop
  ROWS_CASE(11, 3, 4, 2)  // parallel centralized
  ROWS_CASE(10, 2, 2, 2)  // serial ncoop
  ROWS_CASE(10, 4, 2, 2)  // serial coop          (all four outputs)
  ROWS_CASE(10, 4, 4, 2)  // serial centralized
  ROWS_CASE(11, 3, 2, 1)
  return -1;
}
