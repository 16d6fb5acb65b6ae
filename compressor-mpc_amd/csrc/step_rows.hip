// Fused small-batch steps on the row build kernel (build_rows_kernel.h):
// the build kernel runs the K Jacobi iterations of the QPs it built (one
// per lane after its groups, or one per 16-lane row inside each group).
// Compiled with the solver objects' flags (Makefile SOLVERFLAGS).
#include "build_rows_kernel.h"

// fused build + K iterations with the row solver inside each group:
// four-wave workgroups at one wave per SIMD (the row solver's state on top of
// the build's live registers)
#define ROWS_FUSED_CASE(NS_, NY_, NU_, M_)                                            \
  if (ns == NS_ && ny == NY_ && nu == NU_ && m == M_ && P.nd == 2 && P.nu_tot == 4) { \
    if (cmpc_rows_waves_per_group(P.rows) != 4) return -1;                           \
    if (P.rows.per_wave < 4 * (NU_ * M_) * (NU_ * M_)) return -1;                    \
    *solver = CMPC_SOLVE_ROWS;                                                         \
    if (ring) {                                                                        \
      if (trace) return rows_launch<NS_, NY_, NU_, M_, 4, true, 1, 2>(P, s);          \
      return rows_launch<NS_, NY_, NU_, M_, 4, true, 1, 1>(P, s);                     \
    }                                                                                  \
    if (trace) return rows_launch<NS_, NY_, NU_, M_, 4, false, 1, 2>(P, s);           \
    return rows_launch<NS_, NY_, NU_, M_, 4, false, 1, 1>(P, s);                      \
  }
// the same with the lane solver (nV <= 4: faster than the row solver there)
// (a wave solves its groups' QPs after building them all: at most 16 groups
// per wave, one QP per lane)
#define ROWS_FUSED_LANE_CASE(NS_, NY_, NU_, M_)                                       \
  if (ns == NS_ && ny == NY_ && nu == NU_ && m == M_ && P.nd == 2 && P.nu_tot == 4) { \
    if (cmpc_rows_waves_per_group(P.rows) != 4 || ring) return -1;                   \
    if (P.rows.per_wave < (NU_ * M_) * (NU_ * M_) * 64) return -1; /* G / U columns */ \
    /* one QP per lane: at most 16 groups per wave of the launch's 2 (WPE 2) */      \
    /* 4-wave workgroups per CU, fewer if the LDS layout allows fewer */            \
    if ((P.nqp + 3) / 4 > 16 * 4 * P.cus * std::min(2, cmpc_rows_resident_groups(P.rows, 4))) return -1; \
    *solver = CMPC_SOLVE_LANE;                                                         \
    if (trace) return rows_launch<NS_, NY_, NU_, M_, 4, false, 2, 4>(P, s);           \
    return rows_launch<NS_, NY_, NU_, M_, 4, false, 2, 3>(P, s);                      \
  }

int cmpc_launch_step_rows(const BuildParams& P, int ns, int ny, int nu, int m, void* stream, int* solver) {
  hipStream_t s = (hipStream_t)stream;
  if (!P.rows.ok || P.S < 1 || 4 % P.S) return -1;
  bool ring = false;
  for (int c = 0; c < CMPC_MAX_INPUTS; ++c) ring = ring || P.rows.ring[c] > 0;
  if (!ring && P.rows.nseg > 2 * 2) return -1;
  const bool trace = P.sv.trace != nullptr;
#if CMPC_FUSED_LANE_SOLVE
  ROWS_FUSED_LANE_CASE(11, 3, 2, 2)  // parallel coop
  ROWS_FUSED_LANE_CASE(11, 2, 2, 2)  // parallel ncoop
  ROWS_FUSED_LANE_CASE(10, 2, 2, 2)  // serial ncoop
  ROWS_FUSED_LANE_CASE(10, 4, 2, 2)  // serial coop
#endif
  ROWS_FUSED_CASE(11, 3, 2, 2)  // parallel coop
  ROWS_FUSED_CASE(11, 2, 2, 2)  // parallel ncoop
  ROWS_FUSED_CASE(11, 3, 4, 2)  // parallel centralized
  ROWS_FUSED_CASE(10, 2, 2, 2)  // serial ncoop
  ROWS_FUSED_CASE(10, 4, 2, 2)  // serial coop
  ROWS_FUSED_CASE(10, 4, 4, 2)  // serial centralized
  return -1;
}

