// The K Jacobi iterations of one QP per 16-lane row (qp_solver_row.h):
// shared by the row-layout iterate kernel (solve_rows.hip) and the fused
// build + iterate kernels (build_rows.hip, cmpc_kernels.hip), which hand over
// H, f and G in registers instead of through HBM.
//
// Lane l of the row: Hl = row l of H, f_l = f[l], Gl = row l of G (l < N;
// zeros in lanes N..15); q = the row's QP (clamped), active = q is a real QP
// (stores only then); s = its sub-controller, base_lane = lane 0 of the
// scenario's first row; tsh = this row's N x N LDS scratch.  Every lane of
// the wave must call it (the plan exchange reads other rows' lanes).
#pragma once
#include "cmpc_internal.h"
#include "qp_solver_row.h"

// LDSL: the working-set factor in this row's N x N LDS area lsh (registers
// otherwise; qp_solver_row.h LdsMat)
template <int N, int NU, int NVO, bool TRACE, bool EXT, bool LDSL = false>
__device__ __forceinline__ void rows_solve_qp(const SolveParams& P, int q, bool active, int s, int l,
                                              int base_lane, const double (&Hl)[N], double f_l,
                                              const double (&Gl)[NVO > 0 ? NVO : 1], double* tsh,
                                              double* lsh = nullptr) {
  constexpr int M = N / NU;
  constexpr int NVOA = NVO > 0 ? NVO : 1;
  constexpr int SM1 = NVO / N;  // other sub-controllers per scenario
  const bool own = l < N;
  const double* cfg = P.cfg + (size_t)s * P.co.len;

  // every global operand is requested before the first wait (small batches
  // leave one wave per SIMD: the H^-1 factorisation's LDS barriers would
  // otherwise expose one HBM round trip per load group)
  RowQp<N, NU> qp;
  double uo[NU];
#pragma unroll
  for (int c = 0; c < NU; ++c) uo[c] = P.u_old[(size_t)q * P.nu_tot + c];
  uint32_t ws = P.ws[q];
  // the plan, entry l in lane l (without other controllers only the K = 0
  // output reads it)
  double dprev_l = 0.0;
  if constexpr (NVO > 0) {
    if (own) dprev_l = P.du_old[(size_t)q * N + l];
  }
#pragma unroll
  for (int c = 0; c < NU; ++c) {
    qp.lb[c] = cfg[P.co.lower + c] - uo[c];
    qp.ub[c] = cfg[P.co.upper + c] - uo[c];
    qp.lbA[c] = cfg[P.co.rlower + c];
    qp.ubA[c] = cfg[P.co.rupper + c];
  }
  qp.tolerances();
  const RowScan sc = row_scan_consts<N, NU>(qp, l);
  double hr[N];
  const bool pd = hinv_row<N>(Hl, l, hr, tsh);
  double hmax = 0.0;
  {
    double hd[N];
    row_gather<N>(sel<N>(Hl, l < N ? l : N - 1), hd);  // H[i][i] from lane i
#pragma unroll
    for (int i = 0; i < N; ++i) hmax = fabs(hd[i]) > hmax ? fabs(hd[i]) : hmax;
  }
  const double tol_d = TOL_D * (1.0 + hmax);

  double x_l = 0.0;
  QpOut o;
  if (P.init) {  // InitializeQPProblem: cold solve of the step QP, status ignored
    qp_solve_row<false, N, NU, LDSL>(qp, hr, tsh, sc, l, pd, tol_d, f_l, 0u, CMPC_NWSR_MAX, x_l, o, lsh);
    if (active && l == 0) P.ws[q] = o.ws;
    __builtin_amdgcn_wave_barrier();  // tsh is reused by the next QP of this row
    return;
  }
  if constexpr (NVO == 0) {
    if (own) dprev_l = P.du_old[(size_t)q * N + l];
  }
  // the map form (qp_solver_row.h): x_u0 and U = Hinv G once per QP, the map
  // of the current working set kept across the K iterations
  double xu0_l, U_l[NVOA];
  row_jmap_terms<N, NVO>(hr, f_l, Gl, xu0_l, U_l);
  RowMap<N, NVO> mp;
  mp.ws = kWsInvalid;
  for (int k = 0; k < P.K; ++k) {
    {  // fair progress of the SIMD's waves (cf. cmpc_solve_kernel)
      // 3 - floor(4 k / K) by comparisons (a runtime integer division is a
      // long scalar sequence on this target, once per iteration)
      const int level = 3 - (4 * k >= P.K) - (4 * k >= 2 * P.K) - (4 * k >= 3 * P.K);
      if (level <= 0) __builtin_amdgcn_s_setprio(0);
      else if (level == 1) __builtin_amdgcn_s_setprio(1);
      else if (level == 2) __builtin_amdgcn_s_setprio(2);
      else __builtin_amdgcn_s_setprio(3);
    }
    double dother[NVOA];
#pragma unroll
    for (int c = 0; c < NVOA; ++c) dother[c] = 0.0;
    if constexpr (NVO > 0) {
      if constexpr (EXT) {
        // du_last of DistributedController::GetInput (nerve_center.h:283-285)
#pragma unroll
        for (int rk = 0; rk < SM1; ++rk)
#pragma unroll
          for (int mv = 0; mv < M; ++mv)
#pragma unroll
            for (int c = 0; c < NU; ++c)
              dother[mv * (SM1 * NU) + rk * NU + c] = P.du_other[(size_t)q * NVO + rk * N + mv * NU + c];
      } else {
        // the other sub-controllers' plans: entry mv * NU + c of sub-controller
        // s2 sits in lane mv * NU + c of its row
#pragma unroll
        for (int rk = 0; rk < SM1; ++rk) {
          const int s2 = rk + (rk >= s ? 1 : 0);
#pragma unroll
          for (int mv = 0; mv < M; ++mv)
#pragma unroll
            for (int c = 0; c < NU; ++c)
              dother[mv * (SM1 * NU) + rk * NU + c] = __shfl(dprev_l, base_lane + 16 * s2 + mv * NU + c, 64);
        }
      }
    }
    // f_k = f + G du_other, in the map form
    qp_solve_row_map<TRACE, N, NU, NVO, LDSL>(qp, tsh, sc, l, pd, tol_d, xu0_l, U_l, dother, ws, CMPC_NWSR_MAX, x_l,
                                              o, mp, lsh);
    ws = o.ws;
    dprev_l = x_l;
    if (TRACE && active && l == 0 && P.trace) {
      uint32_t* tr = reinterpret_cast<uint32_t*>(P.trace + ((size_t)q * P.K + k) * 16);
#pragma unroll
      for (int t = 0; t < 4; ++t) tr[t] = o.tr[t];
      P.ntrace[(size_t)q * P.K + k] = o.ntrace;
    }
  }
  __builtin_amdgcn_wave_barrier();  // tsh is reused by the next QP of this row
  if (!active) return;
  if (l == 0) {
    P.ws[q] = ws;
    if (P.K > 0) {
      P.status[q] = o.status;
      P.nwsr[q] = o.nchg;
    }
  }
  if (own) {
    P.du[(size_t)q * N + l] = dprev_l;
    P.du_old[(size_t)q * N + l] = dprev_l;
  }
  if ((P.flags & CMPC_APPLY_MOVE) && l < NU) {
    P.u_old[(size_t)q * P.nu_tot + l] = sel<NU>(uo, l) + dprev_l;
  }
}
