// K Jacobi iterations of one QP per lane (qp_solver.h): the body of the
// iterate kernel (cmpc_solve_kernel) and of the fused small-batch step of the
// row build kernel (build_rows.hip), which solves the four QPs it just built
// in lanes 0-3 of the same wave.
//
// rec = the QP's H, f (nV*nV, nV; global, LDS or registers), G[a][c] =
// gb[(a * NVOA + c) * GSTRIDE]; q the QP (clamped), active = stores allowed; s = its
// sub-controller, base_lane = the lane of the scenario's sub-controller 0
// (the plan exchange reads lanes base_lane + s2 of the same wave).
#pragma once
#include <type_traits>

#include "cmpc_internal.h"
#include "qp_solver.h"

#ifndef CMPC_SOLVE_XU_LDS
#define CMPC_SOLVE_XU_LDS 1  // x_u0 in H^-1's unused LDS slots (0: registers)
#endif
#ifndef CMPC_SOLVE_PRIO
#define CMPC_SOLVE_PRIO 1  // priority by Jacobi-iteration progress (iterate 0.049 -> 0.047 ms)
#endif

template <int N, int NU, int NVO, bool TRACE, bool EXT, int GSTRIDE, class HS = HinvRegs<N>>
__device__ __forceinline__ void lane_solve_qp(const SolveParams& P, int q, bool active, int s, int base_lane,
                                              const double* rec, const double* gb, double* hsh = nullptr) {
  constexpr int M = N / NU;
  constexpr int NVOA = NVO > 0 ? NVO : 1;
  constexpr int SM1 = NVO / N;  // other sub-controllers per scenario
  const double* cfg = P.cfg + (size_t)s * P.co.len;
  double H[N][N], f[N];
#pragma unroll
  for (int a = 0; a < N; ++a)
#pragma unroll
    for (int b = 0; b < N; ++b) H[a][b] = rec[a * N + b];
#pragma unroll
  for (int a = 0; a < N; ++a) f[a] = rec[N * N + a];

  // bounds repeat every NU entries (rep_m(lower - u_old), rep_m(rate bounds));
  // H^-1 stays in registers (an LDS copy measured slower: the compiler
  // hoists its loads and spills more)
  // H^-1 in registers, or (HinvStrided) in the caller's LDS column hsh
  Qp<N, NU, NU, HS> qp;
  if constexpr (!std::is_same_v<HS, HinvRegs<N>>) qp.Hinv.p = hsh;
  double uo[NU];
#pragma unroll
  for (int c = 0; c < NU; ++c) uo[c] = P.u_old[(size_t)q * P.nu_tot + c];
#pragma unroll
  for (int c = 0; c < NU; ++c) {
    qp.lb[c] = cfg[P.co.lower + c] - uo[c];
    qp.ub[c] = cfg[P.co.upper + c] - uo[c];
    qp.lbA[c] = cfg[P.co.rlower + c];
    qp.ubA[c] = cfg[P.co.rupper + c];
  }
  qp.tolerances();
  const bool pd = hinv_of<N>(H, qp.Hinv);
  double hmax = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) hmax = fabs(H[i][i]) > hmax ? fabs(H[i][i]) : hmax;
  const double tol_d = TOL_D * (1.0 + hmax);

  uint32_t ws = P.ws[q];
  double x[N];
  QpOut o;
  if (P.init) {  // InitializeQPProblem: cold solve of the step QP, status ignored
    qp_solve_t<false>(qp, pd, tol_d, f, 0u, CMPC_NWSR_MAX, x, o);
    if (active) P.ws[q] = o.ws;
    return;
  }
  double dprev[N];
#pragma unroll
  for (int a = 0; a < N; ++a) dprev[a] = P.du_old[(size_t)q * N + a];
  // the map form (qp_solver.h): x_u0 = -Hinv f and U = Hinv G once per QP,
  // the map of the current working set kept across the K iterations
  // (the iterate kernel, G in its own LDS columns (GSTRIDE > 1): U replaces
  // G there, the map form reads G only here; the fused steps read G from the
  // stored QP: U in registers)
  double xu0[N];
  constexpr bool UIN = GSTRIDE > 1;
  double Ur[UIN ? 1 : N][UIN ? 1 : NVOA];
  if constexpr (UIN) jmap_terms<N, NVO, GSTRIDE>(qp.Hinv, f, const_cast<double*>(gb), xu0);
  else jmap_terms<N, NVO, GSTRIDE>(qp.Hinv, f, gb, xu0, Ur);
  using UAcc = std::conditional_t<UIN, UStrided<NVOA, GSTRIDE>, URegs<N, NVOA>>;
  const UAcc U = [&]() {
    if constexpr (UIN) return UStrided<NVOA, GSTRIDE>{gb};
    else return URegs<N, NVOA>{Ur};
  }();
  // x_u0 into H^-1's unused LDS slots where H^-1 lives in LDS (its 4
  // registers were spilled to scratch across the iterations and reloaded
  // at every map build)
  auto xu0_of = [&]() -> decltype(auto) {
    if constexpr (CMPC_SOLVE_XU_LDS && !std::is_same_v<HS, HinvRegs<N>> && N >= 3) {
      XuStrided<N, HS::kStride> xs{hsh};
#pragma unroll
      for (int r = 0; r < N; ++r) xs.set(r, xu0[r]);
      return xs;
    } else {
      return (xu0);
    }
  };
  decltype(auto) xa = xu0_of();
  JMap<N, NVO> mp;
  mp.ws = kWsInvalid;
  for (int k = 0; k < P.K; ++k) {
#if CMPC_SOLVE_PRIO
    {  // fair progress of the SIMD's waves (cf. build_rows.hip)
      // 3 - floor(4 k / K) by comparisons (a runtime integer division is a
      // long scalar sequence on this target, once per iteration)
      const int level = 3 - (4 * k >= P.K) - (4 * k >= 2 * P.K) - (4 * k >= 3 * P.K);
      if (level <= 0) __builtin_amdgcn_s_setprio(0);
      else if (level == 1) __builtin_amdgcn_s_setprio(1);
      else if (level == 2) __builtin_amdgcn_s_setprio(2);
      else __builtin_amdgcn_s_setprio(3);
    }
#endif
    double dother[NVOA];
#pragma unroll
    for (int c = 0; c < NVOA; ++c) dother[c] = 0.0;
    if (NVO > 0) {
      if constexpr (EXT) {
        // du_last of DistributedController::GetInput: the other controllers'
        // plans, controller-major, then move, then input (nerve_center.h:283-285)
#pragma unroll
        for (int rk = 0; rk < SM1; ++rk)
#pragma unroll
          for (int mv = 0; mv < M; ++mv)
#pragma unroll
            for (int c = 0; c < NU; ++c)
              dother[mv * (SM1 * NU) + rk * NU + c] = P.du_other[(size_t)q * NVO + rk * N + mv * NU + c];
      } else if (SM1 == 1 && !(base_lane & 1)) {
        // two sub-controllers on lanes (2i, 2i + 1), as every caller places
        // a scenario's pair: the other plan is the partner lane's, a
        // quad_perm [1,0,3,2] DPP move instead of an LDS permute
#pragma unroll
        for (int mv = 0; mv < M; ++mv)
#pragma unroll
          for (int c = 0; c < NU; ++c) {
            const double v = dprev[mv * NU + c];
            const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, true);
            const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, true);
            dother[mv * NU + c] = __hiloint2double(hi, lo);
          }
      } else {
#pragma unroll
        for (int rk = 0; rk < SM1; ++rk) {
          const int s2 = rk + (rk >= s ? 1 : 0);
#pragma unroll
          for (int mv = 0; mv < M; ++mv)
#pragma unroll
            for (int c = 0; c < NU; ++c)
              dother[mv * (SM1 * NU) + rk * NU + c] = __shfl(dprev[mv * NU + c], base_lane + s2, 64);
        }
      }
    }
    // f_k = f + (Su_other du_other)' W Su = f + G du_other, in the map form
    qp_solve_map<TRACE, N, NVO>(qp, pd, tol_d, xa, U, dother, ws, CMPC_NWSR_MAX, x, o, mp);
    ws = o.ws;
#pragma unroll
    for (int a = 0; a < N; ++a) dprev[a] = x[a];
    if (TRACE && active && P.trace) {
      uint32_t* tr = reinterpret_cast<uint32_t*>(P.trace + ((size_t)q * P.K + k) * 16);
#pragma unroll
      for (int t = 0; t < 4; ++t) tr[t] = o.tr[t];
      P.ntrace[(size_t)q * P.K + k] = o.ntrace;
    }
  }
  if (!active) return;
  P.ws[q] = ws;
  if (P.K > 0) {
    P.status[q] = o.status;
    P.nwsr[q] = o.nchg;
  }
#pragma unroll
  for (int a = 0; a < N; ++a) {
    P.du[(size_t)q * N + a] = dprev[a];
    P.du_old[(size_t)q * N + a] = dprev[a];
  }
  if (P.flags & CMPC_APPLY_MOVE) {
#pragma unroll
    for (int c = 0; c < NU; ++c) P.u_old[(size_t)q * P.nu_tot + c] = uo[c] + dprev[c];
  }
}
