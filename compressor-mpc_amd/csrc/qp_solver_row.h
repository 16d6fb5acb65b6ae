// Row-parallel form of the QP solver (qp_solver.h) for batches too small to
// fill the GPU with one QP per lane: one QP per 16-lane DPP row, four per
// wave64.  Same specification and arithmetic order as qp_solve_t and
// oracle/or_qp.c, bit for bit:
//  - the O(N^2) products (H^-1 g, H^-1 nu, the LDL' rows of H and the
//    columns of H^-1) are formed row-parallel: lane l computes entry l with
//    exactly the operations the scalar code performs for that entry;
//  - their results are all-gathered inside the row (row_newbcast DPP moves),
//    and everything else -- the working set, the K x K LDL' of N'H^-1 N, the
//    multipliers, the ratio tests, the phase-B scan, the iterate x -- runs
//    replicated in every lane of the row on identical values, so all lanes
//    of a row take the same branches (a wave diverges over its four QPs, not
//    over 64).
// Lane l = lane & 15 of a row: l < N owns row l of H^-1 and entry l of the
// distributed vectors; lanes N..15 run the replicated code on zero rows.
#pragma once
#include <type_traits>

#include "qp_solver.h"

// lane L of this lane's 16-lane row
template <int L>
__device__ __forceinline__ double rbc(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x150 + L, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x150 + L, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
// o[c] = v of lane c of the row, c < N
template <int N, int C = 0>
__device__ __forceinline__ void row_gather(double v, double (&o)[N]) {
  if constexpr (C < N) {
    o[C] = rbc<C>(v);
    row_gather<N, C + 1>(v, o);
  }
}

// f(std::integral_constant<int, 0>), ..., f(<N - 1>): a loop whose index is
// a compile-time constant (DPP lane selects are instruction immediates)
template <int N, int C = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (C < N) {
    f(std::integral_constant<int, C>{});
    static_for<N, C + 1>(f);
  }
}

// No stored H^-1 (the Qp's bounds, thresholds and normals only)
struct NoHinv {
  __device__ __forceinline__ double operator()(int, int) const { return 0.0; }
  __device__ __forceinline__ void set(int, int, double) {}
};
template <int N, int NU>
using RowQp = Qp<N, NU, NU, NoHinv>;

// entry l of H^-1 n (Qp::hinv_n for row l): hr = row l of H^-1
template <int N>
__device__ __forceinline__ double hinv_n_row(const double (&hr)[N], const double (&n)[N]) {
  double t = 0.0;
#pragma unroll
  for (int c = 0; c < N; ++c) t = fma(hr[c], n[c], t);
  return t;
}

// H^-1 (hinv_of: LDL' of H, then one ldl_solve per column, the upper
// triangle from the column solves mirrored).  Hl = row l of H.  The LDL' runs
// row-parallel (lane i forms L[i][j]; row j of L is broadcast once it is
// complete and kept, so every lane ends with all of L); lane c then solves
// column c; the transpose to rows goes through this QP's N x N LDS scratch t.
// Returns false if H is not positive definite (every lane the same).
template <int N>
__device__ __forceinline__ bool hinv_row(const double (&Hl)[N], int l, double (&hr)[N], double* t) {
  double Li[N], Lf[N][N], D[N];
#pragma unroll
  for (int k = 0; k < N; ++k) Li[k] = 0.0;
  bool ok = true;
  static_for<N>([&](auto J) {
    constexpr int j = decltype(J)::value;
    // row j of L (entries k < j, final since column j - 1) and M[j][j]
#pragma unroll
    for (int k = 0; k < j; ++k) Lf[j][k] = rbc<j>(Li[k]);
    double d = rbc<j>(Hl[j]);
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (k < j) d = d - (Lf[j][k] * Lf[j][k]) * D[k];
    ok = ok && (d > 0.0);
    D[j] = d;
    Lf[j][j] = 1.0;
    double sacc = Hl[j];  // M[i][j] of lane i
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (k < j) sacc = sacc - (Li[k] * Lf[j][k]) * D[k];
    if (l > j) Li[j] = sacc / d;
  });
  // column l of H^-1 (ldl_solve_k(N, L, D, e_l)): entries i <= l are H^-1(i, l)
  double e[N], colv[N];
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = (i == l) ? 1.0 : 0.0;
  ldl_solve_k<N>(N, Lf, D, e, colv);
  if (l < N) {
#pragma unroll
    for (int i = 0; i < N; ++i) t[i * N + l] = colv[i];  // t[i][c] = column c's entry i
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // row l: H^-1(l, c) = column c's entry l for c >= l, own column's entry c
  // for c < l (hinv_of's mirror)
#pragma unroll
  for (int c = 0; c < N; ++c) hr[c] = (l >= N) ? 0.0 : (c >= l ? t[l * N + c] : colv[c]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();  // t is reused by the next QP of this row
  return ok;
}

// (re)build M = N' H^-1 N and its LDL' for the current working set
// (wset_factor): H^-1 n_b row-parallel, gathered, the ndots replicated
template <int N, int NU>
__device__ __forceinline__ bool wset_factor_row(const RowQp<N, NU>& q, const double (&hr)[N],
                                                WSet<N, false>& W) {
  double M[N][N];
#pragma unroll
  for (int b = 0; b < N; ++b) {
    double hb[N];
#pragma unroll
    for (int c = 0; c < N; ++c) hb[c] = 0.0;
    if (b < W.K) {
      double nb[N];
      q.normal(W.j[b], W.side[b], nb);
      row_gather<N>(hinv_n_row<N>(hr, nb), hb);
    }
#pragma unroll
    for (int a = 0; a <= b; ++a) {
      double v = 0.0;
      if (b < W.K) {
        double na[N];
        q.normal(W.j[a], W.side[a], na);
        v = ndot<N>(na, hb);
      }
      M[a][b] = v;
      M[b][a] = v;
    }
  }
  return ldl_k<N>(W.K, M, W.L, W.D);
}

// qp_solve_t<TRACE, CACHE = false> for the QP of this row: g_l = entry l of
// the gradient; x (replicated) = the solution (zero on failure).
template <bool TRACE, int N, int NU>
__device__ __forceinline__ void qp_solve_row(const RowQp<N, NU>& q, const double (&hr)[N], int l, bool pd,
                                             double tol_d, double g_l, uint32_t ws_in, int max_chg,
                                             double (&X)[N], QpOut& o) {
  WSet<N, false> W;
  o.status = CMPC_QP_OK;
  o.nchg = 0;
  o.ntrace = 0;
  o.tr[0] = o.tr[1] = o.tr[2] = o.tr[3] = 0xFFFFFFFFu;
  W.K = 0;
#pragma unroll
  for (int a = 0; a < N; ++a) {
    W.j[a] = 0;
    W.side[a] = 0;
    W.lam[a] = 0.0;
  }
  int chg = 0;
  bool done = false;
  bool fact_ok = false;
  if (!pd) {
    o.status = CMPC_QP_NOT_PD;
    done = true;
  }
  double G[N], XU[N];
  row_gather<N>(g_l, G);
  {
    double sacc = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) sacc = sacc + hr[j] * G[j];
    row_gather<N>(-sacc, XU);
  }
  // A. warm start
  {
    uint32_t msk = done ? 0u : (ws_in & ((1u << (2 * N)) - 1u));
#pragma unroll
    for (int a = 0; a < N; ++a) {
      if (msk) {
        const int j = __builtin_ctz(msk);
        msk &= msk - 1u;
        const int sd = (ws_in >> (16 + j)) & 1u;
        W.j[a] = j;
        W.side[a] = sd;
        W.lam[a] = 0.0;
        W.bta[a] = q.beta(j, sd);
        W.K = a + 1;
      }
    }
  }
  for (int it = 0; it <= 2 * N + 2 && !done; ++it) {
    if (!(fact_ok && it == 0)) {
      fact_ok = wset_factor_row<N, NU>(q, hr, W);
      if (!fact_ok) {
        W.K = 0;
        ++chg;
        continue;
      }
    }
    double rhs[N];
#pragma unroll
    for (int a = 0; a < N; ++a) {
      rhs[a] = 0.0;
      if (a < W.K) {
        double na[N];
        q.normal(W.j[a], W.side[a], na);
        rhs[a] = W.bta[a] - ndot<N>(na, XU);
      }
    }
    ldl_solve_k<N>(W.K, W.L, W.D, rhs, W.lam);
    int worst = -1;
    double wv = -tol_d;
#pragma unroll
    for (int a = 0; a < N; ++a)
      if (a < W.K && W.lam[a] < wv) {
        wv = W.lam[a];
        worst = a;
      }
    if (worst < 0) break;
    int wj = 0, wsd = 0;
#pragma unroll
    for (int a = 0; a < N; ++a)
      if (a == worst) {
        wj = W.j[a];
        wsd = W.side[a];
      }
    if (TRACE) trace_push(o, 0, wj, wsd);
    wset_drop<N>(W, worst);
    fact_ok = false;
    if (++chg > max_chg) {
      o.status = CMPC_QP_MAX_NWSR;
      done = true;
    }
  }
#pragma unroll
  for (int r = 0; r < N; ++r) X[r] = 0.0;
  if (!done) {
    // x = xu + sum_a lam_a h_a (per entry, a ascending): entry l here, then gathered
    double xl = sel<N>(XU, l);
#pragma unroll
    for (int a = 0; a < N; ++a) {
      if (a < W.K) {
        double na[N];
        q.normal(W.j[a], W.side[a], na);
        xl = xl + W.lam[a] * hinv_n_row<N>(hr, na);
      }
    }
    row_gather<N>(xl, X);
  }
  // B. Goldfarb–Idnani
  for (int outer = 0; outer <= max_chg + 1 && !done; ++outer) {
    int pj = -1, ps = 0;
    double pv = 0.0;
    bool anyv = false;
#pragma unroll
    for (int j = 0; j < 2 * N; ++j)
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) anyv = anyv | (q.nu_dot(j, sd, X) - q.beta(j, sd) < q.thr(j, sd));
    if (anyv) {
      uint32_t act = 0;
#pragma unroll
      for (int a = 0; a < N; ++a)
        if (a < W.K) act |= 1u << W.j[a];
#pragma unroll
      for (int j = 0; j < 2 * N; ++j) {
        if (!((act >> j) & 1u)) {
#pragma unroll
          for (int sd = 0; sd < 2; ++sd) {
            const double sl = q.nu_dot(j, sd, X) - q.beta(j, sd);
            if (sl < q.thr(j, sd) && (pj < 0 || sl < pv)) {
              pj = j;
              ps = sd;
              pv = sl;
            }
          }
        }
      }
    }
    if (pj < 0) break;  // optimal
    double np_[N];
    q.normal(pj, ps, np_);
    const double bp = q.beta(pj, ps);
    double up = 0.0;
    for (int inner = 0; inner <= max_chg + 1 && !done; ++inner) {
      double HP[N], qv[N], rv[N], Z[N];
      const double hp_l = hinv_n_row<N>(hr, np_);
      row_gather<N>(hp_l, HP);
#pragma unroll
      for (int a = 0; a < N; ++a) {
        qv[a] = 0.0;
        if (a < W.K) {
          double na[N];
          q.normal(W.j[a], W.side[a], na);
          qv[a] = ndot<N>(na, HP);
        }
      }
      ldl_solve_k<N>(W.K, W.L, W.D, qv, rv);
      double zl = hp_l;
#pragma unroll
      for (int a = 0; a < N; ++a) {
        if (a < W.K) {
          double na[N];
          q.normal(W.j[a], W.side[a], na);
          zl = zl - rv[a] * hinv_n_row<N>(hr, na);
        }
      }
      row_gather<N>(zl, Z);
      const double zn = ndot<N>(np_, Z);
      const double den = ndot<N>(np_, HP);
      int k = -1;
      double t1 = 0.0;
#pragma unroll
      for (int a = 0; a < N; ++a)
        if (a < W.K && rv[a] > TOL_R) {
          const double ratio = W.lam[a] / rv[a];
          if (k < 0 || ratio < t1) {
            t1 = ratio;
            k = a;
          }
        }
      if (zn <= TOL_Z * den) {
        if (k < 0) {
          o.status = CMPC_QP_INFEASIBLE;
          done = true;
          break;
        }
#pragma unroll
        for (int a = 0; a < N; ++a)
          if (a < W.K) W.lam[a] = W.lam[a] - t1 * rv[a];
        up = up + t1;
        int kj = 0, ks = 0;
#pragma unroll
        for (int a = 0; a < N; ++a)
          if (a == k) {
            kj = W.j[a];
            ks = W.side[a];
          }
        if (TRACE) trace_push(o, 0, kj, ks);
        wset_drop<N>(W, k);
        if (++chg > max_chg) {
          o.status = CMPC_QP_MAX_NWSR;
          done = true;
          break;
        }
        fact_ok = wset_factor_row<N, NU>(q, hr, W);
        continue;
      }
      const double sl = ndot<N>(np_, X) - bp;
      const double t2 = -sl / zn;
      const bool full = (k < 0) || (t2 <= t1);
      const double t = full ? t2 : t1;
#pragma unroll
      for (int r = 0; r < N; ++r) X[r] = X[r] + t * Z[r];
#pragma unroll
      for (int a = 0; a < N; ++a)
        if (a < W.K) W.lam[a] = W.lam[a] - t * rv[a];
      up = up + t;
      if (full) {
        if (TRACE) trace_push(o, 1, pj, ps);
        wset_add<N>(W, pj, ps, up, np_, bp);
        if (++chg > max_chg) {
          o.status = CMPC_QP_MAX_NWSR;
          done = true;
          break;
        }
        fact_ok = wset_factor_row<N, NU>(q, hr, W);
        break;
      }
      int kj = 0, ks = 0;
#pragma unroll
      for (int a = 0; a < N; ++a)
        if (a == k) {
          kj = W.j[a];
          ks = W.side[a];
        }
      if (TRACE) trace_push(o, 0, kj, ks);
      wset_drop<N>(W, k);
      if (++chg > max_chg) {
        o.status = CMPC_QP_MAX_NWSR;
        done = true;
        break;
      }
      fact_ok = wset_factor_row<N, NU>(q, hr, W);
    }
  }
  o.nchg = chg;
  uint32_t w = 0;
#pragma unroll
  for (int a = 0; a < N; ++a)
    if (a < W.K) w |= (1u << W.j[a]) | ((uint32_t)W.side[a] << (16 + W.j[a]));
  o.ws = w;
  (void)fact_ok;
  if (o.status == CMPC_QP_OK) {
    bool fin = true;
#pragma unroll
    for (int r = 0; r < N; ++r) fin = fin && __builtin_isfinite(X[r]);
    if (!fin) o.status = CMPC_QP_NONFINITE;
  }
  if (o.status == CMPC_QP_OK) {
    const uint32_t bnd = w & ((1u << N) - 1u), upm = (w >> 16) & bnd;
#pragma unroll
    for (int r = 0; r < N; ++r)
      X[r] = ((bnd >> r) & 1u) ? (((upm >> r) & 1u) ? q.ubv(r) : q.lbv(r)) : X[r];
  } else {
#pragma unroll
    for (int r = 0; r < N; ++r) X[r] = 0.0;
  }
}
