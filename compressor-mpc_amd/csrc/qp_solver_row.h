// Row-parallel form of the QP solver (qp_solver.h) for batches too small to
// fill the GPU with one QP per lane: one QP per 16-lane DPP row, four per
// wave64.  Same specification (oracle/or_qp.c, version 4) and arithmetic
// order as qp_solve_t, bit for bit:
//  - vectors stay distributed: lane l < N holds row l of H^-1 (registers and
//    this QP's N x N LDS scratch T), and entry l of x_u, x, H^-1 nu_p, z;
//  - a column of H^-1 (h_j = H^-1 nall_j, one or two LDS reads per lane) and
//    a constraint value nu_j' v of a distributed v (one or two ds_bpermute
//    reads of lanes j, j - nu) take the runtime constraint index directly,
//    with exactly the scalar code's operations (a single subtraction, a
//    negation);
//  - the phase-B scan is lane-parallel: lane c < 2N evaluates constraint c
//    (both sides), a row ballot tells whether any is violated and a DPP
//    butterfly min + lowest-lane ballot picks the most violated, first in
//    (j, side) order on ties, as the scalar scan does;
//  - the working set and its K x K LDL' factor (append / removal updates of
//    qp_solver.h) are replicated in every lane of the row on identical
//    values, so all lanes of a row take the same branches (a wave diverges
//    over its four QPs, not over 64).
// Lanes N..15 hold zero rows and run the replicated code on them.
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
// v of a lane of the same row selected by a DPP control (row_shr, quad_perm,
// mirrors); bound_ctrl: lanes without a source read 0
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
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

// The working set's factor L in LDS (one N x N matrix per row, every lane of
// the row reading and writing the same values): WSet<N, false, LdsMat<N>>
// frees the 2 N (N - 1) / 2 registers of the replicated factor where the row
// solver shares a kernel with other register-hungry code (the fused split step).
template <int N>
struct LdsMat {
  double* p;
  struct Row {
    double* r;
    __device__ __forceinline__ double& operator[](int k) const { return r[k]; }
  };
  __device__ __forceinline__ Row operator[](int i) const { return Row{p + i * N}; }
};
template <int N, bool LDSL>
using RowWSet = WSet<N, false, std::conditional_t<LDSL, LdsMat<N>, double[N][N]>>;

// No stored H^-1 (the Qp's bounds, thresholds and normals only)
struct NoHinv {
  __device__ __forceinline__ double operator()(int, int) const { return 0.0; }
  __device__ __forceinline__ void set(int, int, double) {}
};
template <int N, int NU>
using RowQp = Qp<N, NU, NU, NoHinv>;

// H^-1 (hinv_of: LDL' of H with reciprocal pivots, then one ldl_solve per
// column, the upper triangle from the column solves mirrored).  Hl = row l of
// H.  The LDL' runs row-parallel (lane i forms L[i][j]; row j of L is
// broadcast once it is complete and kept, so every lane ends with all of L);
// lane c then solves column c into this QP's N x N LDS scratch t
// (t[i * N + c] = column c's entry i), which stays valid for the QP's solves
// (hinv_at); hr = row l of H^-1.  Returns false if H is not positive definite
// (every lane the same).
template <int N>
__device__ __forceinline__ bool hinv_row(const double (&Hl)[N], int l, double (&hr)[N], double* t) {
  double Li[N], Lf[N][N], D[N], R[N];
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
      if (k < j) d = fma(-(Lf[j][k] * Lf[j][k]), D[k], d);
    ok = ok && (d > 0.0);
    D[j] = d;
    R[j] = 1.0 / d;
    Lf[j][j] = 1.0;
    double sacc = Hl[j];  // M[i][j] of lane i
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (k < j) sacc = fma(-(Li[k] * Lf[j][k]), D[k], sacc);
    if (l > j) Li[j] = sacc * R[j];
  });
  // column l of H^-1 (ldl_solve_k(N, L, R, e_l)): entries i <= l are H^-1(i, l)
  double e[N], colv[N];
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = (i == l) ? 1.0 : 0.0;
  ldl_solve_k<N>(N, Lf, R, e, colv);
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
  return ok;
}

// H^-1(r, c) of the specification (upper triangle of the column solves,
// mirrored) from the LDS scratch t of hinv_row; r < N
template <int N>
__device__ __forceinline__ double hinv_at(const double* t, int r, int c) {
  return r <= c ? t[r * N + c] : t[c * N + r];
}

// entry l of h = H^-1 nu_{j,side} (or_qp.c hinv_nu): a column, or a
// difference of two columns, of H^-1; 0 on lanes l >= N
template <int N, int NU>
__device__ __forceinline__ double hval(const double* t, int l, int j, int side) {
  if (l >= N) return 0.0;
  const bool rate = j >= N;
  const int i = rate ? j - N : j;
  double v = hinv_at<N>(t, l, i);
  if (rate && i >= NU) v = v - hinv_at<N>(t, l, i - NU);
  return side ? -v : v;
}

// v of lane `src` of this lane's row (ds_bpermute; src runtime)
__device__ __forceinline__ double row_read(double v, int rowbase, int src) {
  return __shfl(v, rowbase + src, 64);
}

// nu_{j,side}' v for a distributed v (entry r in lane r), replicated in the
// row (or_qp.c nu_dot)
template <int N, int NU>
__device__ __forceinline__ double nval(double v, int rowbase, int j, int side) {
  const bool rate = j >= N;
  const int i = rate ? j - N : j;
  double t = row_read(v, rowbase, i);
  if (rate && i >= NU) t = t - row_read(v, rowbase, i - NU);
  return side ? -t : t;
}

// warm start: the LDL' of M (M[i][k] = n_k' h_i, k <= i; wset_factor) with
// the h_i distributed (hv[i] = entry l of h_i) and M's entries formed where
// the factorisation reads them, in ldl_k's order
template <int N, int NU, class WS>
__device__ __forceinline__ bool wset_factor_row(const double* t, int l, int rowbase, WS& W) {
  double hv[N];
#pragma unroll
  for (int i = 0; i < N; ++i) hv[i] = (i < W.K) ? hval<N, NU>(t, l, W.j[i], W.side[i]) : 0.0;
  bool ok = true;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (j < W.K) {
      double d = nval<N, NU>(hv[j], rowbase, W.j[j], W.side[j]);
      const double mjj = d;
#pragma unroll
      for (int k = 0; k < j; ++k) d = fma(-(W.L[j][k] * W.L[j][k]), W.D[k], d);
      ok = ok && (d > TOL_Z * mjj);
      W.D[j] = d;
      const double r = 1.0 / d;
      W.R[j] = r;
      W.L[j][j] = 1.0;
#pragma unroll
      for (int i = j + 1; i < N; ++i) {
        if (i < W.K) {
          double sacc = nval<N, NU>(hv[i], rowbase, W.j[j], W.side[j]);
#pragma unroll
          for (int k = 0; k < j; ++k) sacc = fma(-(W.L[i][k] * W.L[j][k]), W.D[k], sacc);
          W.L[i][j] = sacc * r;
        }
      }
    }
  }
  return ok;
}

// Per-QP constants of the lane-parallel scan: lane c < 2N evaluates
// constraint c (c < N: bound on x_c; else rate row c - N); bounds and
// thresholds of its two sides (Qp::beta, Qp::thr)
struct RowScan {
  double blo, bhi, tlo, thi;  // beta of side 0 / 1, -TOL_P (1 + |beta|)
  bool live;                  // c < 2N
};
template <int N, int NU>
__device__ __forceinline__ RowScan row_scan_consts(const RowQp<N, NU>& q, int l) {
  RowScan s;
  s.live = l < 2 * N;
  const int j = s.live ? l : 0;
  s.blo = q.beta(j, 0);
  s.bhi = q.beta(j, 1);
  s.tlo = q.thr(j, 0);
  s.thi = q.thr(j, 1);
  return s;
}

// the most violated inactive constraint (phase-B scan of qp_solve_t):
// returns pj (-1: none) and its side ps, replicated in the row
template <int N, int NU>
__device__ __forceinline__ int row_scan(double x_l, const RowScan& sc, uint32_t act, int l, int rowbase,
                                        int& ps) {
  // constraint value nu_c' x of lane c: x_c, x_i or x_i - x_{i-NU} (i = c - N)
  const double xs = dpp64<0x110 + N>(x_l);  // row_shr:N  -> x_{c - N}
  double v = l < N ? x_l : xs;
  if constexpr (N > NU) {
    const double xs2 = dpp64<0x110 + N + NU>(x_l);  // row_shr:N+NU -> x_{c - N - NU}
    if (l >= N + NU) v = xs - xs2;
  }
  const bool inact = sc.live && !((act >> (l & 31)) & 1u);
  const double slo = v - sc.blo;
  const double shi = -v - sc.bhi;
  const bool vlo = inact && slo < sc.tlo;
  const bool vhi = inact && shi < sc.thi;
  const unsigned long long any = __ballot(vlo || vhi);
  ps = 0;
  if (((any >> rowbase) & 0xFFFFull) == 0) return -1;
  // the lane's candidate (lower side first on ties), +inf if none
  const bool takelo = vlo && (!vhi || slo <= shi);
  const int side = takelo ? 0 : 1;
  double val = takelo ? slo : (vhi ? shi : __builtin_huge_val());
  double m = val;
  m = fmin(m, dpp64<0xB1>(m));   // quad_perm [1,0,3,2]
  m = fmin(m, dpp64<0x4E>(m));   // quad_perm [2,3,0,1]
  m = fmin(m, dpp64<0x141>(m));  // row_half_mirror
  m = fmin(m, dpp64<0x140>(m));  // row_mirror
  const unsigned long long win = __ballot((vlo || vhi) && val == m);
  const int pj = __builtin_ctzll((win >> rowbase) & 0xFFFFull);
  ps = __shfl(side, rowbase + pj, 64);
  return pj;
}

// Phase B (Goldfarb–Idnani) of the row's QP from the phase-A point x_l and
// multipliers W.lam, then the result (qp_phase_b).
template <bool TRACE, int N, int NU, class WS>
__device__ __forceinline__ void qp_row_phase_b(const RowQp<N, NU>& q, const double* t, const RowScan& sc,
                                               int l, int rowbase, WS& W, double& x_l, int chg,
                                               bool done, int max_chg, QpOut& o) {
  // B. Goldfarb–Idnani
  for (int outer = 0; outer <= max_chg + 1 && !done; ++outer) {
    uint32_t act = 0;
#pragma unroll
    for (int a = 0; a < N; ++a)
      if (a < W.K) act |= 1u << W.j[a];
    int ps = 0;
    const int pj = row_scan<N, NU>(x_l, sc, act, l, rowbase, ps);
    if (pj < 0) break;  // optimal
    const double bp = q.beta(pj, ps);
    const double hp_l = hval<N, NU>(t, l, pj, ps);
    double up = 0.0;
    for (int inner = 0; inner <= max_chg + 1 && !done; ++inner) {
      double qv[N], rv[N], zz[N];
#pragma unroll
      for (int a = 0; a < N; ++a) qv[a] = (a < W.K) ? nval<N, NU>(hp_l, rowbase, W.j[a], W.side[a]) : 0.0;
      ldl_solve_k<N>(W.K, W.L, W.R, qv, rv, zz);
      double z_l = hp_l;
#pragma unroll
      for (int a = 0; a < N; ++a)
        if (a < W.K) z_l = fma(-rv[a], hval<N, NU>(t, l, W.j[a], W.side[a]), z_l);
      const double zn = nval<N, NU>(z_l, rowbase, pj, ps);
      const double den = nval<N, NU>(hp_l, rowbase, pj, ps);
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
      if (zn <= TOL_Z * den || W.K >= N) {  // dependent (n active: always)
        if (k < 0) {
          o.status = CMPC_QP_INFEASIBLE;
          done = true;
          break;
        }
#pragma unroll
        for (int a = 0; a < N; ++a)
          if (a < W.K) W.lam[a] = fma(-t1, rv[a], W.lam[a]);
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
        continue;
      }
      const double rzn = 1.0 / zn;
      const double sl = nval<N, NU>(x_l, rowbase, pj, ps) - bp;
      const double t2 = -sl * rzn;
      const bool full = (k < 0) || (t2 <= t1);
      const double tt = full ? t2 : t1;
      x_l = fma(tt, z_l, x_l);
#pragma unroll
      for (int a = 0; a < N; ++a)
        if (a < W.K) W.lam[a] = fma(-tt, rv[a], W.lam[a]);
      up = up + tt;
      if (full) {
        if (TRACE) trace_push(o, 1, pj, ps);
        double nz[N];  // (unused: the row form keeps no normals)
        wset_add<N>(W, pj, ps, up, nz, bp, zz, zn, rzn);
        if (++chg > max_chg) {
          o.status = CMPC_QP_MAX_NWSR;
          done = true;
        }
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
    }
  }
  o.nchg = chg;
  uint32_t w = 0;
#pragma unroll
  for (int a = 0; a < N; ++a)
    if (a < W.K) w |= (1u << W.j[a]) | ((uint32_t)W.side[a] << (16 + W.j[a]));
  o.ws = w;
  if (o.status == CMPC_QP_OK) {
    const unsigned long long bad = __ballot(l < N && !__builtin_isfinite(x_l));
    if ((bad >> rowbase) & 0xFFFFull) o.status = CMPC_QP_NONFINITE;
  }
  if (o.status == CMPC_QP_OK) {
    if (l < N && ((w >> l) & 1u)) x_l = ((w >> (16 + l)) & 1u) ? q.ubv(l) : q.lbv(l);
  } else {
    x_l = 0.0;
  }
}


// qp_solve_t for the QP of this row: g_l = entry l of
// the gradient, t = hinv_row's LDS scratch, hr = row l of H^-1, sc the scan
// constants; x_l = entry l of the solution (zero on failure).
template <bool TRACE, int N, int NU, bool LDSL = false>
__device__ __forceinline__ void qp_solve_row(const RowQp<N, NU>& q, const double (&hr)[N], const double* t,
                                             const RowScan& sc, int l, bool pd, double tol_d, double g_l,
                                             uint32_t ws_in, int max_chg, double& x_l, QpOut& o,
                                             double* lsh = nullptr) {
  const int rowbase = (int)(__lane_id() & ~15u);
  RowWSet<N, LDSL> W;
  if constexpr (LDSL) W.L.p = lsh;
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
  if (!pd) {
    o.status = CMPC_QP_NOT_PD;
    done = true;
  }
  double xu_l;
  {
    double G[N];
    row_gather<N>(g_l, G);
    double sacc = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) sacc = fma(hr[j], G[j], sacc);
    xu_l = -sacc;
  }
  // A. warm start: slots in ascending j, the full factor
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
        W.K = a + 1;
      }
    }
    if (W.K > 0 && !wset_factor_row<N, NU>(t, l, rowbase, W)) {  // inconsistent warm start: cold
      W.K = 0;
      ++chg;
    }
  }
  for (int it = 0; it <= N && !done; ++it) {
    double rhs[N];
#pragma unroll
    for (int a = 0; a < N; ++a) rhs[a] = (a < W.K) ? wset_beta(q, W, a) - nval<N, NU>(xu_l, rowbase, W.j[a], W.side[a]) : 0.0;
    ldl_solve_k<N>(W.K, W.L, W.R, rhs, W.lam);
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
    if (++chg > max_chg) {
      o.status = CMPC_QP_MAX_NWSR;
      done = true;
    }
  }
  x_l = 0.0;
  if (!done) {
    // x = xu + sum_a lam_a h_a (entry l, a ascending)
    x_l = xu_l;
#pragma unroll
    for (int a = 0; a < N; ++a)
      if (a < W.K) x_l = fma(W.lam[a], hval<N, NU>(t, l, W.j[a], W.side[a]), x_l);
  }
  qp_row_phase_b<TRACE, N, NU>(q, t, sc, l, rowbase, W, x_l, chg, done, max_chg, o);
}

// The map form of the Jacobi iterations (qp_solve_map) for the row's QP:
// lam0, Lam replicated, x0 and X distributed (entry / row l in lane l).
template <int N, int NVO>
struct RowMap {
  static constexpr int NVOA = NVO > 0 ? NVO : 1;
  uint32_t ws, wc;
  int K;
  double lam0[N], Lam[N][NVOA];
  double x0_l, X_l[NVOA];
};

// x_u0 = -Hinv f and U = Hinv G, entry / row l (jmap_terms): f_l, Gl = row l
// of G
template <int N, int NVO>
__device__ __forceinline__ void row_jmap_terms(const double (&hr)[N], double f_l,
                                               const double (&Gl)[RowMap<N, NVO>::NVOA], double& xu0_l,
                                               double (&U_l)[RowMap<N, NVO>::NVOA]) {
  double F[N];
  row_gather<N>(f_l, F);
  double sacc = 0.0;
#pragma unroll
  for (int j = 0; j < N; ++j) sacc = fma(hr[j], F[j], sacc);
  xu0_l = -sacc;
#pragma unroll
  for (int c = 0; c < RowMap<N, NVO>::NVOA; ++c) U_l[c] = 0.0;
#pragma unroll
  for (int c = 0; c < NVO; ++c) {
    double Gc[N];
    row_gather<N>(Gl[c], Gc);
    double u = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) u = fma(hr[j], Gc[j], u);
    U_l[c] = u;
  }
}

template <int N, int NU, int NVO, class WS>
__device__ __forceinline__ void row_jmap_build(const RowQp<N, NU>& q, const double* t, int l, int rowbase,
                                               const WS& W,
                                               double xu0_l, const double (&U_l)[RowMap<N, NVO>::NVOA],
                                               RowMap<N, NVO>& mp) {
  double rhs[N];
#pragma unroll
  for (int a = 0; a < N; ++a) rhs[a] = (a < W.K) ? wset_beta(q, W, a) - nval<N, NU>(xu0_l, rowbase, W.j[a], W.side[a]) : 0.0;
  ldl_solve_k<N>(W.K, W.L, W.R, rhs, mp.lam0);
#pragma unroll
  for (int c = 0; c < NVO; ++c) {
    double lc[N];
#pragma unroll
    for (int a = 0; a < N; ++a) rhs[a] = (a < W.K) ? nval<N, NU>(U_l[c], rowbase, W.j[a], W.side[a]) : 0.0;
    ldl_solve_k<N>(W.K, W.L, W.R, rhs, lc);
#pragma unroll
    for (int a = 0; a < N; ++a) mp.Lam[a][c] = lc[a];
  }
  mp.x0_l = xu0_l;
#pragma unroll
  for (int c = 0; c < NVO; ++c) mp.X_l[c] = -U_l[c];
#pragma unroll
  for (int a = 0; a < N; ++a) {
    if (a < W.K) {
      const double h = hval<N, NU>(t, l, W.j[a], W.side[a]);
      mp.x0_l = fma(mp.lam0[a], h, mp.x0_l);
#pragma unroll
      for (int c = 0; c < NVO; ++c) mp.X_l[c] = fma(mp.Lam[a][c], h, mp.X_l[c]);
    }
  }
}

// qp_solve_map for the row's QP (xu0_l, U_l from row_jmap_terms; d the
// other plans, replicated); mp persists across the QP's iterations
template <bool TRACE, int N, int NU, int NVO, bool LDSL = false>
__device__ __forceinline__ void qp_solve_row_map(const RowQp<N, NU>& q, const double* t, const RowScan& sc, int l,
                                                 bool pd, double tol_d, double xu0_l,
                                                 const double (&U_l)[RowMap<N, NVO>::NVOA],
                                                 const double (&d)[RowMap<N, NVO>::NVOA], uint32_t ws_in,
                                                 int max_chg, double& x_l, QpOut& o, RowMap<N, NVO>& mp,
                                                 double* lsh = nullptr) {
  const int rowbase = (int)(__lane_id() & ~15u);
  RowWSet<N, LDSL> W;
  if constexpr (LDSL) W.L.p = lsh;
  o.status = CMPC_QP_OK;
  o.nchg = 0;
  o.ntrace = 0;
  o.tr[0] = o.tr[1] = o.tr[2] = o.tr[3] = 0xFFFFFFFFu;
  int chg = 0;
  bool done = false, have_w = false;
  if (!pd) {
    o.status = CMPC_QP_NOT_PD;
    done = true;
    W.K = 0;
    have_w = true;
    mp.ws = kWsInvalid;
  } else if (ws_in != mp.ws) {
    wset_fill(q, ws_in, W);
    if (W.K > 0 && !wset_factor_row<N, NU>(t, l, rowbase, W)) {  // inconsistent warm start: cold
      W.K = 0;
      ++chg;
    }
    have_w = true;
    row_jmap_build<N, NU, NVO>(q, t, l, rowbase, W, xu0_l, U_l, mp);
    mp.K = W.K;
    mp.wc = wset_word(W);
    mp.ws = chg ? kWsInvalid : ws_in;
  }
  double lam[N];
  int worst = -1;
  {
    double wv = -tol_d;
#pragma unroll
    for (int a = 0; a < N; ++a) {
      double v = mp.lam0[a];
#pragma unroll
      for (int c = 0; c < NVO; ++c) v = fma(mp.Lam[a][c], d[c], v);
      lam[a] = v;
      if (a < mp.K && v < wv) {
        wv = v;
        worst = a;
      }
    }
  }
  if (done) worst = -1;
  const bool stay = !done && worst < 0;
  x_l = 0.0;
  if (stay) {
    double v = mp.x0_l;
#pragma unroll
    for (int c = 0; c < NVO; ++c) v = fma(mp.X_l[c], d[c], v);
    x_l = v;
    int ps = 0;
    if (row_scan<N, NU>(x_l, sc, mp.wc, l, rowbase, ps) < 0) {  // nothing violated: done
      o.nchg = chg;
      o.ws = mp.wc;
      const unsigned long long bad = __ballot(l < N && !__builtin_isfinite(x_l));
      if ((bad >> rowbase) & 0xFFFFull) o.status = CMPC_QP_NONFINITE;
      if (o.status == CMPC_QP_OK) {
        if (l < N && ((mp.wc >> l) & 1u)) x_l = ((mp.wc >> (16 + l)) & 1u) ? q.ubv(l) : q.lbv(l);
      } else {
        x_l = 0.0;
      }
      return;
    }
  }
  if (!have_w) {
    wset_fill(q, ws_in, W);
    wset_factor_row<N, NU>(t, l, rowbase, W);  // (succeeded when the map was built)
  }
#pragma unroll
  for (int a = 0; a < N; ++a) W.lam[a] = lam[a];
  if (!done && !stay) {
    double xu_l = xu0_l;
#pragma unroll
    for (int c = 0; c < NVO; ++c) xu_l = fma(-U_l[c], d[c], xu_l);
    for (int it = 0; it <= N && !done; ++it) {
      if (it > 0) {
        double rhs[N];
#pragma unroll
        for (int a = 0; a < N; ++a)
          rhs[a] = (a < W.K) ? wset_beta(q, W, a) - nval<N, NU>(xu_l, rowbase, W.j[a], W.side[a]) : 0.0;
        ldl_solve_k<N>(W.K, W.L, W.R, rhs, W.lam);
        worst = -1;
        double wv = -tol_d;
#pragma unroll
        for (int a = 0; a < N; ++a)
          if (a < W.K && W.lam[a] < wv) {
            wv = W.lam[a];
            worst = a;
          }
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
      if (++chg > max_chg) {
        o.status = CMPC_QP_MAX_NWSR;
        done = true;
      }
    }
    if (!done) {
      x_l = xu_l;
#pragma unroll
      for (int a = 0; a < N; ++a)
        if (a < W.K) x_l = fma(W.lam[a], hval<N, NU>(t, l, W.j[a], W.side[a]), x_l);
    }
  }
  qp_row_phase_b<TRACE, N, NU>(q, t, sc, l, rowbase, W, x_l, chg, done, max_chg, o);
}
