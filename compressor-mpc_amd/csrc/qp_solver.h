// Warm-started dual (Goldfarb–Idnani) active-set QP solver, one QP per
// thread.  Same specification and arithmetic order as oracle/or_qp.c (see
// DESIGN.md §QP).  Header-only and __host__ __device__ so that a CPU test
// harness (tests/cpp/qp_host.cpp) can diff this exact code against the
// oracle; the product only instantiates it inside the HIP kernels.
#pragma once
#include <math.h>
#include <stdint.h>

#include "../../include/cmpc.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define CMPC_HD __host__ __device__ __forceinline__
#else
#define CMPC_HD inline
#endif

// ---------------------------------------------------------------------------
// Warm-started dual active-set QP solver (lane per QP).  Same specification
// and arithmetic order as oracle/or_qp.c (version 4: every accumulation
// c +- a b is one fma, here and in the oracle); see DESIGN.md §4.
// ---------------------------------------------------------------------------
#ifndef CMPC_QP_ABL
#define CMPC_QP_ABL 0  // timing-only ablations (results invalid): 1 no phase B, 2 no phase A solve
#endif
#define TOL_P 1e-12
#define TOL_D 1e-12
#define TOL_R 1e-12
#define TOL_Z 1e-12

template <int N>
CMPC_HD double sel(const double (&v)[N], int i) {
  double r = 0.0;
#pragma unroll
  for (int t = 0; t < N; ++t) r = (i == t) ? v[t] : r;
  return r;
}

// Storage of H^-1: registers (default) or a per-lane column of a
// lane-contiguous LDS array (the solve kernel, to keep 2 waves/SIMD).
template <int N>
struct HinvRegs {
  static constexpr bool kColumns = false;  // H^-1 nu by the explicit normal (register-indexed)
  double m[N][N];
  CMPC_HD double operator()(int r, int c) const { return m[r][c]; }
  CMPC_HD void set(int r, int c, double v) { m[r][c] = v; }
};
// the upper triangle in a lane-contiguous LDS array (entry (r, c), r <= c,
// at p[(r * N + c) * STRIDE]), read mirrored: the iterate kernel's map form
// needs H^-1 only to build a map and off the common path
template <int N, int STRIDE>
struct HinvStrided {
  static constexpr bool kColumns = true;  // H^-1 nu by column reads (runtime addresses)
  static constexpr int kStride = STRIDE;
  double* p;
  CMPC_HD double operator()(int r, int c) const { return r <= c ? p[(r * N + c) * STRIDE] : p[(c * N + r) * STRIDE]; }
  CMPC_HD void set(int r, int c, double v) {
    if (r <= c) p[(r * N + c) * STRIDE] = v;
  }
};

// x_u0 = -H^-1 f of the map form in the strictly lower triangle that
// HinvStrided leaves unused (entry r in the r-th slot (i, j), i > j, in row
// order; N >= 3): read only to build a map and to leave one, so it holds no
// registers across the Jacobi iterations
template <int N, int STRIDE>
struct XuStrided {
  static_assert(N >= 3, "needs N lower-triangle slots");
  double* p;
  static constexpr CMPC_HD int slot(int r) {
    int n = 0;
    for (int i = 1; i < N; ++i)
      for (int j = 0; j < i; ++j) {
        if (n == r) return i * N + j;
        ++n;
      }
    return -1;
  }
  CMPC_HD double operator[](int r) const { return p[slot(r) * STRIDE]; }
  CMPC_HD void set(int r, double v) { p[slot(r) * STRIDE] = v; }
};

// NB = stored bound entries: N (general), or NU when the bounds repeat every
// NU entries (the MPC QP: rep_m(lower - u_old), rep_m(rate bounds),
// libs/mpc_qp_solver.cc:53-60), which halves their registers.
template <int N, int NU, int NB = N, class HS = HinvRegs<N>>
struct Qp {
  static_assert(NB == N || NB == NU, "bounds: general or NU-periodic");
  using HS_t = HS;
  HS Hinv;
  double lb[NB], ub[NB], lbA[NB], ubA[NB];
  // phase-B violation thresholds -TOL_P (1 + |beta|) per bound and side,
  // formed where they are compared (registers: the iterate kernel's map form
  // keeps its map beside the bounds)
  CMPC_HD void tolerances() {}
  CMPC_HD double thr(int j, int side) const { return -TOL_P * (1.0 + fabs(beta(j, side))); }
  CMPC_HD double lbv(int j) const { return sel<NB>(lb, j % NB); }
  CMPC_HD double ubv(int j) const { return sel<NB>(ub, j % NB); }

  // nu_{j,side}' v for a compile-time j (the phase-B scan; sel folds away)
  CMPC_HD double nu_dot(int j, int side, const double (&v)[N]) const {
    double t;
    if (j < N) {
      t = sel<N>(v, j);
    } else {
      const int i = j - N;
      t = (i >= NU) ? sel<N>(v, i) - sel<N>(v, i - NU) : sel<N>(v, i);
    }
    return side ? -t : t;
  }
  CMPC_HD double beta(int j, int side) const {
    if (j < N) return side ? -sel<NB>(ub, j % NB) : sel<NB>(lb, j % NB);
    return side ? -sel<NB>(ubA, (j - N) % NB) : sel<NB>(lbA, (j - N) % NB);
  }
  // Normal of constraint (j, side) as an explicit vector (entries 0, +-1):
  // bound j < N: +-e_j; rate row i = j - N: +-(e_i - e_{i-NU}) for i >= NU,
  // +-e_i otherwise.  Products with it are exact, and every sum below has at
  // most two nonzero terms accumulated in ascending column order, so ndot /
  // hinv_n round exactly like the oracle's nu_dot / hinv_nu
  // (round(v_i - v_{i-NU}), negated for the upper side).
  CMPC_HD void normal(int j, int side, double (&n)[N]) const {
    const double sg = side ? -1.0 : 1.0;
    const bool rate = j >= N;
    const int i = rate ? j - N : j;
#pragma unroll
    for (int c = 0; c < N; ++c)
      n[c] = (c == i) ? sg : ((rate && i >= NU && c == i - NU) ? -sg : 0.0);
  }
  // out = Hinv nu_{j,side} by columns (or_qp.c hinv_nu: a column, or a
  // difference of two columns, negated for the upper side); the same values
  // as hinv_n on the explicit normal
  CMPC_HD void hcol(int j, int side, double (&out)[N]) const {
    const bool rate = j >= N;
    const int i = rate ? j - N : j;
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double t = Hinv(r, i);
      if (rate && i >= NU) t = t - Hinv(r, i - NU);
      out[r] = side ? -t : t;
    }
  }
  // out = Hinv n
  CMPC_HD void hinv_n(const double (&n)[N], double (&out)[N]) const {
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double t = 0.0;
#pragma unroll
      for (int c = 0; c < N; ++c) t = fma(Hinv(r, c), n[c], t);
      out[r] = t;
    }
  }
};

// n' v (n an explicit constraint normal; exact as noted at Qp::normal)
template <int N>
CMPC_HD double ndot(const double (&n)[N], const double (&v)[N]) {
  double t = 0.0;
#pragma unroll
  for (int c = 0; c < N; ++c) t = fma(n[c], v[c], t);
  return t;
}

// Working set: slots 0..K-1 in the specification's order (ascending j from
// the warm start, phase-B additions appended), each with its normal, bound
// beta and multiplier, and the LDL' factor of M = N' Hinv N with reciprocal
// pivots R = 1/D (oracle/or_qp.c, spec version 2).  h_a = Hinv * normal_a is
// recomputed where it is used (registers: the solve kernel runs at 2
// waves/SIMD).
// SN (store normals): the explicit normal vectors are kept per slot (N <= 6);
// for larger N they are rebuilt from (j, side) where they are used
// (Qp::normal, the same vector bit for bit), which frees 2 N^2 registers per
// working set: the centralized nV = 8 solve then needs no scratch.
#ifndef CMPC_WSET_STORE_MAX
#define CMPC_WSET_STORE_MAX 0  // largest N whose working sets store their normals and bounds
#endif
// LS: storage of the factor L, indexed L[i][k]: registers (a plain array), or
// an LDS matrix (qp_solver_row.h LdsMat, the fused row solver's registers)
template <int N, bool SN = (N <= CMPC_WSET_STORE_MAX), class LS = double[N][N]>
struct WSet {
  int K;
  int j[N], side[N];
  double lam[N];
  double nrm[SN ? N : 1][N], bta[SN ? N : 1];  // normals and bounds (SN) or rebuilt from (j, side)
  LS L;
  double D[N], R[N];
};

// the normal of slot a (stored, or rebuilt from its constraint index)
template <int N, bool SN, class LS, class Q>
CMPC_HD void wset_normal(const Q& q, const WSet<N, SN, LS>& W, int a, double (&n)[N]) {
  if constexpr (SN) {
#pragma unroll
    for (int c = 0; c < N; ++c) n[c] = W.nrm[a][c];
  } else {
    q.normal(W.j[a], W.side[a], n);
  }
}

// the bound beta of slot a (stored, or from its constraint index)
template <int N, bool SN, class LS, class Q>
CMPC_HD double wset_beta(const Q& q, const WSet<N, SN, LS>& W, int a) {
  if constexpr (SN) return W.bta[a];
  else return q.beta(W.j[a], W.side[a]);
}

// H^-1 n_a of slot a: columns of an LDS-resident H^-1 (runtime addresses),
// else the explicit normal's product (registers take compile-time indices)
template <int N, bool SN, class LS, class Q>
CMPC_HD void wset_h(const Q& q, const WSet<N, SN, LS>& W, int a, double (&out)[N]) {
  if constexpr (Q::HS_t::kColumns) {
    q.hcol(W.j[a], W.side[a], out);
  } else {
    double n[N];
    wset_normal(q, W, a, n);
    q.hinv_n(n, out);
  }
}
// n_a' v of slot a (the explicit normal's FMAs: fewer instructions than
// selecting v's entries by the runtime constraint index)
template <int N, bool SN, class LS, class Q>
CMPC_HD double wset_dot(const Q& q, const WSet<N, SN, LS>& W, int a, const double (&v)[N]) {
  double n[N];
  wset_normal(q, W, a, n);
  return ndot<N>(n, v);
}
// H^-1 nu_{j,side}
template <int N, class Q>
CMPC_HD void q_h(const Q& q, int j, int side, double (&out)[N]) {
  if constexpr (Q::HS_t::kColumns) {
    q.hcol(j, side, out);
  } else {
    double n[N];
    q.normal(j, side, n);
    q.hinv_n(n, out);
  }
}

// LDL' of the leading K x K block of M (lower triangle read) with reciprocal
// pivots R = 1/D (or_qp.c ldl); returns false unless every pivot
// d_j > rel * M_jj (rel = 0: H positive definite; TOL_Z: a working set with
// independent normals).
template <int N, class LM>
CMPC_HD bool ldl_k(int K, const double (&M)[N][N], LM& L, double (&D)[N],
                   double (&R)[N], double rel = 0.0) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (j < K) {
      double d = M[j][j];
#pragma unroll
      for (int k = 0; k < j; ++k) d = fma(-(L[j][k] * L[j][k]), D[k], d);
      ok = ok && (d > rel * M[j][j]);
      D[j] = d;
      const double r = 1.0 / d;
      R[j] = r;
      L[j][j] = 1.0;
#pragma unroll
      for (int i = j + 1; i < N; ++i) {
        if (i < K) {
          double sacc = M[i][j];
#pragma unroll
          for (int k = 0; k < j; ++k) sacc = fma(-(L[i][k] * L[j][k]), D[k], sacc);
          L[i][j] = sacc * r;
        }
      }
    }
  }
  return ok;
}

// x = (L D L')^-1 b on the leading K entries, with the scaled forward vector
// zz = D^-1 L^-1 b (or_qp.c ldl_solve); entries from K on are zero.  Each
// forward step is one block under `i < K`, so a wave skips the steps past the
// largest working set among its lanes; every computed entry has the
// arithmetic of the plain loops, bit for bit.
template <int N, class LM>
CMPC_HD void ldl_solve_k(int K, const LM& L, const double (&R)[N],
                         const double (&b)[N], double (&x)[N], double (&zz)[N]) {
  double y[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    y[i] = 0.0;
    zz[i] = 0.0;
    if (i < K) {
      double v = b[i];
#pragma unroll
      for (int k = 0; k < i; ++k) v = fma(-L[i][k], y[k], v);
      y[i] = v;
      zz[i] = v * R[i];
    }
  }
#pragma unroll
  for (int i = N - 1; i >= 0; --i) {
    if (i < K) {
      double v = zz[i];
#pragma unroll
      for (int k = i + 1; k < N; ++k)
        if (k < K) v = fma(-L[k][i], x[k], v);
      x[i] = v;
    } else {
      x[i] = 0.0;
    }
  }
}
template <int N, class LM>
CMPC_HD void ldl_solve_k(int K, const LM& L, const double (&R)[N],
                         const double (&b)[N], double (&x)[N]) {
  double zz[N];
  ldl_solve_k<N>(K, L, R, b, x, zz);
}

// warm start: M (M[i][k] = n_k' Hinv n_i, k <= i) of the current slots and
// its LDL' (or_qp.c wset_factor)
template <int N, bool SN, class LS, class Q>
CMPC_HD bool wset_factor(const Q& q, WSet<N, SN, LS>& W) {
  double M[N][N];
#pragma unroll
  for (int b = 0; b < N; ++b) {
    double hb[N];
    if (b < W.K) wset_h(q, W, b, hb);
#pragma unroll
    for (int a = 0; a <= b; ++a) {
      double v = 0.0;
      if (b < W.K) {
        double na[N];
        wset_normal(q, W, a, na);
        v = ndot<N>(na, hb);
      }
      M[b][a] = v;
    }
  }
  return ldl_k<N>(W.K, M, W.L, W.D, W.R, TOL_Z);
}

// remove slot a (or_qp.c wset_remove): the other slots keep their order; the
// trailing block of the factor takes the rank-one term D_a w w' (GGMS method
// C1, reciprocal pivots), then rows and columns after a move up by one
template <int N, bool SN, class LS>
CMPC_HD void wset_drop(WSet<N, SN, LS>& W, int a) {
  double w[N];
  double alpha = 0.0;
#pragma unroll
  for (int c = 0; c < N; ++c)
    if (c == a) alpha = W.D[c];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double v = 0.0;
#pragma unroll
    for (int c = 0; c < i; ++c)
      if (c == a) v = W.L[i][c];
    w[i] = v;
  }
#pragma unroll
  for (int j = 1; j < N; ++j) {
    if (j > a && j < W.K) {
      const double p = w[j];
      const double t = alpha * p;
      const double d = fma(t, p, W.D[j]);
      const double r = 1.0 / d;
      const double bt = t * r;
      alpha = alpha * (W.D[j] * r);
      W.D[j] = d;
      W.R[j] = r;
#pragma unroll
      for (int i = j + 1; i < N; ++i)
        if (i < W.K) {
          w[i] = fma(-p, W.L[i][j], w[i]);
          W.L[i][j] = fma(bt, w[i], W.L[i][j]);
        }
    }
  }
#pragma unroll
  for (int i = 0; i + 1 < N; ++i)
    if (i >= a && i + 1 < W.K) {
      W.j[i] = W.j[i + 1];
      W.side[i] = W.side[i + 1];
      W.lam[i] = W.lam[i + 1];
      if constexpr (SN) W.bta[i] = W.bta[i + 1];
      W.D[i] = W.D[i + 1];
      W.R[i] = W.R[i + 1];
      if constexpr (SN) {
#pragma unroll
        for (int c = 0; c < N; ++c) W.nrm[i][c] = W.nrm[i + 1][c];
      }
#pragma unroll
      for (int k = 0; k < i; ++k) W.L[i][k] = (k < a) ? W.L[i + 1][k] : W.L[i + 1][k + 1];
      W.L[i][i] = 1.0;
    }
  W.K--;
}

// append (j, side) as slot K (or_qp.c wset_append): the bordered factor's
// row zz = D^-1 L^-1 qv and pivot zn (= den - qv' M^-1 qv), R = 1/zn
template <int N, bool SN, class LS>
CMPC_HD void wset_add(WSet<N, SN, LS>& W, int j, int side, double lam, const double (&n)[N], double bta,
                      const double (&zz)[N], double zn, double rzn) {
#pragma unroll
  for (int b = 0; b < N; ++b)
    if (b == W.K) {
      W.j[b] = j;
      W.side[b] = side;
      W.lam[b] = lam;
      if constexpr (SN) W.bta[b] = bta;
      if constexpr (SN) {
#pragma unroll
        for (int c = 0; c < N; ++c) W.nrm[b][c] = n[c];
      }
#pragma unroll
      for (int k = 0; k < b; ++k) W.L[b][k] = zz[k];
      W.L[b][b] = 1.0;
      W.D[b] = zn;
      W.R[b] = rzn;
    }
  W.K++;
}

struct QpOut {
  int status, nchg, ntrace;
  uint32_t ws;
  uint32_t tr[4];  // 16 trace bytes
};

CMPC_HD void trace_push(QpOut& o, int add, int j, int side) {
  if (o.ntrace < 16) {
    const uint32_t byte = (add ? 0x80u : 0u) | (side ? 0x40u : 0u) | (uint32_t)j;
    const int w = o.ntrace >> 2, sh = (o.ntrace & 3) * 8;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (t == w) o.tr[t] = (o.tr[t] & ~(0xFFu << sh)) | (byte << sh);
    o.ntrace++;
  }
}

// Hinv = H^-1 via LDL' with reciprocal pivots (oracle/or_qp.c step 0).
// Returns false if not PD.
template <int N, class HS>
CMPC_HD bool hinv_of(const double (&H)[N][N], HS& Hinv) {
  double L[N][N], D[N], R[N];
  if (!ldl_k<N>(N, H, L, D, R)) return false;
#pragma unroll
  for (int c = 0; c < N; ++c) {
    double e[N], colv[N];
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = (i == c) ? 1.0 : 0.0;
    ldl_solve_k<N>(N, L, R, e, colv);
#pragma unroll
    for (int i = 0; i <= c; ++i) Hinv.set(i, c, colv[i]);
  }
#pragma unroll
  for (int c = 0; c < N; ++c)
#pragma unroll
    for (int i = 0; i < c; ++i) Hinv.set(c, i, Hinv(i, c));
  return true;
}

// TRACE = false: the working-set change trace (QpOut::tr, ntrace) is not
// recorded (the iterate kernel without CMPC_TRACE); everything else is equal.
constexpr uint32_t kWsInvalid = 0xFFFFFFFFu;

// the warm start's slots: the constraints of ws_in in ascending j
template <int N, bool SN, class LS, class Q>
CMPC_HD void wset_fill(const Q& q, uint32_t ws_in, WSet<N, SN, LS>& W) {
  W.K = 0;
  uint32_t msk = ws_in & ((1u << (2 * N)) - 1u);
#pragma unroll
  for (int a = 0; a < N; ++a) {
    W.j[a] = 0;
    W.side[a] = 0;
    W.lam[a] = 0.0;
    if (msk) {
      const int j = __builtin_ctz(msk);
      msk &= msk - 1u;
      const int sd = (ws_in >> (16 + j)) & 1u;
      W.j[a] = j;
      W.side[a] = sd;
      if constexpr (SN) q.normal(j, sd, W.nrm[a]);
      if constexpr (SN) W.bta[a] = q.beta(j, sd);
      W.K = a + 1;
    }
  }
}

template <bool TRACE, int N, int NU, int NB, class HS, bool SN, class LS>
CMPC_HD void qp_phase_b(const Qp<N, NU, NB, HS>& q, WSet<N, SN, LS>& W, double (&x)[N], int chg, bool done,
                        int max_chg, QpOut& o);

// The plain solve (standalone QPs, InitializeQPProblem, the coupled
// iteration): g given, the map form with nvo = 0 (or_qp.c).
template <bool TRACE, int N, int NU, int NB, class HS>
CMPC_HD void qp_solve_t(const Qp<N, NU, NB, HS>& q, bool pd, double tol_d, const double (&g)[N],
                         uint32_t ws_in, int max_chg, double (&x)[N], QpOut& o) {
  WSet<N> W;
  o.status = CMPC_QP_OK;
  o.nchg = 0;
  o.ntrace = 0;
  o.tr[0] = o.tr[1] = o.tr[2] = o.tr[3] = 0xFFFFFFFFu;
  int chg = 0;
  bool done = false;
  double xu[N];
  if (!pd) {
    o.status = CMPC_QP_NOT_PD;
    done = true;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double sacc = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) sacc = fma(q.Hinv(i, j), g[j], sacc);
    xu[i] = -sacc;
  }
  // A. warm start: slot a = the a-th active constraint of ws_in in ascending
  // j (the oracle adds them in that order while K < n), then the full factor
  wset_fill(q, done ? 0u : ws_in, W);
  if (W.K > 0 && !wset_factor<N>(q, W)) {  // inconsistent warm start: cold
    W.K = 0;
    ++chg;
  }
  for (int it = 0; it <= N && !done; ++it) {
    double rhs[N];
#pragma unroll
    for (int a = 0; a < N; ++a) {
      rhs[a] = 0.0;
      if (a < W.K) {
        rhs[a] = wset_beta(q, W, a) - wset_dot(q, W, a, xu);
      }
    }
    ldl_solve_k<N>(W.K, W.L, W.R, rhs, W.lam);
    if (CMPC_QP_ABL == 2) break;
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
  if (!done) {
    // x = xu + sum_a lam_a h_a (per r, a ascending as the oracle)
#pragma unroll
    for (int r = 0; r < N; ++r) x[r] = xu[r];
#pragma unroll
    for (int a = 0; a < N; ++a) {
      if (a < W.K) {
        double ha[N];
        wset_h(q, W, a, ha);
#pragma unroll
        for (int r = 0; r < N; ++r) x[r] = fma(W.lam[a], ha[r], x[r]);
      }
    }
  }
  qp_phase_b<TRACE>(q, W, x, chg, done, max_chg, o);
}

// Phase B (Goldfarb–Idnani) from the phase-A point x and multipliers W.lam,
// then the result: working-set word, finite check, bound fixing / zero move.
template <bool TRACE, int N, int NU, int NB, class HS, bool SN, class LS>
CMPC_HD void qp_phase_b(const Qp<N, NU, NB, HS>& q, WSet<N, SN, LS>& W, double (&x)[N], int chg, bool done,
                        int max_chg, QpOut& o) {
  // B. Goldfarb–Idnani
  for (int outer = 0; outer <= max_chg + 1 && !done && CMPC_QP_ABL != 1; ++outer) {
    int pj = -1, ps = 0;
    double pv = 0.0;
    // any violated candidate at all (the compares feed one lane mask, no
    // per-candidate VALU bookkeeping): in most scans there is none, and the
    // ordered selection below (the most violated inactive constraint, first
    // in (j, side) order on ties) is skipped.  An active constraint whose
    // slack rounds below the threshold only sends the lane to the selection,
    // which excludes it as before.
    bool anyv = false;
#pragma unroll
    for (int j = 0; j < 2 * N; ++j)
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) anyv = anyv | (q.nu_dot(j, sd, x) - q.beta(j, sd) < q.thr(j, sd));
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
            const double sl = q.nu_dot(j, sd, x) - q.beta(j, sd);
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
    const double bp = q.beta(pj, ps);
    double up = 0.0;
    for (int inner = 0; inner <= max_chg + 1 && !done; ++inner) {
      double hp[N], qv[N], rv[N], zz[N], z[N];
      q_h<N>(q, pj, ps, hp);
#pragma unroll
      for (int a = 0; a < N; ++a) {
        qv[a] = 0.0;
        if (a < W.K) {
          qv[a] = wset_dot(q, W, a, hp);
        }
      }
      ldl_solve_k<N>(W.K, W.L, W.R, qv, rv, zz);
#pragma unroll
      for (int r = 0; r < N; ++r) z[r] = hp[r];
#pragma unroll
      for (int a = 0; a < N; ++a) {
        if (a < W.K) {
          double ha[N];
          wset_h(q, W, a, ha);
#pragma unroll
          for (int r = 0; r < N; ++r) z[r] = fma(-rv[a], ha[r], z[r]);
        }
      }
      const double zn = q.nu_dot(pj, ps, z);
      const double den = q.nu_dot(pj, ps, hp);
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
      const double sl = q.nu_dot(pj, ps, x) - bp;
      const double t2 = -sl * rzn;
      const bool full = (k < 0) || (t2 <= t1);
      const double t = full ? t2 : t1;
#pragma unroll
      for (int r = 0; r < N; ++r) x[r] = fma(t, z[r], x[r]);
#pragma unroll
      for (int a = 0; a < N; ++a)
        if (a < W.K) W.lam[a] = fma(-t, rv[a], W.lam[a]);
      up = up + t;
      if (full) {
        if (TRACE) trace_push(o, 1, pj, ps);
        double np_[N];
        if constexpr (SN) q.normal(pj, ps, np_);
        wset_add<N>(W, pj, ps, up, np_, bp, zz, zn, rzn);
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
  // a non-finite plan (a NaN or infinite gradient) fails like any other
  // non-success: zero move (or_qp.c; checked before the bound fixing)
  if (o.status == CMPC_QP_OK) {
    bool fin = true;
#pragma unroll
    for (int r = 0; r < N; ++r) fin = fin && __builtin_isfinite(x[r]);
    if (!fin) o.status = CMPC_QP_NONFINITE;
  }
  if (o.status == CMPC_QP_OK) {
    // variables at an active bound are fixed exactly at it; the bound
    // constraints are bits j < N of the working-set word (side at 16 + j),
    // each j at most once, so per variable one select instead of a loop over
    // the slots' runtime indices
    const uint32_t bnd = w & ((1u << N) - 1u), up = (w >> 16) & bnd;
#pragma unroll
    for (int r = 0; r < N; ++r)
      x[r] = ((bnd >> r) & 1u) ? (((up >> r) & 1u) ? q.ubv(r) : q.lbv(r)) : x[r];
  } else {
#pragma unroll
    for (int r = 0; r < N; ++r) x[r] = 0.0;
  }
}

// ---------------------------------------------------------------------------
// Map form of the Jacobi iterations (or_qp.c step A, version 3).  Within one
// control step a QP keeps H, f and G = Su'W Su_other; only the other
// sub-controllers' plans d change between its K solves.  For a working set W
// the multipliers and the point are affine in d:
//   lam = lam0 + Lam d,  x = x0 + X d  (x_u0 = -Hinv f, U = Hinv G,
//   lam0 = M^-1 (beta_W - N' x_u0), Lam = M^-1 N' U, x0 = x_u0 + H_W lam0,
//   X = -U + H_W Lam),
// so an iteration whose working set is the one of the map costs two small
// products.  The map is a deterministic function of (H, f, G, bounds, W):
// JMap keeps the last one built (ws = its working-set word) across the
// iterations, and a rebuilt map equals a kept one bit for bit.
// ---------------------------------------------------------------------------
template <int N, int NVO>
struct JMap {
  static constexpr int NVOA = NVO > 0 ? NVO : 1;
  uint32_t ws;   // the ws_in the map was built for, kWsInvalid: none
  uint32_t wc;   // the working-set word of its slots
  int K;         // its slot count
  double lam0[N], Lam[N][NVOA], x0[N], X[N][NVOA];
};

// U = Hinv G in registers, or in the lane's column of an LDS array
// (element (r, c) at p[(r * NVOA + c) * STRIDE])
template <int N, int NVOA>
struct URegs {
  const double (&U)[N][NVOA];
  CMPC_HD double operator()(int r, int c) const { return U[r][c]; }
};
template <int NVOA, int STRIDE>
struct UStrided {
  const double* p;
  CMPC_HD double operator()(int r, int c) const { return p[(r * NVOA + c) * STRIDE]; }
};

// the map of the WSet's slots (fresh warm-start factor).  Each slot's
// explicit normal is formed once and serves all 1 + NVO right-hand sides
// (N' x_u0 and N' U's columns: FMAs with 0 / +-1 coefficients, exact, the
// oracle's nu_dot values).
template <int N, int NVO, int NU, int NB, class HS, bool SN, class LS, class XU, class UA>
CMPC_HD void jmap_build(const Qp<N, NU, NB, HS>& q, const WSet<N, SN, LS>& W, const XU& xu0v,
                        const UA& U, JMap<N, NVO>& mp) {
  double xu0[N];  // (an array, or XuStrided in LDS)
#pragma unroll
  for (int r = 0; r < N; ++r) xu0[r] = xu0v[r];
  constexpr int NVOA = JMap<N, NVO>::NVOA;
  double rhs0[N], rc[NVOA][N];
#pragma unroll
  for (int a = 0; a < N; ++a) {
    rhs0[a] = 0.0;
#pragma unroll
    for (int c = 0; c < NVOA; ++c) rc[c][a] = 0.0;
    if (a < W.K) {
      double na[N];
      wset_normal(q, W, a, na);
      rhs0[a] = wset_beta(q, W, a) - ndot<N>(na, xu0);
#pragma unroll
      for (int c = 0; c < NVO; ++c) {
        double uc[N];
#pragma unroll
        for (int r = 0; r < N; ++r) uc[r] = U(r, c);
        rc[c][a] = ndot<N>(na, uc);
      }
    }
  }
  ldl_solve_k<N>(W.K, W.L, W.R, rhs0, mp.lam0);
#pragma unroll
  for (int c = 0; c < NVO; ++c) {
    double lc[N];
    ldl_solve_k<N>(W.K, W.L, W.R, rc[c], lc);
#pragma unroll
    for (int a = 0; a < N; ++a) mp.Lam[a][c] = lc[a];  // zero from K on
  }
#pragma unroll
  for (int r = 0; r < N; ++r) {
    mp.x0[r] = xu0[r];
#pragma unroll
    for (int c = 0; c < NVO; ++c) mp.X[r][c] = -U(r, c);
  }
#pragma unroll
  for (int a = 0; a < N; ++a) {
    if (a < W.K) {
      double ha[N];
      wset_h(q, W, a, ha);
#pragma unroll
      for (int r = 0; r < N; ++r) {
        mp.x0[r] = fma(mp.lam0[a], ha[r], mp.x0[r]);
#pragma unroll
        for (int c = 0; c < NVO; ++c) mp.X[r][c] = fma(mp.Lam[a][c], ha[r], mp.X[r][c]);
      }
    }
  }
}

// the working-set word of the first K slots
template <int N, bool SN, class LS>
CMPC_HD uint32_t wset_word(const WSet<N, SN, LS>& W) {
  uint32_t w = 0;
#pragma unroll
  for (int a = 0; a < N; ++a)
    if (a < W.K) w |= (1u << W.j[a]) | ((uint32_t)W.side[a] << (16 + W.j[a]));
  return w;
}

// One Jacobi-iteration solve in the map form: xu0 = -Hinv f and U = Hinv G
// of the step's QP, d the other plans; mp persists across the QP's
// iterations (mp.ws = kWsInvalid before the first).  A solve on the map's
// working set that stays on it (no multiplier below -tol_d, no violated
// constraint) touches only the map; otherwise the working set and its fresh
// factor are rebuilt from ws_in (the same values as when the map was built)
// and the solve continues as the plain one.
template <bool TRACE, int N, int NVO, int NU, int NB, class HS, class XU, class UA>
CMPC_HD void qp_solve_map(const Qp<N, NU, NB, HS>& q, bool pd, double tol_d, const XU& xu0,
                          const UA& U, const double (&d)[JMap<N, NVO>::NVOA], uint32_t ws_in, int max_chg,
                          double (&x)[N], QpOut& o, JMap<N, NVO>& mp) {
  WSet<N> W;
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
    // the warm start (slots, full factor) and its map
    wset_fill(q, ws_in, W);
    if (W.K > 0 && !wset_factor<N>(q, W)) {  // inconsistent warm start: cold
      W.K = 0;
      ++chg;
    }
    have_w = true;
    jmap_build<N, NVO>(q, W, xu0, U, mp);
    mp.K = W.K;
    mp.wc = wset_word(W);
    mp.ws = chg ? kWsInvalid : ws_in;  // (a failed warm start is redone)
  }
  // A. lam = lam0 + Lam d (entries from K on are zero)
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
  bool stay = !done && worst < 0;
  if (stay) {
    // x = x0 + X d, then the phase-B scan: nothing violated -> done here
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double v = mp.x0[r];
#pragma unroll
      for (int c = 0; c < NVO; ++c) v = fma(mp.X[r][c], d[c], v);
      x[r] = v;
    }
    bool anyv = false;
#pragma unroll
    for (int j = 0; j < 2 * N; ++j)
#pragma unroll
      for (int sd = 0; sd < 2; ++sd)
        anyv = anyv | (!((mp.wc >> j) & 1u) && (q.nu_dot(j, sd, x) - q.beta(j, sd) < q.thr(j, sd)));
    if (!anyv && CMPC_QP_ABL != 1) {
      o.nchg = chg;
      o.ws = mp.wc;
      bool fin = true;
#pragma unroll
      for (int r = 0; r < N; ++r) fin = fin && __builtin_isfinite(x[r]);
      if (!fin) o.status = CMPC_QP_NONFINITE;
      if (o.status == CMPC_QP_OK) {
        const uint32_t bnd = mp.wc & ((1u << N) - 1u), up = (mp.wc >> 16) & bnd;
#pragma unroll
        for (int r = 0; r < N; ++r)
          x[r] = ((bnd >> r) & 1u) ? (((up >> r) & 1u) ? q.ubv(r) : q.lbv(r)) : x[r];
      } else {
#pragma unroll
        for (int r = 0; r < N; ++r) x[r] = 0.0;
      }
      return;
    }
  }
  // off the map: the map is dropped (after a working-set change the next
  // ws_in is another anyway), and the working set of ws_in is rebuilt with
  // its fresh factor
  mp.ws = kWsInvalid;
  if (!have_w) {
    wset_fill(q, ws_in, W);
    wset_factor<N>(q, W);  // (succeeded when the map was built)
  }
#pragma unroll
  for (int a = 0; a < N; ++a) W.lam[a] = lam[a];
  if (!done && !stay) {
    // leave the map: x_u = x_u0 - U d, drops by the factor removal
    double xu[N];
#pragma unroll
    for (int r = 0; r < N; ++r) {
      double v = xu0[r];
#pragma unroll
      for (int c = 0; c < NVO; ++c) v = fma(-U(r, c), d[c], v);
      xu[r] = v;
    }
    for (int it = 0; it <= N && !done; ++it) {
      if (it > 0) {
        double rhs[N];
#pragma unroll
        for (int a = 0; a < N; ++a) {
          rhs[a] = 0.0;
          if (a < W.K) {
            rhs[a] = wset_beta(q, W, a) - wset_dot(q, W, a, xu);
          }
        }
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
#pragma unroll
      for (int r = 0; r < N; ++r) x[r] = xu[r];
#pragma unroll
      for (int a = 0; a < N; ++a) {
        if (a < W.K) {
          double ha[N];
          wset_h(q, W, a, ha);
#pragma unroll
          for (int r = 0; r < N; ++r) x[r] = fma(W.lam[a], ha[r], x[r]);
        }
      }
    }
  }
  qp_phase_b<TRACE>(q, W, x, chg, done, max_chg, o);
}

// x_u0 = -Hinv f and U = Hinv G of a QP (the map form's per-step terms):
// G[a][c] = gb[(a * NVOA + c) * GSTRIDE], overwritten by U (column c of U
// once column c of G is read)
template <int N, int NVO, int GSTRIDE, class HS>
CMPC_HD void jmap_terms(const HS& Hinv, const double (&f)[N], double* gb, double (&xu0)[N]) {
  constexpr int NVOA = JMap<N, NVO>::NVOA;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double sacc = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) sacc = fma(Hinv(i, j), f[j], sacc);
    xu0[i] = -sacc;
  }
#pragma unroll
  for (int c = 0; c < NVO; ++c) {
    double gc[N];
#pragma unroll
    for (int j = 0; j < N; ++j) gc[j] = gb[(j * NVOA + c) * GSTRIDE];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double u = 0.0;
#pragma unroll
      for (int j = 0; j < N; ++j) u = fma(Hinv(i, j), gc[j], u);
      gb[(i * NVOA + c) * GSTRIDE] = u;
    }
  }
}

// the same with U in registers (G left in place)
template <int N, int NVO, int GSTRIDE, class HS>
CMPC_HD void jmap_terms(const HS& Hinv, const double (&f)[N], const double* gb, double (&xu0)[N],
                        double (&U)[N][JMap<N, NVO>::NVOA]) {
  constexpr int NVOA = JMap<N, NVO>::NVOA;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double sacc = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) sacc = fma(Hinv(i, j), f[j], sacc);
    xu0[i] = -sacc;
#pragma unroll
    for (int c = 0; c < NVOA; ++c) {
      double u = 0.0;
      if (c < NVO) {
#pragma unroll
        for (int j = 0; j < N; ++j) u = fma(Hinv(i, j), gb[(j * NVOA + c) * GSTRIDE], u);
      }
      U[i][c] = u;
    }
  }
}

template <int N, int NU, int NB, class HS>
CMPC_HD void qp_solve(const Qp<N, NU, NB, HS>& q, bool pd, double tol_d, const double (&g)[N],
                         uint32_t ws_in, int max_chg, double (&x)[N], QpOut& o) {
  qp_solve_t<true>(q, pd, tol_d, g, ws_in, max_chg, x, o);
}
