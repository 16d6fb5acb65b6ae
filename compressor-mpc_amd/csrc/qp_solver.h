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
// and arithmetic order as oracle/or_qp.c; see DESIGN.md §QP.
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
  double m[N][N];
  CMPC_HD double operator()(int r, int c) const { return m[r][c]; }
  CMPC_HD void set(int r, int c, double v) { m[r][c] = v; }
};

// NB = stored bound entries: N (general), or NU when the bounds repeat every
// NU entries (the MPC QP: rep_m(lower - u_old), rep_m(rate bounds),
// libs/mpc_qp_solver.cc:53-60), which halves their registers.
template <int N, int NU, int NB = N, class HS = HinvRegs<N>>
struct Qp {
  static_assert(NB == N || NB == NU, "bounds: general or NU-periodic");
  HS Hinv;
  double lb[NB], ub[NB], lbA[NB], ubA[NB];
  // phase-B violation thresholds -TOL_P (1 + |beta|) per bound and side,
  // fixed per QP (tolerances() after the bounds are set), so that the K
  // Jacobi solves of a QP do not recompute them in every scan
  double tlb[NB], tub[NB], tlbA[NB], tubA[NB];
  CMPC_HD void tolerances() {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      tlb[i] = -TOL_P * (1.0 + fabs(lb[i]));
      tub[i] = -TOL_P * (1.0 + fabs(-ub[i]));
      tlbA[i] = -TOL_P * (1.0 + fabs(lbA[i]));
      tubA[i] = -TOL_P * (1.0 + fabs(-ubA[i]));
    }
  }
  CMPC_HD double thr(int j, int side) const {
    if (j < N) return side ? sel<NB>(tub, j % NB) : sel<NB>(tlb, j % NB);
    return side ? sel<NB>(tubA, (j - N) % NB) : sel<NB>(tlbA, (j - N) % NB);
  }
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
#define CMPC_WSET_STORE_MAX 6  // largest N whose working sets store their normals
#endif
template <int N, bool SN = (N <= CMPC_WSET_STORE_MAX)>
struct WSet {
  int K;
  int j[N], side[N];
  double lam[N];
  double nrm[SN ? N : 1][N], bta[N];
  double L[N][N], D[N], R[N];
};

// the normal of slot a (stored, or rebuilt from its constraint index)
template <int N, bool SN, class Q>
CMPC_HD void wset_normal(const Q& q, const WSet<N, SN>& W, int a, double (&n)[N]) {
  if constexpr (SN) {
#pragma unroll
    for (int c = 0; c < N; ++c) n[c] = W.nrm[a][c];
  } else {
    q.normal(W.j[a], W.side[a], n);
  }
}

// LDL' of the leading K x K block of M (lower triangle read) with reciprocal
// pivots R = 1/D (or_qp.c ldl); returns false on a non-positive pivot.
template <int N>
CMPC_HD bool ldl_k(int K, const double (&M)[N][N], double (&L)[N][N], double (&D)[N],
                   double (&R)[N]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (j < K) {
      double d = M[j][j];
#pragma unroll
      for (int k = 0; k < j; ++k) d = d - (L[j][k] * L[j][k]) * D[k];
      ok = ok && (d > 0.0);
      D[j] = d;
      const double r = 1.0 / d;
      R[j] = r;
      L[j][j] = 1.0;
#pragma unroll
      for (int i = j + 1; i < N; ++i) {
        if (i < K) {
          double sacc = M[i][j];
#pragma unroll
          for (int k = 0; k < j; ++k) sacc = sacc - (L[i][k] * L[j][k]) * D[k];
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
template <int N>
CMPC_HD void ldl_solve_k(int K, const double (&L)[N][N], const double (&R)[N],
                         const double (&b)[N], double (&x)[N], double (&zz)[N]) {
  double y[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    y[i] = 0.0;
    zz[i] = 0.0;
    if (i < K) {
      double v = b[i];
#pragma unroll
      for (int k = 0; k < i; ++k) v = v - L[i][k] * y[k];
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
        if (k < K) v = v - L[k][i] * x[k];
      x[i] = v;
    } else {
      x[i] = 0.0;
    }
  }
}
template <int N>
CMPC_HD void ldl_solve_k(int K, const double (&L)[N][N], const double (&R)[N],
                         const double (&b)[N], double (&x)[N]) {
  double zz[N];
  ldl_solve_k<N>(K, L, R, b, x, zz);
}

// warm start: M (M[i][k] = n_k' Hinv n_i, k <= i) of the current slots and
// its LDL' (or_qp.c wset_factor)
template <int N, bool SN, class Q>
CMPC_HD bool wset_factor(const Q& q, WSet<N, SN>& W) {
  double M[N][N];
#pragma unroll
  for (int b = 0; b < N; ++b) {
    double hb[N];
    if (b < W.K) {
      double nb[N];
      wset_normal(q, W, b, nb);
      q.hinv_n(nb, hb);
    }
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
  return ldl_k<N>(W.K, M, W.L, W.D, W.R);
}

// remove slot a (or_qp.c wset_remove): the other slots keep their order; the
// trailing block of the factor takes the rank-one term D_a w w' (GGMS method
// C1, reciprocal pivots), then rows and columns after a move up by one
template <int N, bool SN>
CMPC_HD void wset_drop(WSet<N, SN>& W, int a) {
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
      const double d = W.D[j] + t * p;
      const double r = 1.0 / d;
      const double bt = t * r;
      alpha = alpha * (W.D[j] * r);
      W.D[j] = d;
      W.R[j] = r;
#pragma unroll
      for (int i = j + 1; i < N; ++i)
        if (i < W.K) {
          w[i] = w[i] - p * W.L[i][j];
          W.L[i][j] = W.L[i][j] + bt * w[i];
        }
    }
  }
#pragma unroll
  for (int i = 0; i + 1 < N; ++i)
    if (i >= a && i + 1 < W.K) {
      W.j[i] = W.j[i + 1];
      W.side[i] = W.side[i + 1];
      W.lam[i] = W.lam[i + 1];
      W.bta[i] = W.bta[i + 1];
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
template <int N, bool SN>
CMPC_HD void wset_add(WSet<N, SN>& W, int j, int side, double lam, const double (&n)[N], double bta,
                      const double (&zz)[N], double zn, double rzn) {
#pragma unroll
  for (int b = 0; b < N; ++b)
    if (b == W.K) {
      W.j[b] = j;
      W.side[b] = side;
      W.lam[b] = lam;
      W.bta[b] = bta;
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
//
// CACHE = true (the Jacobi loop of the iterate kernel): the caller keeps the
// working set of the previous solve of the same QP (same H, other g) in *wc,
// with *wc_ws its working-set word, or kWsInvalid.  When ws_in equals it, the
// warm start takes the slots and the LDL' factor of M = N' H^-1 N from *wc
// instead of rebuilding them: the same values (the warm start's slot order
// and full factor are a deterministic function of H and the working set), so
// the result and the trace are bit-identical to the uncached solve.  *wc_ws
// is set only after a solve that ends OK without a working-set change (an
// update-derived factor, or slots in append order, would differ in rounding
// from the warm start's fresh factor).
constexpr uint32_t kWsInvalid = 0xFFFFFFFFu;

template <bool TRACE, bool CACHE = false, int N, int NU, int NB, class HS>
CMPC_HD void qp_solve_t(const Qp<N, NU, NB, HS>& q, bool pd, double tol_d, const double (&g)[N],
                         uint32_t ws_in, int max_chg, double (&x)[N], QpOut& o,
                         WSet<N>* wc = nullptr, uint32_t* wc_ws = nullptr) {
  WSet<N> Wl;
  WSet<N>& W = CACHE ? *wc : Wl;
  constexpr bool SN = (N <= CMPC_WSET_STORE_MAX);
  const bool cached = CACHE && pd && *wc_ws == ws_in;
  o.status = CMPC_QP_OK;
  o.nchg = 0;
  o.ntrace = 0;
  o.tr[0] = o.tr[1] = o.tr[2] = o.tr[3] = 0xFFFFFFFFu;
  if (!cached) {
    W.K = 0;
#pragma unroll
    for (int a = 0; a < N; ++a) {
      W.j[a] = 0;
      W.side[a] = 0;
      W.lam[a] = 0.0;
    }
  }
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
    for (int j = 0; j < N; ++j) sacc = sacc + q.Hinv(i, j) * g[j];
    xu[i] = -sacc;
  }
  // A. warm start: slot a = the a-th active constraint of ws_in in ascending
  // j (the oracle adds them in that order while K < n), then the full factor
  if (!cached) {
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
        if constexpr (SN) q.normal(j, sd, W.nrm[a]);
        W.bta[a] = q.beta(j, sd);
        W.K = a + 1;
      }
    }
    if (W.K > 0 && !wset_factor<N>(q, W)) {  // inconsistent warm start: cold
      W.K = 0;
      ++chg;
    }
  }
  for (int it = 0; it <= N && !done; ++it) {
    double rhs[N];
#pragma unroll
    for (int a = 0; a < N; ++a) {
      rhs[a] = 0.0;
      if (a < W.K) {
        double na[N];
        wset_normal(q, W, a, na);
        rhs[a] = W.bta[a] - ndot<N>(na, xu);
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
        double na[N], ha[N];
        wset_normal(q, W, a, na);
        q.hinv_n(na, ha);
#pragma unroll
        for (int r = 0; r < N; ++r) x[r] = x[r] + W.lam[a] * ha[r];
      }
    }
  }
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
    double np_[N];
    q.normal(pj, ps, np_);
    const double bp = q.beta(pj, ps);
    double up = 0.0;
    for (int inner = 0; inner <= max_chg + 1 && !done; ++inner) {
      double hp[N], qv[N], rv[N], zz[N], z[N];
      q.hinv_n(np_, hp);
#pragma unroll
      for (int a = 0; a < N; ++a) {
        qv[a] = 0.0;
        if (a < W.K) {
          double na[N];
          wset_normal(q, W, a, na);
          qv[a] = ndot<N>(na, hp);
        }
      }
      ldl_solve_k<N>(W.K, W.L, W.R, qv, rv, zz);
#pragma unroll
      for (int r = 0; r < N; ++r) z[r] = hp[r];
#pragma unroll
      for (int a = 0; a < N; ++a) {
        if (a < W.K) {
          double na[N], ha[N];
          wset_normal(q, W, a, na);
          q.hinv_n(na, ha);
#pragma unroll
          for (int r = 0; r < N; ++r) z[r] = z[r] - rv[a] * ha[r];
        }
      }
      const double zn = ndot<N>(np_, z);
      const double den = ndot<N>(np_, hp);
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
        continue;
      }
      const double rzn = 1.0 / zn;
      const double sl = ndot<N>(np_, x) - bp;
      const double t2 = -sl * rzn;
      const bool full = (k < 0) || (t2 <= t1);
      const double t = full ? t2 : t1;
#pragma unroll
      for (int r = 0; r < N; ++r) x[r] = x[r] + t * z[r];
#pragma unroll
      for (int a = 0; a < N; ++a)
        if (a < W.K) W.lam[a] = W.lam[a] - t * rv[a];
      up = up + t;
      if (full) {
        if (TRACE) trace_push(o, 1, pj, ps);
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
  if (CACHE) *wc_ws = (o.status == CMPC_QP_OK && chg == 0) ? w : kWsInvalid;
  // a non-finite plan (a NaN or infinite gradient) fails like any other
  // non-success: zero move (or_qp.c; checked before the bound fixing).  The
  // cached factors stay valid: they depend on H and the working set only.
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


template <int N, int NU, int NB, class HS>
CMPC_HD void qp_solve(const Qp<N, NU, NB, HS>& q, bool pd, double tol_d, const double (&g)[N],
                         uint32_t ws_in, int max_chg, double (&x)[N], QpOut& o) {
  qp_solve_t<true>(q, pd, tol_d, g, ws_in, max_chg, x, o);
}
