/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * The build's QP solver, restated for the CPU: a warm-started dual
 * (Goldfarb–Idnani) active-set method whose working-set factorisation is
 * updated (append / removal) rather than rebuilt, standing in for qpOASES
 * 3.2.0 SQProblem::hotstart (libs/mpc_qp_solver.cc:62-72; qpOASES is a
 * CMakeLists.txt:20-23 dependency that the reference does not vendor).  The
 * QP is the reference's
 *     min 1/2 x'Hx + g'x
 *     s.t. lb <= x <= ub, lbA <= Ain x <= ubA,
 *     Ain = [I 0 ..; -I I 0 ..; ...]     include/mpc_qp_solver.h:108-123
 * Semantics kept from the reference: at most n_wsr_max = 10 working-set
 * changes (include/mpc_qp_solver.h:24), zero vector on any non-success
 * (libs/mpc_qp_solver.cc:66-69), warm start from the previous working set of
 * the same QP slot (hotstart).
 *
 * Algorithm specification, version 4 (the HIP kernels implement the same
 * steps in the same arithmetic order).  Version 4: every
 * accumulation c +- a b below (the factor, its solves and updates, the
 * products with Hinv, U, the map and the step) is one fused multiply-add,
 * C99 fma() here and v_fma_f64 on the device (one rounding each; the build is
 * -ffp-contract=off everywhere else):
 *   0. H = L D L' with reciprocal pivots R = 1/D (any pivot <= 0 -> NOT_PD);
 *      Hinv column by column from that factor.
 *      nall_j = the normal of constraint j without its side: e_j (j < n),
 *      e_i (rate row i = j - n < nu), e_i - e_{i-nu} (rate row i >= nu).
 *      h_j = Hinv nall_j (a column or a difference of two columns).
 *   A. Warm start: slots = the constraints of ws_in in ascending j.  The
 *      working-set matrix M (M[i][k] = s_i s_k nall_{j_k}' h_{j_i} for
 *      i >= k, s = +1 lower side, -1 upper side) is factored M = L D L',
 *      reciprocal pivots R; a pivot d_j <= tol_z M_jj (dependent normals)
 *      -> cold start (W empty, one change).
 *      The gradient is g = f + G d (version 3): f, and G (n x nvo) times the
 *      other sub-controllers' plans d, the Jacobi iteration's ApplyOtherInput
 *      (include/distributed_solver.h:98-103); nvo = 0 for a plain QP.  The
 *      working set's multipliers and point are affine in d (the map of W):
 *        x_u0 = -Hinv f, U = Hinv G,
 *        lam0 = M^-1 (beta_W - N' x_u0),  Lam = M^-1 N' U (one solve per
 *        column), x0 = x_u0 + sum_a lam0_a h_a,  X = -U + sum_a Lam_a h_a,
 *      lam = lam0 + Lam d.  If no lam_w < -tol_d: x = x0 + X d.  Else
 *      x_u = x_u0 - U d and, while some lam_w < -tol_d: drop the most
 *      negative (lowest slot on ties) by the factor removal below, count one
 *      change, lam = M^-1 (beta_W - N' x_u); then x = x_u + sum_a lam_a h_a.
 *      (h_a = s_a h_{j_a}; sums in ascending index order.)  A Jacobi loop
 *      whose working set does not change evaluates only lam0 + Lam d and
 *      x0 + X d per iteration; with nvo = 0 the map form is the plain
 *      x_u, lam = M^-1 (beta_W - N' x_u), x = x_u + sum_a lam_a h_a.
 *   B. Repeat: pick the most violated inactive constraint p (slack < -tol_p,
 *      most negative; ties -> lowest j, lower side first).  None -> optimal.
 *      Goldfarb–Idnani step loop: hp = s_p h_p, qv = N'hp, r = M^-1 qv (the
 *      solve's scaled forward vector zz kept), z = hp - sum_a r_a s_a h_a,
 *      zn = nu_p'z, den = nu_p'hp, t1 = min_{r_a > tol_r} lam_a / r_a.
 *      If zn <= tol_z den or K = n (dependent): no blocking -> INFEASIBLE, else a dual
 *      step t1 and the blocker is removed.  Else t2 = -slack_p * (1/zn),
 *      t = min(t1, t2) (t2 wins ties): x += t z, lam -= t r, u_p += t; a full
 *      step APPENDS p as the last slot (L row = zz, pivot zn, R = 1/zn: the
 *      bordered factor of [M qv; qv' den]); a partial step removes the
 *      blocker.
 *   Factor removal of slot a (order of the other slots kept): rows and pivots
 *      before a unchanged; rows after a move up one; the trailing block gets
 *      the rank-one term D_a w w' (w = column a below a) by Gill, Golub,
 *      Murray & Saunders (1974) method C1 with reciprocal pivots (remove()).
 *   Every add/drop counts one change; the 11th change -> MAX_NWSR.
 *   On success, variables at an active bound are set exactly to that bound.
 *
 * Decision margins (info->margin; the checker's near-tie flag, not part of
 * the algorithm): every comparison that picks a branch or an index above
 * also records how far its two sides were apart, relative to the scale of
 * the compared quantities, and info->margin is the smallest such distance
 * over the whole solve:
 *   multipliers  lam_a vs -tol_d and vs the chosen most negative one,
 *                scale S_lam = max(|g|_inf, (1 + max|H_ii|) S_x, tol_d)
 *   slacks       slack vs -TOL_P(1 + |beta|) and vs the chosen most violated
 *                one, scale S_x = max of the finite |bounds| and |x_u|_inf
 *   step ratios  lam_a / r_a vs the chosen t1 (cross-multiplied:
 *                lam_a r_k - lam_k r_a over S_lam max(r_a, r_k)); r_a vs TOL_R
 *                over max(1, |r_a|)
 *   dependence   nu_p'z vs TOL_Z nu_p'Hinv nu_p over nu_p'Hinv nu_p
 *   step kind    t2 vs t1 over max(|t1|, |t2|)
 *   factor       the warm start's LDL' pivots vs TOL_Z M_aa over M_aa
 * (tests against a tolerance skip a rounding-noise zero: see mg_tol).
 * A QP whose inputs differ from another's by FP64 reassociation only
 * (~1e-13 relative) takes the same decisions whenever its margin is well
 * above that; tests allow differing working-set sequences only where the
 * margin is below 1e-9 (tests/test_solver_margins.py).
 * Working-set word: bit j = constraint j active (j < n: bound on x_j,
 * j >= n: rate row j - n), bit 16 + j = at its upper side.
 */
#include <math.h>
#include <string.h>

#include "cmpc_oracle.h"

#define QMAX CMPC_MAX_NV
#define TOL_P 1e-12
#define TOL_D 1e-12
#define TOL_R 1e-12
#define TOL_Z 1e-12

typedef struct {
  int n, nu;
  double Hinv[QMAX][QMAX];
  const double *lb, *ub, *lbA, *ubA;
  double s_x, s_lam; /* margin scales */
  double margin;     /* smallest relative decision margin so far */
} qp_t;

/* record |a - b| / scale as a decision margin */
static void mg(qp_t* q, double a, double b, double scale) {
  const double v = fabs(a - b) / (scale > 0 ? scale : 1e-300);
  if (v < q->margin) q->margin = v;
}

/* the same for a test of a against a tolerance thr, |thr| = 1e-12 of the
 * scale (or more).  A value within 1e-3 |thr| of zero is a mathematical zero
 * evaluated with rounding noise: a dependent constraint normal (nu_p'z with
 * nu_p in the span of the active normals), a structural zero of H or of the
 * normals, a constraint that x satisfies with equality by construction.
 * Such a value is zero for any perturbation of H and g, and its noise
 * (~1e-16 of the scale, far under 1e-3 |thr|) cannot carry it across thr on
 * any evaluation order, so it records no margin. */
static void mg_tol(qp_t* q, double a, double thr, double scale) {
  if (fabs(a) > 1e-3 * fabs(thr)) mg(q, a, thr, scale);
}

/* LDL' of the leading n x n block of a symmetric M (lower triangle read),
 * reciprocal pivots R = 1/D; a pivot fails unless d_j > rel M_jj (rel = 0:
 * H's positive definiteness; TOL_Z: a working set whose normals are
 * dependent, e.g. a bound and a rate row with the same normal):
 *   d_j = M_jj - sum_{k<j} (L_jk L_jk) D_k,       R_j = 1 / d_j
 *   L_ij = (M_ij - sum_{k<j} (L_ik L_jk) D_k) R_j  (i > j), k ascending.
 * Returns -(j+1) for the first pivot d_j <= 0 (the rest still computed). */
static int ldl(int n, double M[QMAX][QMAX], double L[QMAX][QMAX], double D[QMAX],
               double R[QMAX], double rel) {
  int rc = 0;
  for (int j = 0; j < n; ++j) {
    double d = M[j][j];
    for (int k = 0; k < j; ++k) d = fma(-(L[j][k] * L[j][k]), D[k], d);
    D[j] = d;
    R[j] = 1.0 / d;
    if (!(d > rel * M[j][j]) && !rc) rc = -(j + 1);
    L[j][j] = 1.0;
    for (int i = j + 1; i < n; ++i) {
      double s = M[i][j];
      for (int k = 0; k < j; ++k) s = fma(-(L[i][k] * L[j][k]), D[k], s);
      L[i][j] = s * R[j];
    }
  }
  return rc;
}

/* x = (L D L')^-1 b; also the forward vector y = L^-1 b and the scaled
 * zz = D^-1 y (the row a bordered factor appends):
 *   y_i = b_i - sum_{k<i} L_ik y_k,  zz_i = y_i R_i,
 *   x_i = zz_i - sum_{k>i} L_ki x_k  (k ascending). */
static void ldl_solve(int n, double L[QMAX][QMAX], const double R[QMAX], const double* b,
                      double* x, double* zz) {
  double y[QMAX];
  for (int i = 0; i < n; ++i) {
    double v = b[i];
    for (int k = 0; k < i; ++k) v = fma(-L[i][k], y[k], v);
    y[i] = v;
  }
  for (int i = 0; i < n; ++i) zz[i] = y[i] * R[i];
  for (int i = n - 1; i >= 0; --i) {
    double v = zz[i];
    for (int k = i + 1; k < n; ++k) v = fma(-L[k][i], x[k], v);
    x[i] = v;
  }
}

/* nu_{j,side}' v */
static double nu_dot(const qp_t* q, int j, int side, const double* v) {
  double t;
  if (j < q->n) {
    t = v[j];
  } else {
    const int i = j - q->n;
    t = (i >= q->nu) ? v[i] - v[i - q->nu] : v[i];
  }
  return side ? -t : t;
}

/* out = Hinv nu_{j,side} */
static void hinv_nu(const qp_t* q, int j, int side, double* out) {
  for (int r = 0; r < q->n; ++r) {
    double t;
    if (j < q->n) {
      t = q->Hinv[r][j];
    } else {
      const int i = j - q->n;
      t = (i >= q->nu) ? q->Hinv[r][i] - q->Hinv[r][i - q->nu] : q->Hinv[r][i];
    }
    out[r] = side ? -t : t;
  }
}

static double beta(const qp_t* q, int j, int side) {
  if (j < q->n) return side ? -q->ub[j] : q->lb[j];
  return side ? -q->ubA[j - q->n] : q->lbA[j - q->n];
}

typedef struct {
  int K;
  int j[QMAX], side[QMAX];
  double lam[QMAX];
  double L[QMAX][QMAX], D[QMAX], R[QMAX];
} wset_t;

/* warm start: M of the current slots and its LDL' */
static int wset_factor(qp_t* q, wset_t* W) {
  double M[QMAX][QMAX], h[QMAX];
  for (int i = 0; i < W->K; ++i) {
    hinv_nu(q, W->j[i], W->side[i], h);
    for (int k = 0; k <= i; ++k) M[i][k] = nu_dot(q, W->j[k], W->side[k], h);
  }
  const int rc = ldl(W->K, M, W->L, W->D, W->R, TOL_Z);
  /* margin of the pivot test d > TOL_Z M_aa (pivots relative to M's
   * diagonal), up to and including a failing pivot */
  const int np = rc ? -rc : W->K;
  for (int a = 0; a < np; ++a) mg(q, W->D[a], TOL_Z * M[a][a], fabs(M[a][a]));
  return rc;
}

/* remove slot a: the other slots keep their order; the factor of the
 * remaining working set by a rank-one update of the trailing block
 * (GGMS method C1):  alpha = D_a, w_i = L_ia (i > a); for j = a+1.. :
 *   p = w_j, t = alpha p, d = D_j + t p, r = 1/d, beta = t r,
 *   alpha = alpha (D_j r), D_j = d, R_j = r;
 *   for i > j: w_i = w_i - p L_ij, L_ij = L_ij + beta w_i.
 * Then rows / columns after a move up by one. */
static void wset_remove(wset_t* W, int a) {
  double w[QMAX];
  double alpha = W->D[a];
  for (int i = a + 1; i < W->K; ++i) w[i] = W->L[i][a];
  for (int j = a + 1; j < W->K; ++j) {
    const double p = w[j];
    const double t = alpha * p;
    const double d = fma(t, p, W->D[j]);
    const double r = 1.0 / d;
    const double bt = t * r;
    alpha = alpha * (W->D[j] * r);
    W->D[j] = d;
    W->R[j] = r;
    for (int i = j + 1; i < W->K; ++i) {
      w[i] = fma(-p, W->L[i][j], w[i]);
      W->L[i][j] = fma(bt, w[i], W->L[i][j]);
    }
  }
  for (int i = a; i + 1 < W->K; ++i) {
    W->j[i] = W->j[i + 1];
    W->side[i] = W->side[i + 1];
    W->lam[i] = W->lam[i + 1];
    W->D[i] = W->D[i + 1];
    W->R[i] = W->R[i + 1];
    for (int k = 0; k < a; ++k) W->L[i][k] = W->L[i + 1][k];
    for (int k = a; k < i; ++k) W->L[i][k] = W->L[i + 1][k + 1];
    W->L[i][i] = 1.0;
  }
  W->K--;
}

/* append p as the last slot: the bordered factor of [M qv; qv' den] is
 * L row zz = D^-1 L^-1 qv and pivot den - qv'M^-1 qv = zn */
static void wset_append(wset_t* W, int j, int side, double lam, const double* zz, double zn,
                        double rzn) {
  const int K = W->K;
  W->j[K] = j;
  W->side[K] = side;
  W->lam[K] = lam;
  for (int k = 0; k < K; ++k) W->L[K][k] = zz[k];
  W->L[K][K] = 1.0;
  W->D[K] = zn;
  W->R[K] = rzn;
  W->K = K + 1;
}

static void trace_push(or_qp_info* info, int add, int j, int side) {
  if (info->ntrace < 16)
    info->trace[info->ntrace++] = (uint8_t)((add ? 0x80 : 0) | (side ? 0x40 : 0) | j);
}

int or_qp_solve_map(int n, int nu, const double* H, const double* f, int nvo,
                    const double* G, const double* d, const double* lb,
                    const double* ub, const double* lbA, const double* ubA,
                    uint32_t ws_in, int max_chg, double* x_out, or_qp_info* info) {
  qp_t q;
  wset_t W;
  double x[QMAX], xu[QMAX];
  memset(info, 0, sizeof *info);
  memset(info->trace, 0xFF, sizeof info->trace);
  q.margin = HUGE_VAL;
  q.n = n;
  q.nu = nu;
  q.lb = lb; q.ub = ub; q.lbA = lbA; q.ubA = ubA;
  int chg = 0, status = CMPC_QP_OK;
  W.K = 0;
  /* 0. Hinv */
  {
    double Hm[QMAX][QMAX], L[QMAX][QMAX], D[QMAX], R[QMAX];
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) Hm[i][j] = H[i * n + j];
    const int rc = ldl(n, Hm, L, D, R, 0.0);
    for (int a = 0; a < (rc ? -rc : n); ++a) mg(&q, D[a], 0.0, fabs(H[a * n + a]));
    if (rc) {
      status = CMPC_QP_NOT_PD;
      goto done;
    }
    for (int c = 0; c < n; ++c) {
      double e[QMAX], col[QMAX], zz[QMAX];
      for (int i = 0; i < n; ++i) e[i] = (i == c) ? 1.0 : 0.0;
      ldl_solve(n, L, R, e, col, zz);
      for (int i = 0; i <= c; ++i) q.Hinv[i][c] = col[i];
    }
    for (int c = 0; c < n; ++c)
      for (int i = 0; i < c; ++i) q.Hinv[c][i] = q.Hinv[i][c];
  }
  double xu0[QMAX], U[QMAX][CMPC_MAX_NVO], g[QMAX];
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int j = 0; j < n; ++j) s = fma(q.Hinv[i][j], f[j], s);
    xu0[i] = -s;
    for (int c = 0; c < nvo; ++c) {
      double u = 0;
      for (int j = 0; j < n; ++j) u = fma(q.Hinv[i][j], G[j * nvo + c], u);
      U[i][c] = u;
    }
    /* the gradient f + G d: the margin scales only (checker) */
    double gi = f[i];
    for (int c = 0; c < nvo; ++c) gi = gi + G[i * nvo + c] * d[c];
    g[i] = gi;
  }
  double hmax = 0;
  for (int i = 0; i < n; ++i)
    if (fabs(H[i * n + i]) > hmax) hmax = fabs(H[i * n + i]);
  const double tol_d = TOL_D * (1.0 + hmax);
  {
    double sx = 0, sg = 0;
    for (int i = 0; i < n; ++i) {
      const double v[5] = {lb[i], ub[i], lbA[i], ubA[i], xu0[i]};
      for (int k = 0; k < 5; ++k)
        if (isfinite(v[k]) && fabs(v[k]) > sx) sx = fabs(v[k]);
      if (fabs(g[i]) > sg) sg = fabs(g[i]);
    }
    q.s_x = sx;
    q.s_lam = fmax(fmax(sg, (1.0 + hmax) * sx), tol_d);
  }

  /* A. warm start from ws_in: slots in ascending j */
  for (int j = 0; j < 2 * n; ++j)
    if ((ws_in & (1u << j)) && W.K < n) {
      W.j[W.K] = j;
      W.side[W.K] = (ws_in >> (16 + j)) & 1u;
      W.lam[W.K] = 0.0;
      W.K++;
    }
  while (W.K > 0 && wset_factor(&q, &W)) { /* inconsistent warm start: cold */
    W.K = 0;
    ++chg;
  }
  {
    /* the map of W: lam0, Lam (solves with the warm start's factor), then
     * lam = lam0 + Lam d */
    double rhs[QMAX], zz[QMAX], lam0[QMAX], Lam[QMAX][CMPC_MAX_NVO];
    for (int a = 0; a < W.K; ++a)
      rhs[a] = beta(&q, W.j[a], W.side[a]) - nu_dot(&q, W.j[a], W.side[a], xu0);
    ldl_solve(W.K, W.L, W.R, rhs, lam0, zz);
    for (int c = 0; c < nvo; ++c) {
      double uc[QMAX], lc[QMAX];
      for (int r = 0; r < n; ++r) uc[r] = U[r][c];
      for (int a = 0; a < W.K; ++a) rhs[a] = nu_dot(&q, W.j[a], W.side[a], uc);
      ldl_solve(W.K, W.L, W.R, rhs, lc, zz);
      for (int a = 0; a < W.K; ++a) Lam[a][c] = lc[a];
    }
    for (int a = 0; a < W.K; ++a) {
      double v = lam0[a];
      for (int c = 0; c < nvo; ++c) v = fma(Lam[a][c], d[c], v);
      W.lam[a] = v;
    }
    int first = 1, dropped = 0;
    for (;;) {
      if (!first) {
        for (int a = 0; a < W.K; ++a)
          rhs[a] = beta(&q, W.j[a], W.side[a]) - nu_dot(&q, W.j[a], W.side[a], xu);
        ldl_solve(W.K, W.L, W.R, rhs, W.lam, zz);
      }
      first = 0;
      int worst = -1;
      double wv = -tol_d;
      for (int a = 0; a < W.K; ++a)
        if (W.lam[a] < wv) {
          wv = W.lam[a];
          worst = a;
        }
      for (int a = 0; a < W.K; ++a) {
        mg_tol(&q, W.lam[a], -tol_d, q.s_lam);
        if (worst >= 0 && a != worst && W.lam[a] < -tol_d) mg(&q, W.lam[a], wv, q.s_lam);
      }
      if (worst < 0) break;
      if (!dropped) { /* leaving the map: x_u = x_u0 - U d */
        for (int r = 0; r < n; ++r) {
          double v = xu0[r];
          for (int c = 0; c < nvo; ++c) v = fma(-U[r][c], d[c], v);
          xu[r] = v;
        }
        dropped = 1;
      }
      trace_push(info, 0, W.j[worst], W.side[worst]);
      wset_remove(&W, worst);
      if (++chg > max_chg) {
        status = CMPC_QP_MAX_NWSR;
        goto done;
      }
    }
    if (!dropped) { /* x = x0 + X d */
      double x0[QMAX], X[QMAX][CMPC_MAX_NVO];
      for (int r = 0; r < n; ++r) {
        x0[r] = xu0[r];
        for (int c = 0; c < nvo; ++c) X[r][c] = -U[r][c];
      }
      for (int a = 0; a < W.K; ++a) {
        double h[QMAX];
        hinv_nu(&q, W.j[a], W.side[a], h);
        for (int r = 0; r < n; ++r) {
          x0[r] = fma(lam0[a], h[r], x0[r]);
          for (int c = 0; c < nvo; ++c) X[r][c] = fma(Lam[a][c], h[r], X[r][c]);
        }
      }
      for (int r = 0; r < n; ++r) {
        double v = x0[r];
        for (int c = 0; c < nvo; ++c) v = fma(X[r][c], d[c], v);
        x[r] = v;
      }
    } else {
      for (int r = 0; r < n; ++r) x[r] = xu[r];
      for (int a = 0; a < W.K; ++a) {
        double h[QMAX];
        hinv_nu(&q, W.j[a], W.side[a], h);
        for (int r = 0; r < n; ++r) x[r] = fma(W.lam[a], h[r], x[r]);
      }
    }
  }

  /* B. Goldfarb–Idnani */
  for (;;) {
    int pj = -1, ps = 0;
    double pv = 0;
    unsigned act = 0;
    for (int a = 0; a < W.K; ++a) act |= 1u << W.j[a];
    for (int j = 0; j < 2 * n; ++j) {
      if (act & (1u << j)) continue;
      for (int s = 0; s < 2; ++s) {
        const double b = beta(&q, j, s);
        const double sl = nu_dot(&q, j, s, x) - b;
        mg_tol(&q, sl, -TOL_P * (1.0 + fabs(b)), q.s_x);
        if (sl < -TOL_P * (1.0 + fabs(b)) && (pj < 0 || sl < pv)) {
          pj = j;
          ps = s;
          pv = sl;
        }
      }
    }
    if (pj >= 0) /* the most violated against the other violated ones */
      for (int j = 0; j < 2 * n; ++j) {
        if (act & (1u << j)) continue;
        for (int s = 0; s < 2; ++s) {
          const double b = beta(&q, j, s);
          const double sl = nu_dot(&q, j, s, x) - b;
          if (sl < -TOL_P * (1.0 + fabs(b)) && !(j == pj && s == ps)) mg(&q, sl, pv, q.s_x);
        }
      }
    if (pj < 0) break; /* optimal */
    double up = 0.0;
    for (;;) {
      double hp[QMAX], qv[QMAX], rv[QMAX], zz[QMAX], z[QMAX];
      hinv_nu(&q, pj, ps, hp);
      for (int a = 0; a < W.K; ++a) qv[a] = nu_dot(&q, W.j[a], W.side[a], hp);
      ldl_solve(W.K, W.L, W.R, qv, rv, zz);
      for (int r = 0; r < n; ++r) z[r] = hp[r];
      for (int a = 0; a < W.K; ++a) {
        double h[QMAX];
        hinv_nu(&q, W.j[a], W.side[a], h);
        for (int r = 0; r < n; ++r) z[r] = fma(-rv[a], h[r], z[r]);
      }
      const double zn = nu_dot(&q, pj, ps, z);
      const double den = nu_dot(&q, pj, ps, hp);
      int k = -1;
      double t1 = 0;
      for (int a = 0; a < W.K; ++a)
        if (rv[a] > TOL_R) {
          const double ratio = W.lam[a] / rv[a];
          if (k < 0 || ratio < t1) {
            t1 = ratio;
            k = a;
          }
        }
      for (int a = 0; a < W.K; ++a) {
        mg_tol(&q, rv[a], TOL_R, fmax(1.0, fabs(rv[a])));
        if (k >= 0 && a != k && rv[a] > TOL_R) /* blocking ratio vs the chosen one */
          mg(&q, W.lam[a] * rv[k], W.lam[k] * rv[a], q.s_lam * fmax(rv[a], rv[k]));
      }
      mg_tol(&q, zn, TOL_Z * den, fabs(den));
      /* nu_p dependent on the active normals (with n active constraints it
       * is, whatever the rounding of zn) */
      if (zn <= TOL_Z * den || W.K >= n) {
        if (k < 0) {
          status = CMPC_QP_INFEASIBLE;
          goto done;
        }
        for (int a = 0; a < W.K; ++a) W.lam[a] = fma(-t1, rv[a], W.lam[a]);
        up = up + t1;
        trace_push(info, 0, W.j[k], W.side[k]);
        wset_remove(&W, k);
        if (++chg > max_chg) {
          status = CMPC_QP_MAX_NWSR;
          goto done;
        }
        continue;
      }
      const double rzn = 1.0 / zn;
      const double sl = nu_dot(&q, pj, ps, x) - beta(&q, pj, ps);
      const double t2 = -sl * rzn;
      if (k >= 0) mg(&q, t2, t1, fmax(fabs(t1), fabs(t2)));
      const int full = (k < 0) || (t2 <= t1);
      const double t = full ? t2 : t1;
      for (int r = 0; r < n; ++r) x[r] = fma(t, z[r], x[r]);
      for (int a = 0; a < W.K; ++a) W.lam[a] = fma(-t, rv[a], W.lam[a]);
      up = up + t;
      if (full) {
        trace_push(info, 1, pj, ps);
        wset_append(&W, pj, ps, up, zz, zn, rzn);
        if (++chg > max_chg) {
          status = CMPC_QP_MAX_NWSR;
          goto done;
        }
        break;
      }
      trace_push(info, 0, W.j[k], W.side[k]);
      wset_remove(&W, k);
      if (++chg > max_chg) {
        status = CMPC_QP_MAX_NWSR;
        goto done;
      }
    }
  }
done:
  info->status = status;
  info->nchg = chg;
  info->margin = q.margin;
  {
    uint32_t w = 0;
    for (int a = 0; a < W.K; ++a)
      w |= (1u << W.j[a]) | ((uint32_t)W.side[a] << (16 + W.j[a]));
    info->ws = w;
  }
  /* a non-finite plan (a NaN or infinite gradient; a NaN Hessian is not PD)
   * is a failure like any other: zero move (libs/mpc_qp_solver.cc:66-69);
   * checked before the bound fixing */
  if (status == CMPC_QP_OK)
    for (int i = 0; i < n; ++i)
      if (!isfinite(x[i])) status = CMPC_QP_NONFINITE;
  info->status = status;
  /* variables at an active bound are fixed exactly at it (qpOASES treats
   * active bounds as fixed variables) */
  if (status == CMPC_QP_OK)
    for (int a = 0; a < W.K; ++a)
      if (W.j[a] < n) x[W.j[a]] = W.side[a] ? ub[W.j[a]] : lb[W.j[a]];
  for (int i = 0; i < n; ++i) x_out[i] = (status == CMPC_QP_OK) ? x[i] : 0.0;
  return status;
}

int or_qp_solve(int n, int nu, const double* H, const double* g,
                const double* lb, const double* ub, const double* lbA,
                const double* ubA, uint32_t ws_in, int max_chg, double* x_out,
                or_qp_info* info) {
  return or_qp_solve_map(n, nu, H, g, 0, NULL, NULL, lb, ub, lbA, ubA, ws_in, max_chg, x_out, info);
}
