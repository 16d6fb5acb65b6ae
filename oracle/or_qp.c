/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * The build's QP solver, restated for the CPU: a warm-started dual
 * (Goldfarb–Idnani) active-set method with dense re-factorisation, standing
 * in for qpOASES 3.2.0 SQProblem::hotstart (libs/mpc_qp_solver.cc:62-72;
 * qpOASES is a CMakeLists.txt:20-23 dependency that the reference does not
 * vendor).  The QP is the reference's
 *     min 1/2 x'Hx + g'x
 *     s.t. lb <= x <= ub, lbA <= Ain x <= ubA,
 *     Ain = [I 0 ..; -I I 0 ..; ...]     include/mpc_qp_solver.h:108-123
 * Semantics kept from the reference: at most n_wsr_max = 10 working-set
 * changes (include/mpc_qp_solver.h:24), zero vector on any non-success
 * (libs/mpc_qp_solver.cc:66-69), warm start from the previous working set of
 * the same QP slot (hotstart).
 *
 * Algorithm specification (the HIP kernel implements the same steps in the
 * same arithmetic order):
 *   0. Hinv = H^-1 via LDL' (no square roots); any pivot <= 0 -> NOT_PD.
 *      x_u = -Hinv g.
 *   A. Warm start: W = ws_in.  Solve the equality QP on W:
 *      lam = (N'Hinv N)^-1 (beta_W - N' x_u), x = x_u + Hinv N lam.
 *      While some lam_w < -tol_d: drop the most negative (lowest j on ties),
 *      count one change, re-solve.
 *   B. Repeat: pick the most violated constraint p (slack < -tol_p, most
 *      negative; ties -> lowest j, lower side first).  None -> optimal.
 *      Goldfarb–Idnani step loop: r = M^-1 N'Hinv nu_p,
 *      z = Hinv nu_p - Hinv N r, t1 = min_{r_w > tol_r} lam_w / r_w,
 *      t2 = -slack_p / (nu_p' z).  If nu_p'z <= tol_z nu_p'Hinv nu_p
 *      (dependent): no blocking -> INFEASIBLE, else dual step t1 and drop.
 *      Else t = min(t1, t2) (t2 wins ties): x += t z, lam -= t r,
 *      u_p += t; full step adds p, partial step drops the blocker.
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
 *   factor       working-set LDL' pivots over the diagonal of M
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

static int ldl(int n, double M[QMAX][QMAX], double L[QMAX][QMAX],
               double D[QMAX]) {
  for (int j = 0; j < n; ++j) {
    double d = M[j][j];
    for (int k = 0; k < j; ++k) d = d - (L[j][k] * L[j][k]) * D[k];
    D[j] = d;
    if (!(d > 0)) return -(j + 1);
    L[j][j] = 1.0;
    for (int i = j + 1; i < n; ++i) {
      double s = M[i][j];
      for (int k = 0; k < j; ++k) s = s - (L[i][k] * L[j][k]) * D[k];
      L[i][j] = s / d;
    }
  }
  return 0;
}

static void ldl_solve(int n, double L[QMAX][QMAX], const double D[QMAX],
                      const double* b, double* x) {
  double y[QMAX];
  for (int i = 0; i < n; ++i) {
    double v = b[i];
    for (int k = 0; k < i; ++k) v = v - L[i][k] * y[k];
    y[i] = v;
  }
  for (int i = 0; i < n; ++i) y[i] = y[i] / D[i];
  for (int i = n - 1; i >= 0; --i) {
    double v = y[i];
    for (int k = i + 1; k < n; ++k) v = v - L[k][i] * x[k];
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
  double h[QMAX][QMAX]; /* h[a] = Hinv nu_a */
  double L[QMAX][QMAX], D[QMAX];
} wset_t;

/* (re)build h, M = N'Hinv N and its LDL' for the current W */
static int wset_factor(qp_t* q, wset_t* W) {
  double M[QMAX][QMAX];
  for (int a = 0; a < W->K; ++a) hinv_nu(q, W->j[a], W->side[a], W->h[a]);
  for (int a = 0; a < W->K; ++a)
    for (int b = a; b < W->K; ++b) {
      const double v = nu_dot(q, W->j[a], W->side[a], W->h[b]);
      M[a][b] = v;
      M[b][a] = v;
    }
  const int rc = ldl(W->K, M, W->L, W->D);
  /* margin of the pivot test d > 0 (pivots relative to M's diagonal), up
   * to and including a failing pivot */
  const int np = rc ? -rc : W->K;
  for (int a = 0; a < np; ++a) mg(q, W->D[a], 0.0, fabs(M[a][a]));
  return rc;
}

static void wset_drop(wset_t* W, int a) {
  for (int b = a; b + 1 < W->K; ++b) {
    W->j[b] = W->j[b + 1];
    W->side[b] = W->side[b + 1];
    W->lam[b] = W->lam[b + 1];
  }
  W->K--;
}

static void wset_add(wset_t* W, int j, int side, double lam) {
  int a = W->K;
  while (a > 0 && W->j[a - 1] > j) {
    W->j[a] = W->j[a - 1];
    W->side[a] = W->side[a - 1];
    W->lam[a] = W->lam[a - 1];
    --a;
  }
  W->j[a] = j;
  W->side[a] = side;
  W->lam[a] = lam;
  W->K++;
}

static void trace_push(or_qp_info* info, int add, int j, int side) {
  if (info->ntrace < 16)
    info->trace[info->ntrace++] = (uint8_t)((add ? 0x80 : 0) | (side ? 0x40 : 0) | j);
}

int or_qp_solve(int n, int nu, const double* H, const double* g,
                const double* lb, const double* ub, const double* lbA,
                const double* ubA, uint32_t ws_in, int max_chg, double* x_out,
                or_qp_info* info) {
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
    double Hm[QMAX][QMAX], L[QMAX][QMAX], D[QMAX];
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) Hm[i][j] = H[i * n + j];
    const int rc = ldl(n, Hm, L, D);
    for (int a = 0; a < (rc ? -rc : n); ++a) mg(&q, D[a], 0.0, fabs(H[a * n + a]));
    if (rc) {
      status = CMPC_QP_NOT_PD;
      goto done;
    }
    for (int c = 0; c < n; ++c) {
      double e[QMAX], col[QMAX];
      for (int i = 0; i < n; ++i) e[i] = (i == c) ? 1.0 : 0.0;
      ldl_solve(n, L, D, e, col);
      for (int i = 0; i <= c; ++i) q.Hinv[i][c] = col[i];
    }
    for (int c = 0; c < n; ++c)
      for (int i = 0; i < c; ++i) q.Hinv[c][i] = q.Hinv[i][c];
  }
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int j = 0; j < n; ++j) s = s + q.Hinv[i][j] * g[j];
    xu[i] = -s;
  }
  double hmax = 0;
  for (int i = 0; i < n; ++i)
    if (fabs(H[i * n + i]) > hmax) hmax = fabs(H[i * n + i]);
  const double tol_d = TOL_D * (1.0 + hmax);
  {
    double sx = 0, sg = 0;
    for (int i = 0; i < n; ++i) {
      const double v[5] = {lb[i], ub[i], lbA[i], ubA[i], xu[i]};
      for (int k = 0; k < 5; ++k)
        if (isfinite(v[k]) && fabs(v[k]) > sx) sx = fabs(v[k]);
      if (fabs(g[i]) > sg) sg = fabs(g[i]);
    }
    q.s_x = sx;
    q.s_lam = fmax(fmax(sg, (1.0 + hmax) * sx), tol_d);
  }

  /* A. warm start from ws_in */
  for (int j = 0; j < 2 * n; ++j)
    if ((ws_in & (1u << j)) && W.K < n) wset_add(&W, j, (ws_in >> (16 + j)) & 1u, 0.0);
  for (;;) {
    if (wset_factor(&q, &W)) { /* inconsistent warm start: cold */
      W.K = 0;
      ++chg;
      continue;
    }
    double rhs[QMAX];
    for (int a = 0; a < W.K; ++a)
      rhs[a] = beta(&q, W.j[a], W.side[a]) - nu_dot(&q, W.j[a], W.side[a], xu);
    ldl_solve(W.K, W.L, W.D, rhs, W.lam);
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
    trace_push(info, 0, W.j[worst], W.side[worst]);
    wset_drop(&W, worst);
    if (++chg > max_chg) {
      status = CMPC_QP_MAX_NWSR;
      goto done;
    }
  }
  for (int r = 0; r < n; ++r) {
    double v = xu[r];
    for (int a = 0; a < W.K; ++a) v = v + W.lam[a] * W.h[a][r];
    x[r] = v;
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
      double hp[QMAX], qv[QMAX], rv[QMAX], z[QMAX];
      hinv_nu(&q, pj, ps, hp);
      for (int a = 0; a < W.K; ++a) qv[a] = nu_dot(&q, W.j[a], W.side[a], hp);
      ldl_solve(W.K, W.L, W.D, qv, rv);
      for (int r = 0; r < n; ++r) {
        double v = hp[r];
        for (int a = 0; a < W.K; ++a) v = v - rv[a] * W.h[a][r];
        z[r] = v;
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
      if (zn <= TOL_Z * den) { /* nu_p dependent on the active normals */
        if (k < 0) {
          status = CMPC_QP_INFEASIBLE;
          goto done;
        }
        for (int a = 0; a < W.K; ++a) W.lam[a] = W.lam[a] - t1 * rv[a];
        up = up + t1;
        trace_push(info, 0, W.j[k], W.side[k]);
        wset_drop(&W, k);
        if (++chg > max_chg) {
          status = CMPC_QP_MAX_NWSR;
          goto done;
        }
        wset_factor(&q, &W);
        continue;
      }
      const double sl = nu_dot(&q, pj, ps, x) - beta(&q, pj, ps);
      const double t2 = -sl / zn;
      if (k >= 0) mg(&q, t2, t1, fmax(fabs(t1), fabs(t2)));
      const int full = (k < 0) || (t2 <= t1);
      const double t = full ? t2 : t1;
      for (int r = 0; r < n; ++r) x[r] = x[r] + t * z[r];
      for (int a = 0; a < W.K; ++a) W.lam[a] = W.lam[a] - t * rv[a];
      up = up + t;
      if (full) {
        trace_push(info, 1, pj, ps);
        wset_add(&W, pj, ps, up);
        if (++chg > max_chg) {
          status = CMPC_QP_MAX_NWSR;
          goto done;
        }
        wset_factor(&q, &W);
        break;
      }
      trace_push(info, 0, W.j[k], W.side[k]);
      wset_drop(&W, k);
      if (++chg > max_chg) {
        status = CMPC_QP_MAX_NWSR;
        goto done;
      }
      wset_factor(&q, &W);
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
