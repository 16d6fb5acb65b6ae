/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Restatement, in the reference's own operation order, of
 *   AugmentedLinearizedSystem::Update reorder   libs/aug_lin_sys.cc:145-177
 *   AComposite()  (Aaug map)                    libs/aug_lin_sys.cc:27-57
 *   AComposite::MultiplyC  (C *= A)             libs/aug_lin_sys.cc:62-86
 *   BComposite()  (Baug map)                    libs/aug_lin_sys.cc:182-199
 *   BComposite::MultiplyC  (C * B)              libs/aug_lin_sys.cc:91-113
 *   GeneratePrediction (O(p^2) Su loop)         libs/aug_lin_sys.cc:260-334
 *   AdjustAllDelayedStates                      include/aug_lin_sys.h:141-154
 *   delta_x0 assembly                           libs/distributed_controller.cc:85-90
 *   MpcQpSolver::SetWeights (W, R)              include/mpc_qp_solver.h:62-80
 *   DistributedSolver::GenerateDistributedQP    include/distributed_solver.h:83-94
 *   MpcQpSolver::GenerateQP                     libs/mpc_qp_solver.cc:16-40
 */
#include <stdlib.h>
#include <string.h>

#include "cmpc_oracle.h"

int or_layout_of(const cmpc_dims* d, cmpc_layout* L) {
  if (d->ns < 1 || d->ns > CMPC_MAX_NS || d->nu_tot < 1 ||
      d->nu_tot > CMPC_MAX_INPUTS || d->nu < 1 || d->nu > d->nu_tot ||
      d->ny < 1 || d->p < 1 || d->m < 1 || d->m > d->p ||
      d->m * d->nu > CMPC_MAX_NV || d->ndist < 0 || d->S < 1 || d->B < 1)
    return -1;
  memset(L, 0, sizeof *L);
  for (int i = 0; i < d->nu_tot; ++i) {
    if (d->delay[i] < 0) return -1;
    if (d->delay[i]) L->nd++;
    L->n_delay_states += d->delay[i];
  }
  L->naug = d->ndist + L->n_delay_states;
  L->nobs = d->ns + d->ndist;
  L->ntot = L->nobs + L->n_delay_states;
  L->nV = d->m * d->nu;
  L->nuo = d->nu_tot - d->nu;
  L->nVo = d->m * L->nuo;
  L->off_A = 0;
  L->off_B = d->ns * d->ns;
  L->off_C = L->off_B + d->ns * d->nu_tot;
  L->off_f = L->off_C + d->ny * L->nobs;
  L->off_x = L->off_f + d->ns;
  L->off_y = L->off_x + L->naug;
  L->rec_len = ((L->off_y + d->ny) + 7) / 8 * 8;
  return 0;
}

int or_lin_record(int plant, double p_in, double p_out, double Ts,
                  const double* x, const double* u_full,
                  const int32_t* input_order, const int32_t* out_idx,
                  const cmpc_dims* d, double* rec) {
  cmpc_layout L;
  int ns, ni, no, nci;
  if (or_layout_of(d, &L)) return -1;
  if (or_plant_dims(plant, &ns, &ni, &no, &nci)) return -1;
  if (ns != d->ns || nci != d->nu_tot) return -1;
  double A[16 * 16], Bc[16 * 8], C[8 * 16], f[16];
  double Ad[16 * 16], Bd[16 * 8], fd[16];
  or_plant_linearize(plant, p_in, p_out, x, u_full, A, Bc, C, f);
  or_discretize_rk4(ns, nci, Ts, A, Bc, f, Ad, Bd, fd);
  memcpy(rec + L.off_A, Ad, sizeof(double) * ns * ns);
  for (int r = 0; r < ns; ++r)
    for (int c = 0; c < nci; ++c)
      rec[L.off_B + r * nci + c] = Bd[r * nci + input_order[c]];
  for (int o = 0; o < d->ny; ++o) {
    for (int k = 0; k < ns; ++k)
      rec[L.off_C + o * L.nobs + k] = C[out_idx[o] * ns + k];
    for (int k = 0; k < d->ndist; ++k) /* C.rightCols<n_dist>() = Identity */
      rec[L.off_C + o * L.nobs + ns + k] = (out_idx[o] == k) ? 1.0 : 0.0;
  }
  memcpy(rec + L.off_f, fd, sizeof(double) * ns);
  return 0;
}

typedef struct {
  const cmpc_dims* d;
  cmpc_layout L;
  const double* Aorig; /* ns x ns */
  const double* Bin;   /* ns x nu_tot */
  int Aaug[512];
  int Baug[CMPC_MAX_INPUTS];
  int delayed_input[CMPC_MAX_INPUTS]; /* k-th delayed input -> control index */
} or_aug;

static int aug_init(or_aug* s, const cmpc_dims* d, const double* rec) {
  s->d = d;
  if (or_layout_of(d, &s->L)) return -1;
  if (s->L.naug > 512) return -1;
  s->Aorig = rec + s->L.off_A;
  s->Bin = rec + s->L.off_B;
  const int ndist = d->ndist, nd = s->L.nd, ns = d->ns;
  /* AComposite::AComposite, libs/aug_lin_sys.cc:27-57 */
  for (int i = 0; i < s->L.naug; ++i) s->Aaug[i] = 0;
  for (int i = 0; i < ndist; ++i) s->Aaug[i] = i;
  for (int i = 0; i < nd; ++i) s->Aaug[ndist + i] = -1;
  int ids = ndist + nd, idi = ndist, k = 0;
  for (int i = 0; i < d->nu_tot; ++i) {
    if (d->delay[i] != 0) {
      const int size_block = d->delay[i] - 1;
      if (ids < s->L.naug) s->Aaug[ids] = idi;
      for (int j = 1; j < size_block; ++j) s->Aaug[ids + j] = ids + j - 1;
      ids += d->delay[i] - 1;
      idi++;
      s->delayed_input[k++] = i;
    }
  }
  /* BComposite::BComposite, libs/aug_lin_sys.cc:182-199 */
  ids = nd;
  for (int i = 0; i < d->nu_tot; ++i) {
    if (d->delay[i] != 0) {
      ids += d->delay[i] - 1;
      s->Baug[i] = ns + ndist + ids - 1;
    } else {
      s->Baug[i] = -1;
    }
  }
  return 0;
}

/* libs/aug_lin_sys.cc:62-86: C (ny x ntot) *= A */
static void a_multiply_c(const or_aug* s, double* C, double* tmp, double* tmp2) {
  const int ny = s->d->ny, ns = s->d->ns, nt = s->L.ntot, na = s->L.naug;
  const int nobs = s->L.nobs, nu_tot = s->d->nu_tot;
  for (int o = 0; o < ny; ++o) {
    memcpy(tmp + o * ns, C + o * nt, sizeof(double) * ns);
    memcpy(tmp2 + o * na, C + o * nt + ns, sizeof(double) * na);
  }
  for (int o = 0; o < ny; ++o)
    for (int j = 0; j < ns; ++j) {
      double acc = 0;
      for (int l = 0; l < ns; ++l) acc += tmp[o * ns + l] * s->Aorig[l * ns + j];
      C[o * nt + j] = acc;
    }
  for (int i = 0; i < na; ++i)
    for (int o = 0; o < ny; ++o)
      C[o * nt + ns + i] = (s->Aaug[i] >= 0) ? tmp2[o * na + s->Aaug[i]] : 0.0;
  for (int k = 0; k < s->L.nd; ++k) {
    const int c = s->delayed_input[k];
    for (int o = 0; o < ny; ++o) {
      double acc = 0;
      for (int l = 0; l < ns; ++l) acc += tmp[o * ns + l] * s->Bin[l * nu_tot + c];
      C[o * nt + nobs + k] += acc;
    }
  }
}

/* libs/aug_lin_sys.cc:91-113: out (ny x nu_tot) = C * B */
static void b_multiply_c(const or_aug* s, const double* C, double* out) {
  const int ny = s->d->ny, ns = s->d->ns, nt = s->L.ntot, nu_tot = s->d->nu_tot;
  for (int i = 0; i < nu_tot; ++i) {
    for (int o = 0; o < ny; ++o) {
      if (s->d->delay[i] == 0) {
        double acc = 0;
        for (int l = 0; l < ns; ++l) acc += C[o * nt + l] * s->Bin[l * nu_tot + i];
        out[o * nu_tot + i] = acc;
      } else {
        out[o * nu_tot + i] = C[o * nt + s->Baug[i]];
      }
    }
  }
}

int or_generate_prediction(const cmpc_dims* d, const double* rec, double* Su,
                           double* Sx, double* Sf, double* Su_other) {
  or_aug s;
  if (aug_init(&s, d, rec)) return -1;
  const int ny = d->ny, ns = d->ns, p = d->p, m = d->m, nu = d->nu;
  const int nt = s.L.ntot, na = s.L.naug, nobs = s.L.nobs;
  const int nuo = s.L.nuo, nu_tot = d->nu_tot;
  const int is_reduced = nu != nu_tot;
  const double* Csel = rec + s.L.off_C;
  double* cta = (double*)calloc((size_t)ny * nt, sizeof(double));
  double* tmp = (double*)malloc(sizeof(double) * ny * ns);
  double* tmp2 = (double*)malloc(sizeof(double) * ny * (na + 1));
  double to_add[8 * CMPC_MAX_INPUTS];
  /* c_times_a <- controlled rows of C, delay columns zero (:274-281) */
  for (int o = 0; o < ny; ++o)
    for (int k = 0; k < nobs; ++k) cta[o * nt + k] = Csel[o * nobs + k];
  const int nV = m * nu, nVo = m * nuo;
  memset(Su, 0, sizeof(double) * p * ny * nV);
  memset(Sx, 0, sizeof(double) * p * ny * na);
  memset(Sf, 0, sizeof(double) * p * ny * ns);
  if (is_reduced && Su_other) memset(Su_other, 0, sizeof(double) * p * ny * nVo);
  for (int o = 0; o < ny; ++o)
    for (int k = 0; k < ns; ++k) Sf[o * ns + k] = cta[o * nt + k];
  for (int i = 0; i < p; ++i) {
    if (i > 0)
      for (int o = 0; o < ny; ++o)
        for (int k = 0; k < ns; ++k)
          Sf[(i * ny + o) * ns + k] = Sf[((i - 1) * ny + o) * ns + k] + cta[o * nt + k];
    b_multiply_c(&s, cta, to_add);
    for (int j = 0; j < p - i; ++j) {
      const int ind_row = i + j;
      const int ind_col = (j < m) ? j : m - 1;
      for (int o = 0; o < ny; ++o) {
        for (int c = 0; c < nu; ++c)
          Su[(ind_row * ny + o) * nV + ind_col * nu + c] += to_add[o * nu_tot + c];
        if (is_reduced && Su_other)
          for (int c = 0; c < nuo; ++c)
            Su_other[(ind_row * ny + o) * nVo + ind_col * nuo + c] +=
                to_add[o * nu_tot + nu + c];
      }
    }
    a_multiply_c(&s, cta, tmp, tmp2);
    for (int o = 0; o < ny; ++o)
      for (int a = 0; a < na; ++a) Sx[(i * ny + o) * na + a] = cta[o * nt + ns + a];
  }
  free(cta);
  free(tmp);
  free(tmp2);
  return 0;
}

int or_build_qp(const cmpc_dims* d, const double* rec, const double* u_old,
                const double* y_ref, const double* ywt, const double* uwt,
                double* H, double* f, double* YPW, double* Su_other,
                double* G) {
  cmpc_layout L;
  if (or_layout_of(d, &L)) return -1;
  const int ny = d->ny, ns = d->ns, p = d->p, nu = d->nu;
  const int na = L.naug, nV = L.nV, nVo = L.nVo, nobs = L.nobs;
  const int R = p * ny;
  /* delta_x0 = [f ; dx_aug.tail(naug)]  (libs/distributed_controller.cc:85-87) */
  double* dx0 = (double*)malloc(sizeof(double) * L.ntot);
  memcpy(dx0, rec + L.off_f, sizeof(double) * ns);
  memcpy(dx0 + ns, rec + L.off_x, sizeof(double) * na);
  /* AdjustAllDelayedStates (include/aug_lin_sys.h:141-154) */
  int ids = nobs + L.nd, idi = nobs;
  for (int i = 0; i < d->nu_tot; ++i) {
    if (d->delay[i] != 0) {
      dx0[idi] -= u_old[i];
      for (int j = 1; j < d->delay[i]; ++j) dx0[ids + j - 1] -= u_old[i];
      ids += d->delay[i] - 1;
      idi++;
    }
  }
  double* Su = (double*)malloc(sizeof(double) * R * nV);
  double* Sx = (double*)malloc(sizeof(double) * R * na);
  double* Sf = (double*)malloc(sizeof(double) * R * ns);
  double* Suo_local = NULL;
  if (!Su_other && nVo) Suo_local = (double*)malloc(sizeof(double) * R * nVo);
  double* Suo = Su_other ? Su_other : Suo_local;
  or_generate_prediction(d, rec, Su, Sx, Sf, nVo ? Suo : NULL);
  /* y_pred_weight_ = y_weight_ * Su, W = blkdiag_p(ywt) (mpc_qp_solver.h:62-80) */
  for (int i = 0; i < p; ++i)
    for (int a = 0; a < ny; ++a)
      for (int c = 0; c < nV; ++c) {
        double acc = 0;
        for (int b = 0; b < ny; ++b)
          acc += ywt[a * ny + b] * Su[(i * ny + b) * nV + c];
        YPW[(i * ny + a) * nV + c] = acc;
      }
  /* H = Su' * YPW + R  (libs/mpc_qp_solver.cc:31) */
  for (int a = 0; a < nV; ++a)
    for (int b = 0; b < nV; ++b) {
      double acc = 0;
      for (int r = 0; r < R; ++r) acc += Su[r * nV + a] * YPW[r * nV + b];
      const int ma = a / nu, mb = b / nu;
      const double rw = (ma == mb) ? uwt[(a % nu) * nu + (b % nu)] : 0.0;
      H[a * nV + b] = acc + rw;
    }
  /* f  (libs/mpc_qp_solver.cc:29,33-37) */
  const double* xh = dx0;
  const double* xa = dx0 + ns;
  const double* yprev = rec + L.off_y;
  double* v1 = (double*)malloc(sizeof(double) * R);
  double* v2 = (double*)malloc(sizeof(double) * R);
  double* v3 = (double*)malloc(sizeof(double) * R);
  for (int r = 0; r < R; ++r) {
    double a1 = 0, a3 = 0;
    for (int k = 0; k < ns; ++k) a1 += Sf[r * ns + k] * xh[k];
    for (int k = 0; k < na; ++k) a3 += Sx[r * na + k] * xa[k];
    v1[r] = a1;
    v3[r] = a3;
    v2[r] = y_ref[r] - yprev[r % ny];
  }
  for (int c = 0; c < nV; ++c) {
    double f1 = 0, f2 = 0, f3 = 0;
    for (int r = 0; r < R; ++r) {
      f1 += v1[r] * YPW[r * nV + c];
      f2 += v2[r] * YPW[r * nV + c];
      f3 += v3[r] * YPW[r * nV + c];
    }
    f[c] = f1 - f2 + f3;
  }
  if (G && nVo) {
    for (int a = 0; a < nV; ++a)
      for (int c = 0; c < nVo; ++c) {
        double acc = 0;
        for (int r = 0; r < R; ++r) acc += YPW[r * nV + a] * Suo[r * nVo + c];
        G[a * nVo + c] = acc;
      }
  }
  free(v1); free(v2); free(v3);
  free(Su); free(Sx); free(Sf); free(dx0);
  if (Suo_local) free(Suo_local);
  return 0;
}
