/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Batched restatement of one NerveCenter control step
 * (include/nerve_center.h:134-182) over B independent scenarios of S
 * sub-controllers, in the product's lin-record format (include/cmpc.h):
 *   GenerateInitialQP per sub-controller      libs/distributed_controller.cc:72-108
 *   [init] InitializeQPProblem (cold solve)   libs/mpc_qp_solver.cc:77-101
 *   Jacobi loop, K iterations                 include/nerve_center.h:146-158
 *     gather other plans                      include/nerve_center.h:280-285
 *     GetInput (copy of qp_, ApplyOtherInput,  include/distributed_controller.h:206-226
 *       SolveQP bounds + solve)               include/distributed_solver.h:98-103,
 *                                             libs/mpc_qp_solver.cc:42-75
 *     scatter own plan                        include/nerve_center.h:293-295
 *   du_old_ = du_prev                         include/nerve_center.h:162
 *   UpdateUOld / SendUHelper (own inputs of    include/nerve_center.h:313-328,
 *     each sub-controller += first move)      include/distributed_controller.h:146-152
 *
 * margin (optional, B*S): per QP slot the smallest decision margin of its
 * solves in this step (or_qp_info.margin), the checker's near-tie flag.
 *
 * Other-controller plans are laid out in Su_other's move-major column order
 * (du_other[mv*nuo + rank*nu + c]); for S = 2 this is exactly the
 * reference's concatenation (nerve_center.h:283-285 vs aug_lin_sys.cc:325-327).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "cmpc_oracle.h"

int or_step(const cmpc_dims* d, const or_cfg* cfg, const double* lin, int K,
            uint32_t flags, int init, int threads, double* u_old,
            double* du_old, uint32_t* ws, double* du, int32_t* status,
            int32_t* nwsr, uint8_t* trace, int32_t* ntrace, double* margin) {
  cmpc_layout L;
  if (or_layout_of(d, &L)) return -1;
  const int S = d->S, B = d->B, nu = d->nu, nu_tot = d->nu_tot, m = d->m;
  const int ny = d->ny, p = d->p, R = p * ny;
  const int nV = L.nV, nVo = L.nVo, nuo = L.nuo;
  const int is_reduced = nu != nu_tot;
  (void)threads;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
#endif
  for (int b = 0; b < B; ++b) {
    double* H = (double*)malloc(sizeof(double) * S * nV * nV);
    double* f = (double*)malloc(sizeof(double) * S * nV);
    double* YPW = (double*)malloc(sizeof(double) * S * R * nV);
    double* Suo = (double*)malloc(sizeof(double) * S * R * (nVo ? nVo : 1));
    double* dprev = (double*)malloc(sizeof(double) * S * nV);
    double* dnew = (double*)malloc(sizeof(double) * S * nV);
    double* v = (double*)malloc(sizeof(double) * R);
    for (int s = 0; s < S; ++s) {
      const size_t q = (size_t)b * S + s;
      or_build_qp(d, lin + q * L.rec_len, u_old + q * nu_tot,
                  cfg->y_ref + (size_t)s * R, cfg->ywt + (size_t)s * ny * ny,
                  cfg->uwt + (size_t)s * nu * nu, H + s * nV * nV, f + s * nV,
                  YPW + (size_t)s * R * nV, nVo ? Suo + (size_t)s * R * nVo : NULL,
                  NULL);
    }
    double lb[CMPC_MAX_NV], ub[CMPC_MAX_NV], lbA[CMPC_MAX_NV], ubA[CMPC_MAX_NV];
    if (margin)
      for (int s = 0; s < S; ++s) margin[(size_t)b * S + s] = HUGE_VAL;
    if (init) {
      for (int s = 0; s < S; ++s) {
        const size_t q = (size_t)b * S + s;
        for (int mv = 0; mv < m; ++mv)
          for (int c = 0; c < nu; ++c) {
            lb[mv * nu + c] = cfg->lower[s * nu + c] - u_old[q * nu_tot + c];
            ub[mv * nu + c] = cfg->upper[s * nu + c] - u_old[q * nu_tot + c];
            lbA[mv * nu + c] = cfg->rate_lower[s * nu + c];
            ubA[mv * nu + c] = cfg->rate_upper[s * nu + c];
          }
        or_qp_info info;
        double xs[CMPC_MAX_NV];
        or_qp_solve(nV, nu, H + s * nV * nV, f + s * nV, lb, ub, lbA, ubA, 0u,
                    CMPC_NWSR_MAX, xs, &info);
        ws[q] = info.ws;
        if (margin && info.margin < margin[q]) margin[q] = info.margin;
      }
    }
    for (int s = 0; s < S; ++s)
      memcpy(dprev + s * nV, du_old + ((size_t)b * S + s) * nV, sizeof(double) * nV);
    for (int k = 0; k < K; ++k) {
      for (int s = 0; s < S; ++s) {
        const size_t q = (size_t)b * S + s;
        double fk[CMPC_MAX_NV];
        memcpy(fk, f + s * nV, sizeof(double) * nV);
        if (is_reduced) {
          double dother[64];
          for (int s2 = 0, rank = 0; s2 < S; ++s2) {
            if (s2 == s) continue;
            for (int mv = 0; mv < m; ++mv)
              for (int c = 0; c < nu; ++c)
                dother[mv * nuo + rank * nu + c] = dprev[s2 * nV + mv * nu + c];
            ++rank;
          }
          /* f += (du_other' Su_other') YPW   (distributed_solver.h:98-103) */
          const double* So = Suo + (size_t)s * R * nVo;
          const double* Y = YPW + (size_t)s * R * nV;
          for (int r = 0; r < R; ++r) {
            double a = 0;
            for (int c = 0; c < nVo; ++c) a += dother[c] * So[r * nVo + c];
            v[r] = a;
          }
          for (int c = 0; c < nV; ++c) {
            double a = 0;
            for (int r = 0; r < R; ++r) a += v[r] * Y[r * nV + c];
            fk[c] += a;
          }
        }
        for (int mv = 0; mv < m; ++mv)
          for (int c = 0; c < nu; ++c) {
            lb[mv * nu + c] = cfg->lower[s * nu + c] - u_old[q * nu_tot + c];
            ub[mv * nu + c] = cfg->upper[s * nu + c] - u_old[q * nu_tot + c];
            lbA[mv * nu + c] = cfg->rate_lower[s * nu + c];
            ubA[mv * nu + c] = cfg->rate_upper[s * nu + c];
          }
        or_qp_info info;
        or_qp_solve(nV, nu, H + s * nV * nV, fk, lb, ub, lbA, ubA, ws[q],
                    CMPC_NWSR_MAX, dnew + s * nV, &info);
        ws[q] = info.ws;
        status[q] = info.status;
        nwsr[q] = info.nchg;
        if (trace) memcpy(trace + (q * K + k) * 16, info.trace, 16);
        if (ntrace) ntrace[q * K + k] = info.ntrace;
        if (margin && info.margin < margin[q]) margin[q] = info.margin;
      }
      memcpy(dprev, dnew, sizeof(double) * S * nV);
    }
    for (int s = 0; s < S; ++s) {
      const size_t q = (size_t)b * S + s;
      memcpy(du + q * nV, dprev + s * nV, sizeof(double) * nV);
      memcpy(du_old + q * nV, dprev + s * nV, sizeof(double) * nV);
      if (flags & CMPC_APPLY_MOVE)
        for (int c = 0; c < nu; ++c) u_old[q * nu_tot + c] += dprev[s * nV + c];
    }
    free(H); free(f); free(YPW); free(Suo); free(dprev); free(dnew); free(v);
  }
  return 0;
}
