/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Restatement of the per-sub-controller observer and receding-horizon update
 * (SURVEY.md §8(f) row 2):
 *   Observer::ObserveAPosteriori          libs/observer.cc:27-44
 *   DistributedController::GenerateInitialQP, x_ += ...
 *                                          libs/distributed_controller.cc:80
 *   Observer::ObserveAPriori              libs/observer.cc:8-22
 *   AdjustFirstDelayedStates              include/aug_lin_sys.h:129-139
 *   AdjustAppliedInput                    include/aug_lin_sys.h:157-163
 *   AComposite::operator* / TimesAugmentedOnly
 *                                          include/aug_lin_sys.h:235-252,
 *                                          libs/aug_lin_sys.cc:125-140
 *   BComposite::operator*                 libs/aug_lin_sys.cc:204-226
 *   DistributedController::UpdateU        include/distributed_controller.h:145-152
 *   C = [C_plant | I]                     libs/aug_lin_sys.cc:20-21, :175
 *
 * Two exact elisions, shared with the product kernels (observer.hip):
 *  - C's identity block: sum_k (o == k) dx[ns + k] is dx[ns + o] plus zero
 *    products, which change nothing but the sign of a zero;
 *  - Aorig * dx' with dx'[:ns] = 0 (ObserveAPriori zeroes the state part
 *    before multiplying) adds +0.0 to every state entry.
 * The observer gain M is a constructor argument of the reference
 * (distributed_controller.cc:14); the harness that chose it
 * (common-simulation.inc) is missing upstream, so these functions are pinned
 * by an independent dense-matrix formulation (tests/test_observer.py) and by
 * the step-0 golden records (where the update is the identity), not by
 * recorded later steps.
 */
#include <string.h>

#include "cmpc_oracle.h"

/* dx: n_total = ns + ndist + n_delay_states (the full AugmentedState);
 * Cp: n_out x ns; M: (ns + ndist) x n_out; ndist == n_out columns of I. */
void or_observe_post(int ns, int ndist, int n_out, const double* Cp, const double* M,
                     const double* y, double* y_old, double* dx, double* x_hat) {
  const int nobs = ns + ndist;
  double v[16];
  for (int o = 0; o < n_out; ++o) {
    double t = 0.0;
    for (int j = 0; j < ns; ++j) t += Cp[o * ns + j] * dx[j];
    if (o < ndist) t = t + dx[ns + o];
    v[o] = (y[o] - y_old[o]) - t;
  }
  for (int k = 0; k < nobs; ++k) {
    double acc = 0.0;
    for (int o = 0; o < n_out; ++o) acc += M[k * n_out + o] * v[o];
    dx[k] = dx[k] + acc;
  }
  for (int o = 0; o < n_out; ++o) y_old[o] = y[o];
  for (int i = 0; i < ns; ++i) x_hat[i] = x_hat[i] + dx[i];
}

/* rec: the step's lin record (B in the sub-controller's input order, f);
 * du_own: first move of the sub-controller's plan (nu entries; the other
 * inputs' entries of the FullControlInput are zero, nerve_center.h:323-328);
 * u_old: nu_tot, updated in place (u_old += du). */
int or_observe_prior(const cmpc_dims* d, const double* rec, const double* du_own,
                     double* u_old, double* dx) {
  cmpc_layout L;
  if (or_layout_of(d, &L)) return -1;
  const int ns = d->ns, nut = d->nu_tot, nobs = L.nobs;
  const double* B = rec + L.off_B;
  const double* f = rec + L.off_f;
  double du[CMPC_MAX_INPUTS], dup[CMPC_MAX_INPUTS];
  int dinput[CMPC_MAX_INPUTS], nd = 0;
  for (int i = 0; i < nut; ++i) {
    if (d->delay[i] == 1) return -1; /* a one-step delay has no delay block */
    du[i] = (i < d->nu) ? du_own[i] : 0.0;
    dup[i] = du[i];
    if (d->delay[i]) {
      dup[i] += u_old[i]; /* AdjustAppliedInput */
      dinput[nd++] = i;
    }
  }
  /* dx' = dx with the state part zeroed, AdjustFirstDelayedStates */
  double seg[CMPC_MAX_INPUTS];
  for (int k = 0; k < nd; ++k) seg[k] = dx[nobs + k] - u_old[dinput[k]];
  /* states: (B du')[:ns] + (A dx')[:ns] + f */
  for (int l = 0; l < ns; ++l) {
    double b = 0.0;
    for (int i = 0; i < nut; ++i)
      if (!d->delay[i]) b += B[l * nut + i] * dup[i];
    double t = 0.0;
    for (int k = 0; k < nd; ++k) t += B[l * nut + dinput[k]] * seg[k];
    dx[l] = (b + t) + f[l];
  }
  /* disturbances: identity.  Delay blocks: the first state moves to the
   * delayed-input slot, the rest shift down by one, the applied input enters
   * at the block's end (Baug). */
  int ids = nobs + nd;
  for (int k = 0; k < nd; ++k) {
    const int i = dinput[k], size = d->delay[i] - 1;
    dx[nobs + k] = dx[ids];
    for (int j = 1; j < size; ++j) dx[ids + j - 1] = dx[ids + j];
    dx[ids + size - 1] = dup[i];
    ids += size;
  }
  for (int i = 0; i < nut; ++i) u_old[i] = u_old[i] + du[i];
  return 0;
}
