/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Restatement of the reference harness's plant simulation (SURVEY.md §8(f)
 * row 3):
 *   SimulationSystem::Integrate            include/simulation_system.h:108-116
 *     boost::numeric::odeint::integrate_const with
 *     controlled_runge_kutta<runge_kutta_dopri5> (Boost 1.60 odeint, not
 *     vendored in the reference), eps_abs = eps_rel = 1e-6, a_x = a_dxdt = 1;
 *     the error norm is the reference's override of vector_space_norm_inf
 *     for Eigen arrays: the 2-norm (simulation_system.h:121-133)
 *   SimulationSystem::SetInput / GetPlantInput
 *                                          include/simulation_system.h:67-88
 *   TimeDelay::GetDelayedInput             include/time_delay.h:41-58
 *
 * odeint semantics restated (Boost 1.60, from its published algorithm):
 *   - integrate_const(stepper, sys, x, t0, tf, dt, obs) runs, per
 *     observation interval [t, t + dt], integrate_adaptive on a COPY of the
 *     controlled stepper (so the FSAL derivative is recomputed at the start
 *     of each interval, with the input the observer just set), with the step
 *     size dt carried by reference from interval to interval;
 *   - integrate_adaptive: while t_end - t > eps: clip dt to t_end - t when
 *     t + dt - t_end > eps; try_step until success (500 failures throw);
 *     integrate_const's max_step_checker throws after 500 steps between two
 *     observer calls (here: return -2, the device sets status 2);
 *   - try_step: one Dormand-Prince 5(4) step; err = ||e_i / (eps_abs +
 *     eps_rel (|x_i| + dt |dxdt_i|))||; err > 1: reject, dt *= max(0.9
 *     err^(-1/3), 0.2); else accept, t += dt and, if err < 0.5,
 *     dt *= 0.9 max(err, 5^-5)^(-1/5);
 *   - the stage combinations are odeint's scale_sumN: a1 t2 + a2 t3 + ...
 *     left to right with a1 = 1 (so x + (dt b_i1) k1 + ...).
 * Pinned by the reference's recorded trajectories (tests/golden/traj_<plant>_
 * <cfg>.json, from results/<plant>/run1/<cfg>.dat): driven by the recorded
 * inputs, the simulation reproduces the recorded plant states to the printed
 * 6 digits.
 */
#include <float.h>
#include <math.h>
#include <string.h>

#include "cmpc_oracle.h"

#define OR_SIM_MAXN 16

static const double a_b21 = 1.0 / 5.0;
static const double a_b31 = 3.0 / 40.0, a_b32 = 9.0 / 40.0;
static const double a_b41 = 44.0 / 45.0, a_b42 = -56.0 / 15.0, a_b43 = 32.0 / 9.0;
static const double a_b51 = 19372.0 / 6561.0, a_b52 = -25360.0 / 2187.0,
                    a_b53 = 64448.0 / 6561.0, a_b54 = -212.0 / 729.0;
static const double a_b61 = 9017.0 / 3168.0, a_b62 = -355.0 / 33.0, a_b63 = 46732.0 / 5247.0,
                    a_b64 = 49.0 / 176.0, a_b65 = -5103.0 / 18656.0;
static const double a_c1 = 35.0 / 384.0, a_c3 = 500.0 / 1113.0, a_c4 = 125.0 / 192.0,
                    a_c5 = -2187.0 / 6784.0, a_c6 = 11.0 / 84.0;

/* one Dormand-Prince step from (x, k1): out, k7 = f(out), xerr */
static void dopri5_step(int plant, double p_in, double p_out, const double* u, int n,
                        const double* x, const double* k1, double dt, double* out, double* k7,
                        double* xerr) {
  const double dc1 = a_c1 - 5179.0 / 57600.0, dc3 = a_c3 - 7571.0 / 16695.0,
               dc4 = a_c4 - 393.0 / 640.0, dc5 = a_c5 - -92097.0 / 339200.0,
               dc6 = a_c6 - 187.0 / 2100.0, dc7 = -1.0 / 40.0;
  double k2[OR_SIM_MAXN], k3[OR_SIM_MAXN], k4[OR_SIM_MAXN], k5[OR_SIM_MAXN], k6[OR_SIM_MAXN];
  double xt[OR_SIM_MAXN];
  for (int i = 0; i < n; ++i) xt[i] = x[i] + dt * a_b21 * k1[i];
  or_plant_derivative(plant, p_in, p_out, xt, u, k2);
  for (int i = 0; i < n; ++i) xt[i] = x[i] + dt * a_b31 * k1[i] + dt * a_b32 * k2[i];
  or_plant_derivative(plant, p_in, p_out, xt, u, k3);
  for (int i = 0; i < n; ++i)
    xt[i] = x[i] + dt * a_b41 * k1[i] + dt * a_b42 * k2[i] + dt * a_b43 * k3[i];
  or_plant_derivative(plant, p_in, p_out, xt, u, k4);
  for (int i = 0; i < n; ++i)
    xt[i] = x[i] + dt * a_b51 * k1[i] + dt * a_b52 * k2[i] + dt * a_b53 * k3[i] +
            dt * a_b54 * k4[i];
  or_plant_derivative(plant, p_in, p_out, xt, u, k5);
  for (int i = 0; i < n; ++i)
    xt[i] = x[i] + dt * a_b61 * k1[i] + dt * a_b62 * k2[i] + dt * a_b63 * k3[i] +
            dt * a_b64 * k4[i] + dt * a_b65 * k5[i];
  or_plant_derivative(plant, p_in, p_out, xt, u, k6);
  for (int i = 0; i < n; ++i)
    out[i] = x[i] + dt * a_c1 * k1[i] + dt * a_c3 * k3[i] + dt * a_c4 * k4[i] +
             dt * a_c5 * k5[i] + dt * a_c6 * k6[i];
  or_plant_derivative(plant, p_in, p_out, out, u, k7);
  for (int i = 0; i < n; ++i)
    xerr[i] = dt * dc1 * k1[i] + dt * dc3 * k3[i] + dt * dc4 * k4[i] + dt * dc5 * k5[i] +
              dt * dc6 * k6[i] + dt * dc7 * k7[i];
}

int or_sim_interval(int plant, double p_in, double p_out, const double* u_full, double* x,
                    double t, double t_end, double* dt_io, double eps_abs, double eps_rel) {
  int n, ni, no, nci;
  if (or_plant_dims(plant, &n, &ni, &no, &nci)) return -1;
  double dxdt[OR_SIM_MAXN], xnew[OR_SIM_MAXN], dxnew[OR_SIM_MAXN], xerr[OR_SIM_MAXN];
  double dt = *dt_io;
  or_plant_derivative(plant, p_in, p_out, x, u_full, dxdt); /* fresh stepper: initialize */
  int count = 0;
  while (t_end - t > DBL_EPSILON) {
    if (count >= 500) { /* max_step_checker: 500 steps between observer calls */
      *dt_io = dt;
      return -2;
    }
    if ((t + dt) - t_end > DBL_EPSILON) dt = t_end - t;
    int fails = 0;
    for (;;) {
      dopri5_step(plant, p_in, p_out, u_full, n, x, dxdt, dt, xnew, dxnew, xerr);
      double acc = 0;
      for (int i = 0; i < n; ++i) {
        const double e = fabs(xerr[i]) / (eps_abs + eps_rel * (1.0 * fabs(x[i]) + dt * fabs(dxdt[i])));
        acc += e * e;
      }
      double err = sqrt(acc);
      if (err > 1.0) {
        const double f = 0.9 * pow(err, -1.0 / 3.0);
        dt *= f > 0.2 ? f : 0.2;
        if (++fails >= 500) {
          *dt_io = dt;
          return -1;
        }
        continue;
      }
      t += dt;
      if (err < 0.5) {
        const double lo = pow(5.0, -5.0);
        if (err < lo) err = lo;
        dt *= 0.9 * pow(err, -1.0 / 5.0);
      }
      memcpy(x, xnew, sizeof(double) * n);
      memcpy(dxdt, dxnew, sizeof(double) * n);
      break;
    }
    ++count;
  }
  *dt_io = dt;
  return count;
}

void or_time_delay(int n_inputs, const int32_t* delays, double* ring, int32_t* cur,
                   const double* u_next, double* u_out) {
  int index_delay_states = 0;
  for (int i = 0; i < n_inputs; ++i) {
    if (delays[i] == 0) {
      u_out[i] = u_next[i];
    } else {
      index_delay_states += delays[i];
      u_out[i] = ring[cur[i]];
      ring[cur[i]] = u_next[i];
      cur[i]++;
      if (cur[i] == index_delay_states) cur[i] -= delays[i];
    }
  }
}

void or_time_delay_init(int n_inputs, const int32_t* delays, double* ring, int32_t* cur) {
  int sum = 0;
  for (int i = 0; i < n_inputs; ++i) {
    cur[i] = sum;
    sum += delays[i];
  }
  for (int k = 0; k < sum; ++k) ring[k] = 0.0;
}

void or_plant_input(int n_inputs, int n_control, const int32_t* control_index,
                    const double* u_offset, const double* u_control, double* u_full) {
  for (int k = 0; k < n_inputs; ++k) u_full[k] = u_offset[k];
  for (int i = 0; i < n_control; ++i) u_full[control_index[i]] += u_control[i];
}
