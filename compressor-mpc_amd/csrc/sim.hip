// Batched plant simulation on the GPU: the harness's
// SimulationSystem for B scenarios at once, one lane per scenario, so a
// closed loop (plant -> observer -> QP build -> Jacobi iterations -> input
// delay line -> plant) never leaves the device.
//
//   SimulationSystem::Integrate    include/simulation_system.h:108-116:
//     odeint integrate_const with controlled_runge_kutta<runge_kutta_dopri5>,
//     one observation interval per call (the harness's callback runs the
//     controller between intervals); step size carried per scenario;
//     error norm = the reference's 2-norm override (:121-133)
//   SimulationSystem::SetInput     :67-70 (TimeDelay::GetDelayedInput,
//                                  include/time_delay.h:41-58, + GetPlantInput :82-88)
//   SimulationSystem::GetOutput    :79
// The arithmetic order is the oracle's (oracle/or_sim.c), which reproduces
// the reference's recorded trajectories to their printed 6 digits.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_internal.h"
#include "plant_model.h"

namespace {

template <int PLANT>
struct PlantF {
  static constexpr int ns = PLANT == CMPC_PLANT_PARALLEL ? 11 : 10;
  static constexpr int ni = PLANT == CMPC_PLANT_PARALLEL ? 9 : 8;
  __device__ static void f(double p_in, double p_out, const double* x, const double* u, double* dx) {
    if (PLANT == CMPC_PLANT_PARALLEL)
      cmpc_plant::parallel_derivative(p_in, p_out, x, u, dx);
    else
      cmpc_plant::serial_derivative(p_in, p_out, x, u, dx);
  }
};

// Dormand-Prince 5(4) tableau (odeint runge_kutta_dopri5)
constexpr double b21 = 1.0 / 5.0;
constexpr double b31 = 3.0 / 40.0, b32 = 9.0 / 40.0;
constexpr double b41 = 44.0 / 45.0, b42 = -56.0 / 15.0, b43 = 32.0 / 9.0;
constexpr double b51 = 19372.0 / 6561.0, b52 = -25360.0 / 2187.0, b53 = 64448.0 / 6561.0,
                 b54 = -212.0 / 729.0;
constexpr double b61 = 9017.0 / 3168.0, b62 = -355.0 / 33.0, b63 = 46732.0 / 5247.0,
                 b64 = 49.0 / 176.0, b65 = -5103.0 / 18656.0;
constexpr double c1 = 35.0 / 384.0, c3 = 500.0 / 1113.0, c4 = 125.0 / 192.0,
                 c5 = -2187.0 / 6784.0, c6 = 11.0 / 84.0;
constexpr double dc1 = c1 - 5179.0 / 57600.0, dc3 = c3 - 7571.0 / 16695.0,
                 dc4 = c4 - 393.0 / 640.0, dc5 = c5 - -92097.0 / 339200.0,
                 dc6 = c6 - 187.0 / 2100.0, dc7 = -1.0 / 40.0;
constexpr double kEps = 2.220446049250313e-16;  // numeric_limits<double>::epsilon()
constexpr int kMaxSteps = 500;                  // odeint max_step_checker default

template <int PLANT>
__global__ __launch_bounds__(64) void cmpc_sim_kernel(SimParams P) {
  using F = PlantF<PLANT>;
  constexpr int N = F::ns, NI = F::ni;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P.B) return;
  // the status is sticky: a scenario that failed in an earlier interval
  // stays where it stopped (the reference's odeint throws and the run ends)
  // until cmpc_sim_reset clears it
  if (P.status[b]) return;
  double x[N], k1[N], u[NI];
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = P.x[(size_t)b * N + i];
#pragma unroll
  for (int i = 0; i < NI; ++i) u[i] = P.u_full[(size_t)b * NI + i];
  double dt = P.dt[b];
  double t = P.t;
  const double t_end = P.t_end;
  int status = 0, steps = 0;
  F::f(P.p_in, P.p_out, x, u, k1);  // a fresh stepper per interval: initialize
  while (t_end - t > kEps) {
    // odeint's max_step_checker: at most 500 steps between two observer calls
    // (every lane leaves the loop even when the step size collapses)
    if (++steps > kMaxSteps) {
      status = 2;
      break;
    }
    if ((t + dt) - t_end > kEps) dt = t_end - t;
    int fails = 0;
    for (;;) {
      double k2[N], k3[N], k4[N], k5[N], k6[N], k7[N], xt[N], xo[N];
#pragma unroll
      for (int i = 0; i < N; ++i) xt[i] = x[i] + dt * b21 * k1[i];
      F::f(P.p_in, P.p_out, xt, u, k2);
#pragma unroll
      for (int i = 0; i < N; ++i) xt[i] = x[i] + dt * b31 * k1[i] + dt * b32 * k2[i];
      F::f(P.p_in, P.p_out, xt, u, k3);
#pragma unroll
      for (int i = 0; i < N; ++i) xt[i] = x[i] + dt * b41 * k1[i] + dt * b42 * k2[i] + dt * b43 * k3[i];
      F::f(P.p_in, P.p_out, xt, u, k4);
#pragma unroll
      for (int i = 0; i < N; ++i)
        xt[i] = x[i] + dt * b51 * k1[i] + dt * b52 * k2[i] + dt * b53 * k3[i] + dt * b54 * k4[i];
      F::f(P.p_in, P.p_out, xt, u, k5);
#pragma unroll
      for (int i = 0; i < N; ++i)
        xt[i] = x[i] + dt * b61 * k1[i] + dt * b62 * k2[i] + dt * b63 * k3[i] + dt * b64 * k4[i] +
                dt * b65 * k5[i];
      F::f(P.p_in, P.p_out, xt, u, k6);
#pragma unroll
      for (int i = 0; i < N; ++i)
        xo[i] = x[i] + dt * c1 * k1[i] + dt * c3 * k3[i] + dt * c4 * k4[i] + dt * c5 * k5[i] +
                dt * c6 * k6[i];
      F::f(P.p_in, P.p_out, xo, u, k7);
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const double e = dt * dc1 * k1[i] + dt * dc3 * k3[i] + dt * dc4 * k4[i] + dt * dc5 * k5[i] +
                         dt * dc6 * k6[i] + dt * dc7 * k7[i];
        const double r = fabs(e) / (P.eps_abs + P.eps_rel * (1.0 * fabs(x[i]) + dt * fabs(k1[i])));
        acc += r * r;
      }
      double err = sqrt(acc);
      if (!(err == err) || err > 1.7976931348623157e308) {  // non-finite error norm
        status = 3;
        break;
      }
      if (err > 1.0) {  // reject: dt *= max(0.9 err^(-1/3), 0.2)
        const double f = 0.9 * pow(err, -1.0 / 3.0);
        dt *= f > 0.2 ? f : 0.2;
        if (++fails >= 500) {
          status = 1;
          break;
        }
        continue;
      }
      t += dt;  // accept
      if (err < 0.5) {
        const double lo = 0.00032;  // 5^-5
        if (err < lo) err = lo;
        dt *= 0.9 * pow(err, -1.0 / 5.0);
      }
      bool finite = true;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        x[i] = xo[i];
        k1[i] = k7[i];  // FSAL
        finite = finite && fabs(xo[i]) <= 1.7976931348623157e308;
      }
      if (!finite) status = 3;
      break;
    }
    if (status) break;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) P.x[(size_t)b * N + i] = x[i];
  P.dt[b] = dt;
  if (status) P.status[b] = status;
}

// SetInput: TimeDelay::GetDelayedInput then GetPlantInput (u_offset + delayed
// control input at ControlInputIndex).  Every scenario's delay line advances
// in step, so the cursors are the host's (P.cur) and the ring is slot-major:
// the read and the write of a slot coalesce across the scenarios of a wave.
__global__ __launch_bounds__(64) void cmpc_sim_input_kernel(SimInputParams P) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P.B) return;
  double out[CMPC_MAX_INPUTS];
  for (int i = 0; i < P.nc; ++i) {
    const double un = P.u_control[(size_t)b * P.nc + i];
    if (P.delay[i] == 0 || !P.use_delay) {
      out[i] = un;
    } else {
      double* slot = P.ring + (size_t)P.cur[i] * P.B + b;
      out[i] = *slot;
      *slot = un;
    }
  }
  double* uf = P.u_full + (size_t)b * P.ni;
  const double* off = P.u_offset + (size_t)b * P.ni;
  for (int k = 0; k < P.ni; ++k) uf[k] = off[k];
  for (int i = 0; i < P.nc; ++i) uf[P.cidx[i]] += out[i];
}

template <int PLANT>
__global__ __launch_bounds__(64) void cmpc_sim_output_kernel(const double* x, double* y, int B) {
  constexpr int N = PLANT == CMPC_PLANT_PARALLEL ? 11 : 10;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double xs[N], ys[4];
#pragma unroll
  for (int i = 0; i < N; ++i) xs[i] = x[(size_t)b * N + i];
  if (PLANT == CMPC_PLANT_PARALLEL)
    cmpc_plant::parallel_output(xs, ys);
  else
    cmpc_plant::serial_output(xs, ys);
#pragma unroll
  for (int o = 0; o < 4; ++o) y[(size_t)b * 4 + o] = ys[o];
}

// u_control[b][order[s][k]] += du[b*S + s][k] for the own inputs k < nu,
// sub-controllers in order (UpdateUOld's expander order)
__global__ __launch_bounds__(64) void cmpc_accumulate_kernel(AccumParams P) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P.B) return;
  double* u = P.u_control + (size_t)b * P.nu_tot;
  for (int s = 0; s < P.S; ++s)
    for (int k = 0; k < P.nu; ++k) {
      const int c = P.order[s][k];
      u[c] = u[c] + P.du[((size_t)b * P.S + s) * P.nV + k];
    }
}

}  // namespace

int cmpc_launch_accumulate(const AccumParams& P, void* stream) {
  if (P.B <= 0) return 0;
  hipLaunchKernelGGL(cmpc_accumulate_kernel, dim3((P.B + 63) / 64), dim3(64), 0, (hipStream_t)stream, P);
  return 0;
}

int cmpc_launch_sim(const SimParams& P, int plant, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (P.B <= 0) return 0;
  const int grid = (P.B + 63) / 64;
  if (plant == CMPC_PLANT_PARALLEL)
    hipLaunchKernelGGL(cmpc_sim_kernel<CMPC_PLANT_PARALLEL>, dim3(grid), dim3(64), 0, s, P);
  else if (plant == CMPC_PLANT_SERIAL)
    hipLaunchKernelGGL(cmpc_sim_kernel<CMPC_PLANT_SERIAL>, dim3(grid), dim3(64), 0, s, P);
  else
    return -1;
  return 0;
}

int cmpc_launch_sim_input(const SimInputParams& P, void* stream) {
  if (P.B <= 0) return 0;
  hipLaunchKernelGGL(cmpc_sim_input_kernel, dim3((P.B + 63) / 64), dim3(64), 0, (hipStream_t)stream, P);
  return 0;
}

int cmpc_launch_sim_output(int plant, const double* x, double* y, int B, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (B <= 0) return 0;
  const int grid = (B + 63) / 64;
  if (plant == CMPC_PLANT_PARALLEL)
    hipLaunchKernelGGL(cmpc_sim_output_kernel<CMPC_PLANT_PARALLEL>, dim3(grid), dim3(64), 0, s, x, y, B);
  else if (plant == CMPC_PLANT_SERIAL)
    hipLaunchKernelGGL(cmpc_sim_output_kernel<CMPC_PLANT_SERIAL>, dim3(grid), dim3(64), 0, s, x, y, B);
  else
    return -1;
  return 0;
}
