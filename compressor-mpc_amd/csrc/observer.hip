// Per-sub-controller observer and receding-horizon update on the GPU
// (SURVEY.md §8(f) row 2): with these, a full closed-loop control step
//   observe a posteriori -> linearise at x_hat -> build -> K Jacobi
//   iterations -> observe a priori + u_old update
// stays on the device, the observer state resident in HBM between steps.
//
//   Observer::ObserveAPosteriori            libs/observer.cc:27-44
//   x_ += (GenerateInitialQP)               libs/distributed_controller.cc:80
//   Observer::ObserveAPriori                libs/observer.cc:8-22, with
//     AdjustFirstDelayedStates / AdjustAppliedInput (include/aug_lin_sys.h:129-163),
//     AComposite / BComposite products      (libs/aug_lin_sys.cc:125-140, :204-226)
//   DistributedController::UpdateU          include/distributed_controller.h:145-152
//
// Observer state of QP slot q (doubles, QP-major, ObserverParams::obs_len each):
//   [x_hat ns][dx_aug ntot = ns + ndist + delay states][y_old n_out][C n_out x ns]
// C is the plant output matrix of the last linearisation (written by the
// producer), as the reference's observer reads it through p_auglinsys_.
//
// One wave per QP: the record and state rows are contiguous, so the lanes'
// loads coalesce; the few cross-lane values (dx head, the innovation, the
// adjusted inputs) pass through LDS.  Arithmetic order, and the two exact
// elisions (the zero products of C's identity block and of Aorig * 0), match
// the oracle (oracle/or_observer.c) term for term.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_internal.h"

namespace {

#define WAVE_SYNC()                                           \
  do {                                                        \
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");    \
    __builtin_amdgcn_wave_barrier();                          \
  } while (0)

constexpr int kWaves = 4;

// Initialize (libs/distributed_controller.cc:36-43): x_ = x_init, observer
// output y_old = y_init, augmented state dx_init (or zero)
__global__ __launch_bounds__(64 * kWaves) void cmpc_obs_init_kernel(ObserverParams P) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (q >= P.nqp) return;
  const int b = q / P.S;
  double* st = P.obs + (size_t)q * P.obs_len;
  if (lane < P.ns) st[lane] = P.x_init[(size_t)b * P.ns + lane];
  for (int e = lane; e < P.ntot; e += 64)
    st[P.ns + e] = P.dx_init ? P.dx_init[(size_t)q * P.ntot + e] : 0.0;
  if (lane < P.n_out) st[P.ns + P.ntot + lane] = P.y[(size_t)b * P.n_out + lane];
}

__global__ __launch_bounds__(64 * kWaves) void cmpc_obs_post_kernel(ObserverParams P) {
  __shared__ double sdx[kWaves][32];
  __shared__ double sv[kWaves][8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x * kWaves + wave;
  if (q >= P.nqp) return;  // (whole waves exit together)
  const int b = q / P.S, s = q - b * P.S;
  const int ns = P.ns, nobs = P.nobs, no = P.n_out;
  double* st = P.obs + (size_t)q * P.obs_len;
  double* dx = st + ns;
  double* yo = dx + P.ntot;
  const double* C = yo + no;
  const double* y = P.y + (size_t)b * no;
  const double* M = P.M + (size_t)s * nobs * no;
  double dxl = 0.0;
  if (lane < nobs) {
    dxl = dx[lane];
    sdx[wave][lane] = dxl;
  }
  WAVE_SYNC();
  // innovation v = (y - y_old) - C dx[:nobs]   (lane o)
  if (lane < no) {
    double t = 0.0;
    for (int j = 0; j < ns; ++j) t += C[lane * ns + j] * sdx[wave][j];
    if (lane < P.ndist) t = t + sdx[wave][ns + lane];
    sv[wave][lane] = (y[lane] - yo[lane]) - t;
  }
  WAVE_SYNC();
  // dx[:nobs] += M v   (lane k);  y_old = y;  x_ += dx[:ns]
  if (lane < nobs) {
    double acc = 0.0;
    for (int o = 0; o < no; ++o) acc += M[lane * no + o] * sv[wave][o];
    dxl = dxl + acc;
    dx[lane] = dxl;
    if (lane < ns) st[lane] = st[lane] + dxl;
  }
  if (lane < no) yo[lane] = y[lane];
}

__global__ __launch_bounds__(64 * kWaves) void cmpc_obs_prior_kernel(ObserverParams P) {
  __shared__ double sdup[kWaves][CMPC_MAX_INPUTS];
  __shared__ double sseg[kWaves][CMPC_MAX_INPUTS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x * kWaves + wave;
  if (q >= P.nqp) return;
  const int ns = P.ns, nobs = P.nobs, nut = P.nu_tot, nd = P.nd;
  double* st = P.obs + (size_t)q * P.obs_len;
  double* dx = st + ns;
  const double* rec = P.lin + (size_t)q * P.rec_len;
  double* uo = P.u_old + (size_t)q * nut;
  // du = own first move (others zero, nerve_center.h:323-328);
  // du' = du + u_old on delayed inputs (AdjustAppliedInput)
  double du = 0.0, u0 = 0.0;
  if (lane < nut) {
    u0 = uo[lane];
    du = (lane < P.nu) ? P.du_old[(size_t)q * P.nV + lane] : 0.0;
    double dup = du;
    if (P.delay[lane]) dup += u0;
    sdup[wave][lane] = dup;
  }
  // dx' delayed-input slots minus u_old (AdjustFirstDelayedStates)
  if (lane < nd) sseg[wave][lane] = dx[nobs + lane] - uo[P.dinput[lane]];
  // aug part (delayed-input slots and delay blocks), two elements per lane:
  // slot k <- first state of block k; a block state <- its successor; the
  // block's last state <- du' of its input (Baug).  Sources are loaded
  // before any store.
  double nv[2];
  int tgt[2], from_du[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int e = nobs + lane + 64 * h;
    tgt[h] = -1;
    from_du[h] = -1;
    nv[h] = 0.0;
    if (e < P.ntot) {
      tgt[h] = e;
      if (e < nobs + nd) {
        nv[h] = dx[P.blk[e - nobs]];
      } else {
        int k = 0;
        while (k + 1 < nd && e >= P.blk[k + 1]) ++k;
        const int i = P.dinput[k];
        if (e - P.blk[k] < P.delay[i] - 2) nv[h] = dx[e + 1];
        else from_du[h] = i;
      }
    }
  }
  WAVE_SYNC();
  // states: (B du')[:ns] + (Adelay seg) + f
  if (lane < ns) {
    const double* Br = rec + P.off_B + lane * nut;
    double bsum = 0.0;
    for (int i = 0; i < nut; ++i)
      if (!P.delay[i]) bsum += Br[i] * sdup[wave][i];
    double t = 0.0;
    for (int k = 0; k < nd; ++k) t += Br[P.dinput[k]] * sseg[wave][k];
    dx[lane] = (bsum + t) + rec[P.off_f + lane];
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (tgt[h] >= 0) dx[tgt[h]] = from_du[h] >= 0 ? sdup[wave][from_du[h]] : nv[h];
  // UpdateU: u_old += du (own inputs; the others add zero)
  if (lane < nut) uo[lane] = u0 + du;
}

}  // namespace

int cmpc_launch_observer(const ObserverParams& P, int mode, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (P.nqp <= 0) return 0;
  const int grid = (P.nqp + kWaves - 1) / kWaves;
  switch (mode) {
    case CMPC_OBS_INIT:
      hipLaunchKernelGGL(cmpc_obs_init_kernel, dim3(grid), dim3(64 * kWaves), 0, s, P);
      return 0;
    case CMPC_OBS_POST:
      hipLaunchKernelGGL(cmpc_obs_post_kernel, dim3(grid), dim3(64 * kWaves), 0, s, P);
      return 0;
    case CMPC_OBS_PRIOR:
      hipLaunchKernelGGL(cmpc_obs_prior_kernel, dim3(grid), dim3(64 * kWaves), 0, s, P);
      return 0;
  }
  return -1;
}
