// Per-sub-controller observer and receding-horizon update on the GPU
// (SURVEY.md §8(f) row 2): with these, a full closed-loop control step
//   observe a posteriori -> linearise at x_hat -> build -> K Jacobi
//   iterations -> observe a priori + u_old update
// stays on the device, the observer state resident in HBM between steps.
//
//   Observer::ObserveAPosteriori            libs/observer.cc:27-44 (in produce.hip)
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
// Instantiated for the two plants (ns = 11 / 10, four outputs and inputs):
// with compile-time dims every load is issued up front and the few
// cross-lane values (dx head, the innovation, the adjusted inputs) move by
// lane shuffles, so a wave pays about one memory round trip.  Arithmetic order, and the two exact
// elisions (the zero products of C's identity block and of Aorig * 0), match
// the oracle (oracle/or_observer.c) term for term.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_internal.h"
#include "observer_body.h"

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

// a posteriori (ObserveAPosteriori, libs/observer.cc:27-44): fused into the
// per-QP producer (produce.hip, cmpc_observe_step), which runs it on the same
// 16-lane rows before linearising at the updated x_hat.

// a priori + u_old update, four QPs per wave (one 16-lane row each).
// The delay blocks of dx are rings: block k's logical state i (i < D - 1,
// D its input's delay) is stored at blk[k] + (i + rot[k]) mod (D - 1), with
// rot the number of a-priori steps since cmpc_observer_init.  The reference's
// shift (AComposite::Aaug: slot k <- the block's first state, a state <- its
// successor, the last state <- du' of the input, BComposite::Baug) is then a
// read of the first state and a write of du' over it, the ring advancing by
// one: 4 + 2 nd entries per QP written instead of the whole aug part (78 for
// the reference plants).  cmpc_get/set_observer_state present the rows in
// the logical order.  Every source value is loaded before any store.
template <int NS, int NUT>
__global__ __launch_bounds__(64 * kWaves) void cmpc_obs_prior_kernel(ObserverParams P) {
  const int q_raw = (blockIdx.x * kWaves + (threadIdx.x >> 6)) * 4 + ((threadIdx.x & 48) >> 4);
  obs_prior_row<NS, NUT>(P, q_raw, threadIdx.x & 63);
}

}  // namespace

// The a-priori kernel's shape for n_aug delay-block entries per QP: one
// 16-lane row per QP whatever the delays (the delay blocks are rings, see
// cmpc_obs_prior_kernel); 0 if a QP's states or inputs do not fit a row.
int cmpc_obs_prior_shape(int n_aug, int nd, int nu_tot) {
  (void)n_aug;
  return (nd <= 16 && nu_tot <= 16) ? 4 : 0;
}

// The observer kernels instantiated below: both compressor plants (ns 11 /
// 10), four outputs and four disturbance states, four inputs.  cmpc_set_observer
// checks the same predicate, so an unsupported shape fails at set-up rather
// than at the first cmpc_observe_step / cmpc_observe_apply.
bool cmpc_obs_supported(int ns, int n_out, int ndist, int n_aug, int nd, int nu_tot) {
  return (ns == 11 || ns == 10) && n_out == 4 && ndist == 4 && nu_tot == 4 &&
         cmpc_obs_prior_shape(n_aug, nd, nu_tot) > 0;
}

int cmpc_launch_observer(const ObserverParams& P, int mode, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (P.nqp <= 0) return 0;
  const int grid = (P.nqp + kWaves - 1) / kWaves;
  switch (mode) {
    case CMPC_OBS_INIT:
      hipLaunchKernelGGL(cmpc_obs_init_kernel, dim3(grid), dim3(64 * kWaves), 0, s, P);
      return 0;
    case CMPC_OBS_PRIOR: {
      if (!cmpc_obs_supported(P.ns, P.n_out, P.ndist, P.ntot - P.nobs, P.nd, P.nu_tot)) return -1;
      const int g = (P.nqp + 4 * kWaves - 1) / (4 * kWaves);
      if (P.ns == 11)
        cmpc_launch((cmpc_obs_prior_kernel<11, 4>), dim3(g), dim3(64 * kWaves), 0, s, P);
      else if (P.ns == 10)
        cmpc_launch((cmpc_obs_prior_kernel<10, 4>), dim3(g), dim3(64 * kWaves), 0, s, P);
      else
        return -1;
      return 0;
    }
  }
  return -1;
}
