// Device record producer: AugmentedLinearizedSystem::
// Update for every scenario of the batch, written straight into the lin
// records the build kernel reads, so a control step needs no host round trip.
//
//   continuous linearisation   plant_model.h (shared with the host producer)
//   DiscretizeRK4 (Taylor-4)   libs/aug_lin_sys.cc:232-255
//   record assembly            cmpc_plant_lin_record (plant.cpp) + the
//                              observer tail dx_aug and the controlled y
//
// One wave per scenario.  Lane 0 runs the scalar plant model into LDS; the
// 11x11 products of the discretisation are spread over the 64 lanes with the
// host's summation order (k ascending, separate multiply and add), and the S
// records of the scenario are written with lane-contiguous stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_internal.h"
#include "plant_model.h"

namespace {

// LDS hand-offs inside one wave: order the stores before the other lanes'
// loads (compiler and hardware, wavefront scope)
#define WAVE_SYNC()                                           \
  do {                                                        \
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");    \
    __builtin_amdgcn_wave_barrier();                          \
  } while (0)

constexpr int kWaves = 4;          // waves (scenarios) per workgroup
constexpr int kMat = 121;          // ns x ns, ns <= 11
constexpr int kWaveLds = 8 * kMat + 4 * 11 * 2 + 11 * 2 + 32;  // doubles per wave

// Z = X Y (n x n), entries spread over the wave: the host's mm order
__device__ __forceinline__ void mm_wave(int n, int lane, const double* X, const double* Y,
                                        double* Z) {
  for (int e = lane; e < n * n; e += 64) {
    const int i = e / n, j = e - i * n;
    double s = 0;
    for (int k = 0; k < n; ++k) s = s + X[i * n + k] * Y[k * n + j];
    Z[e] = s;
  }
}

template <int PLANT>
__global__ __launch_bounds__(64 * kWaves) void cmpc_produce_kernel(ProduceParams P) {
  __shared__ double lds[kWaves * kWaveLds];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.x * kWaves + wave;
  if (b >= P.B) return;  // whole wave exits together
  constexpr int ns = PLANT == CMPC_PLANT_PARALLEL ? 11 : 10;
  constexpr int ni = PLANT == CMPC_PLANT_PARALLEL ? 9 : 8;
  double* w = lds + wave * kWaveLds;
  double *A = w, *A2 = A + kMat, *A3 = A2 + kMat, *Ac = A3 + kMat, *Ad = Ac + kMat;
  double *Bc = Ad + kMat, *Bd = Bc + 44, *Cc = Bd + 44, *fc = Cc + 44, *fd = fc + 11;
  double *xs = fd + 11, *us = xs + 11;

  if (lane < ns) xs[lane] = P.x[(size_t)b * ns + lane];
  if (lane < ni) us[lane] = P.u_full[(size_t)b * ni + lane];
  WAVE_SYNC();
  if (lane == 0) {
    if (PLANT == CMPC_PLANT_PARALLEL)
      cmpc_plant::parallel_linearize(P.p_in, P.p_out, xs, us, A, Bc, Cc, fc);
    else
      cmpc_plant::serial_linearize(P.p_in, P.p_out, xs, us, A, Bc, Cc, fc);
  }
  WAVE_SYNC();

  // DiscretizeRK4: Ac = Ts I + Ts^2/2 A + Ts^3/6 A^2 + Ts^4/24 A^3,
  // Ad = I + Ac A, Bd = Ac B, fd = Ac f
  const double Ts = P.Ts;
  mm_wave(ns, lane, A, A, A2);
  WAVE_SYNC();
  mm_wave(ns, lane, A2, A, A3);
  WAVE_SYNC();
  for (int e = lane; e < ns * ns; e += 64) {
    const int r = e / ns, c = e - r * ns;
    Ac[e] = Ts * (r == c) + Ts * Ts / 2.0 * A[e] + Ts * Ts * Ts / 6.0 * A2[e] +
            Ts * Ts * Ts * Ts / 24.0 * A3[e];
  }
  WAVE_SYNC();
  mm_wave(ns, lane, Ac, A, Ad);
  for (int e = lane; e < ns * 4 + ns; e += 64) {
    if (e < ns * 4) {
      const int i = e / 4, j = e - i * 4;
      double s = 0;
      for (int k = 0; k < ns; ++k) s = s + Ac[i * ns + k] * Bc[k * 4 + j];
      Bd[e] = s;
    } else {
      const int i = e - ns * 4;
      double s = 0;
      for (int k = 0; k < ns; ++k) s = s + Ac[i * ns + k] * fc[k];
      fd[i] = s;
    }
  }
  WAVE_SYNC();
  if (lane < ns) Ad[lane * ns + lane] += 1.0;
  WAVE_SYNC();

  // records of the S sub-controllers of scenario b
  for (int s = 0; s < P.S; ++s) {
    const size_t q = (size_t)b * P.S + s;
    double* rec = P.lin + q * P.rec_len;
    for (int e = lane; e < P.rec_len; e += 64) {
      double v = 0.0;
      if (e >= P.off_A && e < P.off_A + ns * ns) {
        v = Ad[e - P.off_A];
      } else if (e >= P.off_B && e < P.off_B + ns * P.nu_tot) {
        const int r = (e - P.off_B) / P.nu_tot, c = e - P.off_B - r * P.nu_tot;
        v = Bd[r * 4 + P.input_order[s][c]];
      } else if (e >= P.off_C && e < P.off_C + P.ny * P.nobs) {
        const int o = (e - P.off_C) / P.nobs, k = e - P.off_C - o * P.nobs;
        const int oi = P.out_idx[s][o];
        v = (k < ns) ? Cc[oi * ns + k] : ((oi == k - ns) ? 1.0 : 0.0);
      } else if (e >= P.off_f && e < P.off_f + ns) {
        v = fd[e - P.off_f];
      } else if (e >= P.off_x && e < P.off_x + P.naug) {
        v = P.dx_aug ? P.dx_aug[q * P.naug + (e - P.off_x)] : 0.0;
      } else if (e >= P.off_y && e < P.off_y + P.ny) {
        v = P.y[(size_t)b * P.n_outputs + P.out_idx[s][e - P.off_y]];
      }
      rec[e] = v;
    }
  }
}

}  // namespace

int cmpc_launch_produce(const ProduceParams& P, int plant, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int grid = (P.B + kWaves - 1) / kWaves;
  if (plant == CMPC_PLANT_PARALLEL)
    hipLaunchKernelGGL(cmpc_produce_kernel<CMPC_PLANT_PARALLEL>, dim3(grid), dim3(64 * kWaves), 0,
                       s, P);
  else if (plant == CMPC_PLANT_SERIAL)
    hipLaunchKernelGGL(cmpc_produce_kernel<CMPC_PLANT_SERIAL>, dim3(grid), dim3(64 * kWaves), 0, s,
                       P);
  else
    return -1;
  return 0;
}
