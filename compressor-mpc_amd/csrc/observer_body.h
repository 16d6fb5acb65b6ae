// The observer's a-priori update of one QP slot on one 16-lane DPP row
// (cmpc_obs_prior_kernel, observer.hip; and the tail of the one-launch
// control step, cmpc_kernels.hip): ObserveAPriori (libs/observer.cc:8-22)
// with the own first move (other inputs zero, nerve_center.h:323-328), then
// u_old += du (distributed_controller.h:145-152).  q_raw = the row's slot
// (rows past the batch keep the wave's shuffles), lane64 = lane in the wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_internal.h"

#ifndef CMPC_WAVE_SYNC
#define CMPC_WAVE_SYNC()                                      \
  do {                                                        \
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");    \
    __builtin_amdgcn_wave_barrier();                          \
  } while (0)
#endif

template <int NS, int NUT>
__device__ __forceinline__ void obs_prior_row(const ObserverParams& P, int q_raw, int lane64) {
  static_assert(NS <= 16 && NUT <= 16, "a QP's 16-lane row holds a state row per lane and every input");
  const int lane = lane64 & 15, base = lane64 & 48;
  const int nobs = P.nobs, nd = P.nd;
  // delay tables in registers (compile-time indices: a runtime-indexed
  // kernel-argument read is a dependent memory load)
  int dl[NUT], din[NUT], blk[NUT], rot[NUT];
#pragma unroll
  for (int i = 0; i < NUT; ++i) {
    dl[i] = P.delay[i];
    din[i] = P.dinput[i];
    blk[i] = P.blk[i];
    rot[i] = P.rot[i];
  }
  // (a per-lane choice among uniform values: a select chain; written out on
  // scalars, since inside the one-launch control step the compiler turned a
  // chain over a local array into a scratch table)
#define CMPC_PICK(a, k)                                   \
  ([&]() {                                                \
    int v_ = a[0];                                        \
    _Pragma("unroll") for (int i_ = 1; i_ < NUT; ++i_) {  \
      const int c_ = a[i_];                               \
      v_ = ((k) == i_) ? c_ : v_;                         \
    }                                                     \
    return v_;                                            \
  }())
  const bool valid = q_raw < P.nqp;  // (an idle row keeps the wave's shuffles)
  const int q = valid ? q_raw : P.nqp - 1;
  double* st = P.obs + (size_t)q * P.obs_len;
  double* dx = st + NS;
  const double* rec = P.lin + (size_t)q * P.rec_len;
  double* uo = P.u_old + (size_t)q * NUT;
  // lanes < nu_tot: u_old, du = own first move (others zero, nerve_center.h:323-328),
  // or the caller's full input change (DistributedController::UpdateU(du))
  const int li = lane < NUT ? lane : 0;
  const double u0 = uo[li];
  const double du = P.du_full ? ((lane < NUT) ? P.du_full[(size_t)q * NUT + lane] : 0.0)
                              : ((lane < P.nu) ? P.du_old[(size_t)q * P.nV + lane] : 0.0);
  // lanes < nd: delayed-input slot, the block's first state (ring head), the
  // input's u_old
  const int lk = lane < nd ? lane : 0;
  const int ik = CMPC_PICK(P.dinput, lk);
  const int head = CMPC_PICK(P.blk, lk) + CMPC_PICK(P.rot, lk);
  const double slot = dx[nobs + lk];
  const double first = dx[head];
  const double useg = uo[ik];
  // lanes < ns: row of B (sub-controller input order) and f
  const int ls = lane < NS ? lane : 0;
  double brow[NUT];
#pragma unroll
  for (int i = 0; i < NUT; ++i) brow[i] = rec[P.off_B + ls * NUT + i];
  const double fl = rec[P.off_f + ls];
  // du' = du + u_old on delayed inputs (AdjustAppliedInput); dx' slots minus
  // u_old (AdjustFirstDelayedStates)
  const double dup = CMPC_PICK(P.delay, li) ? du + u0 : du;
  const double seg = slot - useg;
  double dupv[NUT];
#pragma unroll
  for (int i = 0; i < NUT; ++i) dupv[i] = __shfl(dup, base + i, 64);
  // states: (B du')[:ns] + (Adelay seg) + f
  double bsum = 0.0;
#pragma unroll
  for (int i = 0; i < NUT; ++i)
    if (!dl[i]) bsum += brow[i] * dupv[i];
  double tsum = 0.0;
#pragma unroll
  for (int k = 0; k < NUT; ++k) {
    const double sk = __shfl(seg, base + k, 64);
    double bk = brow[0];
#pragma unroll
    for (int i = 1; i < NUT; ++i) bk = (din[k] == i) ? brow[i] : bk;
    if (k < nd) tsum += bk * sk;
  }
  const double xn = (bsum + tsum) + fl;
  double last = dupv[0];  // du' of the block's input: its new last state
#pragma unroll
  for (int i = 1; i < NUT; ++i) last = (ik == i) ? dupv[i] : last;
  CMPC_WAVE_SYNC();  // all loads above have completed before the first store
  if (!valid) return;
  if (lane < NS) dx[lane] = xn;
  if (lane < nd) {
    dx[nobs + lane] = first;  // slot k <- first state of block k
    dx[head] = last;          // the ring advances: this entry becomes the last state
  }
  // UpdateU: u_old += du (cmpc_observe_apply: own inputs, the others add zero)
  if (lane < NUT) uo[lane] = u0 + du;
}
