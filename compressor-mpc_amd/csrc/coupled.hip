// Sub-controller-sharded cooperative iteration:
// S_total sub-controllers per scenario spread over the ranks, S_local on this
// one.  Between iterations the ranks all-gather every sub-controller's move
// plan (RCCL, driven by the caller: cmpc/coupled.py); this kernel is one
// Jacobi iteration for the local QPs:
//   f_k = f + G_ext du_other      (ApplyOtherInput, include/distributed_solver.h:98-103,
//                                  with du_other = all other sub-controllers' plans in
//                                  global order, nerve_center.h:280-285)
//   du  = SolveQP(H, f_k)         (libs/mpc_qp_solver.cc:42-75), warm-started
// G_ext (nV x (S_total-1) nV per QP) is stored element-major ([element][qp]) so
// the lane-per-QP reads coalesce; the gathered plans are rank-major
// ([rank][scenario][local sub-controller][nV]), as all_gather_into_tensor
// lays them out.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_internal.h"
#include "qp_solver.h"

namespace {

template <int N, int NU>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void cmpc_coupled_kernel(CoupledParams P) {
  constexpr int M = N / NU;
  const int q_raw = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = q_raw < P.nqp;
  const int q = active ? q_raw : P.nqp - 1;
  const int b = q / P.S_local, sl = q - b * P.S_local;
  const int sg = P.s_offset + sl;  // global sub-controller index
  const int s_cfg = q % P.S_cfg;
  const double* rec = P.qp + (size_t)q * P.qp_len;
  const double* cfg = P.cfg + (size_t)s_cfg * P.co.len;

  double H[N][N], f[N];
#pragma unroll
  for (int a = 0; a < N; ++a)
#pragma unroll
    for (int c = 0; c < N; ++c) H[a][c] = rec[a * N + c];
#pragma unroll
  for (int a = 0; a < N; ++a) f[a] = rec[N * N + a];

  Qp<N, NU, NU> qp;
  double uo[NU];
#pragma unroll
  for (int c = 0; c < NU; ++c) uo[c] = P.u_old[(size_t)q * P.nu_tot + c];
#pragma unroll
  for (int c = 0; c < NU; ++c) {
    qp.lb[c] = cfg[P.co.lower + c] - uo[c];
    qp.ub[c] = cfg[P.co.upper + c] - uo[c];
    qp.lbA[c] = cfg[P.co.rlower + c];
    qp.ubA[c] = cfg[P.co.rupper + c];
  }
  qp.tolerances();
  const bool pd = hinv_of<N>(H, qp.Hinv);
  double hmax = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) hmax = fabs(H[i][i]) > hmax ? fabs(H[i][i]) : hmax;
  const double tol_d = TOL_D * (1.0 + hmax);

  // f_k = f + G_ext du_other (other sub-controllers in global order).  The
  // loop runs over G_ext's column blocks jj (the same for every lane, so each
  // element read is one contiguous row segment of the wave's QPs) and maps
  // jj to the other controller j (skipping this one); four blocks per trip
  // keep 64 G_ext loads per lane in flight.  The sum order (j, then a, then
  // v) is unchanged.
  const int nvo = (P.S_total - 1) * N;
  double fk[N];
#pragma unroll
  for (int a = 0; a < N; ++a) fk[a] = f[a];
  const size_t rs = (size_t)N * P.nqp;  // stride of one column block (N rows of G_ext)
  const double* gq = P.G_ext + q;
#pragma unroll 4
  for (int jj = 0; jj < P.S_total - 1; ++jj) {
    const int j = jj < sg ? jj : jj + 1;
    const int rj = j / P.S_local, slj = j - rj * P.S_local;
    const double* dj = P.du_all + (((size_t)rj * P.B + b) * P.S_local + slj) * N;
    double d[N];
#pragma unroll
    for (int v = 0; v < N; ++v) d[v] = dj[v];
#pragma unroll
    for (int a = 0; a < N; ++a)
#pragma unroll
      for (int v = 0; v < N; ++v)
        fk[a] = fk[a] + gq[(size_t)a * nvo * P.nqp + jj * rs + (size_t)v * P.nqp] * d[v];
  }

  double x[N];
  QpOut o;
  qp_solve<N, NU>(qp, pd, tol_d, fk, P.ws[q], CMPC_NWSR_MAX, x, o);
  if (!active) return;
  P.ws[q] = o.ws;
  P.status[q] = o.status;
  P.nwsr[q] = o.nchg;
#pragma unroll
  for (int a = 0; a < N; ++a) {
    P.du[(size_t)q * N + a] = x[a];
    if (P.du_out) P.du_out[(size_t)q * N + a] = x[a];
  }
  if (P.flags & CMPC_APPLY_MOVE) {  // UpdateUOld (nerve_center.h:313-328), end of the step
#pragma unroll
    for (int a = 0; a < N; ++a) P.du_old[(size_t)q * N + a] = x[a];
#pragma unroll
    for (int c = 0; c < NU; ++c) P.u_old[(size_t)q * P.nu_tot + c] = uo[c] + x[c];
  }
  (void)M;
}

}  // namespace

int cmpc_launch_coupled(const CoupledParams& P, int n, int nu, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int grid = (P.nqp + 255) / 256;
  if (n == 4 && nu == 2) {
    cmpc_launch((cmpc_coupled_kernel<4, 2>), dim3(grid), dim3(256), 0, s, P);
    return 0;
  }
  return -1;
}
