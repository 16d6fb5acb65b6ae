// Jacobi iterate kernel for small batches: one QP per 16-lane DPP row
// (qp_solver_row.h), four QPs per wave.  The same K iterations of
// ApplyOtherInput + SolveQP as cmpc_solve_kernel (include/nerve_center.h:146-172,
// include/distributed_solver.h:98-103, libs/mpc_qp_solver.cc:42-75), the same
// results bit for bit; where cmpc_solve_kernel runs one QP per lane (a wave
// per 64 QPs, every QP a long scalar dependency chain), this kernel spreads
// each QP's H^-1 and its matrix-vector products over the row's lanes, which
// shortens the chain when the batch leaves most SIMDs idle anyway (SURVEY
// configs 2 and 5: 8 192 and 1 024 QPs).
//
// Lane l of row R (QP q = 4 * wave + R): row l of H, of G and of H^-1, entry l
// of f_k; the plan dprev (nV) and the solver's control state replicated in
// the row.  The S sub-controllers of a scenario are adjacent rows of one wave
// (S divides 4); the plan exchange of an iteration reads the other rows'
// lanes (ds_bpermute).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_internal.h"
#include "solve_rows.h"

namespace {

constexpr int kRowsPerBlock = CMPC_SOLVE_THREADS / 16;

template <int N, int NU, int NVO, bool TRACE, bool EXT>
__global__ __launch_bounds__(CMPC_SOLVE_THREADS) void cmpc_solve_rows_kernel(SolveParams P) {
  constexpr int NVOA = NVO > 0 ? NVO : 1;
  __shared__ double tsh[kRowsPerBlock][N * N];
  const int lane = threadIdx.x & 63;
  const int l = lane & 15;
  const int qrow = threadIdx.x >> 4;
  const int q_raw = blockIdx.x * kRowsPerBlock + qrow;
  const bool active = q_raw < P.nqp;
  const int q = active ? q_raw : P.nqp - 1;
  const int s = q % P.S;
  const int lr = l < N ? l : N - 1;
  const bool own = l < N;
  const double* rec = P.qp + (size_t)q * P.qp_len;

  double Hl[N];
#pragma unroll
  for (int c = 0; c < N; ++c) Hl[c] = own ? rec[lr * N + c] : 0.0;
  const double f_l = own ? rec[N * N + lr] : 0.0;
  double Gl[NVOA];
#pragma unroll
  for (int c = 0; c < NVOA; ++c) Gl[c] = (NVO > 0 && own) ? rec[N * N + N + lr * NVO + c] : 0.0;

  const int base_lane = (lane & ~15) - 16 * s;  // lane 0 of the scenario's first row
  rows_solve_qp<N, NU, NVO, TRACE, EXT>(P, q, active, s, l, base_lane, Hl, f_l, Gl, tsh[qrow]);
}

}  // namespace

#define SOLVE_ROWS_CASE(N_, NU_, NVO_)                                                  \
  if (nV == N_ && nu == NU_ && nVo == NVO_) {                                           \
    if (P.qp_len != N_ * N_ + N_ + N_ * NVO_) return -1;                                \
    const int grid = (P.nqp + kRowsPerBlock - 1) / kRowsPerBlock;                       \
    if (P.du_other) {                                                                   \
      if (NVO_ == 0 || P.trace) return -1;                                              \
      cmpc_launch((cmpc_solve_rows_kernel<N_, NU_, NVO_, false, (NVO_ > 0)>), dim3(grid), \
                  dim3(CMPC_SOLVE_THREADS), 0, s, P);                                   \
      return 0;                                                                         \
    }                                                                                   \
    if (P.trace)                                                                        \
      cmpc_launch((cmpc_solve_rows_kernel<N_, NU_, NVO_, true, false>), dim3(grid),     \
                  dim3(CMPC_SOLVE_THREADS), 0, s, P);                                   \
    else                                                                                \
      cmpc_launch((cmpc_solve_rows_kernel<N_, NU_, NVO_, false, false>), dim3(grid),    \
                  dim3(CMPC_SOLVE_THREADS), 0, s, P);                                   \
    return 0;                                                                           \
  }

// -1: not instantiated for these dimensions, or S does not divide the
// four rows of a wave (the plan exchange stays inside a wave)
int cmpc_launch_solve_rows(const SolveParams& P, int nV, int nu, int nVo, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (P.S < 1 || 4 % P.S) return -1;
  SOLVE_ROWS_CASE(4, 2, 4)   // coop / ncoop, S = 2, m = 2
  SOLVE_ROWS_CASE(8, 4, 0)   // centralized, m = 2
  SOLVE_ROWS_CASE(2, 2, 2)   // m = 1
  SOLVE_ROWS_CASE(6, 2, 6)   // m = 3
  return -1;
}
