// MI355X (gfx950) kernels of the condensed-QP hot path.
//
// build  : AdjustAllDelayedStates + GeneratePrediction + GenerateDistributedQP
//          + GenerateQP (libs/aug_lin_sys.cc:260-334, include/aug_lin_sys.h:141-154,
//          include/distributed_solver.h:83-94, libs/mpc_qp_solver.cc:16-40)
//          for one QP per wavefront, prediction matrices never materialised.
// solve  : K Jacobi iterations of ApplyOtherInput + SolveQP
//          (include/nerve_center.h:146-172, include/distributed_solver.h:98-103,
//          libs/mpc_qp_solver.cc:42-75) for one QP per lane, the sub-controllers
//          of a scenario in adjacent lanes exchanging plans by lane shuffles.
//
// Build-kernel layout (one QP = one wave64 = four 16-lane DPP rows):
//   rows o < ny : row o of  P_i = L_W' C A^i        (L_W L_W' = ywt)
//                 lane j < ns          : P_i[o][j]             (broadcast source)
//                 lane ns + c          : P_i[o] . B_c          (raw Markov column c)
//                 lane ns + nu_tot     : z_i[o]                 (free response row)
//   row 3       : free response x_{i+1} = A x_i + f + Adelay w_i  (lanes j < ns)
//                 lanes ns + o         : (L_W' C x_{i+1})[o] + kappa[o] - yhat_i[o]
// One step of both chains is ns v_fmac_f64_dpp (row_newbcast) instructions.
// Because W is folded into P (W = L_W L_W'), H, G and f are plain sums over
// rows o and steps i of products of per-lane values: each step adds
// nV*m DPP-broadcast FMAs into accumulators that live in the Markov lanes,
// and one cross-row reduction at the end yields H (exactly symmetric),
// G = Su' W Su_other and f.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_internal.h"
#include "dpp_blocks.inc"

// ---------------------------------------------------------------------------
// build kernel
// ---------------------------------------------------------------------------
template <int NS, int NY, int NU, int M>
__global__ __launch_bounds__(64 * CMPC_BUILD_WAVES) void cmpc_build_kernel(BuildParams P) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int NV = NU * M;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q_raw = blockIdx.x * CMPC_BUILD_WAVES + wave;
  const bool active = q_raw < P.nqp;
  const int q = active ? q_raw : P.nqp - 1;
  const int row = lane >> 4, col = lane & 15;
  const int s = q % P.S;
  const int nu_tot = P.nu_tot, ND = P.nd, Dmax = P.dmax;
  const double* rec = P.lin + (size_t)q * P.rec_len;
  const double* cfg = P.cfg + (size_t)s * P.co.len;
  const double* uold = P.u_old + (size_t)q * nu_tot;
  const double* lwt = cfg + P.co.lwt;
  double* wl = smem + wave * P.lds_per_wave;  // w[t*ND + k]
  double* ring = wl + Dmax * ND;              // ring[(kd*NY + o)*Dmax + pos]

  // delay-line inputs, AdjustAllDelayedStates applied (include/aug_lin_sys.h:141-154)
  for (int e = lane; e < Dmax * ND; e += 64) {
    const int t = e / ND, k = e - t * ND;
    double v = 0.0;
    if (t < P.dlen[k]) {
      const double x = (t == 0) ? rec[P.off_x + P.ndist + k] : rec[P.off_x + P.boff[k] + t - 1];
      v = x - uold[P.dinput[k]];
    }
    wl[e] = v;
  }
  for (int e = lane; e < ND * NY * Dmax; e += 64) ring[e] = 0.0;
  __syncthreads();

  const int nobs = P.nobs;
  const double* A = rec + P.off_A;
  const double* Bin = rec + P.off_B;
  const double* Cs = rec + P.off_C;
  const double* xh = rec + P.off_f;
  const bool prow = row < NY;
  const bool srow = row == 3;

  // per-lane operands of the broadcast FMA
  double m[NS];
  double pv = 0.0, xadd = 0.0;
  double ad[CMPC_ND_MAX];
#pragma unroll
  for (int k = 0; k < CMPC_ND_MAX; ++k) ad[k] = 0.0;
#pragma unroll
  for (int l = 0; l < NS; ++l) {
    double v = 0.0;
    if (prow) {
      if (col < NS) v = A[l * NS + col];
      else if (col < NS + nu_tot) v = Bin[l * nu_tot + (col - NS)];
    } else if (srow) {
      if (col < NS) {
        v = A[col * NS + l];
      } else if (col < NS + NY) {
        const int o = col - NS;
        for (int o2 = o; o2 < NY; ++o2) v += lwt[o * NY + o2] * Cs[o2 * nobs + l];
      }
    }
    m[l] = v;
  }
  if (prow && col < NS) {
    for (int o2 = row; o2 < NY; ++o2) pv += lwt[row * NY + o2] * Cs[o2 * nobs + col];
  }
  if (srow && col < NS) {
    for (int k = 0; k < ND && k < CMPC_ND_MAX; ++k) ad[k] = Bin[col * nu_tot + P.dinput[k]];
    xadd = xh[col];
    double x1 = xh[col];
    for (int k = 0; k < ND && k < CMPC_ND_MAX; ++k) x1 += ad[k] * wl[k];
    pv = x1;  // x_1 = f + Adelay w_0  (x_0 = 0)
  }
  if (srow && col >= NS && col < NS + NY) {
    const int o = col - NS;
    const double* xa = rec + P.off_x;
    const double* yp = rec + P.off_y;
    for (int o2 = o; o2 < NY; ++o2) {
      double dist = 0.0;
      for (int d = 0; d < P.ndist; ++d) dist += Cs[o2 * nobs + NS + d] * xa[d];
      xadd += lwt[o * NY + o2] * (dist + yp[o2]);
    }
  }

  // Markov / z lanes
  const int c_in = col - NS;
  const bool mlane = prow && col >= NS && col < NS + nu_tot;
  const bool zlane = prow && col == NS + nu_tot;
  const int D = mlane ? P.delay[c_in] : 0;
  const int kd = mlane ? P.dindex[c_in] : -1;
  const bool rlane = mlane && D > 0;
  double* rbase = ring + (rlane ? (kd * NY + row) * Dmax : 0);
  int rpos = 0;
  double hist[M], ssum = 0.0;
#pragma unroll
  for (int k = 0; k < M; ++k) hist[k] = 0.0;
  double acc[NV * M];
#pragma unroll
  for (int k = 0; k < NV * M; ++k) acc[k] = 0.0;
  const double* yhat = cfg + P.co.yhat;
  const int oz = (col >= NS && col < NS + NY) ? col - NS : 0;
  const int zsrc = 48 + NS + (row < NY ? row : 0);

  for (int r = 0; r < P.p; ++r) {
    double a0 = 0.0, a1 = 0.0;
    prop_dpp<NS>(pv, m, a0, a1);
    const double qv = a0 + a1;
    double simx = qv + xadd;
    if (r + 1 < Dmax) {
#pragma unroll
      for (int k = 0; k < CMPC_ND_MAX; ++k)
        if (k < ND) simx += ad[k] * wl[(r + 1) * ND + k];
    }
    const double zq = qv + xadd - yhat[r * NY + oz];
    pv = srow ? simx : qv;
    double hv = qv;
    if (rlane) {
      const double old = rbase[rpos];
      rbase[rpos] = qv;
      hv = old;
      rpos = (rpos + 1 == D) ? 0 : rpos + 1;
    }
    const double zval = __shfl(zq, zsrc, 64);
#pragma unroll
    for (int k = M - 1; k > 0; --k) hist[k] = hist[k - 1];
    hist[0] = hv;
    ssum += hist[M - 1];
    double v[M];
#pragma unroll
    for (int k = 0; k < M; ++k) {
      const double mv = (k < M - 1) ? hist[k] : ssum;
      v[k] = mlane ? mv : ((zlane && k == 0) ? zval : 0.0);
    }
    accum_dpp<NS, NU, M>(v, acc);
  }

  // reduce over the ny rows and store row 0 of lanes ns .. ns + nu_tot
  double tot[NV * M];
#pragma unroll
  for (int k = 0; k < NV * M; ++k) {
    double t = acc[k];
    for (int o = 1; o < NY; ++o) t += __shfl(acc[k], (lane + 16 * o) & 63, 64);
    tot[k] = t;
  }
  if (active && row == 0 && col >= NS && col <= NS + nu_tot) {
    double* out = P.qp + (size_t)q * P.qp_len;
    const int c = col - NS;
    const int nuo = nu_tot - NU, nVo = M * nuo;
    const double* uwt = cfg + P.co.uwt;
    if (c < NU) {
#pragma unroll
      for (int a = 0; a < NV; ++a)
#pragma unroll
        for (int k = 0; k < M; ++k) {
          const int b = k * NU + c;
          const double rw = (a / NU == k) ? uwt[(a % NU) * NU + c] : 0.0;
          out[a * NV + b] = tot[a * M + k] + rw;
        }
    } else if (c < nu_tot) {
#pragma unroll
      for (int a = 0; a < NV; ++a)
#pragma unroll
        for (int k = 0; k < M; ++k) out[NV * NV + NV + a * nVo + k * nuo + (c - NU)] = tot[a * M + k];
    } else {
#pragma unroll
      for (int a = 0; a < NV; ++a) out[NV * NV + a] = tot[a * M];
    }
  }
}

#include "qp_solver.h"

// ---------------------------------------------------------------------------
// Jacobi iterate kernel (lane per QP)
// ---------------------------------------------------------------------------
template <int N, int NU, int NVO>
__global__ __launch_bounds__(CMPC_SOLVE_THREADS) void cmpc_solve_kernel(SolveParams P) {
  constexpr int M = N / NU;
  constexpr int NVOA = NVO > 0 ? NVO : 1;
  constexpr int SM1 = NVO / N;  // other sub-controllers per scenario
  const int q_raw = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = q_raw < P.nqp;
  const int q = active ? q_raw : P.nqp - 1;
  const int s = q % P.S;
  const int lane = threadIdx.x & 63;
  const int base_lane = lane - s;
  const double* rec = P.qp + (size_t)q * P.qp_len;
  const double* cfg = P.cfg + (size_t)s * P.co.len;

  double H[N][N], f[N], G[N][NVOA];
#pragma unroll
  for (int a = 0; a < N; ++a)
#pragma unroll
    for (int b = 0; b < N; ++b) H[a][b] = rec[a * N + b];
#pragma unroll
  for (int a = 0; a < N; ++a) f[a] = rec[N * N + a];
#pragma unroll
  for (int a = 0; a < N; ++a)
#pragma unroll
    for (int c = 0; c < NVOA; ++c) G[a][c] = (NVO > 0) ? rec[N * N + N + a * NVO + c] : 0.0;

  Qp<N, NU> qp;
  double uo[NU];
#pragma unroll
  for (int c = 0; c < NU; ++c) uo[c] = P.u_old[(size_t)q * P.nu_tot + c];
#pragma unroll
  for (int mv = 0; mv < M; ++mv)
#pragma unroll
    for (int c = 0; c < NU; ++c) {
      qp.lb[mv * NU + c] = cfg[P.co.lower + c] - uo[c];
      qp.ub[mv * NU + c] = cfg[P.co.upper + c] - uo[c];
      qp.lbA[mv * NU + c] = cfg[P.co.rlower + c];
      qp.ubA[mv * NU + c] = cfg[P.co.rupper + c];
    }
  const bool pd = hinv_of<N>(H, qp.Hinv);
  double hmax = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) hmax = fabs(H[i][i]) > hmax ? fabs(H[i][i]) : hmax;
  const double tol_d = TOL_D * (1.0 + hmax);

  uint32_t ws = P.ws[q];
  double x[N];
  QpOut o;
  if (P.init) {  // InitializeQPProblem: cold solve of the step QP, status ignored
    qp_solve<N, NU>(qp, pd, tol_d, f, 0u, CMPC_NWSR_MAX, x, o);
    if (active) P.ws[q] = o.ws;
    return;
  }
  double dprev[N];
#pragma unroll
  for (int a = 0; a < N; ++a) dprev[a] = P.du_old[(size_t)q * N + a];
  for (int k = 0; k < P.K; ++k) {
    double fk[N];
#pragma unroll
    for (int a = 0; a < N; ++a) fk[a] = f[a];
    if (NVO > 0) {
      double dother[NVOA];
#pragma unroll
      for (int rk = 0; rk < SM1; ++rk) {
        const int s2 = rk + (rk >= s ? 1 : 0);
#pragma unroll
        for (int mv = 0; mv < M; ++mv)
#pragma unroll
          for (int c = 0; c < NU; ++c)
            dother[mv * (SM1 * NU) + rk * NU + c] = __shfl(dprev[mv * NU + c], base_lane + s2, 64);
      }
      // f_k = f + (Su_other du_other)' W Su  ==  f + G du_other
#pragma unroll
      for (int a = 0; a < N; ++a) {
        double t = fk[a];
#pragma unroll
        for (int c = 0; c < NVOA; ++c) t = t + G[a][c] * dother[c];
        fk[a] = t;
      }
    }
    qp_solve<N, NU>(qp, pd, tol_d, fk, ws, CMPC_NWSR_MAX, x, o);
    ws = o.ws;
#pragma unroll
    for (int a = 0; a < N; ++a) dprev[a] = x[a];
    if (active && P.trace) {
      uint32_t* tr = reinterpret_cast<uint32_t*>(P.trace + ((size_t)q * P.K + k) * 16);
#pragma unroll
      for (int t = 0; t < 4; ++t) tr[t] = o.tr[t];
      P.ntrace[(size_t)q * P.K + k] = o.ntrace;
    }
  }
  if (!active) return;
  P.ws[q] = ws;
  if (P.K > 0) {
    P.status[q] = o.status;
    P.nwsr[q] = o.nchg;
  }
#pragma unroll
  for (int a = 0; a < N; ++a) {
    P.du[(size_t)q * N + a] = dprev[a];
    P.du_old[(size_t)q * N + a] = dprev[a];
  }
  if (P.flags & CMPC_APPLY_MOVE) {
#pragma unroll
    for (int c = 0; c < NU; ++c) P.u_old[(size_t)q * P.nu_tot + c] = uo[c] + dprev[c];
  }
}

// standalone batched solve (parity and KKT tests)
template <int N, int NU>
__global__ __launch_bounds__(CMPC_SOLVE_THREADS) void cmpc_qp_batch_kernel(QpBatchParams P) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P.nqp) return;
  double H[N][N], g[N];
  Qp<N, NU> qp;
#pragma unroll
  for (int a = 0; a < N; ++a) {
#pragma unroll
    for (int b = 0; b < N; ++b) H[a][b] = P.H[(size_t)q * N * N + a * N + b];
    g[a] = P.g[(size_t)q * N + a];
    qp.lb[a] = P.lb[(size_t)q * N + a];
    qp.ub[a] = P.ub[(size_t)q * N + a];
    qp.lbA[a] = P.lbA[(size_t)q * N + a];
    qp.ubA[a] = P.ubA[(size_t)q * N + a];
  }
  const bool pd = hinv_of<N>(H, qp.Hinv);
  double hmax = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) hmax = fabs(H[i][i]) > hmax ? fabs(H[i][i]) : hmax;
  double x[N];
  QpOut o;
  qp_solve<N, NU>(qp, pd, TOL_D * (1.0 + hmax), g, P.ws_in[q], P.max_chg, x, o);
#pragma unroll
  for (int a = 0; a < N; ++a) P.x[(size_t)q * N + a] = x[a];
  P.status[q] = o.status;
  P.nchg[q] = o.nchg;
  P.ws_out[q] = o.ws;
  P.ntrace[q] = o.ntrace;
  uint32_t* tr = reinterpret_cast<uint32_t*>(P.trace + (size_t)q * 16);
#pragma unroll
  for (int t = 0; t < 4; ++t) tr[t] = o.tr[t];
}

// ---------------------------------------------------------------------------
// launchers — explicit instantiation list (cf. the reference's *_list.h)
// ---------------------------------------------------------------------------
#define BUILD_CASE(NS_, NY_, NU_, M_)                                                  \
  if (ns == NS_ && ny == NY_ && nu == NU_ && m == M_) {                                \
    const int grid = (P.nqp + CMPC_BUILD_WAVES - 1) / CMPC_BUILD_WAVES;                \
    const size_t lds = sizeof(double) * (size_t)P.lds_per_wave * CMPC_BUILD_WAVES;     \
    hipLaunchKernelGGL((cmpc_build_kernel<NS_, NY_, NU_, M_>), dim3(grid),             \
                       dim3(64 * CMPC_BUILD_WAVES), lds, s, P);                        \
    return 0;                                                                          \
  }

int cmpc_launch_build(const BuildParams& P, int ns, int ny, int nu, int m, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  BUILD_CASE(11, 3, 2, 2)  // parallel coop        (ControlledOutputIndices <0,1,3>)
  BUILD_CASE(11, 2, 2, 2)  // parallel ncoop       (NCControlledOutputIndices)
  BUILD_CASE(11, 3, 4, 2)  // parallel centralized
  BUILD_CASE(10, 2, 2, 2)  // serial ncoop
  BUILD_CASE(11, 3, 2, 1)
  BUILD_CASE(11, 3, 2, 3)
  return -1;
}

#define SOLVE_CASE(N_, NU_, NVO_)                                                      \
  if (nV == N_ && nu == NU_ && nVo == NVO_) {                                          \
    const int grid = (P.nqp + CMPC_SOLVE_THREADS - 1) / CMPC_SOLVE_THREADS;            \
    hipLaunchKernelGGL((cmpc_solve_kernel<N_, NU_, NVO_>), dim3(grid),                 \
                       dim3(CMPC_SOLVE_THREADS), 0, s, P);                             \
    return 0;                                                                          \
  }

int cmpc_launch_solve(const SolveParams& P, int nV, int nu, int nVo, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  SOLVE_CASE(4, 2, 4)   // coop / ncoop, S = 2, m = 2
  SOLVE_CASE(8, 4, 0)   // centralized, m = 2
  SOLVE_CASE(2, 2, 2)   // m = 1
  SOLVE_CASE(6, 2, 6)   // m = 3
  return -1;
}

int cmpc_launch_qp_batch(const QpBatchParams& P, int n, int nu, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int grid = (P.nqp + CMPC_SOLVE_THREADS - 1) / CMPC_SOLVE_THREADS;
  if (n == 4 && nu == 2) {
    hipLaunchKernelGGL((cmpc_qp_batch_kernel<4, 2>), dim3(grid), dim3(CMPC_SOLVE_THREADS), 0, s, P);
    return 0;
  }
  if (n == 8 && nu == 4) {
    hipLaunchKernelGGL((cmpc_qp_batch_kernel<8, 4>), dim3(grid), dim3(CMPC_SOLVE_THREADS), 0, s, P);
    return 0;
  }
  return -1;
}
