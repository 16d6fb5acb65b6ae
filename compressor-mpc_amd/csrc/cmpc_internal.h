// Internal launch parameters shared by cmpc_abi.cpp (host) and
// cmpc_kernels.hip (device).  Not part of the public ABI.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cmpc.h"

// Kernel timing (cmpc_enable_timing).  cmpc_abi.cpp sets these events around
// a timed launch (null otherwise); the launchers hand them to
// hipExtLaunchKernelGGL, which stamps the kernel's own start and end into
// them from its dispatch packet.  hipEventRecord markers before and after
// each kernel cost ~7 us per bench step (tools/time_step_gaps.py).  One
// context per host thread (cmpc.h), hence thread_local.
struct LaunchEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local LaunchEvents cmpc_launch_events;
template <typename F, typename... A>
inline void cmpc_launch(F kernel, dim3 grid, dim3 block, size_t lds, hipStream_t stream, A... args) {
  if (cmpc_launch_events.start || cmpc_launch_events.stop)
    hipExtLaunchKernelGGL(kernel, grid, block, (std::uint32_t)lds, stream, cmpc_launch_events.start,
                          cmpc_launch_events.stop, 0u, args...);
  else  // the plain launch path: ~8 us of host time per hipExtLaunchKernel
        // call in the B = 1 step's --hip-trace (profiles/r4e_b1_hip_api_stats.csv)
    hipLaunchKernelGGL(kernel, grid, block, (std::uint32_t)lds, stream, args...);
}

// Resident workgroups per CU of `kernel` at `threads` x `lds` bytes, from the
// occupancy query, cached per (kernel, threads, lds): the query costs ~9 us of
// host time per call (B = 1 step --hip-trace), once per launch before.
// 0 when the query fails.  One context per host thread, hence thread_local.
template <typename F>
inline int cmpc_blocks_per_cu(F kernel, int threads, size_t lds) {
  struct Entry {
    const void* k;
    int threads;
    size_t lds;
    int blocks;
  };
  static thread_local Entry cache[32];
  static thread_local int n = 0;
  const void* key = reinterpret_cast<const void*>(kernel);
  for (int i = 0; i < n && i < 32; ++i)
    if (cache[i].k == key && cache[i].threads == threads && cache[i].lds == lds) return cache[i].blocks;
  int v = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kernel, threads, lds) != hipSuccess) v = 0;
  cache[n % 32] = Entry{key, threads, lds, v};
  ++n;
  return v;
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (device, kernel,
// size): a launcher that set it on every launch paid its host time per step
// (a config-5 step: 57 us of wall time per 41 us kernel).  The attribute
// belongs to the function object of the current device, so a host thread
// that drives contexts on two devices sets it on each.
inline void cmpc_allow_lds(const void* kernel, size_t bytes) {
  struct Entry {
    int dev;
    const void* k;
    size_t bytes;
  };
  static thread_local Entry cache[32];
  static thread_local int n = 0;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  for (int i = 0; i < n && i < 32; ++i)
    if (cache[i].dev == dev && cache[i].k == kernel && cache[i].bytes >= bytes) return;
  (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  cache[n % 32] = Entry{dev, kernel, bytes};
  ++n;
}

#define CMPC_ND_MAX 4            // delayed inputs supported by the build kernel
#define CMPC_BUILD_WAVES 4       // waves per build workgroup (one QP per wave at a time)
#ifndef CMPC_ROWS_U
#define CMPC_ROWS_U 5            // horizon unroll of the row build kernel (4 or 5; 5: p = 50 in whole blocks, +0.7%)
#endif
#ifndef CMPC_ROWS_U2
#define CMPC_ROWS_U2 10          // ... for ny = 2 (config 3: 211 -> 205 us; profiles/r6f_stride_u10_ab/)
#endif
// the row build kernel's horizon unroll for ny outputs (the kernel and its
// LDS layout, rows_layout.cpp, take it from here)
__host__ __device__ constexpr int cmpc_rows_unroll(int ny) { return ny == 2 ? CMPC_ROWS_U2 : CMPC_ROWS_U; }
#define CMPC_ROWS_NSEG 16        // loop segment bounds of the row build kernel
#define CMPC_REC_CHUNKS 3        // 16-byte lin-record chunks per lane (rec_len <= 384)
// QPs (= lanes) per solve workgroup: one wave, so a batch of fewer waves than
// CUs spreads one wave per CU (the CU's scalar unit and instruction fetch
// are shared by its waves): config 2 iterate (K = 9, 128 waves) 11.6 -> 9.8 us
// against 256; level at the bench size (profiles/r5h_solve_wg_ab.txt)
#ifndef CMPC_SOLVE_THREADS
#define CMPC_SOLVE_THREADS 64
#endif
#define CMPC_HOST_OUT_MAX_QP 64  // up to this many QPs: du/status/nWSR live in page-locked host memory
#ifndef CMPC_SOLVE_ROWS_MAX_QP
#define CMPC_SOLVE_ROWS_MAX_QP 16384  // CMPC_SOLVE_AUTO: the row solve kernel below this many QPs
#endif

// Per sub-controller configuration block in device memory (doubles):
//   [lwt  : ny*ny ]  L_W' with ywt = L_W L_W' (upper triangular)
//   [yhat : p*ny  ]  L_W' y_ref_r
//   [uwt  : nu*nu ]  input weight block of R = blkdiag_m(uwt)
//   [lower, upper, rate_lower, rate_upper : nu each]
struct CfgOffsets {
  int lwt, yhat, uwt, lower, upper, rlower, rupper, len;
};

// LDS layout of the row-layout build kernel (build_rows.hip), doubles.
// Block region: [zeros 16][yhat S x NY x yls (output-major)][lwt][uwt].
// Wave region : [hand-off 4 x LQ][C_hat 4 x NY x 16][w 4 x ND x WL].
// Hand-off area of one QP, in entries of NY doubles ([entry][output]): per
// input c at lo[c] a ring of U + 1 entries (undelayed) or m - 1 zero entries
// + max(0, p - D_c) values (delayed); then a dump area, the free-response z
// entries and a zero area (U entries each).
// A delayed input's line is a ring of D + m entries when its p - D values
// would need more (p > 2 D + 1): the writer and the two gather readers step
// back by ring[c] entries at each of their wrap steps (every ring[c] steps),
// which are loop segment bounds too (at most CMPC_ROWS_NSEG of them).  The C_hat rows overlay the hand-off areas: they are read in the
// prologue only, before the zero areas are written.
struct RowsLayout {
  int ok;                        // the row kernel can run these dimensions
  int lds_block, per_wave;
  int yl_off, yls, lw_off, uw_off;
  int LQ, lo[CMPC_MAX_INPUTS], dump_off, z_off, zr_off;
  int ring[CMPC_MAX_INPUTS];      // entries of a wrapping delayed line, 0: a plain line
  int ch_off, w_off, WL;
  int nseg, seg[CMPC_ROWS_NSEG];  // ascending distinct D, p - D and wrap steps inside (0, p)
  int U;                          // the kernel's horizon unroll (cmpc_rows_unroll)
};

struct SolveParams {
  const double* qp;
  const double* cfg;
  double* u_old;      // nqp * nu_tot
  double* du_old;     // nqp * nV
  uint32_t* ws;       // nqp
  double* du;         // nqp * nV
  int32_t* status;    // nqp
  int32_t* nwsr;      // nqp
  uint8_t* trace;     // nqp * K * 16 or null
  int32_t* ntrace;    // nqp * K or null
  int nqp, S, K, nu_tot, qp_len;
  CfgOffsets co;
  uint32_t flags;
  int init;           // 1: InitializeQPProblem (cold, f only, ws only)
  const double* du_other;  // nqp * nVo other controllers' plans (cmpc_get_input), or null:
                           // the in-scenario exchange of cmpc_iterate
};

struct BuildParams {
  const double* lin;     // nqp * rec_len
  const double* cfg;     // S * cfg.len
  const double* u_old;   // nqp * nu_tot
  double* qp;            // nqp * qp_len   [H nV*nV | f nV | G nV*nVo]
  int nqp, S, p, nu_tot, ndist, nd, dmax, rec_len, qp_len;
  int off_A, off_B, off_C, off_f, off_x, off_y, nobs;
  CfgOffsets co;
  int delay[CMPC_MAX_INPUTS];    // per input
  int dindex[CMPC_MAX_INPUTS];   // per input: delayed index kd or -1
  int dinput[CMPC_ND_MAX];       // per delayed index: input c
  int dlen[CMPC_ND_MAX];         // per delayed index: delay D
  int boff[CMPC_ND_MAX];         // per delayed index: offset of its shift block in dx_aug
  // LDS layout (doubles), computed on the host by build_lds_layout() so that
  // the per-step hand-off reads/writes are free of bank conflicts
  int lds_block;                 // block-shared: yhat (S x yl_stride), lwt, uwt, zeros
  int yl_stride;                 // per sub-controller yhat stride (multiple of 32)
  int lds_per_wave;              // per-wave region (multiple of 32)
  int line_off[CMPC_MAX_INPUTS]; // delay line of input c inside a row
  int line_rs;                   // delay-line row stride (one row per output)
  int w_off;                     // w table
  int zs_off;                    // free-response hand-off slots (NY x 4), or the
                                 // ny = 4 pre-pass z lines (NY x zl_stride)
  int zl_stride;
  int nbound;                    // distinct delays 0 < D < p, ascending (loop segments)
  int bound[CMPC_MAX_INPUTS];
  int grid;                      // workgroups needed (one QP per wave); launcher caps it
  int split;                     // cmpc_launch_build: the role-split kernel (ny <= 3)
  int cus;                       // compute units of the device
  RowsLayout rows;               // row-layout kernel (four QPs per wave)
  // fused step (cmpc_step on small batches): the K Jacobi iterations run in
  // the build kernel on the QPs it just built (solve_rows.h), with these
  // parameters (sv.qp unused: H, f, G stay in registers)
  SolveParams sv;
};


// Standalone batched solver (parity / KKT tests).  G (nqp * n * nvo) and d
// (nqp * nvo) non-null: the Jacobi iteration's map-form solve with g = f + G d
// (cmpc_qp_solve_batch_map); g is f then.
struct QpBatchParams {
  const double *H, *g, *lb, *ub, *lbA, *ubA;
  const uint32_t* ws_in;
  double* x;
  int32_t *status, *nchg, *ntrace;
  uint32_t* ws_out;
  uint8_t* trace;
  int nqp, max_chg;
  const double *G = nullptr, *d = nullptr;
  int nvo = 0;
};

// Device record producer (produce.hip): one scenario's plant linearisation
// -> its S lin records.
#define CMPC_MAX_S_PRODUCE 8
struct ProduceParams {
  double* lin;                  // B*S*rec_len, written
  const double* x;              // B*ns
  const double* u_full;         // B*n_inputs
  const double* dx_aug;         // B*S*naug or null (zeros)
  const double* y;              // B*n_outputs
  int B, S, rec_len, nu_tot, ny, nobs, naug, n_outputs;
  int off_A, off_B, off_C, off_f, off_x, off_y;
  double p_in, p_out, Ts;
  int input_order[CMPC_MAX_S_PRODUCE][CMPC_MAX_INPUTS];
  int out_idx[CMPC_MAX_S_PRODUCE][4];
  // per-QP mode (the observer's closed loop): one linearisation per QP slot
  // q at x + q * x_stride, dx_aug row stride dx_stride, and the plant's full
  // output matrix (n_outputs x ns) stored to c_out + q * c_stride
  int per_qp, x_stride, dx_stride, c_stride;
  double* c_out;
  // per-QP mode: dx_aug's delay blocks are rings (observer.hip): block k
  // spans dx_aug entries [rb[k], rb[k] + rlen[k]), logical entry i stored at
  // rb[k] + (i + rot[k]) mod rlen[k]
  int nring, rb[CMPC_ND_MAX], rlen[CMPC_ND_MAX], rot[CMPC_ND_MAX];
  // per-QP mode, cmpc_observe_step: the observer's a-posteriori update of the
  // slot (ObserveAPosteriori, in or_observe_post's arithmetic order) runs first in
  // the same kernel, x = the observer rows (x_hat, then dx of obs_ntot
  // entries, y_old, C): obs_M = S x nobs x n_outputs gains, or null
  const double* obs_M;
  double* obs;  // the observer rows (x above, writable)
  int obs_ntot;
};

// Observer kernels (observer.hip)
#define CMPC_OBS_INIT 0
#define CMPC_OBS_PRIOR 2
struct ObserverParams {
  double* obs;              // nqp * obs_len state rows
  const double* M;          // S * nobs * n_out observer gains
  const double* y;          // B * n_out plant outputs (init / post)
  const double* x_init;     // B * ns (init)
  const double* dx_init;    // nqp * ntot or null (init)
  const double* lin;        // step records (prior: B, f)
  const double* du_old;     // nqp * nV plans (prior)
  double* u_old;            // nqp * nu_tot (prior)
  const double* du_full;    // nqp * nu_tot applied input change (cmpc_update_u), or null:
                            // the own first move of du_old (cmpc_observe_apply)
  int nqp, S, ns, ndist, nobs, ntot, n_out, obs_len;
  int nu, nu_tot, nV, nd, rec_len, off_B, off_f;
  int delay[CMPC_MAX_INPUTS];   // per input (sub-controller order)
  int dinput[CMPC_MAX_INPUTS];  // k-th delayed input -> input index
  int blk[CMPC_MAX_INPUTS];     // first dx index of delay block k
  int rot[CMPC_MAX_INPUTS];     // ring position of block k's first state (step count mod D - 1)
};

// One-launch control step (cmpc_control_step, cmpc_kernels.hip): the
// producer (per-QP mode with the a-posteriori update), the fused build + K
// iterations and the observer's a-priori update of a small batch.  pr_off:
// the producer rows' LDS offset (doubles) after its element table.
struct ControlStepParams {
  BuildParams b;
  ProduceParams pr;
  ObserverParams ob;
  int pr_off;
  // one-workgroup launches: after the last phase, seq is stored to *done
  // (page-locked host memory) with a system-scope release, so the host can
  // wait for the results by polling instead of a stream synchronisation
  uint32_t* done;
  uint32_t seq;
};
int cmpc_launch_control_step(const ControlStepParams& C, int ns, int ny, int nu, int m, void* stream,
                             int* solver);

// One Jacobi iteration of the sub-controller-sharded cooperative loop
// (coupled.hip).
struct CoupledParams {
  const double* qp;       // nqp * qp_len (H, f from cmpc_build)
  const double* cfg;
  CfgOffsets co;
  double* u_old;          // nqp * nu_tot
  double* du_old;         // nqp * nV
  uint32_t* ws;
  double* du;             // nqp * nV (context buffer)
  double* du_out;         // nqp * nV caller buffer (the next all-gather's input) or null
  int32_t *status, *nwsr;
  const double* G_ext;    // [nV * (S_total-1) * nV][nqp], element-major
  const double* du_all;   // [world][B][S_local][nV], all-gathered plans
  int nqp, qp_len, nu_tot, S_cfg, S_total, S_local, s_offset, B;
  uint32_t flags;
};

// Kernel launchers (cmpc_kernels.hip, produce.hip, coupled.hip).  Return 0 or -1 (unsupported dims).
int cmpc_launch_build(const BuildParams& P, int ns, int ny, int nu, int m,
                      void* stream);
// Row-layout build kernel (build_rows.hip); -1 when not instantiated / not usable.
int cmpc_launch_build_rows(const BuildParams& P, int ns, int ny, int nu, int m,
                           void* stream);
// Fused step (step_rows.hip): the row build kernel running the K Jacobi
// iterations of its QPs itself (P.sv); -1 when not available.  *solver:
// the solver it runs (CMPC_SOLVE_ROWS or CMPC_SOLVE_LANE).
int cmpc_launch_step_rows(const BuildParams& P, int ns, int ny, int nu, int m, void* stream, int* solver);
// the same on the one-QP-per-wave build kernel (cmpc_kernels.hip)
int cmpc_launch_step_wave(const BuildParams& P, int ns, int ny, int nu, int m, void* stream, int* solver);
// Waves per workgroup the row kernel launches with for layout R (4, 2 or 1;
// 0: does not fit) (build_rows.hip).
int cmpc_rows_waves_per_group(const RowsLayout& R);
// workgroups of w waves per CU that the layout's LDS lets run at once
int cmpc_rows_resident_groups(const RowsLayout& R, int w);
// LDS layout of the row kernel, chosen by a bank-conflict model of its
// horizon loop (rows_layout.cpp); cached per dimension set, thread-safe.
void cmpc_rows_layout(const cmpc_dims& d, int nd, int nobs, int rec_len, RowsLayout* out);
// modelled extra LDS cycles per wave-step of the horizon loop for one wave
double cmpc_rows_layout_conflicts(const cmpc_dims& d, int nd, const RowsLayout& R, int wave);
int cmpc_launch_solve(const SolveParams& P, int nV, int nu, int nVo,
                      void* stream);
// Row-layout iterate kernel (solve_rows.hip): one QP per 16-lane row;
// -1 when not instantiated for these dimensions or S does not divide 4.
int cmpc_launch_solve_rows(const SolveParams& P, int nV, int nu, int nVo, void* stream);
int cmpc_launch_qp_batch(const QpBatchParams& P, int n, int nu, void* stream);
int cmpc_launch_qp_batch_map(const QpBatchParams& P, int n, int nu, int nvo, void* stream);
// the (n, nu[, nvo]) the two launchers above have instances for
bool cmpc_qp_batch_supported(int n, int nu);
bool cmpc_qp_batch_map_supported(int n, int nu, int nvo);
// Plant simulation (sim.hip)
struct SimParams {
  double* x;              // B * ns
  double* dt;             // B (controlled stepper's step, carried between intervals)
  const double* u_full;   // B * n_inputs
  int32_t* status;        // B or null (1: step-size control failed)
  int B;
  double t, t_end, eps_abs, eps_rel, p_in, p_out;
};
struct SimInputParams {
  const double* u_control;  // B * nc
  const double* u_offset;   // B * ni
  double* u_full;           // B * ni
  double* ring;             // ring_len * B, slot-major: slot k of every scenario is contiguous
  int B, nc, ni, ring_len, use_delay;
  int delay[CMPC_MAX_INPUTS];
  int cidx[CMPC_MAX_INPUTS];
  int cur[CMPC_MAX_INPUTS];  // ring slot of each delayed input (the same for every scenario)
};
struct AccumParams {
  const double* du;   // nqp * nV
  double* u_control;  // B * nu_tot
  int B, S, nu, nu_tot, nV;
  int order[CMPC_MAX_S_PRODUCE][CMPC_MAX_INPUTS];
};
int cmpc_launch_accumulate(const AccumParams& P, void* stream);
int cmpc_launch_sim(const SimParams& P, int plant, void* stream);
int cmpc_launch_sim_input(const SimInputParams& P, void* stream);
int cmpc_launch_sim_output(int plant, const double* x, double* y, int B, void* stream);

int cmpc_launch_produce(const ProduceParams& P, int plant, void* stream);
int cmpc_obs_prior_shape(int n_aug, int nd, int nu_tot);
bool cmpc_obs_supported(int ns, int n_out, int ndist, int n_aug, int nd, int nu_tot);
int cmpc_launch_observer(const ObserverParams& P, int mode, void* stream);
int cmpc_launch_coupled(const CoupledParams& P, int n, int nu, void* stream);
