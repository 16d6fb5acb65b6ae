/*
 * cmpc.h — C ABI of the MI355X-native condensed-QP hot path of
 * katie-jones/compressor-mpc (cooperative / non-cooperative / centralized
 * linear-time-varying MPC).
 *
 * Plain C, POD arguments only, int status returns (0 = ok, <0 = error; the
 * message is in cmpc_last_error()).  One context per (device, stream, host
 * thread); a context is not thread-safe.  All batched device buffers are
 * owned by the library; host arrays are owned by the caller.
 *
 * What each entry point replaces in the reference (paths relative to the
 * reference root):
 *
 *   cmpc_create            MpcQpSolver ctor  libs/mpc_qp_solver.cc:3-14,
 *                          DistributedController ctor libs/distributed_controller.cc:6-22,
 *                          NerveCenter ctor include/nerve_center.h:89-95
 *   cmpc_set_weights       MpcQpSolver::SetWeights include/mpc_qp_solver.h:62-80,
 *                          NerveCenter::SetWeights include/nerve_center.h:107-116
 *   cmpc_set_constraints   InputConstraints include/input_constraints.h:12-26
 *   cmpc_set_reference     MpcQpSolver::SetOutputReference include/mpc_qp_solver.h:94,
 *                          NerveCenter::SetOutputReference include/nerve_center.h:119-122
 *   cmpc_set_state         DistributedController::Initialize (u_old_) libs/distributed_controller.cc:27-67,
 *                          NerveCenter du_old_ include/nerve_center.h:73,94
 *   cmpc_upload_lin        AugmentedLinearizedSystem::Update result (A,B,C,f)
 *                          libs/aug_lin_sys.cc:145-177 + Observer state estimate
 *   cmpc_build             GenerateInitialQP libs/distributed_controller.cc:72-108 =
 *                          AdjustAllDelayedStates include/aug_lin_sys.h:141-154
 *                          + GeneratePrediction libs/aug_lin_sys.cc:260-334
 *                          + GenerateDistributedQP include/distributed_solver.h:83-94
 *                          + GenerateQP libs/mpc_qp_solver.cc:16-40
 *   cmpc_init_warmstart    MpcQpSolver::InitializeQPProblem libs/mpc_qp_solver.cc:77-101
 *   cmpc_iterate           Jacobi loop include/nerve_center.h:146-172 (SolveQPHelper :276-296,
 *                          DistributedController::GetInput include/distributed_controller.h:206-226,
 *                          ApplyOtherInput include/distributed_solver.h:98-103,
 *                          SolveQP libs/mpc_qp_solver.cc:42-75, UpdateUOld/SendUHelper
 *                          include/nerve_center.h:313-328)
 *   cmpc_step              cmpc_build + cmpc_iterate = NerveCenter::GetNextInputWithTiming
 *                          include/nerve_center.h:134-182
 *   cmpc_control_step      the same with the observer (ObserveAPosteriori, Update,
 *                          UpdateU: libs/observer.cc:8-44, libs/distributed_controller.cc:72-108,
 *                          include/distributed_controller.h:145-152) = GetNextInput
 *
 * The QP solver is this library's own warm-started dual active-set method
 * (qpOASES 3.2.0 SQProblem::hotstart is not vendored in the reference); it
 * keeps the reference's n_wsr_max = 10 cap (include/mpc_qp_solver.h:24) and
 * the zero-move fallback on any non-success (libs/mpc_qp_solver.cc:66-69).
 */
#ifndef CMPC_H
#define CMPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CMPC_MAX_INPUTS 8   /* nu_tot */
#define CMPC_MAX_NV 8       /* m * nu */
#define CMPC_MAX_NS 15      /* plant states (+ inputs <= 16 lanes) */
#define CMPC_NWSR_MAX 10    /* include/mpc_qp_solver.h:24 */

/* QP status words (per QP slot, last solve of the step) */
#define CMPC_QP_OK 0          /* qpOASES::SUCCESSFUL_RETURN */
#define CMPC_QP_MAX_NWSR 1    /* > n_wsr_max working-set changes -> zero move */
#define CMPC_QP_INFEASIBLE 2  /* -> zero move */
#define CMPC_QP_NOT_PD 3      /* Hessian not positive definite -> zero move */
#define CMPC_QP_NONFINITE 4   /* non-finite plan (NaN / infinite gradient) -> zero move */

/* cmpc_iterate / cmpc_step flags */
#define CMPC_APPLY_MOVE 1u    /* u_old += first move (UpdateUOld/SendUHelper) */
#define CMPC_TRACE 2u         /* record working-set change sequences */

/* Problem dimensions.  All sub-controllers of a context share them
 * (coop: every sub-controller has nu own inputs, nu_tot - nu other inputs). */
typedef struct cmpc_dims {
  int32_t ns;      /* plant states                   AugmentedLinearizedSystem::n_states */
  int32_t ndist;   /* disturbance/integrator states  n_disturbance_states */
  int32_t nu_tot;  /* plant control inputs           n_control_inputs */
  int32_t nu;      /* own inputs per sub-controller  n_sub_control_inputs */
  int32_t ny;      /* controlled outputs             ControlledOutputIndices::size */
  int32_t p;       /* prediction horizon */
  int32_t m;       /* move horizon */
  int32_t delay[CMPC_MAX_INPUTS]; /* Delays, per sub-controller-ordered input */
  int32_t S;       /* sub-controllers per scenario (NerveCenter pack size) */
  int32_t B;       /* independent scenarios in the batch */
} cmpc_dims;

/* Derived sizes and the packed per-QP input record ("lin record").
 * One record per QP slot q = b * S + s (scenario-major), doubles, row-major:
 *   [off_A ] Aorig   ns x ns        discrete A       (AComposite::Aorig)
 *   [off_B ] Bin     ns x nu_tot    column c = input c of this sub-controller's
 *                                   ordering: Borig column if delay[c]==0,
 *                                   Adelay column otherwise (BComposite/AComposite)
 *   [off_C ] Csel    ny x nobs      controlled rows of C = [Cplant | I_dist]
 *   [off_f ] fd      ns             discrete affine term (GetDerivative())
 *   [off_x ] dxaug   naug           observer augmented state tail: ndist
 *                                   disturbance, nd delayed-input slots, then
 *                                   per delayed input delay-1 shift states
 *                                   (raw: AdjustAllDelayedStates is applied here)
 *   [off_y ] yprev   ny             controlled part of the measured output
 * stride = rec_len (multiple of 8 doubles). */
typedef struct cmpc_layout {
  int32_t nd, n_delay_states, naug, nobs, ntot, nV, nuo, nVo;
  int32_t off_A, off_B, off_C, off_f, off_x, off_y, rec_len;
} cmpc_layout;

/* Fill *L from *d.  Returns 0, or <0 if the dimensions are unsupported. */
int cmpc_layout_of(const cmpc_dims* d, cmpc_layout* L);

typedef struct cmpc_ctx cmpc_ctx;

/* Context on HIP device `device`, all work on a private non-blocking stream
 * unless cmpc_set_stream() is called. */
int cmpc_create(cmpc_ctx** ctx, const cmpc_dims* dims, int device);
int cmpc_destroy(cmpc_ctx* ctx);
int cmpc_set_stream(cmpc_ctx* ctx, void* hip_stream);
const char* cmpc_last_error(void);
int cmpc_get_layout(const cmpc_ctx* ctx, cmpc_layout* L);

/* Per sub-controller configuration (s = 0..S-1), shared by all scenarios. */
int cmpc_set_weights(cmpc_ctx* ctx, int s, const double* uwt /* nu x nu */,
                     const double* ywt /* ny x ny */);
int cmpc_set_constraints(cmpc_ctx* ctx, int s, const double* lower,
                         const double* upper, const double* rate_lower,
                         const double* rate_upper); /* each nu */
int cmpc_set_reference(cmpc_ctx* ctx, int s, const double* y_ref /* p x ny */);

/* Mutable per-slot state.  Any pointer may be NULL (left unchanged).
 * u_old  : B*S*nu_tot  sub-controller's u_old_ in its own input ordering
 * du_old : B*S*nV      previous step's move plans (NerveCenter::du_old_)
 * ws     : B*S         warm-start working-set words */
int cmpc_set_state(cmpc_ctx* ctx, const double* u_old, const double* du_old,
                   const uint32_t* ws);
int cmpc_get_state(cmpc_ctx* ctx, double* u_old, double* du_old, uint32_t* ws);
/* Bind external device-resident state arrays (shapes as above, on the ctx
 * device, 8-byte aligned): every later call reads and updates them in place
 * of the context's own state, as if they were the context's.  All three
 * pointers, or all NULL to re-bind the context's own buffers.  Lets one
 * context serve several sets of B scenarios in rotation (cmpc_bind_lin for
 * their records), each set warm-started from its own previous step, as each
 * reference controller hot-starts its own QProblem (libs/mpc_qp_solver.cc:42-75). */
int cmpc_bind_state(cmpc_ctx* ctx, double* u_old_device, double* du_old_device,
                    uint32_t* ws_device);

/* Inputs: B*S lin records from host memory (H2D copy on the ctx stream), or
 * written in place by a device-side producer through cmpc_lin_device(). */
int cmpc_upload_lin(cmpc_ctx* ctx, const double* lin_host);
void* cmpc_lin_device(cmpc_ctx* ctx);
/* Copy the context's own record buffer to the host (B*S*rec_len doubles),
 * e.g. to inspect what cmpc_produce_lin wrote. */
int cmpc_download_lin(cmpc_ctx* ctx, double* lin_host);
/* Bind an external device-resident record array (B*S*rec_len doubles on the
 * ctx device, 16-byte aligned, e.g. the output of a device-side producer);
 * NULL re-binds the context's own buffer.  Takes effect for the next
 * cmpc_build.  cmpc_bind_lin and cmpc_bind_state check that each pointer is
 * device memory of the context's device inside an allocation of the
 * required size, once per (pointer, size) and context: re-binding a buffer
 * freed and re-allocated at the same address is not re-checked. */
int cmpc_bind_lin(cmpc_ctx* ctx, const double* lin_device);

/* Hot path. */
int cmpc_build(cmpc_ctx* ctx);
/* Build-kernel selection for cmpc_build (same H, f, G within rounding):
 * CMPC_BUILD_ROWS four QPs per wave, one per 16-lane DPP row (m <= 2, LDS
 * fits); CMPC_BUILD_WAVE one QP per wave (every instantiated dimension set);
 * CMPC_BUILD_SPLIT one QP per two waves, the DPP chain in one and the gather
 * in the other (every ny, the ny = 4 simulation pre-pass included);
 * CMPC_BUILD_AUTO (default) rows where its LDS fits and the batch fills the
 * SIMDs, else split up to one QP per SIMD, else wave.  WAVE and SPLIT give
 * the same QP bit for bit; ROWS sums in another order (agreement within
 * rounding, 1e-11 relative). */
#define CMPC_BUILD_AUTO 0
#define CMPC_BUILD_WAVE 1
#define CMPC_BUILD_ROWS 2
#define CMPC_BUILD_SPLIT 3
int cmpc_set_build_variant(cmpc_ctx* ctx, int variant);
/* The build kernel the last cmpc_build, cmpc_step or cmpc_control_step
 * launched (CMPC_BUILD_WAVE, CMPC_BUILD_ROWS or CMPC_BUILD_SPLIT), 0 before the
 * first build, <0 on a null context. */
int cmpc_last_build_kernel(cmpc_ctx* ctx);
/* Solve-kernel selection for cmpc_iterate / cmpc_init_warmstart /
 * cmpc_get_input (the same results bit for bit):
 * CMPC_SOLVE_LANE one QP per lane (large batches); CMPC_SOLVE_ROWS one QP per
 * 16-lane DPP row, its H^-1 and matrix-vector products spread over the row
 * (batches that leave most SIMDs idle; needs S | 4); CMPC_SOLVE_AUTO
 * (default) rows for nV >= 6 below CMPC_SOLVE_ROWS_MAX_QP QPs and for smaller
 * nV up to four QPs per SIMD, where available. */
#define CMPC_SOLVE_AUTO 0
#define CMPC_SOLVE_LANE 1
#define CMPC_SOLVE_ROWS 2
int cmpc_set_solve_variant(cmpc_ctx* ctx, int variant);
/* The solve kernel the last iterate / init / get-input launched. */
int cmpc_last_solve_kernel(cmpc_ctx* ctx);
/* cmpc_step as one launch (the build kernel runs the K Jacobi iterations of
 * the QPs it built, H, f, G handed over in registers; the same results bit
 * for bit as cmpc_build + cmpc_iterate with the row solve kernel):
 * CMPC_STEP_SPLIT two launches; CMPC_STEP_FUSED one (an error where no fused
 * kernel exists for the dimensions); CMPC_STEP_AUTO (default) fused for
 * nV >= 6 from one QP per CU up to CMPC_SOLVE_ROWS_MAX_QP QPs, two launches
 * otherwise (measured faster there: DESIGN.md §3.0). */
#define CMPC_STEP_AUTO 0
#define CMPC_STEP_SPLIT 1
#define CMPC_STEP_FUSED 2
int cmpc_set_step_variant(cmpc_ctx* ctx, int variant);
/* 1 if the last cmpc_step ran fused, 0 if split, <0 on a null context. */
int cmpc_last_step_fused(cmpc_ctx* ctx);
/* Diagnostic (no GPU needed): the row kernel's LDS layout for *dims as
 * cmpc_build chooses it.  Writes the bank-conflict model's extra LDS cycles
 * per wave-step of the horizon loop (wave 0) for the packed layout (regions
 * back to back) and for the chosen one, and the chosen layout's LDS bytes per
 * workgroup.  Returns 0, or -1 if the row kernel cannot run these dims. */
int cmpc_rows_lds_model(const cmpc_dims* dims, double* packed_cycles, double* chosen_cycles,
                        int32_t* lds_bytes);
int cmpc_init_warmstart(cmpc_ctx* ctx);
int cmpc_iterate(cmpc_ctx* ctx, int K, uint32_t flags);
int cmpc_step(cmpc_ctx* ctx, int K, uint32_t flags);
int cmpc_synchronize(cmpc_ctx* ctx);

/* Results of the last cmpc_iterate (any pointer may be NULL).
 * du: B*S*nV move plans; status/nwsr: B*S of the last solve. */
int cmpc_download(cmpc_ctx* ctx, double* du, int32_t* status, int32_t* nwsr);
/* The condensed QPs of the last cmpc_build (parity/debug):
 * H: B*S*nV*nV (row-major), f: B*S*nV, G: B*S*nV*nVo (G = Su' W Su_other). */
int cmpc_download_qp(cmpc_ctx* ctx, double* H, double* f, double* G);
/* Working-set change sequences of the last traced cmpc_iterate:
 * trace: B*S*K*16 bytes (bit7 add, bit6 upper side, bits0-5 constraint j;
 * 0xFF terminates), ntrace: B*S*K counts. */
int cmpc_download_trace(cmpc_ctx* ctx, uint8_t* trace, int32_t* ntrace);

/* Per-kernel device time (HIP events stamped by the kernel's own dispatch,
 * opt-in).  enable: 0 off, 1 every kernel, or an OR of CMPC_TIME_ONLY(k)
 * to time only those kernels (the others launch without events). */
#define CMPC_KERNEL_BUILD 0
#define CMPC_KERNEL_ITERATE 1         /* cmpc_iterate, cmpc_coupled_iterate */
#define CMPC_KERNEL_PRODUCE 2         /* cmpc_produce_lin; cmpc_observe_step (a posteriori + per-QP producer, one kernel) */
#define CMPC_KERNEL_OBSERVE_POST 3    /* no launches since the a posteriori update runs in the producer (kept for the numbering) */
#define CMPC_KERNEL_OBSERVE_PRIOR 4   /* cmpc_observe_apply */
#define CMPC_KERNEL_STEP 5            /* cmpc_step as one fused build + K-iteration launch */
#define CMPC_KERNEL_COUNT 6
#define CMPC_TIME_ONLY(kernel) (2 << (kernel))
int cmpc_enable_timing(cmpc_ctx* ctx, int enable);
int cmpc_kernel_time(cmpc_ctx* ctx, int kernel, double* total_ms,
                     int64_t* launches);
/* Time only every stride-th launch of each timed kernel (1, the default:
 * every launch).  An event-stamped launch costs the stream a few us after
 * the kernel; sampling keeps the mean launch time while the untimed launches
 * run as in production.  Counted from the last cmpc_enable_timing. */
int cmpc_set_timing_stride(cmpc_ctx* ctx, int stride);

/* The batched QP solver alone, on device `device`, for host arrays of nqp
 * QPs of size n (nu inputs per move): H nqp*n*n, g/lb/ub/lbA/ubA nqp*n,
 * ws_in nqp; outputs x nqp*n, status/nchg nqp, ws_out nqp, trace nqp*16,
 * ntrace nqp.  (Parity and known-answer tests of the solver.) */
int cmpc_qp_solve_batch(int device, int n, int nu, int nqp, const double* H,
                        const double* g, const double* lb, const double* ub,
                        const double* lbA, const double* ubA,
                        const uint32_t* ws_in, int max_chg, double* x,
                        int32_t* status, int32_t* nchg, uint32_t* ws_out,
                        uint8_t* trace, int32_t* ntrace);
/* The same for one Jacobi-iteration solve (the map form of DESIGN.md §4):
 * g = f + G d with G nqp*n*nvo (row-major per QP, columns in the order of the
 * other sub-controllers' plans d, nqp*nvo: controller-major within each move,
 * include/nerve_center.h:283-285).  Replaces ApplyOtherInput + SolveQP of
 * DistributedSolver::UpdateAndSolveQP (include/distributed_solver.h:69-80,
 * 98-103; libs/mpc_qp_solver.cc:42-75); bit-identical to the solves inside
 * cmpc_iterate / cmpc_get_input.  nvo = 0: cmpc_qp_solve_batch. */
int cmpc_qp_solve_batch_map(int device, int n, int nu, int nvo, int nqp,
                            const double* H, const double* f, const double* G,
                            const double* d, const double* lb, const double* ub,
                            const double* lbA, const double* ubA,
                            const uint32_t* ws_in, int max_chg, double* x,
                            int32_t* status, int32_t* nchg, uint32_t* ws_out,
                            uint8_t* trace, int32_t* ntrace);

/* Upstream producer (host, untimed): AugmentedLinearizedSystem::Update for the
 * reference plants — linearise the plant at (x, u_full), discretise
 * (Taylor-4, libs/aug_lin_sys.cc:232-255), reorder the inputs by input_order
 * (ControlInputIndices) and fill off_A..off_f of one lin record for the
 * controlled outputs out_idx[0..ny-1].  plant: 0 parallel, 1 serial. */
#define CMPC_PLANT_PARALLEL 0
#define CMPC_PLANT_SERIAL 1
int cmpc_plant_dims(int plant, int* ns, int* n_inputs, int* n_outputs,
                    int* n_control_inputs);
int cmpc_plant_default(int plant, double* x, double* u_full);
int cmpc_plant_output(int plant, const double* x, double* y);
int cmpc_plant_lin_record(int plant, double p_in, double p_out, double Ts,
                          const double* x, const double* u_full,
                          const int32_t* input_order, const int32_t* out_idx,
                          const cmpc_dims* dims, double* record);

/* One stand-alone sub-controller per QP slot (the reference's per-object
 * DistributedController API; the NerveCenter path is cmpc_iterate /
 * cmpc_observe_apply):
 *   cmpc_get_input  DistributedController::GetInput(&du, du_last)
 *                   (include/distributed_controller.h:206-226): f_k = f + G du_last
 *                   (ApplyOtherInput, distributed_solver.h:98-103) and one
 *                   warm-started SolveQP; du_last: device, B*S*nVo doubles per
 *                   slot, the other controllers' plans controller-major, then
 *                   move, then input (nerve_center.h:283-285); NULL for a full
 *                   (centralized, nVo = 0) controller: SolveQP(qp_, u_old_).
 *                   Results through cmpc_download (du, status, nwsr); flags as
 *                   cmpc_iterate (CMPC_APPLY_MOVE: u_old += first move)
 *   cmpc_update_u   DistributedController::UpdateU(du) (:145-152): ObserveAPriori
 *                   (du, u_old_) and u_old_ += du with the caller's full input
 *                   change du (device, B*S*nu_tot, the slot's input order);
 *                   NerveCenter passes only the own inputs, the others zero
 *                   (nerve_center.h:323-328; cmpc_observe_apply does that)
 * The _host variants take host arrays (staged on the context's stream). */
int cmpc_get_input(cmpc_ctx* ctx, const double* du_last, uint32_t flags);
int cmpc_get_input_host(cmpc_ctx* ctx, const double* du_last, uint32_t flags);
int cmpc_update_u(cmpc_ctx* ctx, const double* du_full);
int cmpc_update_u_host(cmpc_ctx* ctx, const double* du_full);

/* Sub-controller-sharded cooperative iteration.
 * S_total sub-controllers per scenario are spread over the ranks, S_local of
 * them on this context (QP slot q = scenario * S_local + local index; global
 * index s_offset + local index); the context's H, f come from cmpc_build.
 * One Jacobi iteration (nerve_center.h:146-172 with ApplyOtherInput
 * distributed_solver.h:98-103):
 *   f_k = f + G_ext du_other,   du = SolveQP(H, f_k) warm-started
 * G_ext: device, [nV * (S_total-1) * nV][B*S_local] (element-major),
 *        column block j = the j-th other sub-controller in global order.
 * du_all: device, all-gathered plans [world][B][S_local][nV] (rank-major),
 *        world = S_total / S_local: the kernel reads all of it.
 * G_ext_len, du_all_len: the element counts (doubles) of the caller's two
 *        buffers.  The call is refused (-1, cmpc_last_error) unless
 *        G_ext_len >= nV*(S_total-1)*nV * B*S_local and
 *        du_all_len >= S_total * B * nV, i.e. unless every read of the
 *        kernel falls inside them (a rank layout that does not cover
 *        S_total would otherwise read past the gathered plans).
 * du_out: device [B*S_local][nV] or NULL: this rank's new plans (the next
 *        all-gather's input).  CMPC_APPLY_MOVE on the last iteration of a
 *        step applies the first move (UpdateUOld) and stores du_old.
 * The caller all-gathers between calls (RCCL; cmpc/coupled.py). */
/* The checks cmpc_coupled_iterate makes before any launch, for a context of
 * these dims (B scenarios x S = B*S local QPs): 0, or -1 with
 * cmpc_last_error().  Host only, no device needed. */
int cmpc_coupled_validate(const cmpc_dims* dims, int S_total, int S_local, int s_offset,
                          size_t G_ext_len, size_t du_all_len);
int cmpc_coupled_iterate(cmpc_ctx* ctx, int S_total, int S_local, int s_offset,
                         const double* G_ext, size_t G_ext_len, const double* du_all,
                         size_t du_all_len, double* du_out, uint32_t flags);

/* Observer and receding-horizon update on the device (SURVEY.md §8(f)
 * row 2).  Each QP slot keeps the state of its sub-controller's
 * DistributedController (observer.h:53-56, distributed_controller.h:104-111)
 * in HBM, a row of cmpc_observer_len() doubles:
 *   [x_hat ns][dx_aug ntot][y_old n_outputs][C n_outputs x ns][padding]
 * (rows padded to a multiple of 16 doubles, one 128-byte line;
 * ntot = ns + ndist + delay states, the full AugmentedState; C = the plant
 * output matrix of the last linearisation).  A closed-loop control step is
 *   cmpc_observe_step(u_full, y)   ObserveAPosteriori + x_ += (observer.cc:27-44,
 *                                  distributed_controller.cc:80), then
 *                                  Update(x_, u_full) per QP slot: the lin
 *                                  records (GenerateInitialQP, :75-110)
 *   cmpc_build, cmpc_iterate(K, 0) the QP and the Jacobi iterations (no
 *                                  CMPC_APPLY_MOVE: the update below applies it)
 *   cmpc_observe_apply()           UpdateU (distributed_controller.h:145-152):
 *                                  ObserveAPriori (observer.cc:8-22) with the own
 *                                  first move (other inputs zero,
 *                                  nerve_center.h:323-328), then u_old += du
 * All device pointers; asynchronous on the context's stream.
 * Not graph-capturable: the delay blocks' ring phase (a-priori steps since
 * cmpc_observer_init) is host state that reaches the kernels as a launch
 * argument and advances per cmpc_observe_apply call, so a replayed capture
 * would reuse the phase it was captured with.  The same holds for
 * cmpc_sim_set_input (the TimeDelay cursors).  cmpc_build, cmpc_iterate and
 * cmpc_step carry no such host state. */
/* ObserverMatrix M of sub-controller s ((ns + ndist) x n_outputs, row-major;
 * the DistributedController constructor argument, distributed_controller.cc:14).
 * n_outputs (the plant's outputs, ObserverOutputIndices) must agree for all s. */
int cmpc_set_observer(cmpc_ctx* ctx, int s, int n_outputs, const double* M);
int cmpc_observer_len(const cmpc_ctx* ctx);
/* DistributedController::Initialize (distributed_controller.cc:30-43):
 * x_hat = x_init[b] (B x ns), y_old = y_init[b] (B x n_outputs), dx_aug =
 * dx_init (B*S x ntot, or NULL for zero), then the records at x_init (as
 * cmpc_produce_lin, input_order / out_idx as there).  Follow with cmpc_build
 * and cmpc_init_warmstart (InitializeQPProblem). */
int cmpc_observer_init(cmpc_ctx* ctx, int plant, double p_in, double p_out, double Ts,
                       const int32_t* input_order, const int32_t* out_idx,
                       const double* x_init, const double* u_full, const double* y_init,
                       const double* dx_init);
/* u_full: B x n_inputs plant input at the linearisation (NerveCenter
 * u_old_ + u_offset, nerve_center.h:139); y: B x n_outputs measured outputs. */
int cmpc_observe_step(cmpc_ctx* ctx, const double* u_full, const double* y);
int cmpc_observe_apply(cmpc_ctx* ctx);
/* The same two calls with HOST arrays (staged to the device on the
 * context's stream), for host-side harnesses such as the C++ adapter. */
int cmpc_observer_init_host(cmpc_ctx* ctx, int plant, double p_in, double p_out, double Ts,
                            const int32_t* input_order, const int32_t* out_idx,
                            const double* x_init, const double* u_full, const double* y_init,
                            const double* dx_init);
int cmpc_observe_step_host(cmpc_ctx* ctx, const double* u_full, const double* y);
/* NerveCenter::GetNextInput (include/nerve_center.h:134-182) on the device:
 * cmpc_observe_step(u_full, y) + cmpc_step(K, 0) + cmpc_observe_apply() with
 * the same results bit for bit, as ONE kernel launch for batches of up to
 * four QPs per CU (AUTO variants, no trace): observer a posteriori +
 * linearisation, the QP build,
 * K Jacobi iterations and the a-priori update in one workgroup per four QP
 * slots.  Elsewhere the three calls.  Plans, statuses and nWSR through
 * cmpc_download; u_old has moved by the own first moves. */
int cmpc_control_step(cmpc_ctx* ctx, const double* u_full, const double* y, int K);
int cmpc_control_step_host(cmpc_ctx* ctx, const double* u_full, const double* y, int K);
/* cmpc_control_step_host + cmpc_download (host arrays in and out; any output
 * pointer may be NULL), the C++ NerveCenter::GetNextInput path: a one-
 * workgroup launch (up to four QP slots) marks its completion in page-locked
 * host memory, which the call polls instead of synchronising the stream. */
int cmpc_control_step_download(cmpc_ctx* ctx, const double* u_full, const double* y, int K,
                               double* du, int32_t* status, int32_t* nwsr);
/* Host copies of the observer state rows (B*S x cmpc_observer_len()). */
int cmpc_get_observer_state(cmpc_ctx* ctx, double* host);
int cmpc_set_observer_state(cmpc_ctx* ctx, const double* host);

/* Batched plant simulation: the harness's
 * SimulationSystem for B scenarios on the GPU, one lane per scenario.
 *   cmpc_sim_reset      SimulationSystem(p_sys, u_offset, x_in) + TimeDelay()
 *                       (simulation_system.h:50-56, time_delay.h:26-38):
 *                       x0 (B x ns), u_offset (B x n_inputs), device; dt0 =
 *                       the integrate_const step (the sampling time)
 *   cmpc_sim_set_input  SetInput(u) (simulation_system.h:67-70): u_control
 *                       (B x n_control, device) through the input delay line
 *                       (time_delay.h:41-58) onto u_offset (GetPlantInput)
 *   cmpc_sim_integrate  one observation interval [t, t_end] of Integrate
 *                       (simulation_system.h:108-116): controlled
 *                       Dormand-Prince with Boost odeint's semantics and the
 *                       reference's 2-norm error (:121-133); the step size
 *                       carries over between intervals as in integrate_const
 *   cmpc_sim_set_offset SetOffset(u_offset) (simulation_system.h:64): the
 *                       plant-input offset (B x n_inputs, device) that the next
 *                       cmpc_sim_set_input adds the control inputs to; the
 *                       current plant input is unchanged until then (the
 *                       setup files' `simulation` segments, a step of an
 *                       unmeasured input such as the discharge valve)
 *   cmpc_sim_restart    a new Integrate call (simulation_system.h:108-116):
 *                       integrate_const's controlled stepper starts again from
 *                       the step size dt0 (the harness integrates each setup
 *                       segment with its own call)
 *   cmpc_sim_output     GetOutput() (B x n_outputs, device)
 *   cmpc_sim_plant_input GetPlantInput(u_control) without the delay line (the
 *                       controller's linearisation input, nerve_center.h:139)
 *   cmpc_sim_plant_input_offset  the same over a given offset (B x n_inputs,
 *                       device): the controller's own u_offset_, which keeps
 *                       its Initialize value when the plant's steps
 * Device arrays: cmpc_sim_state (x), cmpc_sim_input (plant input u_),
 * cmpc_sim_step_size (dt), cmpc_sim_status (1 = step-size control failed:
 * 500 rejected tries of one step; 2 = more than 500 steps in one interval,
 * odeint's max_step_checker; 3 = non-finite error norm or state). A status
 * is sticky: the scenario's state stays where it stopped and later
 * cmpc_sim_integrate calls skip it (the reference's odeint throws and ends
 * the run) until cmpc_sim_reset clears it, so one read after a run counts
 * every scenario that failed in any interval. */
typedef struct cmpc_sim cmpc_sim;
int cmpc_sim_create(cmpc_sim** sim, int plant, int B, int device, double p_in, double p_out,
                    int n_control, const int32_t* delays /* n_control, control order */,
                    const int32_t* control_index /* ControlInputIndex: plant input of each */);
int cmpc_sim_destroy(cmpc_sim* sim);
int cmpc_sim_set_stream(cmpc_sim* sim, void* hip_stream);
int cmpc_sim_reset(cmpc_sim* sim, const double* x0, const double* u_offset, double dt0);
int cmpc_sim_set_input(cmpc_sim* sim, const double* u_control);
int cmpc_sim_set_offset(cmpc_sim* sim, const double* u_offset);
int cmpc_sim_restart(cmpc_sim* sim, double dt0);
int cmpc_sim_plant_input(cmpc_sim* sim, const double* u_control, double* u_full_out);
int cmpc_sim_plant_input_offset(cmpc_sim* sim, const double* u_control, const double* u_offset,
                                double* u_full_out);
int cmpc_sim_integrate(cmpc_sim* sim, double t, double t_end, double eps_abs, double eps_rel);
int cmpc_sim_output(cmpc_sim* sim, double* y);
int cmpc_sim_synchronize(cmpc_sim* sim);
/* Host-array variants of reset / set_input / set_offset / output (staged
 * through the simulator's own device buffer; each returns once done). */
int cmpc_sim_reset_host(cmpc_sim* sim, const double* x0, const double* u_offset, double dt0);
int cmpc_sim_set_input_host(cmpc_sim* sim, const double* u_control);
int cmpc_sim_set_offset_host(cmpc_sim* sim, const double* u_offset);
int cmpc_sim_output_host(cmpc_sim* sim, double* y);
/* Host copies (any pointer may be NULL): x B x ns, plant input B x n_inputs,
 * step size B, status B. */
int cmpc_sim_download(cmpc_sim* sim, double* x, double* u_full, double* dt, int32_t* status);
double* cmpc_sim_state(cmpc_sim* sim);
double* cmpc_sim_input(cmpc_sim* sim);
double* cmpc_sim_step_size(cmpc_sim* sim);
int32_t* cmpc_sim_status(cmpc_sim* sim);
/* NerveCenter::UpdateUOld (nerve_center.h:313-319): u_control (device,
 * B x nu_tot, plant control order) += each sub-controller's first move of its
 * own inputs (du_old after cmpc_iterate; input_order as cmpc_produce_lin). */
int cmpc_accumulate_moves(cmpc_ctx* ctx, const int32_t* input_order, double* u_control);

/* Device producer: AugmentedLinearizedSystem::Update
 * (libs/aug_lin_sys.cc:145-177, DiscretizeRK4 :232-255) for every scenario b
 * of the context's batch, on the GPU.  Linearises the plant at (x[b],
 * u_full[b]), discretises with sampling time Ts and writes the S lin records
 * of b into the context's own record buffer (replacing any cmpc_bind_lin
 * binding): input columns in input_order[s] order (host, S x nu_tot),
 * controlled rows out_idx[s] (host, S x ny), the observer tail dx_aug
 * (B*S x naug, or NULL for zeros) and y_prev = y[b][out_idx[s]].
 * x (B x ns), u_full (B x n_inputs), dx_aug and y (B x n_outputs) are DEVICE
 * pointers; the call is asynchronous on the context's stream. */
int cmpc_produce_lin(cmpc_ctx* ctx, int plant, double p_in, double p_out, double Ts,
                     const int32_t* input_order, const int32_t* out_idx, const double* x,
                     const double* u_full, const double* dx_aug, const double* y);

#ifdef __cplusplus
}
#endif
#endif /* CMPC_H */
