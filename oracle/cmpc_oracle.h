/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * CPU restatement of the reference's condensed-QP hot path
 * (katie-jones/compressor-mpc):
 *   or_plant.c     plant linearisation + Taylor-4 discretisation (upstream
 *                  producer, needed to pin against the step-0 golden records)
 *   or_condense.c  AugmentedLinearizedSystem (Update reorder, AComposite,
 *                  BComposite, GeneratePrediction, AdjustAllDelayedStates),
 *                  MpcQpSolver::SetWeights/GenerateQP/SolveQP bounds,
 *                  DistributedSolver::GenerateDistributedQP/ApplyOtherInput,
 *                  in the reference's own operation order (O(p^2) Su loop,
 *                  dense products)
 *   or_qp.c        the build's warm-started dual active-set QP solver
 *                  (replaces qpOASES 3.2.0 SQProblem::hotstart, which is not
 *                  vendored in the reference; parity of the QP arithmetic to
 *                  qpOASES itself is pinned only through the unique optimum
 *                  and the six step-0 golden records)
 *   or_nerve.c     NerveCenter Jacobi loop / DistributedController::GetInput
 *                  over a batch in the product's lin-record format
 *   or_observer.c  Observer a posteriori / a priori and UpdateU
 *   or_sim.c       the harness's plant simulation (controlled Dormand-Prince,
 *                  TimeDelay, GetPlantInput)
 *
 * The product must never route through this library.
 */
#ifndef CMPC_ORACLE_H
#define CMPC_ORACLE_H

#include <stdint.h>

#include "../include/cmpc.h"

#ifdef __cplusplus
extern "C" {
#endif

#define OR_PLANT_PARALLEL 0
#define OR_PLANT_SERIAL 1

/* ---- plant (or_plant.c) ---- */
int or_plant_dims(int plant, int* ns, int* ni, int* no, int* nci);
void or_plant_default(int plant, double* x, double* u);
void or_plant_linearize(int plant, double p_in, double p_out, const double* x,
                        const double* u, double* A, double* B, double* C,
                        double* f);
void or_plant_output(int plant, const double* x, double* y);
void or_discretize_rk4(int ns, int nci, double Ts, const double* A,
                       const double* B, const double* f, double* Ad,
                       double* Bd, double* fd);

/* ---- layout (restates cmpc.h's documented record format) ---- */
int or_layout_of(const cmpc_dims* d, cmpc_layout* L);

/* AugmentedLinearizedSystem::Update (libs/aug_lin_sys.cc:145-177) +
 * controlled-row selection of C: fills off_A..off_f of a lin record. */
int or_lin_record(int plant, double p_in, double p_out, double Ts,
                  const double* x, const double* u_full,
                  const int32_t* input_order, const int32_t* out_idx,
                  const cmpc_dims* d, double* rec);

/* ---- condensation (or_condense.c) ---- */
/* GeneratePrediction (libs/aug_lin_sys.cc:260-334).  Row-major outputs:
 * Su (p*ny) x (m*nu), Sx (p*ny) x naug, Sf (p*ny) x ns,
 * Su_other (p*ny) x (m*nuo) (may be NULL when nuo == 0). */
int or_generate_prediction(const cmpc_dims* d, const double* rec, double* Su,
                           double* Sx, double* Sf, double* Su_other);

/* Full sub-controller build = GenerateInitialQP: delta_x0 assembly
 * (libs/distributed_controller.cc:85-90), AdjustAllDelayedStates,
 * GeneratePrediction, GenerateDistributedQP (YPW = W*Su) and GenerateQP.
 * Outputs H (nV x nV, row-major, not symmetrised — as the reference),
 * f (nV), YPW ((p*ny) x nV), Su_other ((p*ny) x nVo), G = Su'W Su_other
 * (nV x nVo, for cross-checks only; the oracle's iterate uses YPW/Su_other). */
int or_build_qp(const cmpc_dims* d, const double* rec, const double* u_old,
                const double* y_ref, const double* ywt, const double* uwt,
                double* H, double* f, double* YPW, double* Su_other,
                double* G);

/* ---- QP (or_qp.c) ---- */
typedef struct or_qp_info {
  int32_t status;  /* CMPC_QP_* */
  int32_t nchg;    /* working-set changes used */
  uint32_t ws;     /* working set on exit */
  int32_t ntrace;
  uint8_t trace[16];
  double margin;   /* smallest relative decision margin (checker only; or_qp.c header) */
} or_qp_info;

/* min 1/2 x'Hx + g'x  s.t. lb <= x <= ub, lbA <= A x <= ubA with the
 * reference's rate-constraint matrix A (include/mpc_qp_solver.h:108-123). */
int or_qp_solve(int n, int nu, const double* H, const double* g,
                const double* lb, const double* ub, const double* lbA,
                const double* ubA, uint32_t ws_in, int max_chg, double* x,
                or_qp_info* info);
/* The same QP with g = f + G d (G: n x nvo row-major, d: nvo), solved in the
 * map form of the Jacobi iterations (or_qp.c header, step A); nvo = 0 is
 * or_qp_solve. */
#define CMPC_MAX_NVO 64
int or_qp_solve_map(int n, int nu, const double* H, const double* f, int nvo,
                    const double* G, const double* d, const double* lb,
                    const double* ub, const double* lbA, const double* ubA,
                    uint32_t ws_in, int max_chg, double* x, or_qp_info* info);

/* ---- batched NerveCenter step (or_nerve.c) ---- */
typedef struct or_cfg {
  const double* y_ref; /* S x (p*ny) */
  const double* ywt;   /* S x (ny*ny) */
  const double* uwt;   /* S x (nu*nu) */
  const double* lower; /* S x nu each */
  const double* upper;
  const double* rate_lower;
  const double* rate_upper;
} or_cfg;

/* One control step for all B scenarios (build + K Jacobi iterations), on
 * `threads` OpenMP threads (1 = the reference's execution model).
 * State in/out: u_old (B*S*nu_tot), du_old (B*S*nV), ws (B*S).
 * Outputs: du (B*S*nV), status/nwsr (B*S), optional trace (B*S*K*16 bytes)
 * and ntrace (B*S*K). init != 0 first runs InitializeQPProblem (cold solve,
 * status ignored) on each QP.  Returns 0. */
int or_step(const cmpc_dims* d, const or_cfg* cfg, const double* lin, int K,
            uint32_t flags, int init, int threads, double* u_old,
            double* du_old, uint32_t* ws, double* du, int32_t* status,
            int32_t* nwsr, uint8_t* trace, int32_t* ntrace, double* margin);

/* ---- plant simulation (or_plant.c, or_sim.c) ---- */
/* GetDerivative of the plant (parallel_compressors.cc:9-26, serial_compressors.cc:8-26). */
int or_plant_derivative(int plant, double p_in, double p_out, const double* x,
                        const double* u, double* dx);
/* One observation interval [t, t_end] of SimulationSystem::Integrate
 * (controlled Dormand-Prince, odeint semantics, see or_sim.c); x in/out,
 * dt in/out (carried between intervals).  Returns accepted steps; -1 after
 * 500 rejected tries of one step, -2 after 500 steps in the interval. */
int or_sim_interval(int plant, double p_in, double p_out, const double* u_full, double* x,
                    double t, double t_end, double* dt_io, double eps_abs, double eps_rel);
/* TimeDelay (time_delay.h:26-58): ring = sum(delays) doubles, cur = n_inputs. */
void or_time_delay_init(int n_inputs, const int32_t* delays, double* ring, int32_t* cur);
void or_time_delay(int n_inputs, const int32_t* delays, double* ring, int32_t* cur,
                   const double* u_next, double* u_out);
/* SimulationSystem::GetPlantInput (simulation_system.h:82-88). */
void or_plant_input(int n_inputs, int n_control, const int32_t* control_index,
                    const double* u_offset, const double* u_control, double* u_full);

/* ---- observer (or_observer.c) ---- */
/* ObserveAPosteriori + x_ += (libs/observer.cc:27-44,
 * distributed_controller.cc:80).  dx: full AugmentedState (ns + ndist +
 * delay states); Cp: n_out x ns plant C of the last linearisation;
 * M: (ns + ndist) x n_out. */
void or_observe_post(int ns, int ndist, int n_out, const double* Cp,
                     const double* M, const double* y, double* y_old,
                     double* dx, double* x_hat);
/* UpdateU: ObserveAPriori (libs/observer.cc:8-22) with the step's record,
 * then u_old += du (include/distributed_controller.h:145-152); du = own
 * first move, zero for the other inputs (nerve_center.h:323-328). */
int or_observe_prior(const cmpc_dims* d, const double* rec, const double* du_own,
                     double* u_old, double* dx);

#ifdef __cplusplus
}
#endif
#endif
