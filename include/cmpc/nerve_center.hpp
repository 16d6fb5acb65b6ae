// nerve_center.hpp — C++ host adapter over the C ABI (include/cmpc.h) that
// keeps the reference's controller API, so a harness written against
// katie-jones/compressor-mpc's NerveCenter / DistributedController changes its
// type names, not its call pattern.  Header-only, C++17, no Eigen: vectors
// are plain `const double*` (matrices row-major).
//
// Reference interface mirrored (paths relative to the reference root):
//   ControllerInterface<System>::GetNextInput(y)      include/controller_interface.h:46
//   NerveCenter ctor (controllers, n_solver_iterations) include/nerve_center.h:89-95
//   DistributedController(sys, constraints, M)         include/distributed_controller.h:126-128
//   DistributedController::{Initialize, SetWeights, SetOutputReference,
//     UpdateU, GenerateInitialQP, GetInput, GetStateEstimate}, incl. the
//     timed overloads on a CpuTimer (boost::timer::cpu_timer's role)
//                                                       include/distributed_controller.h:131-191
//   NerveCenter::Initialize(x, u, u_full, y, dx)      include/nerve_center.h:98-104
//   NerveCenter::SetWeights(uwt, ywt)                 include/nerve_center.h:107-110
//   NerveCenter::SetWeights(uwt, {ywt_s})             include/nerve_center.h:113-116
//   NerveCenter::SetOutputReference(y_ref)            include/nerve_center.h:119-122
//   NerveCenter::GetNextInputWithTiming(y, n, t)      include/nerve_center.h:134-182
//   InputConstraints<nu> (per sub-controller ctor arg) include/input_constraints.h:12-26
//   read_files.h setup-file reader                    include/read_files.h:13-81
//   MpcQpSolver::{SetWeights, GenerateQP, SolveQP, InitializeQPProblem,
//     SetOutputReference, GetOutputReference}          include/mpc_qp_solver.h:53-97
//   DistributedSolver::{UpdateAndSolveQP, GenerateDistributedQP}
//                                                       include/distributed_solver.h:69-94
//   ParallelCompressors(p_in, p_out), Ts              include/parallel_compressors.h:44-55,
//                                                       include/common-variables.h (sampling time)
//
// Two ways to run a step:
//  - with the observer (the reference's own pattern): SetObserver(s, M) for
//    every sub-controller (M is the DistributedController constructor
//    argument, distributed_controller.cc:14), then Initialize(...) and
//    GetNextInput(y) / GetNextInputWithTiming(y, n, t) exactly as the
//    reference.  Each sub-controller's observer (observer.cc:6-40), its
//    linearisation at its own estimate, the QP build, K Jacobi iterations and
//    UpdateU run on the GPU, the state estimates resident in device memory.
//    The reference runs' M is ReferenceObserverGain(spec) = [0; I] (set in
//    the harness's missing common-simulation.inc, identified from the
//    recorded runs).
//  - with an external estimate: GetNextInput(y, x_hat, dx_aug) takes the state
//    estimate from the caller; the linearisation runs on the host
//    (cmpc_plant_lin_record), the rest on the GPU.
#pragma once

#include <chrono>
#include <cstdint>
#include <memory>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../cmpc.h"

namespace cmpc {

class Error : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

inline void Check(int rc, const char* what) {
  if (rc != 0) {
    const char* m = cmpc_last_error();
    throw Error(std::string(what) + ": " + (m ? m : "error"));
  }
}

// The reference's boost::timer::cpu_timer as its harness uses it (the timed
// overloads of DistributedController, distributed_controller.h:155-183, and
// NerveCenter's per-controller helpers, nerve_center.h:261-310): a wall clock
// that accumulates between resume() and stop().  Boost is not a dependency
// here; elapsed().wall is in nanoseconds like boost's cpu_times::wall.
class CpuTimer {
 public:
  struct Times {
    int64_t wall = 0;  // nanoseconds
  };
  CpuTimer() { start(); }
  /// (re)start from zero, running (boost: start()).
  void start() {
    acc_ = 0;
    stopped_ = false;
    t0_ = std::chrono::steady_clock::now();
  }
  /// stop accumulating (boost: stop()); no-op when stopped.
  void stop() {
    if (stopped_) return;
    acc_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0_).count();
    stopped_ = true;
  }
  /// continue accumulating (boost: resume()); no-op when running.
  void resume() {
    if (!stopped_) return;
    stopped_ = false;
    t0_ = std::chrono::steady_clock::now();
  }
  bool is_stopped() const { return stopped_; }
  /// the accumulated time, including the running interval (boost: elapsed()).
  Times elapsed() const {
    Times t;
    t.wall = acc_;
    if (!stopped_)
      t.wall += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0_).count();
    return t;
  }

 private:
  int64_t acc_ = 0;
  bool stopped_ = false;
  std::chrono::steady_clock::time_point t0_{};
};

enum class PlantType { Parallel = CMPC_PLANT_PARALLEL, Serial = CMPC_PLANT_SERIAL };
enum class ControllerType { Centralized, Cooperative, NonCooperative };

// The reference's compile-time controller configuration, as run-time values
// (include/parallel_compressors_constants.h:68-94,
//  include/serial_compressors_constants.h:82-110, include/common-variables.h).
struct ControllerSpec {
  PlantType plant = PlantType::Parallel;
  ControllerType type = ControllerType::Cooperative;
  int ns = 0, n_inputs = 0, n_outputs = 0, nu_tot = 0;  // plant
  int nu = 0, ny = 0, ndist = 4, p = 100, m = 2;        // per sub-controller
  std::vector<int> delays;                              // Delays, plant control-input order
  std::vector<std::vector<int>> input_order;            // ControlInputIndices per sub-controller
  std::vector<std::vector<int>> out_idx;                // ControlledOutputIndices per sub-controller
  std::vector<int> plant_input_index;                   // ControlInputIndex (GetPlantInput)
  // plant parameters of the linearisation: suction / discharge pressure
  // (ParallelCompressors(p_in, p_out), parallel_compressors.h:44-55; the
  // serial plant's SerialCompressors(p_in, p_out), serial_compressors.h) and
  // the sampling time of the discretisation (common-variables.h: 0.05 s)
  double p_in = 1.0, p_out = 1.0, Ts = 0.05;

  int S() const { return static_cast<int>(input_order.size()); }
  int nV() const { return m * nu; }

  static ControllerSpec Reference(PlantType plant, ControllerType type, int p = 100, int m = 2) {
    ControllerSpec c;
    c.plant = plant;
    c.type = type;
    c.p = p;
    c.m = m;
    int nci = 0;
    Check(cmpc_plant_dims(static_cast<int>(plant), &c.ns, &c.n_inputs, &c.n_outputs, &nci),
          "cmpc_plant_dims");
    c.nu_tot = nci;
    c.delays = {0, 40, 0, 40};                 // ConstexprArray<0, 40, 0, 40>
    c.plant_input_index = {0, 3, 4, 7};        // ConstexprArray<0, 3, 4, 7>
    const std::vector<int> ci1{0, 1, 2, 3}, ci2{2, 3, 0, 1};  // ControlInputIndices1/2
    std::vector<int> ctrl_out;
    std::vector<std::vector<int>> nc_out;
    if (plant == PlantType::Parallel) {
      ctrl_out = {0, 1, 3};
      nc_out = {{0, 3}, {1, 3}};
    } else {
      ctrl_out = {0, 1, 2, 3};
      nc_out = {{0, 1}, {2, 3}};
    }
    switch (type) {
      case ControllerType::Centralized:
        c.nu = 4;
        c.input_order = {ci1};
        c.out_idx = {ctrl_out};
        break;
      case ControllerType::Cooperative:
        c.nu = 2;
        c.input_order = {ci1, ci2};
        c.out_idx = {ctrl_out, ctrl_out};
        break;
      case ControllerType::NonCooperative:
        c.nu = 2;
        c.input_order = {ci1, ci2};
        c.out_idx = nc_out;
        break;
    }
    c.ny = static_cast<int>(c.out_idx[0].size());
    return c;
  }
};

// Setup file of the reference (setup/setup-<ctrl>-<plant>), read like
// include/read_files.h:13-81: a key line, then whitespace-separated values.
struct SetupFile {
  int n_iterations = 1, n_timing_iterations = 1;
  std::vector<double> yref, uwt, ywt, lower, upper, rate_lower, rate_upper;
  // `simulation`: segments of n_inputs plant-input offset changes (from the
  // default input) and an end time, in file order
  std::vector<double> simulation;
  std::string folder_name, output_filename;

  static SetupFile Read(const std::string& path) {
    std::ifstream in(path);
    if (!in) throw Error("cannot open setup file " + path);
    static const char* keys[] = {"n-iterations", "n-timing-iterations", "folder-name",
                                 "output-filename", "yref", "uwt", "ywt",
                                 "constraints-lower", "constraints-upper",
                                 "constraints-rate-lower", "constraints-rate-upper",
                                 "simulation"};
    SetupFile s;
    std::string line, key;
    std::vector<double>* dst = nullptr;
    std::vector<double> scratch;
    while (std::getline(in, line)) {
      std::istringstream ls(line);
      std::string tok;
      if (!(ls >> tok)) continue;
      bool is_key = false;
      for (const char* k : keys) is_key = is_key || tok == k;
      if (is_key) {
        key = tok;
        dst = key == "yref" ? &s.yref : key == "uwt" ? &s.uwt : key == "ywt" ? &s.ywt
            : key == "constraints-lower" ? &s.lower : key == "constraints-upper" ? &s.upper
            : key == "constraints-rate-lower" ? &s.rate_lower
            : key == "constraints-rate-upper" ? &s.rate_upper
            : key == "simulation" ? &s.simulation : &scratch;
        continue;
      }
      if (key.empty()) throw Error("Error reading setup file at line: " + line);
      if (key == "folder-name") s.folder_name = tok;
      if (key == "output-filename") s.output_filename = tok;
      if (key == "folder-name" || key == "output-filename") continue;
      std::istringstream vs(line);
      double v;
      std::vector<double> vals;
      while (vs >> v) vals.push_back(v);
      if (key == "n-iterations" && !vals.empty()) s.n_iterations = static_cast<int>(vals[0]);
      if (key == "n-timing-iterations" && !vals.empty())
        s.n_timing_iterations = static_cast<int>(vals[0]);
      dst->insert(dst->end(), vals.begin(), vals.end());
    }
    return s;
  }
};

// The observer gain M of the reference's runs, (ns + ndist) x n_outputs
// row-major: M = [0; I], the innovation corrects the disturbance states at
// unit gain.  The reference harness sets M in its missing
// common-simulation.inc; this one reproduces every recorded run
// (tests/test_closed_loop_golden.py).
inline std::vector<double> ReferenceObserverGain(const ControllerSpec& spec) {
  std::vector<double> M(static_cast<size_t>(spec.ns + spec.ndist) * spec.n_outputs, 0.0);
  for (int o = 0; o < spec.ndist && o < spec.n_outputs; ++o) M[(spec.ns + o) * spec.n_outputs + o] = 1.0;
  return M;
}

// InputConstraints<nu> (include/input_constraints.h:12-26): bounds on one
// sub-controller's own inputs, nu values each.  As in the reference the rate
// rows are always part of the QP and use_rate_constraints is never read
// (SURVEY.md 8, quirk 9).
struct InputConstraints {
  std::vector<double> lower_bound, upper_bound, lower_rate_bound, upper_rate_bound;
  bool use_rate_constraints = false;
};

// The C ABI dimensions of sub-controller s of spec (delays in its own input
// order) for B scenarios and S sub-controllers per scenario.
inline cmpc_dims SubControllerDims(const ControllerSpec& spec, int s, int S, int B) {
  cmpc_dims d{};
  d.ns = spec.ns;
  d.ndist = spec.ndist;
  d.nu_tot = spec.nu_tot;
  d.nu = spec.nu;
  d.ny = spec.ny;
  d.p = spec.p;
  d.m = spec.m;
  d.S = S;
  d.B = B;
  for (int c = 0; c < spec.nu_tot; ++c) d.delay[c] = spec.delays[spec.input_order[s][c]];
  return d;
}

// MpcQpSolver<...>::QP (include/mpc_qp_solver.h:45-50): H (nV x nV,
// row-major as the reference's RowMajor H) and f; plus, for a reduced
// (distributed) sub-controller, G = Su' W Su_other (nV x nVo, row-major), the
// factor ApplyOtherInput multiplies the other controllers' plans with
// (distributed_solver.h:98-103: f += (du_other' Su_other') y_pred_weight_).
// This build forms G in the condensation kernel, never Su_other itself.
struct QP {
  std::vector<double> H, f, G;
};

// MpcQpSolver<n_total_states, n_outputs, n_control_inputs, p, m>
// (include/mpc_qp_solver.h:21-139, libs/mpc_qp_solver.cc) for sub-controller
// s of spec: its own one-slot device context builds the QP (GenerateQP) and
// its qpOASES SQProblem's role -- the working set a hotstart starts from --
// is kept here between SolveQP calls.  SolveQP runs the product's solver
// (cmpc_qp_solve_batch: the dual active-set method of DESIGN.md §4, nWSR cap
// 10, zero move on any failure, as libs/mpc_qp_solver.cc:42-75), so for the
// same QP, u_old and warm start it returns what the batched iterate kernel
// does, bit for bit.
//
// GenerateQP takes what this library condenses from instead of the reference's
// Prediction (Su, Sx, Sf, never formed here): the sub-controller's lin record
// (cmpc_layout: the discrete linearisation, the observer's augmented state,
// y_prev) and the linearisation input u_old (AdjustAllDelayedStates), or the
// plant state and input, linearised on the host (cmpc_plant_lin_record).
class MpcQpSolver {
 public:
  MpcQpSolver(const ControllerSpec& spec, int s, InputConstraints u_constraints,
              const std::vector<double>& y_ref = {}, const std::vector<double>& u_weight = {},
              const std::vector<double>& y_weight = {}, int device = 0)
      : spec_(spec), s_(s), device_(device), c_(std::move(u_constraints)) {
    if (s < 0 || s >= spec.S()) throw Error("MpcQpSolver: bad sub-controller index");
    for (const auto* v : {&c_.lower_bound, &c_.upper_bound, &c_.lower_rate_bound, &c_.upper_rate_bound})
      if (static_cast<int>(v->size()) != spec.nu) throw Error("InputConstraints: nu values per bound");
    d_ = SubControllerDims(spec, s, 1, 1);
    Check(cmpc_create(&ctx_, &d_, device), "cmpc_create");
    Check(cmpc_get_layout(ctx_, &L_), "cmpc_get_layout");
    Check(cmpc_set_constraints(ctx_, 0, c_.lower_bound.data(), c_.upper_bound.data(), c_.lower_rate_bound.data(),
                               c_.upper_rate_bound.data()),
          "cmpc_set_constraints");
    // the reference's defaults: y_ref = 0, identity weights (mpc_qp_solver.h:53-57)
    y_ref_ = y_ref.empty() ? std::vector<double>(static_cast<size_t>(spec.p) * spec.ny, 0.0) : y_ref;
    std::vector<double> uw = u_weight, yw = y_weight;
    if (uw.empty()) uw = Identity(spec.nu);
    if (yw.empty()) yw = Identity(spec.ny);
    SetWeights(uw.data(), yw.data());
    SetOutputReference(y_ref_.data());
  }
  virtual ~MpcQpSolver() {
    if (ctx_) cmpc_destroy(ctx_);
  }
  MpcQpSolver(const MpcQpSolver&) = delete;
  MpcQpSolver& operator=(const MpcQpSolver&) = delete;
  MpcQpSolver(MpcQpSolver&& o) noexcept { *this = std::move(o); }
  MpcQpSolver& operator=(MpcQpSolver&& o) noexcept {
    if (this != &o) {
      if (ctx_) cmpc_destroy(ctx_);
      spec_ = std::move(o.spec_);
      s_ = o.s_;
      device_ = o.device_;
      c_ = std::move(o.c_);
      d_ = o.d_;
      L_ = o.L_;
      ctx_ = o.ctx_;
      o.ctx_ = nullptr;
      y_ref_ = std::move(o.y_ref_);
      ws_ = o.ws_;
      status_ = o.status_;
      nchg_ = o.nchg_;
    }
    return *this;
  }

  /// SetWeights(uwt, ywt) (mpc_qp_solver.h:62-80): uwt nu x nu, ywt ny x ny,
  /// row-major (W = blkdiag_p(ywt), R = blkdiag_m(uwt)).
  void SetWeights(const double* uwt, const double* ywt) { Check(cmpc_set_weights(ctx_, 0, uwt, ywt), "cmpc_set_weights"); }
  /// SetOutputReference(y_ref) (:89): p x ny, prediction-major.
  void SetOutputReference(const double* y_ref) {
    y_ref_.assign(y_ref, y_ref + static_cast<size_t>(spec_.p) * spec_.ny);
    Check(cmpc_set_reference(ctx_, 0, y_ref), "cmpc_set_reference");
  }
  /// GetOutputReference() (:92).
  std::vector<double> GetOutputReference() const { return y_ref_; }

  /// GenerateQP (mpc_qp_solver.h:83-87 / libs/mpc_qp_solver.cc:16-40) from
  /// the sub-controller's lin record (cmpc_layout().rec_len doubles) and its
  /// linearisation input u_old (nu_tot, this controller's input order).
  QP GenerateQP(const double* lin_record, const double* u_old) {
    const std::vector<double> du(L_.nV, 0.0);
    const uint32_t ws = 0;
    Check(cmpc_set_state(ctx_, u_old, du.data(), &ws), "cmpc_set_state");
    Check(cmpc_upload_lin(ctx_, lin_record), "cmpc_upload_lin");
    Check(cmpc_build(ctx_), "cmpc_build");
    QP qp;
    qp.H.resize(static_cast<size_t>(L_.nV) * L_.nV);
    qp.f.resize(L_.nV);
    qp.G.resize(static_cast<size_t>(L_.nV) * L_.nVo);
    Check(cmpc_download_qp(ctx_, qp.H.data(), qp.f.data(), L_.nVo ? qp.G.data() : nullptr), "cmpc_download_qp");
    return qp;
  }
  /// GenerateQP at a plant state: x (ns), u_full (the plant's n_inputs), the
  /// observer's augmented-state tail dx_aug (naug, null = 0), y_prev
  /// (n_outputs), u_old (nu_tot, this controller's order).  The
  /// linearisation and discretisation run on the host (the reference's
  /// AugmentedLinearizedSystem::Update, aug_lin_sys.cc:145-177).
  QP GenerateQP(const double* x, const double* u_full, const double* dx_aug, const double* y_prev,
                const double* u_old) {
    std::vector<double> rec(L_.rec_len, 0.0);
    Check(cmpc_plant_lin_record(static_cast<int>(spec_.plant), spec_.p_in, spec_.p_out, spec_.Ts, x, u_full,
                                spec_.input_order[s_].data(), spec_.out_idx[s_].data(), &d_, rec.data()),
          "cmpc_plant_lin_record");
    for (int i = 0; i < L_.naug; ++i) rec[L_.off_x + i] = dx_aug ? dx_aug[i] : 0.0;
    for (int o = 0; o < spec_.ny; ++o) rec[L_.off_y + o] = y_prev[spec_.out_idx[s_][o]];
    return GenerateQP(rec.data(), u_old);
  }

  /// InitializeQPProblem(qp, u_old) (libs/mpc_qp_solver.cc:77-101): a cold
  /// solve whose working set the next hotstart starts from; its status is
  /// ignored, as the reference's.
  void InitializeQPProblem(const QP& qp, const double* u_old) {
    std::vector<double> x(L_.nV);
    Solve(qp, qp.f.data(), u_old, 0u, x.data());
  }
  /// SolveQP(qp, u_old) (libs/mpc_qp_solver.cc:42-75): hotstart from the
  /// last solve's working set, nWSR <= 10; the zero vector on any failure.
  /// u_old: this controller's own inputs (nu).
  std::vector<double> SolveQP(const QP& qp, const double* u_old) {
    std::vector<double> x(L_.nV);
    Solve(qp, qp.f.data(), u_old, ws_, x.data());
    return x;
  }
  /// Solver status word (CMPC_QP_*) and working-set changes of the last solve.
  int last_status() const { return status_; }
  int last_nwsr() const { return nchg_; }
  /// the working-set word the next hotstart starts from
  uint32_t working_set() const { return ws_; }
  const cmpc_layout& layout() const { return L_; }
  cmpc_ctx* handle() { return ctx_; }

 protected:
  void Solve(const QP& qp, const double* f, const double* u_old, uint32_t ws_in, double* x) {
    const int nV = L_.nV, nu = spec_.nu;
    if (static_cast<int>(qp.H.size()) != nV * nV || static_cast<int>(qp.f.size()) != nV)
      throw Error("MpcQpSolver::SolveQP: QP of another size");
    // lb = rep_m(lower - u_old), ub = rep_m(upper - u_old), lbA/ubA = rep_m(rate)
    std::vector<double> lb(nV), ub(nV), lbA(nV), ubA(nV);
    for (int i = 0; i < nV; ++i) {
      lb[i] = c_.lower_bound[i % nu] - u_old[i % nu];
      ub[i] = c_.upper_bound[i % nu] - u_old[i % nu];
      lbA[i] = c_.lower_rate_bound[i % nu];
      ubA[i] = c_.upper_rate_bound[i % nu];
    }
    int32_t status = 0, nchg = 0, ntrace = 0;
    uint32_t ws_out = 0;
    uint8_t trace[16];
    Check(cmpc_qp_solve_batch(device_, nV, nu, 1, qp.H.data(), f, lb.data(), ub.data(), lbA.data(), ubA.data(),
                              &ws_in, CMPC_NWSR_MAX, x, &status, &nchg, &ws_out, trace, &ntrace),
          "cmpc_qp_solve_batch");
    ws_ = ws_out;
    status_ = status;
    nchg_ = nchg;
  }
  static std::vector<double> Identity(int n) {
    std::vector<double> I(static_cast<size_t>(n) * n, 0.0);
    for (int i = 0; i < n; ++i) I[i * n + i] = 1.0;
    return I;
  }

  ControllerSpec spec_;
  int s_ = 0, device_ = 0;
  InputConstraints c_;
  cmpc_dims d_{};
  cmpc_layout L_{};
  cmpc_ctx* ctx_ = nullptr;
  std::vector<double> y_ref_;
  uint32_t ws_ = 0;
  int status_ = 0, nchg_ = 0;
};

// DistributedSolver<...> (include/distributed_solver.h:12-123): MpcQpSolver
// plus the update of a QP by the other sub-controllers' plans.
class DistributedSolver : public MpcQpSolver {
 public:
  /// DistributedSolver(index, u_constraints, y_ref, u_weight, y_weight)
  /// (distributed_solver.h:57-64); index = the sub-controller s of spec.
  DistributedSolver(const ControllerSpec& spec, int index, InputConstraints u_constraints,
                    const std::vector<double>& y_ref = {}, const std::vector<double>& u_weight = {},
                    const std::vector<double>& y_weight = {}, int device = 0)
      : MpcQpSolver(spec, index, std::move(u_constraints), y_ref, u_weight, y_weight, device) {}

  /// GenerateDistributedQP(qp, ...) (:83-94): the step's QP incl. G.
  void GenerateDistributedQP(QP* qp, const double* lin_record, const double* u_old) {
    *qp = GenerateQP(lin_record, u_old);
  }
  /// UpdateAndSolveQP(qp, du_out, u_old, Su_other, du_other) (:69-80):
  /// ApplyOtherInput on *qp (f += G du_other; the caller passes a copy of
  /// the step's QP, as distributed_controller.h:214 does), then the solve of
  /// that Jacobi iteration: the map form of the iterate kernels
  /// (cmpc_qp_solve_batch_map on the step's f, G and du_other), so the plan is
  /// bit-identical to DistributedController::GetInput's.  du_other: the other
  /// controllers' plans, controller-major, then move, then input
  /// (nerve_center.h:283-285), m * (nu_tot - nu) values.
  void UpdateAndSolveQP(QP* qp, std::vector<double>* du_out, const double* u_old, const double* du_other) {
    const int nV = L_.nV, nVo = L_.nVo;
    if (!nVo) {
      *du_out = SolveQP(*qp, u_old);
      return;
    }
    // the sizes Solve checks, before ApplyOtherInput writes f and SolveMap
    // reads H, f and G into host copies of nV x nV, nV and nV x nVo doubles
    if (static_cast<int>(qp->H.size()) != nV * nV || static_cast<int>(qp->f.size()) != nV)
      throw Error("UpdateAndSolveQP: QP of the wrong size");
    if (static_cast<int>(qp->G.size()) != nV * nVo) throw Error("UpdateAndSolveQP: QP without G");
    const std::vector<double> f0 = qp->f;  // the step's f
    const std::vector<double> d = OtherPlans(du_other);
    ApplyOtherInput(qp, d);
    std::vector<double> x(nV);
    SolveMap(*qp, f0.data(), d.data(), u_old, ws_, x.data());
    *du_out = x;
  }

 private:
  // du_other (controller-major) in G's column order (move, then other input)
  std::vector<double> OtherPlans(const double* du_other) const {
    const int nV = L_.nV, nVo = L_.nVo, nu = spec_.nu;
    const int sm1 = nVo / nV, m = spec_.m;
    std::vector<double> d(nVo);
    for (int rk = 0; rk < sm1; ++rk)
      for (int mv = 0; mv < m; ++mv)
        for (int c = 0; c < nu; ++c) d[mv * (sm1 * nu) + rk * nu + c] = du_other[rk * nV + mv * nu + c];
    return d;
  }
  // f_k[a] = f[a] + sum_c G[a][c] d[c], c ascending, each product rounded
  // before the add (the reference's ApplyOtherInput on the caller's copy)
  void ApplyOtherInput(QP* qp, const std::vector<double>& d) {
    const int nV = L_.nV, nVo = L_.nVo;
    for (int a = 0; a < nV; ++a) {
      double t = qp->f[a];
      for (int c = 0; c < nVo; ++c) {
        volatile double prod = qp->G[a * nVo + c] * d[c];  // no contraction into an FMA
        t = t + prod;
      }
      qp->f[a] = t;
    }
  }
  void SolveMap(const QP& qp, const double* f0, const double* d, const double* u_old, uint32_t ws_in, double* x) {
    const int nV = L_.nV, nu = spec_.nu;
    std::vector<double> lb(nV), ub(nV), lbA(nV), ubA(nV);
    for (int i = 0; i < nV; ++i) {
      lb[i] = c_.lower_bound[i % nu] - u_old[i % nu];
      ub[i] = c_.upper_bound[i % nu] - u_old[i % nu];
      lbA[i] = c_.lower_rate_bound[i % nu];
      ubA[i] = c_.upper_rate_bound[i % nu];
    }
    int32_t status = 0, nchg = 0, ntrace = 0;
    uint32_t ws_out = 0;
    uint8_t trace[16];
    Check(cmpc_qp_solve_batch_map(device_, nV, nu, L_.nVo, 1, qp.H.data(), f0, qp.G.data(), d, lb.data(), ub.data(),
                                  lbA.data(), ubA.data(), &ws_in, CMPC_NWSR_MAX, x, &status, &nchg, &ws_out, trace,
                                  &ntrace),
          "cmpc_qp_solve_batch_map");
    ws_ = ws_out;
    status_ = status;
    nchg_ = nchg;
  }
};

// DistributedController<AugLinSys, ...>(sys, constraints, M)
// (include/distributed_controller.h:126-128).  Two uses, as in the reference:
//  - the constructor arguments of one sub-controller of a NerveCenter
//    (DistributedController(constraints, M)); its template arguments (plant,
//    index maps, delays, p, m) are the ControllerSpec; M is the
//    (ns + ndist) x n_outputs observer gain, row-major (empty: no device
//    observer, see NerveCenter);
//  - a stand-alone sub-controller (DistributedController(spec, s, constraints,
//    M)): sub-controller s of spec on its own one-slot device context, driven
//    through the reference's member functions (distributed_controller.h:131-191)
//    by a harness that runs the cooperative iteration itself.  Vectors are in
//    the reference's orders: FullControlInput = this controller's input order
//    (own inputs first), Output / Input = the plant's.
class DistributedController {
 public:
  explicit DistributedController(InputConstraints constraints, std::vector<double> M = {})
      : constraints_(std::move(constraints)), M_(std::move(M)) {}
  DistributedController(const ControllerSpec& spec, int s, InputConstraints constraints,
                        std::vector<double> M, int device = 0)
      : constraints_(std::move(constraints)), M_(std::move(M)), dev_(std::make_unique<Device>()) {
    if (s < 0 || s >= spec.S()) throw Error("DistributedController: bad sub-controller index");
    if (static_cast<int>(M_.size()) != (spec.ns + spec.ndist) * spec.n_outputs)
      throw Error("DistributedController: M must be (ns + ndist) x n_outputs");
    for (const auto* v : {&constraints_.lower_bound, &constraints_.upper_bound,
                          &constraints_.lower_rate_bound, &constraints_.upper_rate_bound})
      if (static_cast<int>(v->size()) != spec.nu) throw Error("InputConstraints: nu values per bound");
    dev_->spec = spec;
    dev_->s = s;
    cmpc_dims d = SubControllerDims(spec, s, 1, 1);
    Check(cmpc_create(&dev_->ctx, &d, device), "cmpc_create");
    Check(cmpc_get_layout(dev_->ctx, &dev_->L), "cmpc_get_layout");
    Check(cmpc_set_constraints(dev_->ctx, 0, constraints_.lower_bound.data(), constraints_.upper_bound.data(),
                               constraints_.lower_rate_bound.data(), constraints_.upper_rate_bound.data()),
          "cmpc_set_constraints");
    Check(cmpc_set_observer(dev_->ctx, 0, spec.n_outputs, M_.data()), "cmpc_set_observer");
  }
  // The reference's controllers are values that NerveCenter copies into its
  // tuple (nerve_center.h:95).  The constructor-argument form copies as a
  // value; a stand-alone controller owns its device context (state estimate,
  // u_old, warm start), which a copy would share, so it can only be moved.
  DistributedController(const DistributedController& o) : constraints_(o.constraints_), M_(o.M_) {
    if (o.dev_) throw Error("DistributedController: a stand-alone controller owns its device context; move it");
  }
  DistributedController& operator=(const DistributedController& o) {
    if (o.dev_) throw Error("DistributedController: a stand-alone controller owns its device context; move it");
    constraints_ = o.constraints_;
    M_ = o.M_;
    dev_.reset();
    return *this;
  }
  DistributedController(DistributedController&&) noexcept = default;
  DistributedController& operator=(DistributedController&&) noexcept = default;

  const InputConstraints& constraints() const { return constraints_; }
  const std::vector<double>& observer_matrix() const { return M_; }

  /// Initialize(x_init, u_init, full_u_old, y_init, dx_init)
  /// (distributed_controller.cc:27-67): x_init ns, u_init nu_tot (this
  /// controller's order), full_u_old n_inputs, y_init n_outputs, dx_init the
  /// AugmentedState (ntot) or null for zero.  Builds the QP at x_init and runs
  /// InitializeQPProblem.
  void Initialize(const double* x_init, const double* u_init, const double* full_u_old,
                  const double* y_init, const double* dx_init = nullptr) {
    Device& D = dev();
    const std::vector<double> du0(D.L.nV, 0.0);
    const uint32_t ws0 = 0;
    Check(cmpc_set_state(D.ctx, u_init, du0.data(), &ws0), "cmpc_set_state");
    Check(cmpc_observer_init_host(D.ctx, static_cast<int>(D.spec.plant), D.spec.p_in, D.spec.p_out, D.spec.Ts,
                                  D.spec.input_order[D.s].data(), D.spec.out_idx[D.s].data(), x_init,
                                  full_u_old, y_init, dx_init),
          "cmpc_observer_init_host");
    Check(cmpc_build(D.ctx), "cmpc_build");
    Check(cmpc_init_warmstart(D.ctx), "cmpc_init_warmstart");
    Check(cmpc_synchronize(D.ctx), "cmpc_synchronize");
  }
  /// SetWeights(uwt, ywt) (:136-138): uwt nu x nu, ywt ny x ny, row-major.
  void SetWeights(const double* uwt, const double* ywt) {
    Check(cmpc_set_weights(dev().ctx, 0, uwt, ywt), "cmpc_set_weights");
  }
  /// SetOutputReference(y_ref) (:141-143): p x ny, prediction-major.
  void SetOutputReference(const double* y_ref) {
    Check(cmpc_set_reference(dev().ctx, 0, y_ref), "cmpc_set_reference");
  }
  /// UpdateU(du) (:146-152): ObserveAPriori(du, u_old_), u_old_ += du; du is
  /// nu_tot in this controller's order.
  void UpdateU(const double* du) { Check(cmpc_update_u_host(dev().ctx, du), "cmpc_update_u_host"); }
  /// UpdateU(time_out, du) (:155-159): the same, with time_out resumed
  /// around it (the reference's boost::timer::cpu_timer -> CpuTimer).
  void UpdateU(CpuTimer* time_out, const double* du) {
    time_out->resume();
    UpdateU(du);
    time_out->stop();
  }
  /// GenerateInitialQP(y, full_u_old) (distributed_controller.cc:72-108):
  /// a-posteriori observer update, linearisation at the estimate, the QP.
  void GenerateInitialQP(const double* y, const double* full_u_old) {
    Device& D = dev();
    Check(cmpc_observe_step_host(D.ctx, full_u_old, y), "cmpc_observe_step_host");
    Check(cmpc_build(D.ctx), "cmpc_build");
  }
  /// GenerateInitialQP(time_out, y, full_u_old) (:165-170): timed; the
  /// build is complete on the device when the timer stops.
  void GenerateInitialQP(CpuTimer* time_out, const double* y, const double* full_u_old) {
    time_out->resume();
    GenerateInitialQP(y, full_u_old);
    Check(cmpc_synchronize(dev().ctx), "cmpc_synchronize");
    time_out->stop();
  }
  /// GetInput(&u_solution, du_last) (:173-183, :206-226): the QP with the other
  /// controllers' plans du_last (m * (nu_tot - nu) values, controller-major;
  /// ignored by a centralized controller), warm-started; u_solution gets nV
  /// moves (zero on a solver failure, as the reference).
  void GetInput(double* u_solution, const double* du_last) {
    Device& D = dev();
    Check(cmpc_get_input_host(D.ctx, D.L.nVo > 0 ? du_last : nullptr, 0u), "cmpc_get_input_host");
    Check(cmpc_download(D.ctx, u_solution, &D.status, &D.nwsr), "cmpc_download");
  }
  /// GetInput(time_out, &u_solution, du_last) (:176-183): timed.
  void GetInput(CpuTimer* time_out, double* u_solution, const double* du_last) {
    time_out->resume();
    GetInput(u_solution, du_last);
    time_out->stop();
  }
  /// GetStateEstimate() (:186-191): the observer's x_ (ns values).
  std::vector<double> GetStateEstimate() {
    std::vector<double> x(dev().spec.ns);
    GetStateEstimate(x.data());
    return x;
  }
  void GetStateEstimate(double* x_out) {
    Device& D = dev();
    std::vector<double> row(static_cast<size_t>(cmpc_observer_len(D.ctx)));
    Check(cmpc_get_observer_state(D.ctx, row.data()), "cmpc_get_observer_state");
    for (int i = 0; i < D.spec.ns; ++i) x_out[i] = row[i];
  }
  /// The step's QP (H, f, G) as GenerateInitialQP built it.
  QP GetQP() {
    Device& D = dev();
    QP qp;
    qp.H.resize(static_cast<size_t>(D.L.nV) * D.L.nV);
    qp.f.resize(D.L.nV);
    qp.G.resize(static_cast<size_t>(D.L.nV) * D.L.nVo);
    Check(cmpc_download_qp(D.ctx, qp.H.data(), qp.f.data(), D.L.nVo ? qp.G.data() : nullptr), "cmpc_download_qp");
    return qp;
  }
  /// The lin record the last build read (the linearisation at the estimate,
  /// the augmented state, y_prev; cmpc_layout) and this controller's u_old_
  /// (nu_tot, its own input order).
  std::vector<double> GetLinRecord() {
    Device& D = dev();
    std::vector<double> rec(D.L.rec_len);
    Check(cmpc_download_lin(D.ctx, rec.data()), "cmpc_download_lin");
    return rec;
  }
  std::vector<double> GetUOld() {
    Device& D = dev();
    std::vector<double> u(D.spec.nu_tot), du(D.L.nV);
    uint32_t ws = 0;
    Check(cmpc_get_state(D.ctx, u.data(), du.data(), &ws), "cmpc_get_state");
    return u;
  }
  /// status word and working-set change count of the last GetInput
  int last_status() { return dev().status; }
  int last_nwsr() { return dev().nwsr; }
  cmpc_ctx* handle() { return dev().ctx; }

 private:
  struct Device {
    ControllerSpec spec;
    int s = 0;
    cmpc_ctx* ctx = nullptr;
    cmpc_layout L{};
    int32_t status = 0, nwsr = 0;
    ~Device() {
      if (ctx) cmpc_destroy(ctx);
    }
  };
  Device& dev() {
    if (!dev_) throw Error("DistributedController: constructed as NerveCenter arguments; use "
                           "DistributedController(spec, s, constraints, M) to drive it directly");
    return *dev_;
  }
  InputConstraints constraints_;
  std::vector<double> M_;
  std::unique_ptr<Device> dev_;
};

// ControllerInterface<System> (include/controller_interface.h:18-50): the
// pure-virtual interface every reference controller implements.  A harness
// that holds its controller as ControllerInterface* keeps doing so.
class ControllerInterface {
 public:
  virtual ~ControllerInterface() = default;
  /// const ControlInput GetNextInput(const Output& y) (controller_interface.h:46)
  virtual std::vector<double> GetNextInput(const double* y) = 0;
};

// NerveCenter<System, n_total_states, SubControllers...> for one plant
// (B = 1, as the reference); `handle()` exposes the context for the batched
// entry points of include/cmpc.h.
class NerveCenter : public ControllerInterface {
 public:
  NerveCenter(const ControllerSpec& spec, int n_solver_iterations, int device = 0)
      : spec_(spec), K_(n_solver_iterations) {
    d_ = SubControllerDims(spec, 0, spec.S(), 1);
    // delays in each sub-controller's input order; the ABI shares them
    for (int c = 0; c < spec.nu_tot; ++c)
      for (int s = 1; s < spec.S(); ++s)
        if (spec.delays[spec.input_order[s][c]] != d_.delay[c])
          throw Error("sub-controllers with different delay orderings");
    Check(cmpc_create(&ctx_, &d_, device), "cmpc_create");
    Check(cmpc_get_layout(ctx_, &L_), "cmpc_get_layout");
    u_old_.assign(spec.nu_tot, 0.0);
    u_offset_.assign(spec.n_inputs, 0.0);
    rec_.assign(static_cast<size_t>(spec.S()) * L_.rec_len, 0.0);
  }
  /// NerveCenter(controllers, n_solver_iterations) (nerve_center.h:89-95):
  /// from the sub-controllers, in sub-controller order, as the reference
  /// harness builds NvCtr from its DistributedController tuple.
  NerveCenter(const ControllerSpec& spec, const std::vector<DistributedController>& controllers,
              int n_solver_iterations, int device = 0)
      : NerveCenter(spec, n_solver_iterations, device) {
    if (static_cast<int>(controllers.size()) != spec.S())
      throw Error("NerveCenter: " + std::to_string(controllers.size()) + " sub-controllers for a " +
                  std::to_string(spec.S()) + "-controller spec");
    for (int s = 0; s < spec.S(); ++s) {
      const InputConstraints& c = controllers[s].constraints();
      for (const auto* v : {&c.lower_bound, &c.upper_bound, &c.lower_rate_bound, &c.upper_rate_bound})
        if (static_cast<int>(v->size()) != spec.nu) throw Error("InputConstraints: nu values per bound");
      SetConstraints(s, c.lower_bound.data(), c.upper_bound.data(), c.lower_rate_bound.data(),
                     c.upper_rate_bound.data());
      if (!controllers[s].observer_matrix().empty()) {
        if (static_cast<int>(controllers[s].observer_matrix().size()) !=
            (spec.ns + spec.ndist) * spec.n_outputs)
          throw Error("DistributedController: M must be (ns + ndist) x n_outputs");
        SetObserver(s, controllers[s].observer_matrix().data());
      }
    }
  }
  ~NerveCenter() {
    if (ctx_) cmpc_destroy(ctx_);
  }
  NerveCenter(const NerveCenter&) = delete;
  NerveCenter& operator=(const NerveCenter&) = delete;

  cmpc_ctx* handle() { return ctx_; }
  const ControllerSpec& spec() const { return spec_; }

  /// SetWeights(uwt, ywt): uwt n_control_inputs^2, ywt n_outputs^2 (row-major);
  /// each sub-controller takes uwt[own, own] and ywt[controlled, controlled].
  void SetWeights(const double* uwt, const double* ywt) {
    std::vector<const double*> per(spec_.S(), nullptr);
    std::vector<std::vector<double>> tmp(spec_.S());
    for (int s = 0; s < spec_.S(); ++s) {
      tmp[s].resize(spec_.ny * spec_.ny);
      for (int a = 0; a < spec_.ny; ++a)
        for (int b = 0; b < spec_.ny; ++b)
          tmp[s][a * spec_.ny + b] =
              ywt[spec_.out_idx[s][a] * spec_.n_outputs + spec_.out_idx[s][b]];
      per[s] = tmp[s].data();
    }
    SetWeights(uwt, per);
  }
  /// SetWeights(uwt, {ywt_s}): one ny x ny output weight per sub-controller.
  void SetWeights(const double* uwt, const std::vector<const double*>& ywt_sub) {
    for (int s = 0; s < spec_.S(); ++s) {
      std::vector<double> u(spec_.nu * spec_.nu);
      for (int a = 0; a < spec_.nu; ++a)
        for (int b = 0; b < spec_.nu; ++b)
          u[a * spec_.nu + b] =
              uwt[spec_.input_order[s][a] * spec_.nu_tot + spec_.input_order[s][b]];
      Check(cmpc_set_weights(ctx_, s, u.data(), ywt_sub[s]), "cmpc_set_weights");
    }
  }
  /// SetOutputReference: y_ref is p_max x n_outputs (prediction-major).
  void SetOutputReference(const double* y_ref) {
    for (int s = 0; s < spec_.S(); ++s) {
      std::vector<double> r(spec_.p * spec_.ny);
      for (int i = 0; i < spec_.p; ++i)
        for (int o = 0; o < spec_.ny; ++o)
          r[i * spec_.ny + o] = y_ref[i * spec_.n_outputs + spec_.out_idx[s][o]];
      Check(cmpc_set_reference(ctx_, s, r.data()), "cmpc_set_reference");
    }
  }
  /// InputConstraints<nu> of sub-controller s (the reference passes them to
  /// each DistributedController's constructor).
  void SetConstraints(int s, const double* lower, const double* upper, const double* rate_lower,
                      const double* rate_upper) {
    Check(cmpc_set_constraints(ctx_, s, lower, upper, rate_lower, rate_upper),
          "cmpc_set_constraints");
  }

  /// ObserverMatrix of sub-controller s, (ns + ndist) x n_outputs row-major
  /// (the DistributedController constructor argument).  Once set for every
  /// sub-controller, the observer runs on the device (see the header note).
  void SetObserver(int s, const double* M) {
    Check(cmpc_set_observer(ctx_, s, spec_.n_outputs, M), "cmpc_set_observer");
    if (has_M_.empty()) has_M_.assign(spec_.S(), 0);
    has_M_[s] = 1;
  }
  bool observer_on() const {
    if (has_M_.empty()) return false;
    for (int v : has_M_)
      if (!v) return false;
    return true;
  }

  /// Initialize(x_init, u_init, u_init_full, y_init, dx_init): linearise at
  /// (x_init, u_init_full), build every sub-controller's QP and run the cold
  /// InitializeQPProblem solve (its working sets warm-start step 0).
  /// dx_init: the augmented-state tail (naug) without the observer, the full
  /// AugmentedState (ns + naug) with it (distributed_controller.cc:30-43).
  void Initialize(const double* x_init, const double* u_init, const double* u_init_full,
                  const double* y_init, const double* dx_init = nullptr) {
    u_offset_.assign(u_init_full, u_init_full + spec_.n_inputs);
    u_old_.assign(u_init, u_init + spec_.nu_tot);
    std::vector<double> u_sub(static_cast<size_t>(spec_.S()) * spec_.nu_tot);
    for (int s = 0; s < spec_.S(); ++s)
      for (int c = 0; c < spec_.nu_tot; ++c)
        u_sub[s * spec_.nu_tot + c] = u_init[spec_.input_order[s][c]];
    std::vector<double> du(static_cast<size_t>(spec_.S()) * spec_.nV(), 0.0);
    std::vector<uint32_t> ws(spec_.S(), 0u);
    Check(cmpc_set_state(ctx_, u_sub.data(), du.data(), ws.data()), "cmpc_set_state");
    if (observer_on()) {
      std::vector<int32_t> io, oi;
      for (int s = 0; s < spec_.S(); ++s) {
        io.insert(io.end(), spec_.input_order[s].begin(), spec_.input_order[s].end());
        oi.insert(oi.end(), spec_.out_idx[s].begin(), spec_.out_idx[s].end());
      }
      std::vector<double> dx;
      if (dx_init)
        for (int s = 0; s < spec_.S(); ++s) dx.insert(dx.end(), dx_init, dx_init + L_.ntot);
      Check(cmpc_observer_init_host(ctx_, static_cast<int>(spec_.plant), spec_.p_in, spec_.p_out, spec_.Ts, io.data(),
                                    oi.data(), x_init, u_init_full, y_init,
                                    dx_init ? dx.data() : nullptr),
            "cmpc_observer_init_host");
    } else {
      FillRecords(x_init, u_init_full, dx_init, y_init);
      Check(cmpc_upload_lin(ctx_, rec_.data()), "cmpc_upload_lin");
    }
    Check(cmpc_build(ctx_), "cmpc_build");
    Check(cmpc_init_warmstart(ctx_), "cmpc_init_warmstart");
    Check(cmpc_synchronize(ctx_), "cmpc_synchronize");
  }

  /// ControllerInterface::GetNextInput(y) (controller_interface.h:46), the
  /// observer on the device (SetObserver).
  std::vector<double> GetNextInput(const double* y) override {
    return GetNextInputWithTiming(y, -1, nullptr);
  }

  /// NerveCenter::GetNextInputWithTiming(y, n_timing_iterations, time_out)
  /// (nerve_center.h:134-182), the observer on the device.  Timing as the
  /// reference's cpu_timer: it runs from the call to the end of the step and
  /// is stopped from the start of Jacobi iteration n_timing_iterations to the
  /// end of the loop (if 0 <= n_timing_iterations < K), so UpdateUOld and
  /// SendUHelper (here the download and the observer's a-priori update) are
  /// inside the time.
  std::vector<double> GetNextInputWithTiming(const double* y, int n_timing_iterations,
                                             int64_t* time_out_ns = nullptr) {
    if (!observer_on()) throw Error("GetNextInput(y) needs SetObserver for every sub-controller");
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<double> u_full(u_offset_);
    for (int c = 0; c < spec_.nu_tot; ++c) u_full[spec_.plant_input_index[c]] += u_old_[c];
    if (K_ > 0 && (n_timing_iterations < 0 || n_timing_iterations >= K_)) {
      // the whole step (a posteriori + Update, build, K iterations, UpdateU)
      // as one launch where the batch allows (cmpc_control_step)
      du_.resize(static_cast<size_t>(spec_.S()) * spec_.nV());
      status_.resize(spec_.S());
      nwsr_.resize(spec_.S());
      Check(cmpc_control_step_download(ctx_, u_full.data(), y, K_, du_.data(), status_.data(), nwsr_.data()),
            "cmpc_control_step_download");
      return Finish(0, t0, time_out_ns);
    }
    // ObserveAPosteriori + Update at each sub-controller's estimate
    Check(cmpc_observe_step_host(ctx_, u_full.data(), y), "cmpc_observe_step_host");
    const int64_t stopped = Step(n_timing_iterations, 0u);
    Download();
    // UpdateU of every sub-controller (observer a priori + its u_old_)
    Check(cmpc_observe_apply(ctx_), "cmpc_observe_apply");
    if (time_out_ns) Check(cmpc_synchronize(ctx_), "cmpc_synchronize");  // the a-priori update is timed
    return Finish(stopped, t0, time_out_ns);
  }

  /// ControllerInterface::GetNextInput with the observer's estimate supplied.
  std::vector<double> GetNextInput(const double* y, const double* x_hat,
                                   const double* dx_aug = nullptr) {
    return GetNextInputWithTiming(y, x_hat, dx_aug);
  }

  /// GetNextInputWithTiming: the wall time of the step without Jacobi
  /// iterations n_timing_iterations .. K-1 (if 0 <= n_timing_iterations < K)
  /// is returned in *time_out_ns, as the reference's cpu_timer
  /// (nerve_center.h:137-179).
  std::vector<double> GetNextInputWithTiming(const double* y, const double* x_hat,
                                             const double* dx_aug = nullptr,
                                             int n_timing_iterations = -1,
                                             int64_t* time_out_ns = nullptr) {
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<double> u_full(u_offset_);
    for (int c = 0; c < spec_.nu_tot; ++c) u_full[spec_.plant_input_index[c]] += u_old_[c];
    FillRecords(x_hat, u_full.data(), dx_aug, y);
    Check(cmpc_upload_lin(ctx_, rec_.data()), "cmpc_upload_lin");
    const int64_t stopped = Step(n_timing_iterations, CMPC_APPLY_MOVE);
    Download();
    return Finish(stopped, t0, time_out_ns);
  }

  /// Sub-controller s's observer estimate x_ (ns values; the device observer,
  /// DistributedController::GetStateEstimate of its s-th controller).
  std::vector<double> GetStateEstimate(int s) {
    std::vector<double> rows(static_cast<size_t>(spec_.S()) * cmpc_observer_len(ctx_));
    Check(cmpc_get_observer_state(ctx_, rows.data()), "cmpc_get_observer_state");
    const double* r = rows.data() + static_cast<size_t>(s) * cmpc_observer_len(ctx_);
    return std::vector<double>(r, r + spec_.ns);
  }

  /// Move plans (S x nV), QP status words and working-set change counts of the last step.
  const std::vector<double>& last_plans() const { return du_; }
  const std::vector<int32_t>& last_status() const { return status_; }
  const std::vector<int32_t>& last_nwsr() const { return nwsr_; }

 private:
  // K Jacobi iterations, the last with `last_flags`.  If 0 <= n < K, the
  // reference stops its timer before iteration n and resumes it after the
  // loop (nerve_center.h:151,158): returns that stopped span (ns), else 0.
  // build + K Jacobi iterations: one cmpc_step (a single fused launch for
  // small batches), or, when the timing stops at iteration n, the build and
  // the first n iterations, then the untimed rest
  int64_t Step(int n_timing_iterations, uint32_t last_flags) {
    if (n_timing_iterations >= 0 && n_timing_iterations < K_) {
      Check(cmpc_build(ctx_), "cmpc_build");
      Check(cmpc_iterate(ctx_, n_timing_iterations, 0u), "cmpc_iterate");
      Check(cmpc_synchronize(ctx_), "cmpc_synchronize");
      const auto stop = std::chrono::steady_clock::now();
      Check(cmpc_iterate(ctx_, K_ - n_timing_iterations, last_flags), "cmpc_iterate");
      Check(cmpc_synchronize(ctx_), "cmpc_synchronize");
      return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - stop)
          .count();
    }
    if (K_ > 0) {
      Check(cmpc_step(ctx_, K_, last_flags), "cmpc_step");
    } else {
      Check(cmpc_build(ctx_), "cmpc_build");
      Check(cmpc_iterate(ctx_, 0, last_flags), "cmpc_iterate");
    }
    return 0;
  }
  void Download() {
    du_.resize(static_cast<size_t>(spec_.S()) * spec_.nV());
    status_.resize(spec_.S());
    nwsr_.resize(spec_.S());
    Check(cmpc_download(ctx_, du_.data(), status_.data(), nwsr_.data()), "cmpc_download");
  }
  // UpdateUOld (include/nerve_center.h:313-319): apply each first move; the
  // step's time without the stopped span
  std::vector<double> Finish(int64_t stopped, std::chrono::steady_clock::time_point t0,
                             int64_t* time_out_ns) {
    for (int s = 0; s < spec_.S(); ++s)
      for (int c = 0; c < spec_.nu; ++c) u_old_[spec_.input_order[s][c]] += du_[s * spec_.nV() + c];
    if (time_out_ns)
      *time_out_ns =
          std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() -
          stopped;
    return u_old_;
  }

  // AugmentedLinearizedSystem::Update + observer state tail + y_prev for every
  // sub-controller (the inputs GenerateInitialQP reads).
  void FillRecords(const double* x, const double* u_full, const double* dx_aug, const double* y) {
    for (int s = 0; s < spec_.S(); ++s) {
      double* r = rec_.data() + static_cast<size_t>(s) * L_.rec_len;
      Check(cmpc_plant_lin_record(static_cast<int>(spec_.plant), spec_.p_in, spec_.p_out, spec_.Ts, x, u_full,
                                  spec_.input_order[s].data(), spec_.out_idx[s].data(), &d_, r),
            "cmpc_plant_lin_record");
      for (int i = 0; i < L_.naug; ++i) r[L_.off_x + i] = dx_aug ? dx_aug[i] : 0.0;
      for (int o = 0; o < spec_.ny; ++o) r[L_.off_y + o] = y[spec_.out_idx[s][o]];
    }
  }

  ControllerSpec spec_;
  int K_;
  cmpc_dims d_{};
  cmpc_layout L_{};
  cmpc_ctx* ctx_ = nullptr;
  std::vector<double> u_old_, u_offset_, rec_, du_;
  std::vector<int32_t> status_, nwsr_;
  std::vector<int> has_M_;
};

}  // namespace cmpc
