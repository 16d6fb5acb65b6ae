// The reference's per-object DistributedController API
// (include/distributed_controller.h:131-191) driven the way NerveCenter drives
// it (include/nerve_center.h:134-182, 276-328), against cmpc::NerveCenter on
// the same inputs.  Each sub-controller is a stand-alone
// cmpc::DistributedController on its own one-slot device context; this
// program runs the cooperative Jacobi loop on the host:
//   GenerateInitialQP(y, u_full_old) per controller,
//   K x { GetInput(&du_s, du_prev without its own segment) },
//   UpdateUOld, SendUHelper: UpdateU(du with only the own inputs set),
//   on odd steps through the timed overloads (CpuTimer),
// and checks, step by step, that the applied inputs, the move plans, the QP
// status words and every controller's GetStateEstimate equal NerveCenter's
// bit for bit.  Beside each controller runs a DistributedSolver (the
// reference's MpcQpSolver / DistributedSolver API, mpc_qp_solver.h:53-97,
// distributed_solver.h:69-94) on the controller's own lin record and u_old:
// its GenerateDistributedQP must equal the controller's QP, and every
// UpdateAndSolveQP (SolveQP for a full controller) the controller's GetInput,
// bit for bit.
//
// usage: distributed_controller_loop <setup-file> <par|ser> <cent|coop|ncoop> [p] [steps]
// Prints one line per step; exit 0 if every step matched, 3 otherwise.
#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <vector>

#include "cmpc/nerve_center.hpp"

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <setup-file> <par|ser> <cent|coop|ncoop> [p] [steps]\n", argv[0]);
    return 2;
  }
  try {
    using namespace cmpc;
    const PlantType plant = std::strcmp(argv[2], "ser") == 0 ? PlantType::Serial : PlantType::Parallel;
    const ControllerType type = std::strcmp(argv[3], "cent") == 0 ? ControllerType::Centralized
                                : std::strcmp(argv[3], "ncoop") == 0 ? ControllerType::NonCooperative
                                                                    : ControllerType::Cooperative;
    const int p = argc > 4 ? std::atoi(argv[4]) : 100;
    const int steps = argc > 5 ? std::atoi(argv[5]) : 6;
    const ControllerSpec spec = ControllerSpec::Reference(plant, type, p);
    const SetupFile setup = SetupFile::Read(argv[1]);
    const int S = spec.S(), nV = spec.nV(), nu = spec.nu, nut = spec.nu_tot, K = setup.n_iterations;

    // observer gain: 0.5 on the disturbance states (the innovation moves them)
    const int nobs = spec.ns + spec.ndist;
    std::vector<double> M(static_cast<size_t>(nobs) * spec.n_outputs, 0.0);
    for (int o = 0; o < spec.ndist && o < spec.n_outputs; ++o) M[(spec.ns + o) * spec.n_outputs + o] = 0.5;
    auto sub = [&](const std::vector<double>& v, int s) {
      std::vector<double> r(nu);
      for (int c = 0; c < nu; ++c) r[c] = static_cast<int>(v.size()) == nu ? v[c] : v[spec.input_order[s][c]];
      return r;
    };
    std::vector<InputConstraints> ics(S);
    for (int s = 0; s < S; ++s) {
      ics[s].lower_bound = sub(setup.lower, s);
      ics[s].upper_bound = sub(setup.upper, s);
      ics[s].lower_rate_bound = sub(setup.rate_lower, s);
      ics[s].upper_rate_bound = sub(setup.rate_upper, s);
    }
    // (a) NerveCenter over the sub-controllers
    std::vector<DistributedController> args;
    for (int s = 0; s < S; ++s) args.emplace_back(ics[s], M);
    NerveCenter nc(spec, args, K);
    // (b) the same sub-controllers, stand-alone
    std::vector<DistributedController> ctrl;
    for (int s = 0; s < S; ++s) ctrl.emplace_back(spec, s, ics[s], M);

    // weights, output reference: NerveCenter takes the plant-wide arrays,
    // each controller its own block (NerveCenter::SetWeights/SetOutputReference)
    const int blk = spec.ny * spec.ny;
    std::vector<const double*> ywt(S);
    for (int s = 0; s < S; ++s)
      ywt[s] = setup.ywt.data() + (static_cast<int>(setup.ywt.size()) == blk * S ? s * blk : 0);
    nc.SetWeights(setup.uwt.data(), ywt);
    std::vector<double> y_ref(static_cast<size_t>(p) * spec.n_outputs);
    for (int i = 0; i < p; ++i)
      for (int o = 0; o < spec.n_outputs; ++o) y_ref[i * spec.n_outputs + o] = setup.yref[o];
    nc.SetOutputReference(y_ref.data());
    for (int s = 0; s < S; ++s) {
      std::vector<double> uw(nu * nu), yr(static_cast<size_t>(p) * spec.ny);
      for (int a = 0; a < nu; ++a)
        for (int b = 0; b < nu; ++b) uw[a * nu + b] = setup.uwt[spec.input_order[s][a] * nut + spec.input_order[s][b]];
      for (int i = 0; i < p; ++i)
        for (int o = 0; o < spec.ny; ++o) yr[i * spec.ny + o] = y_ref[i * spec.n_outputs + spec.out_idx[s][o]];
      ctrl[s].SetWeights(uw.data(), ywt[s]);
      ctrl[s].SetOutputReference(yr.data());
    }

    std::vector<double> x0(spec.ns), u_off(spec.n_inputs), y0(spec.n_outputs);
    Check(cmpc_plant_default(static_cast<int>(plant), x0.data(), u_off.data()), "cmpc_plant_default");
    Check(cmpc_plant_output(static_cast<int>(plant), x0.data(), y0.data()), "cmpc_plant_output");
    const std::vector<double> u0(nut, 0.0);
    nc.Initialize(x0.data(), u0.data(), u_off.data(), y0.data());
    for (int s = 0; s < S; ++s) ctrl[s].Initialize(x0.data(), u0.data(), u_off.data(), y0.data());

    // (c) a DistributedSolver per sub-controller on the controller's records
    std::vector<DistributedSolver> ds;
    for (int s = 0; s < S; ++s) {
      std::vector<double> uw(nu * nu), yr(static_cast<size_t>(p) * spec.ny);
      for (int a = 0; a < nu; ++a)
        for (int b = 0; b < nu; ++b) uw[a * nu + b] = setup.uwt[spec.input_order[s][a] * nut + spec.input_order[s][b]];
      for (int i = 0; i < p; ++i)
        for (int o = 0; o < spec.ny; ++o) yr[i * spec.ny + o] = y_ref[i * spec.n_outputs + spec.out_idx[s][o]];
      ds.emplace_back(spec, s, ics[s], yr, uw, std::vector<double>(ywt[s], ywt[s] + blk));
    }
    bool solver_equal = true;
    auto same_qp = [](const QP& a, const QP& b) { return a.H == b.H && a.f == b.f && a.G == b.G; };
    std::vector<QP> qps(S);
    for (int s = 0; s < S; ++s) {  // InitializeQPProblem on the initial QP
      const std::vector<double> uo = ctrl[s].GetUOld();
      ds[s].GenerateDistributedQP(&qps[s], ctrl[s].GetLinRecord().data(), uo.data());
      solver_equal = solver_equal && same_qp(qps[s], ctrl[s].GetQP());
      ds[s].InitializeQPProblem(qps[s], uo.data());
    }

    // NerveCenter's own state for the hand-driven loop (nerve_center.h:71-75)
    std::vector<double> u_old(nut, 0.0), du_old(static_cast<size_t>(S) * nV, 0.0);
    bool all_equal = true;
    // odd steps run (b) through the timed overloads (distributed_controller.h:
    // 155-183) with one CpuTimer per controller and phase, as the reference's
    // TimeInitializeQPHelper / TimeSolveQPHelper would (nerve_center.h:261-310)
    std::vector<CpuTimer> t_build(S), t_solve(S), t_update(S);
    for (int s = 0; s < S; ++s) {
      t_build[s].stop();
      t_solve[s].stop();
      t_update[s].stop();
    }
    for (int k = 0; k < steps; ++k) {
      const bool timed = k % 2 == 1;
      std::vector<double> y(y0);
      for (int o = 0; o < spec.n_outputs; ++o) y[o] = y0[o] * (1.0 + 2e-3 * std::sin(1.3 * k + o));
      // (a)
      const std::vector<double> u_nc = nc.GetNextInput(y.data());
      // (b) GetNextInputWithTiming's body with the per-object calls
      std::vector<double> u_full(u_off);
      for (int c = 0; c < nut; ++c) u_full[spec.plant_input_index[c]] += u_old[c];
      std::vector<std::vector<double>> uo_s(S);
      for (int s = 0; s < S; ++s) {
        if (timed) ctrl[s].GenerateInitialQP(&t_build[s], y.data(), u_full.data());
        else ctrl[s].GenerateInitialQP(y.data(), u_full.data());
        uo_s[s] = ctrl[s].GetUOld();
        ds[s].GenerateDistributedQP(&qps[s], ctrl[s].GetLinRecord().data(), uo_s[s].data());
        solver_equal = solver_equal && same_qp(qps[s], ctrl[s].GetQP());
      }
      std::vector<double> du_prev(du_old), du_new(du_old.size());
      std::vector<int> status(S, 0);
      for (int i = 0; i < K; ++i) {
        for (int s = 0; s < S; ++s) {
          std::vector<double> du_last;  // the others' plans, controller-major (:283-285)
          for (int s2 = 0; s2 < S; ++s2)
            if (s2 != s) du_last.insert(du_last.end(), du_prev.begin() + s2 * nV, du_prev.begin() + (s2 + 1) * nV);
          if (timed) ctrl[s].GetInput(&t_solve[s], du_new.data() + s * nV, du_last.empty() ? nullptr : du_last.data());
          else ctrl[s].GetInput(du_new.data() + s * nV, du_last.empty() ? nullptr : du_last.data());
          status[s] = ctrl[s].last_status();
          // the same solve through the reference's solver API, on a copy of
          // the step's QP (distributed_controller.h:214)
          QP copy = qps[s];
          std::vector<double> du_ds;
          if (du_last.empty()) du_ds = ds[s].SolveQP(copy, uo_s[s].data());
          else ds[s].UpdateAndSolveQP(&copy, &du_ds, uo_s[s].data(), du_last.data());
          solver_equal = solver_equal && ds[s].last_status() == status[s] &&
                         std::equal(du_ds.begin(), du_ds.end(), du_new.begin() + s * nV);
          if (k == 0 && i == 0 && !du_last.empty()) {
            // a mis-sized QP is an Error, not an out-of-bounds host access
            // (Solve's size check, repeated before ApplyOtherInput)
            bool refused = true;
            for (int bad = 0; bad < 2; ++bad) {
              QP wrong = qps[s];
              if (bad == 0) wrong.H.pop_back();
              else wrong.f.pop_back();
              std::vector<double> du_w;
              try {
                ds[s].UpdateAndSolveQP(&wrong, &du_w, uo_s[s].data(), du_last.data());
                refused = false;
              } catch (const Error&) {
              }
            }
            std::printf("mis-sized QP: %s\n", refused ? "refused" : "ACCEPTED");
            solver_equal = solver_equal && refused;
          }
        }
        du_prev = du_new;
      }
      du_old = du_prev;
      // UpdateUOld, then SendUHelper: each controller gets du with only its own
      // inputs set (nerve_center.h:313-328)
      std::vector<double> du_applied(nut, 0.0);
      for (int s = 0; s < S; ++s)
        for (int c = 0; c < nu; ++c) {
          u_old[spec.input_order[s][c]] += du_old[s * nV + c];
          du_applied[spec.input_order[s][c]] = du_old[s * nV + c];
        }
      for (int s = 0; s < S; ++s) {
        std::vector<double> du_s(nut, 0.0);
        for (int c = 0; c < nu; ++c) du_s[c] = du_applied[spec.input_order[s][c]];
        if (timed) ctrl[s].UpdateU(&t_update[s], du_s.data());
        else ctrl[s].UpdateU(du_s.data());
      }
      // compare
      bool eq = u_nc == u_old && nc.last_plans() == du_old;
      for (int s = 0; s < S; ++s) {
        eq = eq && nc.last_status()[s] == status[s];
        eq = eq && nc.GetStateEstimate(s) == ctrl[s].GetStateEstimate();
      }
      double dmax = 0;
      for (int c = 0; c < nut; ++c) dmax = std::fmax(dmax, std::fabs(u_nc[c] - u_old[c]));
      std::printf("step %d: u", k);
      for (double v : u_old) std::printf(" %.9g", v);
      std::printf("  status");
      for (int v : status) std::printf(" %d", v);
      std::printf("  %s (max |du| %.3g)  solver API %s%s\n", eq ? "equal" : "DIFFERENT", dmax,
                  solver_equal ? "equal" : "DIFFERENT", timed ? "  (timed overloads)" : "");
      all_equal = all_equal && eq && solver_equal;
    }
    for (int s = 0; s < S; ++s)
      std::printf("controller %d timed overloads: GenerateInitialQP %.1f us, GetInput %.1f us, UpdateU %.1f us "
                  "(summed over the timed steps)\n",
                  s, t_build[s].elapsed().wall * 1e-3, t_solve[s].elapsed().wall * 1e-3,
                  t_update[s].elapsed().wall * 1e-3);
    bool timers_ok = true;
    for (int s = 0; s < S; ++s)
      timers_ok = timers_ok && (steps < 2 || (t_build[s].elapsed().wall > 0 && t_solve[s].elapsed().wall > 0 &&
                                             t_update[s].elapsed().wall > 0 && t_build[s].is_stopped()));
    if (!timers_ok) std::printf("timers: not accumulated\n");
    return all_equal && timers_ok ? 0 : 3;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
