// Step-0 driver through the C++ adapter (include/cmpc/nerve_center.hpp), the
// way the reference's tests/<ctrl>-<plant>-with-timing.cc drive NerveCenter:
// read the setup file, set weights / output reference / constraints,
// Initialize at the plant's default operating point, then one
// GetNextInputWithTiming.  Prints the applied control input u(t = 0) with 6
// significant digits (the precision of the reference's results/*.dat).
//
// usage: nerve_center_step0 <setup-file> <par|ser> <cent|coop|ncoop> [p] [observer|iface]
// "observer": SetObserver for every sub-controller (an arbitrary gain: the
// t = 0 correction is zero) and the reference's GetNextInputWithTiming(y, n, t).
#include <cstdio>
#include <cstring>
#include <vector>

#include "cmpc/nerve_center.hpp"

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <setup-file> <par|ser> <cent|coop|ncoop> [p]\n", argv[0]);
    return 2;
  }
  try {
    using namespace cmpc;
    const PlantType plant = std::strcmp(argv[2], "ser") == 0 ? PlantType::Serial : PlantType::Parallel;
    const ControllerType type = std::strcmp(argv[3], "cent") == 0 ? ControllerType::Centralized
                                : std::strcmp(argv[3], "ncoop") == 0 ? ControllerType::NonCooperative
                                                                    : ControllerType::Cooperative;
    const int p = argc > 4 ? std::atoi(argv[4]) : 100;
    const ControllerSpec spec = ControllerSpec::Reference(plant, type, p);
    const SetupFile setup = SetupFile::Read(argv[1]);

    // "iface": as "observer", called through the ControllerInterface base
    // (controller_interface.h:46), the way a harness holding any controller does
    const bool iface = argc > 5 && std::strcmp(argv[5], "iface") == 0;
    const bool observer = iface || (argc > 5 && std::strcmp(argv[5], "observer") == 0);
    // the sub-controllers (InputConstraints, observer gain M), then the
    // NerveCenter over them, as the reference harness builds NvCtr
    std::vector<DistributedController> subs;
    for (int s = 0; s < spec.S(); ++s) {
      // nu values, or nu_tot in plant control-input order
      auto sub = [&](const std::vector<double>& v) {
        std::vector<double> r(spec.nu);
        for (int c = 0; c < spec.nu; ++c)
          r[c] = static_cast<int>(v.size()) == spec.nu ? v[c] : v[spec.input_order[s][c]];
        return r;
      };
      InputConstraints ic;
      ic.lower_bound = sub(setup.lower);
      ic.upper_bound = sub(setup.upper);
      ic.lower_rate_bound = sub(setup.rate_lower);
      ic.upper_rate_bound = sub(setup.rate_upper);
      std::vector<double> M;
      if (observer) {  // an arbitrary gain: the t = 0 correction is zero
        const int nobs = spec.ns + spec.ndist;
        M.assign(static_cast<size_t>(nobs) * spec.n_outputs, 0.0);
        for (int o = 0; o < spec.ndist && o < spec.n_outputs; ++o) M[(spec.ns + o) * spec.n_outputs + o] = 0.5;
      }
      subs.emplace_back(ic, M);
    }
    NerveCenter nc(spec, subs, setup.n_iterations);
    // weights: uwt is n_control_inputs^2; ywt one ny x ny block per sub-controller
    const int blk = spec.ny * spec.ny;
    std::vector<const double*> ywt(spec.S());
    for (int s = 0; s < spec.S(); ++s)
      ywt[s] = setup.ywt.data() + (static_cast<int>(setup.ywt.size()) == blk * spec.S() ? s * blk : 0);
    nc.SetWeights(setup.uwt.data(), ywt);
    // output reference replicated over the horizon
    std::vector<double> y_ref(static_cast<size_t>(spec.p) * spec.n_outputs);
    for (int i = 0; i < spec.p; ++i)
      for (int o = 0; o < spec.n_outputs; ++o) y_ref[i * spec.n_outputs + o] = setup.yref[o];
    nc.SetOutputReference(y_ref.data());
    // operating point: the plant's default state and input (u_offset)
    std::vector<double> x0(spec.ns), u_full(spec.n_inputs), y0(spec.n_outputs);
    Check(cmpc_plant_default(static_cast<int>(plant), x0.data(), u_full.data()), "cmpc_plant_default");
    Check(cmpc_plant_output(static_cast<int>(plant), x0.data(), y0.data()), "cmpc_plant_output");
    const std::vector<double> u0(spec.nu_tot, 0.0);
    nc.Initialize(x0.data(), u0.data(), u_full.data(), y0.data());
    int64_t ns_time = 0;
    // t = 0: the observer's a-posteriori correction is zero, x_hat = x0
    cmpc::ControllerInterface& ctrl = nc;
    const std::vector<double> u =
        iface ? ctrl.GetNextInput(y0.data())
        : observer ? nc.GetNextInputWithTiming(y0.data(), setup.n_timing_iterations, &ns_time)
                   : nc.GetNextInputWithTiming(y0.data(), x0.data(), nullptr,
                                               setup.n_timing_iterations, &ns_time);
    for (int c = 0; c < spec.nu_tot; ++c) std::printf("%s%.6g", c ? " " : "", u[c]);
    std::printf("\n");
    std::fprintf(stderr, "status:");
    for (int st : nc.last_status()) std::fprintf(stderr, " %d", st);
    std::fprintf(stderr, "  step time %.1f us\n", ns_time * 1e-3);
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
