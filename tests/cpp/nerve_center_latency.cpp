// Step latency of the reference's own call pattern (B = 1: one plant, one
// NerveCenter::GetNextInput per control step, include/nerve_center.h:134-182)
// through the C++ adapter (include/cmpc/nerve_center.hpp) -> C ABI -> GPU:
// observer a posteriori + linearisation, build, K Jacobi iterations, download,
// a-priori update, all of one step, on the host clock around each call.
// bench.py's `configs` section runs it for SURVEY config 1 (cent-ser, p = 100)
// and the coop-par B = 1 step.
//
// usage: nerve_center_latency <setup-file> <par|ser> <cent|coop|ncoop> [p] [steps]
// Prints one JSON line {"steps", "mean_us", "median_us", "min_us", "p90_us"}.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
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
    const int steps = argc > 5 ? std::atoi(argv[5]) : 400;
    const ControllerSpec spec = ControllerSpec::Reference(plant, type, p);
    const SetupFile setup = SetupFile::Read(argv[1]);
    const int S = spec.S(), nu = spec.nu;
    auto sub = [&](const std::vector<double>& v, int s) {
      std::vector<double> r(nu);
      for (int c = 0; c < nu; ++c) r[c] = static_cast<int>(v.size()) == nu ? v[c] : v[spec.input_order[s][c]];
      return r;
    };
    const std::vector<double> M = ReferenceObserverGain(spec);
    std::vector<DistributedController> ctrl;
    for (int s = 0; s < S; ++s) {
      InputConstraints ic;
      ic.lower_bound = sub(setup.lower, s);
      ic.upper_bound = sub(setup.upper, s);
      ic.lower_rate_bound = sub(setup.rate_lower, s);
      ic.upper_rate_bound = sub(setup.rate_upper, s);
      ctrl.emplace_back(ic, M);
    }
    NerveCenter nc(spec, ctrl, setup.n_iterations);
    const int blk = spec.ny * spec.ny;
    std::vector<const double*> ywt(S);
    for (int s = 0; s < S; ++s)
      ywt[s] = setup.ywt.data() + (static_cast<int>(setup.ywt.size()) == blk * S ? s * blk : 0);
    nc.SetWeights(setup.uwt.data(), ywt);
    std::vector<double> y_ref(static_cast<size_t>(p) * spec.n_outputs);
    for (int i = 0; i < p; ++i)
      for (int o = 0; o < spec.n_outputs; ++o) y_ref[i * spec.n_outputs + o] = setup.yref[o];
    nc.SetOutputReference(y_ref.data());
    std::vector<double> x0(spec.ns), u_off(spec.n_inputs), y0(spec.n_outputs);
    Check(cmpc_plant_default(static_cast<int>(plant), x0.data(), u_off.data()), "cmpc_plant_default");
    Check(cmpc_plant_output(static_cast<int>(plant), x0.data(), y0.data()), "cmpc_plant_output");
    const std::vector<double> u0(spec.nu_tot, 0.0);
    nc.Initialize(x0.data(), u0.data(), u_off.data(), y0.data());
    std::vector<double> t_us;
    std::vector<double> y(y0);
    const int warm = 50;
    for (int k = 0; k < warm + steps; ++k) {
      for (int o = 0; o < spec.n_outputs; ++o) y[o] = y0[o] * (1.0 + 1e-3 * std::sin(0.7 * k + o));
      const auto t0 = std::chrono::steady_clock::now();
      const std::vector<double> u = nc.GetNextInput(y.data());
      const auto t1 = std::chrono::steady_clock::now();
      if (k >= warm) t_us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      (void)u;
    }
    std::vector<double> s = t_us;
    std::sort(s.begin(), s.end());
    double mean = 0;
    for (double v : s) mean += v;
    mean /= s.size();
    std::printf("{\"steps\": %d, \"mean_us\": %.3f, \"median_us\": %.3f, \"min_us\": %.3f, \"p90_us\": %.3f}\n",
                steps, mean, s[s.size() / 2], s.front(), s[(s.size() * 9) / 10]);
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
