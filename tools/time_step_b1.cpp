// Where the time of one B = 1 GetNextInputWithTiming goes (the reference's
// own use: one plant, one controller step per sampling instant).  Times each
// C ABI call of the step with a device synchronisation after it, over N steps
// of the coop-par closed loop (plant simulation included, untimed).
// build: see tools/Makefile.b1;  usage: time_step_b1 <setup-file> [steps]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "cmpc/nerve_center.hpp"
#include "cmpc/simulation_system.hpp"

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}

int main(int argc, char** argv) {
  using namespace cmpc;
  if (argc < 2) return 2;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 2000;
  try {
    const ControllerSpec spec = ControllerSpec::Reference(PlantType::Parallel, ControllerType::Cooperative);
    const SetupFile setup = SetupFile::Read(argv[1]);
    std::vector<DistributedController> subs;
    for (int s = 0; s < spec.S(); ++s) {
      InputConstraints ic;
      for (int c = 0; c < spec.nu; ++c) {
        ic.lower_bound.push_back(setup.lower[c]);
        ic.upper_bound.push_back(setup.upper[c]);
        ic.lower_rate_bound.push_back(setup.rate_lower[c]);
        ic.upper_rate_bound.push_back(setup.rate_upper[c]);
      }
      subs.emplace_back(ic, ReferenceObserverGain(spec));
    }
    NerveCenter nc(spec, subs, setup.n_iterations);
    const int blk = spec.ny * spec.ny;
    std::vector<const double*> ywt(spec.S());
    for (int s = 0; s < spec.S(); ++s) ywt[s] = setup.ywt.data() + (setup.ywt.size() == size_t(blk * spec.S()) ? s * blk : 0);
    nc.SetWeights(setup.uwt.data(), ywt);
    std::vector<double> y_ref(static_cast<size_t>(spec.p) * spec.n_outputs);
    for (int i = 0; i < spec.p; ++i)
      for (int o = 0; o < spec.n_outputs; ++o) y_ref[i * spec.n_outputs + o] = setup.yref[o];
    nc.SetOutputReference(y_ref.data());
    std::vector<double> x0(spec.ns), u_def(spec.n_inputs), y0(spec.n_outputs);
    Check(cmpc_plant_default(0, x0.data(), u_def.data()), "default");
    Check(cmpc_plant_output(0, x0.data(), y0.data()), "output");
    SimulationSystem sim(PlantType::Parallel, u_def, x0);
    nc.Initialize(x0.data(), std::vector<double>(4, 0.0).data(), u_def.data(), y0.data());
    double t_whole = 0, t_sim = 0;
    std::vector<double> samples;
    sim.Integrate(0.0, steps * 0.05, 0.05, [&](const std::vector<double>&, double) {
      const auto a = clk::now();
      const std::vector<double> y = sim.GetOutput();
      const auto b = clk::now();
      int64_t ns = 0;
      const std::vector<double> u = nc.GetNextInputWithTiming(y.data(), setup.n_timing_iterations, &ns);
      const auto c = clk::now();
      sim.SetInput(u);
      const auto d = clk::now();
      t_whole += us(b, c);
      t_sim += us(a, b) + us(c, d);
      samples.push_back(ns * 1e-3);
    });
    const size_t n = samples.size();
    std::printf("{\"steps\": %zu, \"get_next_input_us\": %.2f, \"sim_io_us\": %.2f}\n", n, t_whole / n, t_sim / n);
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
