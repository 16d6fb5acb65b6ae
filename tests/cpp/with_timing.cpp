// The reference's closed-loop timing executables (tests/<ctrl>-<plant>-with-
// timing.cc, whose driver common-simulation.inc is missing upstream), over
// the C++ adapter: cmpc::NerveCenter (include/cmpc/nerve_center.hpp) and
// cmpc::SimulationSystem (include/cmpc/simulation_system.hpp), i.e. the GPU
// behind the C ABI.  What the missing driver did is reconstructed from the
// surviving pieces and from the recorded runs:
//
//   read the setup file (read_files.h:13-81)
//   sub-controllers (InputConstraints, observer gain M = [0; I]) -> NvCtr
//   SetWeights / SetOutputReference; Initialize at the plant's default point
//   per `simulation` segment: SetOffset(default input + change), then
//     Integrate(t_start, t_end, Ts, callback)       simulation_system.h:108-116
//   callback(x, t): y = GetOutput(); u = GetNextInputWithTiming(y, n_timing,
//     &time); SetInput(u); keep the record (x, u, y, time)
//   write t_final / Ts records in the 6-line .dat format,
//     record k labelled k * Ts
//
// usage: with_timing <setup-file> <par|ser> <cent|coop|ncoop> [output-dir] [max-records]
// Writes <output-dir>/<folder-name>/<output-filename> (default output-dir ".").
#include <sys/stat.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "cmpc/nerve_center.hpp"
#include "cmpc/simulation_system.hpp"

namespace {

// Eigen's default output of a vector printed transposed: every coefficient
// with the stream's default precision (6, %g), right-aligned to the widest
// one, separated by one space.
std::string EigenRow(const std::vector<double>& v) {
  std::vector<std::string> s;
  size_t w = 0;
  for (double d : v) {
    char buf[64];
    std::snprintf(buf, sizeof buf, "%g", d);
    s.emplace_back(buf);
    w = std::max(w, s.back().size());
  }
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (i) out += ' ';
    out += std::string(w - s[i].size(), ' ') + s[i];
  }
  return out;
}

struct Record {
  std::vector<double> x, u, y;
  int64_t ns;
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <setup-file> <par|ser> <cent|coop|ncoop> [output-dir] [max-records]\n",
                 argv[0]);
    return 2;
  }
  try {
    using namespace cmpc;
    const PlantType plant = std::strcmp(argv[2], "ser") == 0 ? PlantType::Serial : PlantType::Parallel;
    const ControllerType type = std::strcmp(argv[3], "cent") == 0 ? ControllerType::Centralized
                                : std::strcmp(argv[3], "ncoop") == 0 ? ControllerType::NonCooperative
                                                                    : ControllerType::Cooperative;
    const std::string out_dir = argc > 4 ? argv[4] : ".";
    const long max_records = argc > 5 ? std::atol(argv[5]) : -1;
    const ControllerSpec spec = ControllerSpec::Reference(plant, type);
    const SetupFile setup = SetupFile::Read(argv[1]);
    const double Ts = 0.05;

    std::vector<DistributedController> subs;
    for (int s = 0; s < spec.S(); ++s) {
      auto sub = [&](const std::vector<double>& v) {  // nu values, or nu_tot in control order
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
      subs.emplace_back(ic, ReferenceObserverGain(spec));
    }
    NerveCenter nc(spec, subs, setup.n_iterations);
    const int blk = spec.ny * spec.ny;
    std::vector<const double*> ywt(spec.S());
    for (int s = 0; s < spec.S(); ++s)
      ywt[s] = setup.ywt.data() + (static_cast<int>(setup.ywt.size()) == blk * spec.S() ? s * blk : 0);
    nc.SetWeights(setup.uwt.data(), ywt);
    std::vector<double> y_ref(static_cast<size_t>(spec.p) * spec.n_outputs);
    for (int i = 0; i < spec.p; ++i)
      for (int o = 0; o < spec.n_outputs; ++o) y_ref[i * spec.n_outputs + o] = setup.yref[o];
    nc.SetOutputReference(y_ref.data());

    std::vector<double> x0(spec.ns), u_default(spec.n_inputs), y0(spec.n_outputs);
    Check(cmpc_plant_default(static_cast<int>(plant), x0.data(), u_default.data()), "cmpc_plant_default");
    Check(cmpc_plant_output(static_cast<int>(plant), x0.data(), y0.data()), "cmpc_plant_output");
    SimulationSystem sim(plant, u_default, x0);
    const std::vector<double> u0(spec.nu_tot, 0.0);
    nc.Initialize(x0.data(), u0.data(), u_default.data(), y0.data());

    const int seg_len = spec.n_inputs + 1;
    if (setup.simulation.empty() || setup.simulation.size() % seg_len)
      throw Error("setup: `simulation` needs segments of n_inputs + 1 numbers");
    const double t_final = setup.simulation.back();
    long n_records = std::lround(t_final / Ts);
    if (max_records >= 0 && max_records < n_records) n_records = max_records;
    std::vector<Record> recs;
    recs.reserve(n_records);
    auto callback = [&](const std::vector<double>& x, double) {
      if (static_cast<long>(recs.size()) >= n_records) return;  // the run is recorded
      const std::vector<double> y = sim.GetOutput();
      int64_t ns = 0;
      const std::vector<double> u = nc.GetNextInputWithTiming(y.data(), setup.n_timing_iterations, &ns);
      sim.SetInput(u);
      recs.push_back({x, u, y, ns});
    };
    double t_start = 0.0;
    for (size_t i = 0; i < setup.simulation.size() && static_cast<long>(recs.size()) < n_records;
         i += seg_len) {
      std::vector<double> off(u_default);
      for (int k = 0; k < spec.n_inputs; ++k) off[k] += setup.simulation[i + k];
      const double t_end = setup.simulation[i + spec.n_inputs];
      sim.SetOffset(off);
      // a shortened run stops integrating once its records are taken
      const double t_stop = t_start + Ts * static_cast<double>(n_records - static_cast<long>(recs.size()));
      sim.Integrate(t_start, std::min(t_end, t_stop), Ts, callback);
      t_start = t_end;
    }

    const std::string dir = out_dir + "/" + (setup.folder_name.empty() ? "." : setup.folder_name);
    mkdir(out_dir.c_str(), 0755);
    mkdir(dir.c_str(), 0755);
    const std::string path = dir + "/" + (setup.output_filename.empty() ? "out.dat" : setup.output_filename);
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) throw Error("cannot write " + path);
    double mean_ns = 0;
    for (size_t k = 0; k < recs.size(); ++k) {
      std::fprintf(f, "%g\n%s\n%s\n%s\n%lld\n\n", k * Ts, EigenRow(recs[k].x).c_str(),
                   EigenRow(recs[k].u).c_str(), EigenRow(recs[k].y).c_str(),
                   static_cast<long long>(recs[k].ns));
      mean_ns += recs[k].ns;
    }
    std::fclose(f);
    // the same u and y at full precision (%.17g), one record per line, beside
    // the %g file: the tests tell a rounding-boundary tie of the printed
    // sixth digit from a real difference (tests/golden_cases.py)
    FILE* ff = std::fopen((path + ".full").c_str(), "w");
    if (!ff) throw Error("cannot write " + path + ".full");
    for (const Record& r : recs) {
      for (double v : r.u) std::fprintf(ff, "%.17g ", v);
      std::fprintf(ff, "|");
      for (double v : r.y) std::fprintf(ff, " %.17g", v);
      std::fprintf(ff, "\n");
    }
    std::fclose(ff);
    std::printf("{\"records\": %zu, \"file\": \"%s\", \"mean_step_us\": %.2f}\n", recs.size(), path.c_str(),
                recs.empty() ? 0.0 : mean_ns / recs.size() * 1e-3);
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
