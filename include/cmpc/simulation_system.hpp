// cmpc::SimulationSystem — the reference harness's plant simulation
// (include/simulation_system.h) over the device simulator of the C ABI
// (cmpc_sim_*, include/cmpc.h), for one scenario with host arrays, with the
// reference's member functions:
//
//   SimulationSystem(p_sys, u_offset, x_in)   simulation_system.h:50-56
//   GetCurrentState() / GetCurrentInput()     :59-62
//   SetOffset(u_offset)                       :64
//   SetInput(u)  (TimeDelay, GetPlantInput)   :67-70, time_delay.h:41-58
//   GetOutput()                               :79
//   Integrate(t0, tf, dt, callback)           :108-116 (integrate_const with a
//       controlled Dormand-Prince stepper, eps 1e-6, the 2-norm error; the
//       callback at t0, t0 + dt, ..., and at the end, the step size carried
//       between observations and started afresh at dt by every call)
//
// The plant is selected at run time (cmpc::PlantType) instead of the
// reference's template argument (simulation_system.h:17); the System object's
// inlet/outlet pressures and the Delays / InputIndices template arguments
// (:17, :50) are constructor arguments whose defaults are the reference
// plants' (p_in = p_out = 1, delays (0, 40, 0, 40), control inputs at plant
// inputs (0, 3, 4, 7)).
#pragma once

#include <functional>
#include <vector>

#include "cmpc/nerve_center.hpp"

namespace cmpc {

class SimulationSystem {
 public:
  /// callback(x, t) at every observation instant (IntegrationCallbackPtr)
  using IntegrationCallback = std::function<void(const std::vector<double>& x, double t)>;

  SimulationSystem(PlantType plant, const std::vector<double>& u_offset, const std::vector<double>& x_in,
                   int device = 0, double dt0 = 0.05, double p_in = 1.0, double p_out = 1.0,
                   const std::vector<int32_t>& delays = {0, 40, 0, 40},
                   const std::vector<int32_t>& input_indices = {0, 3, 4, 7})
      : plant_(plant) {
    int nci = 0;
    Check(cmpc_plant_dims(static_cast<int>(plant), &ns_, &ni_, &no_, &nci), "cmpc_plant_dims");
    if (static_cast<int>(u_offset.size()) != ni_ || static_cast<int>(x_in.size()) != ns_)
      throw Error("SimulationSystem: u_offset needs n_inputs, x_in n_states values");
    if (delays.size() != input_indices.size() || delays.empty())
      throw Error("SimulationSystem: one delay per control input");
    nc_ = static_cast<int>(delays.size());
    Check(cmpc_sim_create(&sim_, static_cast<int>(plant), 1, device, p_in, p_out, nc_, delays.data(),
                          input_indices.data()),
          "cmpc_sim_create");
    Check(cmpc_sim_reset_host(sim_, x_in.data(), u_offset.data(), dt0), "cmpc_sim_reset_host");
  }
  ~SimulationSystem() {
    if (sim_) cmpc_sim_destroy(sim_);
  }
  SimulationSystem(const SimulationSystem&) = delete;
  SimulationSystem& operator=(const SimulationSystem&) = delete;

  std::vector<double> GetCurrentState() const {
    std::vector<double> x(ns_);
    Check(cmpc_sim_download(sim_, x.data(), nullptr, nullptr, nullptr), "cmpc_sim_download");
    return x;
  }
  std::vector<double> GetCurrentInput() const {
    std::vector<double> u(ni_);
    Check(cmpc_sim_download(sim_, nullptr, u.data(), nullptr, nullptr), "cmpc_sim_download");
    return u;
  }
  void SetOffset(const std::vector<double>& u_offset) {
    if (static_cast<int>(u_offset.size()) != ni_) throw Error("SetOffset: n_inputs values");
    Check(cmpc_sim_set_offset_host(sim_, u_offset.data()), "cmpc_sim_set_offset_host");
  }
  void SetInput(const std::vector<double>& u_control) {
    if (static_cast<int>(u_control.size()) != nc_) throw Error("SetInput: one value per control input");
    Check(cmpc_sim_set_input_host(sim_, u_control.data()), "cmpc_sim_set_input_host");
  }
  std::vector<double> GetOutput() const {
    std::vector<double> y(no_);
    Check(cmpc_sim_output_host(sim_, y.data()), "cmpc_sim_output_host");
    return y;
  }

  /// integrate_const(controlled dopri5, *this, x_, t0, tf, dt, callback):
  /// observe at t0 + k dt while t0 + (k+1) dt <= tf, integrating between
  /// observations, then observe once more at the end.
  void Integrate(double t0, double tf, double dt, const IntegrationCallback& callback,
                 double max_rel_error = 1e-6, double max_abs_error = 1e-6) {
    Check(cmpc_sim_restart(sim_, dt), "cmpc_sim_restart");  // a fresh stepper per call
    const double eps = 2.220446049250313e-16;
    double t = t0;
    long step = 0;
    while ((t0 + static_cast<double>(step + 1) * dt) - tf <= eps) {
      callback(GetCurrentState(), t);
      // integrate_adaptive(stepper, sys, x, time, time + dt, dt): the interval
      // ends at time + dt, the next observation is at t0 + (step + 1) dt
      Check(cmpc_sim_integrate(sim_, t, t + dt, max_abs_error, max_rel_error), "cmpc_sim_integrate");
      int32_t st = 0;
      Check(cmpc_sim_download(sim_, nullptr, nullptr, nullptr, &st), "cmpc_sim_download");
      if (st) throw Error(st == 2   ? "Integrate: more than 500 steps in one observation interval"
                          : st == 3 ? "Integrate: non-finite state or error norm"
                                    : "Integrate: step size control failed");
      ++step;
      t = t0 + static_cast<double>(step) * dt;
    }
    callback(GetCurrentState(), t);
  }

  int n_states() const { return ns_; }
  int n_inputs() const { return ni_; }
  int n_outputs() const { return no_; }

 private:
  PlantType plant_;
  int ns_ = 0, ni_ = 0, no_ = 0, nc_ = 0;
  cmpc_sim* sim_ = nullptr;
};

}  // namespace cmpc
