// Upstream producer of the hot path's inputs (host, untimed): the reference
// plants linearised and discretised exactly as
// AugmentedLinearizedSystem::Update does (libs/aug_lin_sys.cc:145-177):
//   Compressor<has_input_tank>  systems/compressor.cc:14-221
//   Tank                        systems/tank.cc:10-49
//   ValveEqs                    include/valve_eqs.h:16-50
//   ParallelCompressors         systems/parallel_compressors.cc:28-128
//   SerialCompressors           systems/serial_compressors.cc:8-117
//   DiscretizeRK4               libs/aug_lin_sys.cc:232-255
// The plant model itself is plant_model.h (shared with the device producer
// cmpc_produce_lin, produce.hip); this file is the host API.
#include <cmath>
#include <cstring>

#include "../../include/cmpc.h"

#include "plant_model.h"

namespace {

using namespace cmpc_plant;

// DiscretizeRK4 (libs/aug_lin_sys.cc:232-255).  Products accumulate with fma
// in k order: the device producer's DPP chains (produce.hip) do the same.
void discretize(int ns, double Ts, const double* A, const double* B, const double* f, double* Ad,
                double* Bd, double* fd) {
  double A2[256], A3[256], Ac[256];
  auto mm = [ns](const double* X, const double* Y, double* Z) {
    for (int i = 0; i < ns; ++i)
      for (int j = 0; j < ns; ++j) {
        double s = 0;
        for (int k = 0; k < ns; ++k) s = std::fma(X[i * ns + k], Y[k * ns + j], s);
        Z[i * ns + j] = s;
      }
  };
  mm(A, A, A2);
  mm(A2, A, A3);
  for (int i = 0; i < ns * ns; ++i) {
    const int r = i / ns, c = i % ns;
    Ac[i] = Ts * (r == c) + Ts * Ts / 2.0 * A[i] + Ts * Ts * Ts / 6.0 * A2[i] +
            Ts * Ts * Ts * Ts / 24.0 * A3[i];
  }
  mm(Ac, A, Ad);
  for (int i = 0; i < ns; ++i) Ad[i * ns + i] += 1.0;
  for (int i = 0; i < ns; ++i) {
    for (int j = 0; j < 4; ++j) {
      double s = 0;
      for (int k = 0; k < ns; ++k) s = std::fma(Ac[i * ns + k], B[k * 4 + j], s);
      Bd[i * 4 + j] = s;
    }
    double s = 0;
    for (int k = 0; k < ns; ++k) s = std::fma(Ac[i * ns + k], f[k], s);
    fd[i] = s;
  }
}

}  // namespace

extern "C" {

int cmpc_plant_dims(int plant, int* ns, int* ni, int* no, int* nci) {
  if (plant != CMPC_PLANT_PARALLEL && plant != CMPC_PLANT_SERIAL) return -1;
  const bool par = plant == CMPC_PLANT_PARALLEL;
  if (ns) *ns = par ? 11 : 10;
  if (ni) *ni = par ? 9 : 8;
  if (no) *no = 4;
  if (nci) *nci = 4;
  return 0;
}

int cmpc_plant_default(int plant, double* x, double* u) {
  static const double xp[11] = {0.916, 1.145, 0.152, 440, 0, 0.916, 1.145, 0.152, 440, 0, 1.12};
  static const double up[9] = {0.304, 0.43, 1.0, 0, 0.304, 0.43, 1.0, 0, 0.7};
  static const double xs[10] = {0.867, 1.03, 0.176, 395, 0, 0.999, 1.19, 0.176, 395, 0};
  static const double us[8] = {0.304, 0.405, 1, 0, 0.304, -1, 0.393, 0};
  if (plant == CMPC_PLANT_PARALLEL) {
    if (x) std::memcpy(x, xp, sizeof xp);
    if (u) std::memcpy(u, up, sizeof up);
    return 0;
  }
  if (plant == CMPC_PLANT_SERIAL) {
    if (x) std::memcpy(x, xs, sizeof xs);
    if (u) std::memcpy(u, us, sizeof us);
    return 0;
  }
  return -1;
}

int cmpc_plant_output(int plant, const double* x, double* y) {
  Compressor comp{CompressorParams(), true};
  double y0[2], y1[2];
  if (plant == CMPC_PLANT_PARALLEL) {
    comp.output(x, y0);
    comp.output(x + 5, y1);
    y[0] = y0[1];
    y[1] = y1[1];
    y[2] = y0[0] - y1[0];
    y[3] = x[10];
    return 0;
  }
  if (plant == CMPC_PLANT_SERIAL) {
    comp.output(x, y);
    comp.output(x + 5, y + 2);
    return 0;
  }
  return -1;
}

int cmpc_plant_lin_record(int plant, double p_in, double p_out, double Ts, const double* x,
                          const double* u_full, const int32_t* input_order, const int32_t* out_idx,
                          const cmpc_dims* d, double* rec) {
  int ns, ni, no, nci;
  if (cmpc_plant_dims(plant, &ns, &ni, &no, &nci)) return -1;
  cmpc_layout L;
  if (cmpc_layout_of(d, &L)) return -1;
  if (d->ns != ns || d->nu_tot != nci || d->ndist > no) return -1;
  double A[121], B[44], C[44], f[11], Ad[121], Bd[44], fd[11];
  if (plant == CMPC_PLANT_PARALLEL)
    parallel_linearize(p_in, p_out, x, u_full, A, B, C, f);
  else
    serial_linearize(p_in, p_out, x, u_full, A, B, C, f);
  discretize(ns, Ts, A, B, f, Ad, Bd, fd);
  std::memcpy(rec + L.off_A, Ad, sizeof(double) * ns * ns);
  for (int r = 0; r < ns; ++r)
    for (int c = 0; c < nci; ++c) rec[L.off_B + r * nci + c] = Bd[r * 4 + input_order[c]];
  for (int o = 0; o < d->ny; ++o) {
    if (out_idx[o] < 0 || out_idx[o] >= no) return -1;
    for (int k = 0; k < ns; ++k) rec[L.off_C + o * L.nobs + k] = C[out_idx[o] * ns + k];
    for (int k = 0; k < d->ndist; ++k) rec[L.off_C + o * L.nobs + ns + k] = (out_idx[o] == k) ? 1.0 : 0.0;
  }
  std::memcpy(rec + L.off_f, fd, sizeof(double) * ns);
  return 0;
}

}  // extern "C"
