// The reference plants as __host__ __device__ code: one source for the host
// record producer (plant.cpp, cmpc_plant_lin_record) and the device producer
// (produce.hip, cmpc_produce_lin).  Restates
//   Compressor<has_input_tank>  systems/compressor.cc:14-221
//   Tank                        systems/tank.cc:10-49
//   ValveEqs                    include/valve_eqs.h:16-50
//   ParallelCompressors         systems/parallel_compressors.cc:28-128
//   SerialCompressors           systems/serial_compressors.cc:8-117
// (continuous-time linearisation, AugmentedLinearizedSystem::Update,
// libs/aug_lin_sys.cc:145-177).  Compiled with -ffp-contract=off on both
// sides, so host and device agree to the last bit except where exp() is
// used (the recycle-valve dead-zone, < 1 ulp apart between libm and OCML).
#pragma once
#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define CMPC_PHD __host__ __device__ inline
#else
#define CMPC_PHD inline
#endif

namespace cmpc_plant {

constexpr double kPi = 3.14159265358979323846;
constexpr double kC2 = 340.0 * 340.0;  // speed of sound squared

CMPC_PHD void zero(double* p, int n) {
  for (int i = 0; i < n; ++i) p[i] = 0.0;
}

struct CompressorParams {
  double J = (0.4 + 0.2070) * 0.4;
  double tau_r = 1 / 0.5;
  double m_in_c = 0.0051, m_out_c = 0.017, torque_drive_c = 15000;
  double delta_bar = 0.1, n_bar = 1e2, SD_multiplier = 100;
  double A[12] = {0.000299749505193654, -0.000171254191089237, 3.57321648097597e-05,
                  -9.1783572200945e-07, -0.252701086129365,   0.136885752773673,
                  -0.02642368327081,    0.00161012740365743,  54.8046725371143,
                  -29.9550791497765,    5.27827499839098,     0.693826282579158};
  double C[8] = {-0.423884232813775, 0.626400271518973, -0.0995040168384753,
                 0.0201535563630318, -0.490814924104294, 0.843580880467905,
                 -0.423103455111209, 0.0386841406482887};
  double D[8] = {-0.0083454, -0.0094965, 0.16826, -0.032215,
                 -0.61199,   0.94175,    -0.48522, 0.10369};
  double m_rec_ss_c[2] = {0.0047, 0.0263};
  double T_ss_c[3] = {2.5543945754982, 47.4222669576423, 0.6218};
  double SD_c[2] = {5.55, 0.66};
  double V1 = 2 * kPi * 0.3 * 0.3 * 2.0 + kPi * 0.04 * 0.04 * 8.191;
  double V2 = kPi * 0.3 * 0.3 * 2.0 + kPi * 0.04 * 0.04 * 5.940;
  double AdivL = kPi * 0.04 * 0.04 / 3 * 0.1;
};

struct TankParams {
  double volume = 20 * kPi * 0.3 * 0.3 * 2 + kPi * 0.04 * 0.04 * 5.940;
  double D[8] = {-0.0083454, -0.0094965, 0.16826, -0.032215,
                 -0.61199,   0.94175,    -0.48522, 0.10369};
  double m_out_c = 0.017;
};

CMPC_PHD double sgn(double v) { return (double)((v > 0) - (v < 0)); }

CMPC_PHD double valve_dpdp(double pin, double pout, double u, const double* C, double vol) {
  const double map = ((u * u * u) * C[0] + (u * u) * C[1]) + (u * C[2] + C[3]);
  return kC2 / vol * 1e-5 * (sgn(pin - pout) / 2. * 100 / sqrt(fabs(pin * 100 - pout * 100))) * map;
}

CMPC_PHD double valve_flow(double pin, double pout, double u, const double* C, double m_off) {
  const double dp = 10 * sqrt(fabs(pin - pout)) * sgn(pin - pout);
  const double basis[8] = {dp * u * u * u, dp * u * u, dp * u, dp, u * u * u, u * u, u, 1};
  double acc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) acc += C[k] * basis[k];
  return acc + m_off;
}

struct Compressor {
  CompressorParams P;
  bool input_tank;
  // u = {torque, u_input, u_out, u_rec, m_in|p_in, p_out}
  CMPC_PHD void derivative(const double* x, const double* u, double* dx, double* m_out) const {
    const double p1 = x[0], p2 = x[1], mc = x[2], wc = x[3], mr = x[4];
    const double m_in = input_tank ? valve_flow(u[4], p1, u[1], P.C, P.m_in_c) : u[4];
    *m_out = valve_flow(p2, u[5], u[2], P.D, P.m_out_c);
    const double mrec = (P.m_rec_ss_c[0] * (sqrt(p2 * 1e5 - p1 * 1e5) * u[3]) + P.m_rec_ss_c[1]) *
                        (u[3] > 1e-2 ? 1.0 : 0.0);
    const double mc2 = mc * mc, mc3 = mc2 * mc, wc2 = wc * wc;
    const double mono[12] = {wc2 * mc3, wc2 * mc2, wc2 * mc, wc2, wc * mc3, wc * mc2,
                             wc * mc,   wc,        mc3,      mc2, mc,       1};
    double pr = 0;
#pragma unroll
    for (int k = 0; k < 12; ++k) pr += P.A[k] * mono[k];
    dx[0] = kC2 / P.V1 * (m_in + mr - mc) * 1e-5;
    dx[1] = kC2 / P.V2 * (mc - mr - *m_out) * 1e-5;
    dx[2] = P.AdivL * (pr * p1 - p2) * 1e5;
    dx[3] = (u[0] * P.torque_drive_c / wc - (P.T_ss_c[0] + P.T_ss_c[1] * mc + P.T_ss_c[2])) / P.J;
    dx[4] = P.tau_r * (mrec - mr);
  }
  CMPC_PHD void output(const double* x, double* y) const {
    y[0] = x[1];
    y[1] = P.SD_multiplier * (-(x[1] / x[0]) / P.SD_c[0] + P.SD_c[1] / P.SD_c[0] + x[2]);
  }
  // A 5x5, B 5x2, C 2x5 (row-major), f 5
  CMPC_PHD void linearize(const double* x, const double* u, double* A, double* B, double* C, double* f,
                 double* m_out) const {
    const double p1 = x[0], p2 = x[1], mc = x[2], wc = x[3];
    const double k1 = kC2 / P.V1 * 1e-5, k2 = kC2 / P.V2 * 1e-5;
    zero(A, 25);
    A[0] = input_tank ? -valve_dpdp(u[4], p1, u[1], P.C, P.V1) : -1.0;
    A[2] = -k1;
    A[4] = k1;
    A[6] = -valve_dpdp(p2, u[5], u[2], P.D, P.V2);
    A[7] = k2;
    A[9] = -k2;
    const double mc2 = mc * mc, mc3 = mc2 * mc, wc2 = wc * wc;
    const double mono[12] = {wc2 * mc3, wc2 * mc2, wc2 * mc, wc2, wc * mc3, wc * mc2,
                             wc * mc,   wc,        mc3,      mc2, mc,       1};
    const double dm[12] = {3 * wc2 * mc2, 2 * wc2 * mc, wc2, 0, 3 * wc * mc2, 2 * wc * mc,
                           wc,            0,            3 * mc2, 2 * mc, 1, 0};
    const double dw[12] = {2 * wc * mc3, 2 * wc * mc2, 2 * wc * mc, 2 * wc, mc3, mc2,
                           mc,           1,            0,           0,      0,   0};
    double pr = 0, prm = 0, prw = 0;
    for (int k = 0; k < 12; ++k) {
      pr += P.A[k] * mono[k];
      prm += P.A[k] * dm[k];
      prw += P.A[k] * dw[k];
    }
    A[10] = P.AdivL * (pr * 1e5);
    A[11] = -P.AdivL * 1e5;
    A[12] = P.AdivL * (p1 * 1e5) * prm;
    A[13] = P.AdivL * (p1 * 1e5) * prw;
    A[17] = -1.0 / P.J * P.T_ss_c[1];
    A[18] = -1.0 / P.J * u[0] * P.torque_drive_c / wc2;
    const double root = sqrt(p2 * 1e5 - p1 * 1e5);
    const double rec = P.tau_r * (P.m_rec_ss_c[0] * 1 / 2 * u[3] / root * 1e5);
    A[20] = -rec;
    A[21] = rec;
    A[24] = -P.tau_r;
    double dmr = P.tau_r * P.m_rec_ss_c[0] * root;
    if (u[3] < 2e-2) {  // exponential dead-zone approximation
      const double a = (u[3] >= 1e-2) ? P.delta_bar + (1 - P.delta_bar) * exp(P.n_bar * (u[3] - 1e-2))
                                      : 2 - (1 - P.delta_bar) * exp(-P.n_bar * u[3]);
      dmr = a * dmr;
    }
    zero(B, 10);
    B[6] = 1.0 / P.J * P.torque_drive_c / wc;
    B[9] = dmr;
    zero(C, 10);
    C[1] = 1;
    C[5] = 100 * p2 / (P.SD_c[0] * p1 * p1);
    C[6] = -100. / (P.SD_c[0] * p1);
    C[7] = 100;
    derivative(x, u, f, m_out);
  }
};

// Continuous linearisation of the parallel plant, split so that the device
// producer runs the two compressors on two lanes: part(i) writes compressor
// i's blocks and leaves its outlet flow and tank coupling in tk[2i], tk[2i+1];
// tank() then adds the tank terms in the order of the single-lane loop.
CMPC_PHD void parallel_linearize_part(int i, double p_in, const double* x, const double* u, double* A,
                                      double* B, double* C, double* f, double* tk) {
  const int ns = 11;
  Compressor comp{CompressorParams(), true};
  TankParams tank;
  const double uc[6] = {u[4 * i], u[4 * i + 1], u[4 * i + 2], u[4 * i + 3], p_in, x[10]};
  double cA[25], cB[10], cC[10], cf[5], mo;
  comp.linearize(x + 5 * i, uc, cA, cB, cC, cf, &mo);
  for (int r = 0; r < 5; ++r) {
    for (int k = 0; k < 5; ++k) A[(5 * i + r) * ns + 5 * i + k] = cA[r * 5 + k];
    B[(5 * i + r) * 4 + 2 * i] = cB[r * 2];
    B[(5 * i + r) * 4 + 2 * i + 1] = cB[r * 2 + 1];
    f[5 * i + r] = cf[r];
  }
  for (int k = 0; k < 5; ++k) C[i * ns + 5 * i + k] = cC[5 + k];
  tk[2 * i] = valve_flow(x[5 * i + 1], x[10], u[4 * i + 2], comp.P.D, comp.P.m_out_c);
  const double to_tank = valve_dpdp(x[5 * i + 1], x[10], u[4 * i + 2], comp.P.D, tank.volume);
  tk[2 * i + 1] = to_tank;
  A[10 * ns + 5 * i + 1] = to_tank;
  A[(5 * i + 1) * ns + 10] = valve_dpdp(x[5 * i + 1], x[10], u[4 * i + 2], comp.P.D, comp.P.V2);
  for (int k = 0; k < 5; ++k) C[2 * ns + 5 * i + k] = i ? -cC[k] : cC[k];
}

CMPC_PHD void parallel_linearize_tank(double p_out, const double* x, const double* u, double* A,
                                      double* C, double* f, const double* tk) {
  const int ns = 11;
  TankParams tank;
  double a = 0.0, flow_total = 0.0;
  for (int i = 0; i < 2; ++i) {
    flow_total += tk[2 * i];
    a += -tk[2 * i + 1];
  }
  A[10 * ns + 10] = a + -valve_dpdp(x[10], p_out, u[8], tank.D, tank.volume);
  C[3 * ns + 10] = 1;
  f[10] = kC2 / tank.volume * (flow_total - valve_flow(x[10], p_out, u[8], tank.D, tank.m_out_c)) * 1e-5;
}

// Continuous linearisation of a reference plant: A ns x ns, B ns x 4, C 4 x ns, f ns.
// zero_out = false: A, B, C are already zero (the device producer clears
// them with the whole wave; one lane then writes only the nonzeros)
CMPC_PHD void parallel_linearize(double p_in, double p_out, const double* x, const double* u, double* A,
                        double* B, double* C, double* f, bool zero_out = true) {
  const int ns = 11;
  if (zero_out) {
    zero(A, ns * ns);
    zero(B, ns * 4);
    zero(C, 4 * ns);
  }
  double tk[4];
  for (int i = 0; i < 2; ++i) parallel_linearize_part(i, p_in, x, u, A, B, C, f, tk);
  parallel_linearize_tank(p_out, x, u, A, C, f, tk);
}

// ParallelCompressors::GetDerivative (systems/parallel_compressors.cc:9-26;
// tank: systems/tank.cc:10-24)
CMPC_PHD void parallel_derivative(double p_in, double p_out, const double* x, const double* u,
                                  double* dx) {
  Compressor comp{CompressorParams(), true};
  TankParams tank;
  double flow_total = 0, mo;
  for (int i = 0; i < 2; ++i) {
    const double uc[6] = {u[4 * i], u[4 * i + 1], u[4 * i + 2], u[4 * i + 3], p_in, x[10]};
    comp.derivative(x + 5 * i, uc, dx + 5 * i, &mo);
    flow_total += mo;
  }
  dx[10] = kC2 / tank.volume * (flow_total - valve_flow(x[10], p_out, u[8], tank.D, tank.m_out_c)) * 1e-5;
}

// GetOutput (systems/parallel_compressors.cc:112-127, serial: both compressors' outputs)
CMPC_PHD void parallel_output(const double* x, double* y) {
  Compressor comp{CompressorParams(), true};
  double y0[2], y1[2];
  comp.output(x, y0);
  comp.output(x + 5, y1);
  y[0] = y0[1];
  y[1] = y1[1];
  y[2] = y0[0] - y1[0];
  y[3] = x[10];
}
CMPC_PHD void serial_output(const double* x, double* y) {
  Compressor comp{CompressorParams(), true};
  comp.output(x, y);
  comp.output(x + 5, y + 2);
}

CMPC_PHD void serial_derivative(double p_in, double p_out, const double* x, const double* u, double* dx) {
  Compressor first{CompressorParams(), true}, follower{CompressorParams(), false};
  double m_out = -1;
  const double u0[6] = {u[0], u[1], u[2], u[3], p_in, x[5]};
  first.derivative(x, u0, dx, &m_out);
  const double u1[6] = {u[4], u[5], u[6], u[7], m_out, p_out};
  follower.derivative(x + 5, u1, dx + 5, &m_out);
}

CMPC_PHD void serial_linearize(double p_in, double p_out, const double* x, const double* u, double* A,
                      double* B, double* C, double* f, bool zero_out = true) {
  const int ns = 10;
  Compressor first{CompressorParams(), true}, follower{CompressorParams(), false};
  if (zero_out) {
    zero(A, ns * ns);
    zero(B, ns * 4);
    zero(C, 4 * ns);
  }
  double cA[25], cB[10], cC[10], cf[5], mo;
  const double u0[6] = {u[0], u[1], u[2], u[3], p_in, x[5]};
  first.linearize(x, u0, cA, cB, cC, cf, &mo);
  for (int r = 0; r < 5; ++r) {
    for (int k = 0; k < 5; ++k) A[r * ns + k] = cA[r * 5 + k];
    B[r * 4] = cB[r * 2];
    B[r * 4 + 1] = cB[r * 2 + 1];
  }
  for (int r = 0; r < 2; ++r)
    for (int k = 0; k < 5; ++k) C[r * ns + k] = cC[r * 5 + k];
  A[5 * ns + 1] = valve_dpdp(x[1], x[5], u[2], first.P.D, follower.P.V1);
  // follower linearised with GetCompressorInput (p_in = -1), as the reference does
  const double u1[6] = {u[4], u[5], u[6], u[7], -1, p_out};
  follower.linearize(x + 5, u1, cA, cB, cC, cf, &mo);
  for (int r = 0; r < 5; ++r) {
    for (int k = 0; k < 5; ++k) A[(5 + r) * ns + 5 + k] = cA[r * 5 + k];
    B[(5 + r) * 4 + 2] = cB[r * 2];
    B[(5 + r) * 4 + 3] = cB[r * 2 + 1];
  }
  A[5 * ns + 5] = -valve_dpdp(x[1], x[5], u[2], first.P.D, follower.P.V1);
  A[1 * ns + 5] = valve_dpdp(x[1], x[5], u[2], first.P.D, first.P.V2);
  for (int r = 0; r < 2; ++r)
    for (int k = 0; k < 5; ++k) C[(2 + r) * ns + 5 + k] = cC[r * 5 + k];
  serial_derivative(p_in, p_out, x, u, f);
}

}  // namespace cmpc_plant
