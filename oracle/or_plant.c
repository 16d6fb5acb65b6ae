/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into the product.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as a checker / CPU baseline.
 *
 * Plain-C restatement of the reference's compressor plant models and of the
 * Taylor-4 ("RK4") discretisation, used to produce the linearisations that
 * feed the condensed-QP hot path when pinning the oracle against the
 * reference's step-0 golden records (results/<plant>/run1/<cfg>.dat line 3).
 *
 *   ValveEqs                      include/valve_eqs.h:16-50
 *   Compressor<>::GetDerivative   systems/compressor.cc:14-66
 *   CompressorBase::GetOutput     systems/compressor.cc:68-78
 *   Compressor<>::GetLinearized.. systems/compressor.cc:80-175
 *   CompressorBase::Parameters    systems/compressor.cc:177-221
 *   Tank                          systems/tank.cc:10-49
 *   ParallelCompressors           systems/parallel_compressors.cc:9-128,
 *                                 include/parallel_compressors.h:44-98
 *   SerialCompressors             systems/serial_compressors.cc:8-117,
 *                                 include/serial_compressors.h:49-127
 *   DiscretizeRK4                 libs/aug_lin_sys.cc:232-255
 */
#include <math.h>
#include <string.h>

#include "cmpc_oracle.h"

static const double kPi = 3.14159265358979323846;
static const double kSound = 340.0;

typedef struct {
  double J, tau_r, m_in_c, m_out_c, torque_drive_c, delta_bar, n_bar;
  double V1, V2, AdivL, SD_multiplier;
  double C[8], D[8], A[12], m_rec_ss_c[2], SD_c[2], T_ss_c[3];
} comp_params;

typedef struct {
  double volume, D[8], m_out_c;
} tank_params;

/* systems/compressor.cc:177-221 */
static void comp_default(comp_params* p) {
  static const double A[12] = {0.000299749505193654,  -0.000171254191089237,
                               3.57321648097597e-05,  -9.1783572200945e-07,
                               -0.252701086129365,    0.136885752773673,
                               -0.02642368327081,     0.00161012740365743,
                               54.8046725371143,      -29.9550791497765,
                               5.27827499839098,      0.693826282579158};
  static const double C[8] = {-0.423884232813775, 0.626400271518973,
                              -0.0995040168384753, 0.0201535563630318,
                              -0.490814924104294, 0.843580880467905,
                              -0.423103455111209, 0.0386841406482887};
  static const double D[8] = {-0.0083454, -0.0094965, 0.16826, -0.032215,
                              -0.61199,   0.94175,    -0.48522, 0.10369};
  p->J = (0.4 + 0.2070) * 0.4;
  p->tau_r = 1 / 0.5;
  memcpy(p->A, A, sizeof A);
  memcpy(p->C, C, sizeof C);
  memcpy(p->D, D, sizeof D);
  p->m_in_c = 0.0051;
  p->m_rec_ss_c[0] = 0.0047;
  p->m_rec_ss_c[1] = 0.0263;
  p->m_out_c = 0.017;
  p->T_ss_c[0] = 2.5543945754982;
  p->T_ss_c[1] = 47.4222669576423;
  p->T_ss_c[2] = 0.6218;
  p->SD_c[0] = 5.55;
  p->SD_c[1] = 0.66;
  p->SD_multiplier = 100;
  p->torque_drive_c = 15000;
  p->delta_bar = 0.1;
  p->n_bar = 1e2;
  p->V1 = 2 * kPi * (0.60 / 2.0) * (0.60 / 2.0) * 2.0 +
          kPi * (0.08 / 2.0) * (0.08 / 2.0) * 8.191;
  p->V2 = kPi * (0.60 / 2.0) * (0.60 / 2.0) * 2.0 +
          kPi * (0.08 / 2.0) * (0.08 / 2.0) * 5.940;
  p->AdivL = kPi * (0.08 / 2) * (0.08 / 2) / 3 * 0.1;
}

/* systems/tank.cc:43-49 */
static void tank_default(tank_params* t) {
  static const double D[8] = {-0.0083454, -0.0094965, 0.16826, -0.032215,
                              -0.61199,   0.94175,    -0.48522, 0.10369};
  t->volume = 20 * kPi * (0.60 / 2) * (0.60 / 2) * 2 +
              kPi * (0.08 / 2) * (0.08 / 2) * 5.940;
  memcpy(t->D, D, sizeof D);
  t->m_out_c = 0.017;
}

static double sgn(double v) { return (double)((v > 0) - (v < 0)); }

/* include/valve_eqs.h:16-27 */
static double valve_derivative(double p_in, double p_out, double u,
                               const double* C, double volume) {
  const double M = u * u * u * C[0] + u * u * C[1] + u * C[2] + C[3];
  return kSound * kSound / volume * 1e-5 *
         (sgn(p_in - p_out) / 2. * 100 / sqrt(fabs(p_in * 100 - p_out * 100))) *
         M;
}

/* include/valve_eqs.h:37-48 */
static double valve_mass_flow(double p_in, double p_out, double u,
                              const double* C, double m_offset) {
  const double dp = 10 * sqrt(fabs(p_in - p_out)) * sgn(p_in - p_out);
  const double M3[8] = {dp * u * u * u, dp * u * u, dp * u, dp,
                        u * u * u,      u * u,      u,      1};
  double s = 0;
  for (int i = 0; i < 8; ++i) s += C[i] * M3[i];
  return s + m_offset;
}

/* systems/compressor.cc:14-66.  u = {torque, u_input, u_out, u_rec, m_in|p_in, p_out} */
static void comp_derivative(const comp_params* P, int has_tank, double* m_out,
                            const double* x, const double* u, double* dx) {
  const double p1 = x[0], p2 = x[1], mc = x[2], wc = x[3], mr = x[4];
  const double td = u[0] * P->torque_drive_c / wc;
  const double u_input = u[1], u_out = u[2], u_rec = u[3], p_out = u[5];
  const double m_in =
      has_tank ? valve_mass_flow(u[4], p1, u_input, P->C, P->m_in_c) : u[4];
  *m_out = valve_mass_flow(p2, p_out, u_out, P->D, P->m_out_c);
  const double m_rec_ss =
      (P->m_rec_ss_c[0] * (sqrt(p2 * 1e5 - p1 * 1e5) * u_rec) +
       P->m_rec_ss_c[1] * 1) *
      (u_rec > 1e-2);
  const double mc2 = mc * mc, mc3 = mc * mc2, wc2 = wc * wc;
  const double M[12] = {wc2 * mc3, wc2 * mc2, wc2 * mc, wc2, wc * mc3, wc * mc2,
                        wc * mc,   wc,        mc3,      mc2, mc,       1};
  double p_ratio = 0;
  for (int i = 0; i < 12; ++i) p_ratio += P->A[i] * M[i];
  const double T_ss_model = P->T_ss_c[0] + P->T_ss_c[1] * mc + P->T_ss_c[2];
  dx[0] = kSound * kSound / P->V1 * (m_in + mr - mc) * 1e-5;
  dx[1] = kSound * kSound / P->V2 * (mc - mr - *m_out) * 1e-5;
  dx[2] = P->AdivL * (p_ratio * p1 - p2) * 1e5;
  dx[3] = (td - T_ss_model) / P->J;
  dx[4] = P->tau_r * (m_rec_ss - mr);
}

/* systems/compressor.cc:68-78 */
static void comp_output(const comp_params* P, const double* x, double* y) {
  const double p1 = x[0], p2 = x[1], mass_flow = x[2];
  y[0] = p2;
  y[1] = P->SD_multiplier *
         (-(p2 / p1) / P->SD_c[0] + P->SD_c[1] / P->SD_c[0] + mass_flow);
}

/* systems/compressor.cc:80-175.  A 5x5, B 5x2, C 2x5 row-major. */
static void comp_linearize(const comp_params* P, int has_tank, double* m_out,
                           const double* x, const double* u, double* A,
                           double* B, double* C, double* f) {
  const double p1 = x[0], p2 = x[1], mc = x[2], wc = x[3];
  const double td_in = u[0], u_input = u[1], u_out = u[2], u_rec = u[3];
  const double p_out = u[5];
  const double k1 = kSound * kSound / P->V1 * 1e-5;
  const double k2 = kSound * kSound / P->V2 * 1e-5;
  memset(A, 0, 25 * sizeof(double));
  A[0] = -1; A[2] = -k1; A[4] = k1;
  if (has_tank) A[0] = -valve_derivative(u[4], p1, u_input, P->C, P->V1);
  A[5 + 1] = -valve_derivative(p2, p_out, u_out, P->D, P->V2);
  A[5 + 2] = k2;
  A[5 + 4] = -k2;
  const double wc2 = wc * wc, mc2 = mc * mc, mc3 = mc * mc2;
  const double dM_dm[12] = {3 * wc2 * mc2, 2 * wc2 * mc, wc2, 0,
                            3 * wc * mc2,  2 * wc * mc,  wc,  0,
                            3 * mc2,       2 * mc,       1,   0};
  const double dM_dw[12] = {2 * wc * mc3, 2 * wc * mc2, 2 * wc * mc, 2 * wc,
                            mc3,          mc2,          mc,          1,
                            0,            0,            0,           0};
  const double M[12] = {wc2 * mc3, wc2 * mc2, wc2 * mc, wc2, wc * mc3, wc * mc2,
                        wc * mc,   wc,        mc3,      mc2, mc,       1};
  double p_ratio = 0, a_dm = 0, a_dw = 0;
  for (int i = 0; i < 12; ++i) {
    p_ratio += P->A[i] * M[i];
    a_dm += P->A[i] * dM_dm[i];
    a_dw += P->A[i] * dM_dw[i];
  }
  A[10 + 0] = P->AdivL * (p_ratio * 1e5);
  A[10 + 1] = -P->AdivL * 1e5;
  A[10 + 2] = P->AdivL * (p1 * 1e5) * a_dm;
  A[10 + 3] = P->AdivL * (p1 * 1e5) * a_dw;
  A[15 + 2] = -1.0 / P->J * P->T_ss_c[1];
  A[15 + 3] = -1.0 / P->J * td_in * P->torque_drive_c / wc2;
  const double sq = sqrt(p2 * 1e5 - p1 * 1e5);
  const double qr = P->tau_r * (P->m_rec_ss_c[0] * 1 / 2 * u_rec / sq * 1e5);
  A[20 + 0] = -qr;
  A[20 + 1] = qr;
  A[20 + 4] = -P->tau_r;
  double dmr_ur = P->tau_r * P->m_rec_ss_c[0] * sq;
  const double x0 = 1e-2;
  if (u_rec < 2 * x0) {
    double a;
    if (u_rec >= x0)
      a = P->delta_bar + (1 - P->delta_bar) * exp(P->n_bar * (u_rec - x0));
    else
      a = 2 - (1 - P->delta_bar) * exp(-P->n_bar * u_rec);
    dmr_ur = a * dmr_ur;
  }
  memset(B, 0, 10 * sizeof(double));
  B[3 * 2 + 0] = 1.0 / P->J * P->torque_drive_c / wc;
  B[4 * 2 + 1] = dmr_ur;
  memset(C, 0, 10 * sizeof(double));
  C[1] = 1;
  C[5 + 0] = 100 * p2 / (P->SD_c[0] * p1 * p1);
  C[5 + 1] = -100. / (P->SD_c[0] * p1);
  C[5 + 2] = 100;
  comp_derivative(P, has_tank, m_out, x, u, f);
}

/* -------------------------------------------------------------------------- */
/* Parallel plant: ns=11, ni=9, no=4, control inputs <0,3,4,7>                 */

static void par_comp_input(const double* u_in, int i, const double* x,
                           double p_in, double* u) {
  for (int k = 0; k < 4; ++k) u[k] = u_in[i * 4 + k];
  u[4] = p_in;
  u[5] = x[10];
}

/* systems/parallel_compressors.cc:28-110 */
static void par_linearize(double p_in, double p_out, const double* x,
                          const double* u, double* A, double* B, double* C,
                          double* f) {
  comp_params cp;
  tank_params tp;
  comp_default(&cp);
  tank_default(&tp);
  const int ns = 11, nci = 4;
  memset(A, 0, ns * ns * sizeof(double));
  memset(B, 0, ns * nci * sizeof(double));
  memset(C, 0, 4 * ns * sizeof(double));
  memset(f, 0, ns * sizeof(double));
  double cA[2][25], cB[2][10], cC[2][10], cf[2][5], m_out;
  double mass_flow_total = 0;
  for (int i = 0; i < 2; ++i) {
    double uc[6];
    par_comp_input(u, i, x, p_in, uc);
    comp_linearize(&cp, 1, &m_out, x + 5 * i, uc, cA[i], cB[i], cC[i], cf[i]);
    for (int r = 0; r < 5; ++r)
      for (int c = 0; c < 5; ++c) A[(5 * i + r) * ns + 5 * i + c] = cA[i][r * 5 + c];
    for (int r = 0; r < 5; ++r)
      for (int c = 0; c < 2; ++c) B[(5 * i + r) * nci + 2 * i + c] = cB[i][r * 2 + c];
    for (int c = 0; c < 5; ++c) C[i * ns + 5 * i + c] = cC[i][5 + c];
    mass_flow_total +=
        valve_mass_flow(x[5 * i + 1], x[10], u[4 * i + 2], cp.D, cp.m_out_c);
    const double dv_tank =
        valve_derivative(x[5 * i + 1], x[10], u[4 * i + 2], cp.D, tp.volume);
    A[10 * ns + 5 * i + 1] = dv_tank;
    A[(5 * i + 1) * ns + 10] =
        valve_derivative(x[5 * i + 1], x[10], u[4 * i + 2], cp.D, cp.V2);
    A[10 * ns + 10] += -dv_tank;
    for (int r = 0; r < 5; ++r) f[5 * i + r] = cf[i][r];
  }
  /* tank: u = {u_tank, p_out, mass_flow_in}; systems/tank.cc:26-40 */
  const double pd = x[10], u_tank = u[8];
  A[10 * ns + 10] += -valve_derivative(pd, p_out, u_tank, tp.D, tp.volume);
  for (int c = 0; c < 5; ++c) {
    C[2 * ns + c] = cC[0][c];
    C[2 * ns + 5 + c] = -cC[1][c];
  }
  C[3 * ns + 10] = 1;
  const double m_out_t = valve_mass_flow(pd, p_out, u_tank, tp.D, tp.m_out_c);
  f[10] = kSound * kSound / tp.volume * (mass_flow_total - m_out_t) * 1e-5;
}

/* systems/parallel_compressors.cc:113-128 */
static void par_output(const double* x, double* y) {
  comp_params cp;
  comp_default(&cp);
  double y0[2], y1[2];
  comp_output(&cp, x, y0);
  comp_output(&cp, x + 5, y1);
  y[0] = y0[1];
  y[1] = y1[1];
  y[2] = y0[0] - y1[0];
  y[3] = x[10];
}

/* -------------------------------------------------------------------------- */
/* Serial plant: ns=10, ni=8, no=4, control inputs <0,3,4,7>                   */

/* include/serial_compressors.h:105-127 */
static void ser_comp_input(const double* u_in, int i, const double* x,
                           double p_in_, double p_out_, double* u) {
  const double p_in = (i == 0) ? p_in_ : -1;
  const double p_out = (i == 1) ? p_out_ : x[(i + 1) * 5];
  for (int k = 0; k < 4; ++k) u[k] = u_in[i * 4 + k];
  u[4] = p_in;
  u[5] = p_out;
}

/* systems/serial_compressors.cc:8-26 */
static void ser_derivative(double p_in, double p_out, const double* x,
                           const double* u, double* dx) {
  comp_params cp;
  comp_default(&cp);
  double m_out = -1;
  for (int i = 0; i < 2; ++i) {
    double uc[6];
    ser_comp_input(u, i, x, p_in, p_out, uc);
    if (i > 0) uc[4] = m_out;
    comp_derivative(&cp, i == 0, &m_out, x + 5 * i, uc, dx + 5 * i);
  }
}

/* systems/serial_compressors.cc:28-106 (the follower is linearised with
 * GetCompressorInput(), not u_sub, exactly as the reference does; the only
 * quantity that differs, f, is overwritten by the full derivative). */
static void ser_linearize(double p_in, double p_out, const double* x,
                          const double* u, double* A, double* B, double* C,
                          double* f) {
  comp_params cp;
  comp_default(&cp);
  const int ns = 10, nci = 4;
  memset(A, 0, ns * ns * sizeof(double));
  memset(B, 0, ns * nci * sizeof(double));
  memset(C, 0, 4 * ns * sizeof(double));
  memset(f, 0, ns * sizeof(double));
  double cA[25], cB[10], cC[10], cf[5], m_out = 0, uc[6];
  ser_comp_input(u, 0, x, p_in, p_out, uc);
  comp_linearize(&cp, 1, &m_out, x, uc, cA, cB, cC, cf);
  for (int r = 0; r < 5; ++r)
    for (int c = 0; c < 5; ++c) A[r * ns + c] = cA[r * 5 + c];
  for (int r = 0; r < 5; ++r)
    for (int c = 0; c < 2; ++c) B[r * nci + c] = cB[r * 2 + c];
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 5; ++c) C[r * ns + c] = cC[r * 5 + c];
  A[5 * ns + 1] = valve_derivative(x[1], x[5], u[2], cp.D, cp.V1);
  for (int i = 1; i < 2; ++i) {
    ser_comp_input(u, i, x, p_in, p_out, uc);
    comp_linearize(&cp, 0, &m_out, x + 5 * i, uc, cA, cB, cC, cf);
    for (int r = 0; r < 5; ++r)
      for (int c = 0; c < 5; ++c) A[(5 * i + r) * ns + 5 * i + c] = cA[r * 5 + c];
    A[(5 * i) * ns + 5 * i] = -valve_derivative(
        x[(i - 1) * 5 + 1], x[i * 5], u[(i - 1) * 4 + 2], cp.D, cp.V1);
    A[((i - 1) * 5 + 1) * ns + i * 5] = valve_derivative(
        x[(i - 1) * 5 + 1], x[i * 5], u[(i - 1) * 4 + 2], cp.D, cp.V2);
    for (int r = 0; r < 5; ++r)
      for (int c = 0; c < 2; ++c) B[(5 * i + r) * nci + 2 * i + c] = cB[r * 2 + c];
    for (int r = 0; r < 2; ++r)
      for (int c = 0; c < 5; ++c) C[(2 * i + r) * ns + 5 * i + c] = cC[r * 5 + c];
    ser_derivative(p_in, p_out, x, u, f);
  }
}

/* systems/serial_compressors.cc:108-117 */
static void ser_output(const double* x, double* y) {
  comp_params cp;
  comp_default(&cp);
  comp_output(&cp, x, y);
  comp_output(&cp, x + 5, y + 2);
}

/* -------------------------------------------------------------------------- */

int or_plant_dims(int plant, int* ns, int* ni, int* no, int* nci) {
  if (plant == OR_PLANT_PARALLEL) {
    *ns = 11; *ni = 9; *no = 4; *nci = 4;
    return 0;
  }
  if (plant == OR_PLANT_SERIAL) {
    *ns = 10; *ni = 8; *no = 4; *nci = 4;
    return 0;
  }
  return -1;
}

void or_plant_default(int plant, double* x, double* u) {
  if (plant == OR_PLANT_PARALLEL) {
    /* include/parallel_compressors.h:74-86 */
    static const double xd[11] = {0.916, 1.145, 0.152, 440, 0, 0.916,
                                  1.145, 0.152, 440,   0,   1.12};
    static const double ud[9] = {0.304, 0.43, 1.0, 0, 0.304, 0.43, 1.0, 0, 0.7};
    if (x) memcpy(x, xd, sizeof xd);
    if (u) memcpy(u, ud, sizeof ud);
  } else {
    /* include/serial_compressors.h:85-95 */
    static const double xd[10] = {0.867, 1.03, 0.176, 395, 0,
                                  0.999, 1.19, 0.176, 395, 0};
    static const double ud[8] = {0.304, 0.405, 1, 0, 0.304, -1, 0.393, 0};
    if (x) memcpy(x, xd, sizeof xd);
    if (u) memcpy(u, ud, sizeof ud);
  }
}

void or_plant_linearize(int plant, double p_in, double p_out, const double* x,
                        const double* u, double* A, double* B, double* C,
                        double* f) {
  if (plant == OR_PLANT_PARALLEL)
    par_linearize(p_in, p_out, x, u, A, B, C, f);
  else
    ser_linearize(p_in, p_out, x, u, A, B, C, f);
}

void or_plant_output(int plant, const double* x, double* y) {
  if (plant == OR_PLANT_PARALLEL)
    par_output(x, y);
  else
    ser_output(x, y);
}

/* libs/aug_lin_sys.cc:232-255.  Row-major; A ns x ns, B ns x nci. */
void or_discretize_rk4(int ns, int nci, double Ts, const double* A,
                       const double* B, const double* f, double* Ad,
                       double* Bd, double* fd) {
  double A2[16 * 16], A3[16 * 16], Ac[16 * 16];
  for (int i = 0; i < ns; ++i)
    for (int j = 0; j < ns; ++j) {
      double s = 0;
      for (int k = 0; k < ns; ++k) s += A[i * ns + k] * A[k * ns + j];
      A2[i * ns + j] = s;
    }
  for (int i = 0; i < ns; ++i)
    for (int j = 0; j < ns; ++j) {
      double s = 0;
      for (int k = 0; k < ns; ++k) s += A2[i * ns + k] * A[k * ns + j];
      A3[i * ns + j] = s;
    }
  for (int i = 0; i < ns; ++i)
    for (int j = 0; j < ns; ++j)
      Ac[i * ns + j] = Ts * (i == j) + Ts * Ts / 2.0 * A[i * ns + j] +
                       Ts * Ts * Ts / 6.0 * A2[i * ns + j] +
                       Ts * Ts * Ts * Ts / 24.0 * A3[i * ns + j];
  for (int i = 0; i < ns; ++i)
    for (int j = 0; j < ns; ++j) {
      double s = 0;
      for (int k = 0; k < ns; ++k) s += Ac[i * ns + k] * A[k * ns + j];
      Ad[i * ns + j] = (i == j) + s;
    }
  for (int i = 0; i < ns; ++i)
    for (int j = 0; j < nci; ++j) {
      double s = 0;
      for (int k = 0; k < ns; ++k) s += Ac[i * ns + k] * B[k * nci + j];
      Bd[i * nci + j] = s;
    }
  for (int i = 0; i < ns; ++i) {
    double s = 0;
    for (int k = 0; k < ns; ++k) s += Ac[i * ns + k] * f[k];
    fd[i] = s;
  }
}

/* ParallelCompressors::GetDerivative (systems/parallel_compressors.cc:9-26,
 * tank: systems/tank.cc:10-24), SerialCompressors::GetDerivative
 * (systems/serial_compressors.cc:8-26). */
int or_plant_derivative(int plant, double p_in, double p_out, const double* x,
                        const double* u, double* dx) {
  if (plant == OR_PLANT_PARALLEL) {
    comp_params cp;
    tank_params tp;
    comp_default(&cp);
    tank_default(&tp);
    double mass_flow_total = 0, m_out;
    for (int i = 0; i < 2; ++i) {
      double uc[6];
      par_comp_input(u, i, x, p_in, uc);
      comp_derivative(&cp, 1, &m_out, x + 5 * i, uc, dx + 5 * i);
      mass_flow_total += m_out;
    }
    const double m_out_t = valve_mass_flow(x[10], p_out, u[8], tp.D, tp.m_out_c);
    dx[10] = kSound * kSound / tp.volume * (mass_flow_total - m_out_t) * 1e-5;
    return 0;
  }
  if (plant == OR_PLANT_SERIAL) {
    ser_derivative(p_in, p_out, x, u, dx);
    return 0;
  }
  return -1;
}
