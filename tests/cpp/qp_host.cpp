// Test harness: the product's QP solver (compressor-mpc_amd/csrc/qp_solver.h)
// compiled for the host, so tests can diff that exact code against the
// oracle without a GPU.  Not part of the product.
#include <string.h>

#include "../../compressor-mpc_amd/csrc/qp_solver.h"

template <int N, int NU>
static void run(const double* Hp, const double* gp, const double* lb, const double* ub,
                const double* lbA, const double* ubA, uint32_t ws_in, int max_chg, double* xo,
                int32_t* st, int32_t* nchg, uint32_t* ws_out, uint8_t* trace, int32_t* ntrace) {
  double H[N][N], g[N];
  Qp<N, NU> qp;
  for (int a = 0; a < N; ++a) {
    for (int b = 0; b < N; ++b) H[a][b] = Hp[a * N + b];
    g[a] = gp[a];
    qp.lb[a] = lb[a]; qp.ub[a] = ub[a]; qp.lbA[a] = lbA[a]; qp.ubA[a] = ubA[a];
  }
  qp.tolerances();
  const bool pd = hinv_of<N>(H, qp.Hinv);
  double hmax = 0.0;
  for (int i = 0; i < N; ++i) hmax = fabs(H[i][i]) > hmax ? fabs(H[i][i]) : hmax;
  double x[N];
  QpOut o;
  qp_solve<N, NU>(qp, pd, TOL_D * (1.0 + hmax), g, ws_in, max_chg, x, o);
  for (int a = 0; a < N; ++a) xo[a] = x[a];
  *st = o.status; *nchg = o.nchg; *ws_out = o.ws; *ntrace = o.ntrace;
  memcpy(trace, o.tr, 16);
}

extern "C" int qp_host_solve(int n, int nu, const double* H, const double* g, const double* lb,
                             const double* ub, const double* lbA, const double* ubA,
                             uint32_t ws_in, int max_chg, double* x, int32_t* st, int32_t* nchg,
                             uint32_t* ws_out, uint8_t* trace, int32_t* ntrace) {
  if (n == 4 && nu == 2) run<4, 2>(H, g, lb, ub, lbA, ubA, ws_in, max_chg, x, st, nchg, ws_out, trace, ntrace);
  else if (n == 8 && nu == 4) run<8, 4>(H, g, lb, ub, lbA, ubA, ws_in, max_chg, x, st, nchg, ws_out, trace, ntrace);
  else return -1;
  return 0;
}
