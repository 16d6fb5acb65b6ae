// Test harness: the product's QP solver (compressor-mpc_amd/csrc/qp_solver.h)
// compiled for the host, so tests can diff that exact code against the
// oracle without a GPU.  Not part of the product.
#include <string.h>

#include <type_traits>

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

// K Jacobi-iteration solves of one QP in the map form (qp_solve_map), the
// working set carried from solve to solve and the map kept across them as
// the iterate kernel keeps it: H, f, G (n x nvo row-major), d (K x nvo).
// Outputs per iteration k: x[k*n..], st[k], nchg[k], ws_out[k], trace[k*16..],
// ntrace[k].
template <int N, int NU, int NVO, bool LDS_HINV = false>
static void run_map(const double* Hp, const double* fp, const double* Gp, const double* dp, int K,
                    const double* lb, const double* ub, const double* lbA, const double* ubA,
                    uint32_t ws_in, int max_chg, double* xo, int32_t* st, int32_t* nchg, uint32_t* ws_out,
                    uint8_t* trace, int32_t* ntrace) {
  constexpr int NVOA = JMap<N, NVO>::NVOA;
  double H[N][N], f[N];
  // H^-1 in registers, or (LDS_HINV) as the iterate kernel keeps it: the
  // upper triangle in a strided array read by columns
  using HS = std::conditional_t<LDS_HINV, HinvStrided<N, 3>, HinvRegs<N>>;
  double hbuf[N * N * 3];
  Qp<N, NU, N, HS> qp;
  if constexpr (LDS_HINV) qp.Hinv.p = hbuf;
  for (int a = 0; a < N; ++a) {
    for (int b = 0; b < N; ++b) H[a][b] = Hp[a * N + b];
    f[a] = fp[a];
    qp.lb[a] = lb[a]; qp.ub[a] = ub[a]; qp.lbA[a] = lbA[a]; qp.ubA[a] = ubA[a];
  }
  qp.tolerances();
  const bool pd = hinv_of<N>(H, qp.Hinv);
  double hmax = 0.0;
  for (int i = 0; i < N; ++i) hmax = fabs(H[i][i]) > hmax ? fabs(H[i][i]) : hmax;
  double xu0[N], Ub[N * NVOA];
  for (int i = 0; i < N * NVOA; ++i) Ub[i] = NVO > 0 ? Gp[i] : 0.0;
  jmap_terms<N, NVO, 1>(qp.Hinv, f, Ub, xu0);
  const UStrided<NVOA, 1> U{Ub};
  JMap<N, NVO> mp;
  mp.ws = kWsInvalid;
  uint32_t ws = ws_in;
  for (int k = 0; k < K; ++k) {
    double d[NVOA] = {0.0}, x[N];
    for (int c = 0; c < NVO; ++c) d[c] = dp[k * NVO + c];
    QpOut o;
    qp_solve_map<true, N, NVO>(qp, pd, TOL_D * (1.0 + hmax), xu0, U, d, ws, max_chg, x, o, mp);
    ws = o.ws;
    for (int a = 0; a < N; ++a) xo[k * N + a] = x[a];
    st[k] = o.status; nchg[k] = o.nchg; ws_out[k] = o.ws; ntrace[k] = o.ntrace;
    memcpy(trace + 16 * k, o.tr, 16);
  }
}

extern "C" int qp_host_jacobi(int n, int nu, int nvo, const double* H, const double* f, const double* G,
                              const double* d, int K, const double* lb, const double* ub, const double* lbA,
                              const double* ubA, uint32_t ws_in, int max_chg, double* x, int32_t* st,
                              int32_t* nchg, uint32_t* ws_out, uint8_t* trace, int32_t* ntrace) {
  if (n == 4 && nu == 2 && nvo == 4)
    run_map<4, 2, 4>(H, f, G, d, K, lb, ub, lbA, ubA, ws_in, max_chg, x, st, nchg, ws_out, trace, ntrace);
  else if (n == 4 && nu == 2 && nvo == -4)  // H^-1 stored as the iterate kernel's LDS copy
    run_map<4, 2, 4, true>(H, f, G, d, K, lb, ub, lbA, ubA, ws_in, max_chg, x, st, nchg, ws_out, trace, ntrace);
  else if (n == 6 && nu == 2 && nvo == 6)
    run_map<6, 2, 6>(H, f, G, d, K, lb, ub, lbA, ubA, ws_in, max_chg, x, st, nchg, ws_out, trace, ntrace);
  else if (n == 8 && nu == 4 && nvo == 0)
    run_map<8, 4, 0>(H, f, G, d, K, lb, ub, lbA, ubA, ws_in, max_chg, x, st, nchg, ws_out, trace, ntrace);
  else
    return -1;
  return 0;
}
