#include <algorithm>
// MI355X (gfx950) kernels of the condensed-QP hot path.
//
// build  : AdjustAllDelayedStates + GeneratePrediction + GenerateDistributedQP
//          + GenerateQP (libs/aug_lin_sys.cc:260-334, include/aug_lin_sys.h:141-154,
//          include/distributed_solver.h:83-94, libs/mpc_qp_solver.cc:16-40)
//          for one QP per wavefront, prediction matrices never materialised.
// solve  : K Jacobi iterations of ApplyOtherInput + SolveQP
//          (include/nerve_center.h:146-172, include/distributed_solver.h:98-103,
//          libs/mpc_qp_solver.cc:42-75) for one QP per lane, the sub-controllers
//          of a scenario in adjacent lanes exchanging plans by lane shuffles.
//
// Build-kernel layout (one QP = one wave64 = four 16-lane DPP rows):
//   rows o < ny : row o of  P_i = L_W' C A^i        (L_W L_W' = ywt)
//                 lane j < ns          : P_i[o][j]             (broadcast source)
//                 lane ns + c          : P_i[o] . B_c          (raw Markov column c)
//                 lane ns + nu_tot     : z_i[o]                 (free response row)
//   row 3       : free response x_{i+1} = A x_i + f + Adelay w_i  (lanes j < ns)
//                 lanes ns + o         : (L_W' C x_{i+1})[o] + kappa[o] - yhat_i[o]
// One step of both chains is ns v_fmac_f64_dpp (row_newbcast) instructions.
// Because W is folded into P (W = L_W L_W'), H, G and f are plain sums over
// rows o and steps i of products of per-lane values: each step adds
// nV*m DPP-broadcast FMAs into accumulators that live in the Markov lanes,
// and one cross-row reduction at the end yields H (exactly symmetric),
// G = Su' W Su_other and f.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "cmpc_internal.h"
#include "dpp_blocks.inc"
#include "observer_body.h"
#include "produce_body.h"
#include "solve_rows.h"
#include "lane_solve.h"

// Ablation switches for timing experiments (tools/ablate.sh); the product
// build uses CMPC_EXP = 0.
#ifndef CMPC_EXP
#define CMPC_EXP 0
#endif
#if CMPC_EXP == 1
#define CMPC_EXP_GACC(v, acc) (void)0
#else
#define CMPC_EXP_GACC(v, acc) gacc_dpp<NUT, NU, M>(v, acc)
#endif
#if CMPC_EXP == 2
#define CMPC_EXP_HAND(...) rd = a;
#else
#define CMPC_EXP_HAND(...) __VA_ARGS__
#endif
#if CMPC_EXP == 3
#define CMPC_EXP_PROP(pv, m, a) prop1_dpp<6>(pv, m, a)
#else
#define CMPC_EXP_PROP(pv, m, a) prop1w_dpp<NS, ND>(pv, m, a)
#endif
#if CMPC_EXP == 4
#define CMPC_EXP_YH(...) yh = yh * 0.5
#else
#define CMPC_EXP_YH(...) __VA_ARGS__
#endif
#ifndef CMPC_BUILD_ILP
#define CMPC_BUILD_ILP 1
#endif

#if CMPC_BUILD_ILP == 4
#define CMPC_ILP_PROP(pv, m, ax) prop4w_dpp<NS, ND>(pv, m, ax)
#define CMPC_ILP_SUM(ax) (((ax)[0] + (ax)[1]) + ((ax)[2] + (ax)[3]))
#elif CMPC_BUILD_ILP == 3
#define CMPC_ILP_PROP(pv, m, ax) prop3w_dpp<NS, ND>(pv, m, ax)
#define CMPC_ILP_SUM(ax) (((ax)[0] + (ax)[1]) + (ax)[2])
#elif CMPC_BUILD_ILP == 2
#define CMPC_ILP_PROP(pv, m, ax) prop2w_dpp<NS, ND>(pv, m, (ax)[0], (ax)[1])
#define CMPC_ILP_SUM(ax) ((ax)[0] + (ax)[1])
#endif
#if CMPC_EXP == 5
#define CMPC_EXP_STEP(pv, m, a, va, acc)                  \
  {                                                       \
    va = __builtin_fma(smask, va, rd);                    \
    double a1_ = 0.0;                                     \
    prop2w_dpp<NS, ND>(pv, m, a, a1_);                    \
    a = a + a1_;                                          \
    CMPC_EXP_GACC(va, acc);                               \
  }
#elif CMPC_EXP == 6
#define CMPC_EXP_STEP(pv, m, a, va, acc)                  \
  {                                                       \
    va = __builtin_fma(smask, va, rd);                    \
    prop1w_gacc_dpp<NS, ND, NUT, NU, M>(pv, m, a, va, acc); \
  }
#elif CMPC_BUILD_ILP > 1
// several partial accumulators per chain (small batches: one wave per SIMD
// has no other wave to hide the dependent FP64 latency); the gather column
// update runs after the chain, off its critical path
#define CMPC_EXP_STEP(pv, m, a, va, acc)                                   \
  {                                                                        \
    double ax_[CMPC_BUILD_ILP];                                            \
    ax_[0] = a;                                                            \
    for (int k_ = 1; k_ < CMPC_BUILD_ILP; ++k_) ax_[k_] = 0.0;             \
    CMPC_ILP_PROP(pv, m, ax_);                                             \
    a = CMPC_ILP_SUM(ax_);                                                 \
    va = __builtin_fma(smask, va, rd);                                     \
    CMPC_EXP_GACC(va, acc);                                                \
  }
#else
// the gather column update consumes the previous step's hand-off read (rd)
// after the chain, so the LDS round trip hides behind it
#define CMPC_EXP_STEP(pv, m, a, va, acc)  \
  {                                       \
    CMPC_EXP_PROP(pv, m, a);              \
    va = __builtin_fma(smask, va, rd);    \
    CMPC_EXP_GACC(va, acc);               \
  }
#endif

// the role split's chain (build_wave_body SPLIT): CMPC_SPLIT_ILP partial
// accumulators per chain (its wave has no gather FMAs to interleave; 1 = the
// single chain of SPLIT = false)
#ifndef CMPC_SPLIT_ILP
#define CMPC_SPLIT_ILP 1
#endif
#if CMPC_SPLIT_ILP == 2
#define CMPC_SPLIT_CHAIN(pv, m, a)                  \
  {                                                 \
    double a1_ = 0.0;                               \
    prop2w_dpp<NS, ND>(pv, m, a, a1_);              \
    a = a + a1_;                                    \
  }
#elif CMPC_SPLIT_ILP == 3
#define CMPC_SPLIT_CHAIN(pv, m, a)                  \
  {                                                 \
    double ax_[3] = {a, 0.0, 0.0};                  \
    prop3w_dpp<NS, ND>(pv, m, ax_);                 \
    a = (ax_[0] + ax_[1]) + ax_[2];                 \
  }
#else
#define CMPC_SPLIT_CHAIN(pv, m, a) CMPC_EXP_PROP(pv, m, a)
#endif

// Diagnostic build (tools/rows_timing.py ... wave): per-wave s_memtime cycle
// totals of the QP phases of the one-QP-per-wave kernel, written over the QP
// output as the row kernel's CMPC_ROWS_TIMING (results invalid).
#ifndef CMPC_WAVE_TIMING
#define CMPC_WAVE_TIMING 0
#endif
#if CMPC_WAVE_TIMING
#define CMPC_WT(i)                                         \
  {                                                        \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();    \
    tsum[i] += now_ - tlast;                               \
    tlast = now_;                                          \
  }
#else
#define CMPC_WT(i)
#endif

// ---------------------------------------------------------------------------
// build kernel
// ---------------------------------------------------------------------------
// FUSE (cmpc_step on small batches, one QP per wave): 1/2 (centralized,
// S = 1): after a QP is built its wave runs the K Jacobi iterations on it
// (solve_rows.h: row 0 is the QP's solver row, rows 1-3 shadow it without
// stores); 3/4 (S divides 4, nV <= 4): the workgroup's QPs, built and stored
// one per wave, are solved one per lane of wave 0 after a workgroup barrier
// (lane_solve.h; a scenario's sub-controllers are adjacent waves, so adjacent
// lanes); 5 (the same, nV <= 4): solved one per DPP row of wave 0 by the row
// solver (solve_rows.h; faster than the lane solver at a few QPs).  Even FUSE
// values record the working-set trace.  The QP is stored either way
// (cmpc_download_qp).
//
// SPLIT (role split, small batches): two waves per QP, SW waves per
// workgroup (2: the split build kernel; 4: the one-launch control step, two
// QPs).  The even wave of a pair stages the record and runs the prologue and
// the DPP chain of every step (P rows and the free response; ny = 4: the
// pre-pass too), storing the raw Markov values into the delay lines and z
// into a two-block ring; the odd wave runs the gather FMAs one block behind,
// reading those values, then the epilogue (and the fused solve).  One
// workgroup barrier per block of up to U steps.  A pair uses two per-wave LDS
// regions (the QP's, then the ring's).  The same FMAs in the same order per
// lane: bit-identical to SPLIT = false, with the two waves' instructions
// sharing a SIMD's issue slots (one wave per SIMD issues an FP64 VALU about
// every 8 cycles).
template <int NS, int NY, int NUT, int NU, int M, int ND, int FUSE, bool SPLIT = false, int SW = 2>
__device__ __forceinline__ void build_wave_body(const BuildParams& P) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int NV = NU * M;
  constexpr int NG = M * NUT + 1;  // gather lanes per row: QP columns (move k, input c), then z
  constexpr int NDW = ND > 0 ? ND : 1;
  constexpr int NCH = CMPC_REC_CHUNKS;  // 16-byte record chunks per lane
  constexpr int U = 4;                  // horizon-loop unroll (immediate LDS offsets)
  static_assert(NG <= 16 && NS + NUT <= 16 && NS + NY + ND <= 16, "lane budget");
  static_assert(ND <= NY, "w table shares the yhat stride");
  static_assert(NY <= 4, "one DPP row per output");
  // ny = 4 leaves no DPP row for the free response: it then runs as a
  // pre-pass (every row simulating, row 3 storing z_r into per-output lines)
  // and the main pass has four P rows whose z lanes read those lines
  constexpr bool PRE = NY == 4;
  static_assert(!SPLIT || SW == 2 || SW == 4, "role split: two-wave pairs");
  constexpr int WGW = SPLIT ? SW : CMPC_BUILD_WAVES;      // waves per workgroup
  constexpr int QPG = SPLIT ? SW / 2 : CMPC_BUILD_WAVES;  // QPs per workgroup at a time
  const int lane = threadIdx.x & 63;
  const int wave = SPLIT ? (threadIdx.x >> 7) : (threadIdx.x >> 6);  // QP slot of the workgroup
  const bool wA = !SPLIT || ((threadIdx.x >> 6) & 1) == 0;           // chain (and prologue) wave
  const bool wB = !SPLIT || ((threadIdx.x >> 6) & 1) == 1;           // gather (and epilogue) wave
  const int row = lane >> 4, col = lane & 15;
  const int pp = P.p, S = P.S;
  const int nobs = P.nobs, rec_len = P.rec_len;
  const int nwaves = gridDim.x * QPG;
  const int nchunk = rec_len / 2;

  // Delay lines: one per (row o, input c), length D_c + M - 1 + p; the first
  // D_c + M - 1 entries are zero (history before t = 0), raw Markov value of
  // step r at index D_c + M - 1 + r.  Reading index (M - 1 - k) + r yields the
  // column (move k, input c) of row r for every c: the delay shifts out.
  // (offsets chosen on the host for conflict-free banking: build_lds_layout)
  int coff[NUT];
#pragma unroll
  for (int c = 0; c < NUT; ++c) coff[c] = P.line_off[c];
  const int rowlen = P.line_rs;

  // ---- LDS layout (doubles) ----
  // block: [yhat S x yl_stride][lwt S x NY x NY][uwt S x NU x NU][zeros 16]
  // wave : [rec rec_len][uold 8][chat NY x nobs][kappa 4]   (prologue only)
  //        overlaid by [delay lines NY x rowlen] (horizon loop), then by the
  //        row reduction (epilogue); followed by
  //        [w (p+3) x NY][z slots NY x U][scratch 64 + U]
  double* yl_all = smem;
  double* lw_all = yl_all + S * P.yl_stride;
  double* uw_all = lw_all + S * NY * NY;
  double* zeros = uw_all + S * NU * NU;
  double* recl = smem + P.lds_block + (SPLIT ? 2 * wave : wave) * P.lds_per_wave;
  const int o_uold = rec_len, o_chat = o_uold + 8, o_kap = o_chat + NY * nobs;
  const int o_line = 0, o_w = P.w_off, o_zl = P.zs_off;
  // Delay parameters in registers (compile-time indices only): a runtime-
  // indexed read of the kernel-argument struct inside the QP loop would be a
  // global load whose vmcnt(0) wait also drains the record prefetch.
  int wdl[NDW], wbo[NDW], wdi[NDW];
#pragma unroll
  for (int k = 0; k < NDW; ++k) {
    wdl[k] = (k < ND) ? P.dlen[k] : 0;
    wbo[k] = (k < ND) ? P.boff[k] : 0;
    wdi[k] = (k < ND) ? P.dinput[k] : 0;
  }
  const int nbound = P.nbound;
  int bnd[NUT];
#pragma unroll
  for (int c = 0; c < NUT; ++c) bnd[c] = P.bound[c];
  double* uol = recl + o_uold;
  double* chat = recl + o_chat;
  double* kap = recl + o_kap;
  double* wl = recl + o_w;
  double* lines = recl + o_line;
  double* zl = recl + o_zl;
  double* red = lines;
  for (int e = threadIdx.x; e < S * P.yl_stride; e += 64 * WGW) {
    const int ss = e / P.yl_stride, t = e - ss * P.yl_stride;
    yl_all[e] = (t < pp * NY) ? P.cfg[(size_t)ss * P.co.len + P.co.yhat + t] : 0.0;
  }
  for (int e = threadIdx.x; e < S * NY * NY; e += 64 * WGW)
    lw_all[e] = P.cfg[(size_t)(e / (NY * NY)) * P.co.len + P.co.lwt + e % (NY * NY)];
  for (int e = threadIdx.x; e < S * NU * NU; e += 64 * WGW)
    uw_all[e] = P.cfg[(size_t)(e / (NU * NU)) * P.co.len + P.co.uwt + e % (NU * NU)];
  if (threadIdx.x < 16) zeros[threadIdx.x] = 0.0;
  __syncthreads();

  // ---- static lane roles and LDS gather descriptors (same for every QP) ----
  const bool prow = row < NY;
  const bool srow = !PRE && row == 3;
  const int c_in = col - NS;
  const bool mlane = prow && col >= NS && col < NS + NUT;       // raw Markov writer
  const bool slane = srow && col >= NS && col < NS + NY;        // free-response writer
  const bool glane = prow && col < NG;                          // gather (accumulating) lane
  const bool wlane = srow && col >= 16 - ND;                    // delayed-input carrier lane
  const int oz = slane ? col - NS : 0;
  const int kw = wlane ? col - (16 - ND) : 0;
  const double ym = slane ? 1.0 : wlane ? -1.0 : 0.0;
  const double* zero_p = zeros;
  // m[l] = mb[l * ms]
  const double* mb = zero_p;
  int ms = 0;
  if (prow && col < NS) { mb = recl + P.off_A + col; ms = NS; }
  else if (mlane) { mb = recl + P.off_B + c_in; ms = NUT; }
  else if (srow && col < NS) { mb = recl + P.off_A + col * NS; ms = 1; }
  else if (slane) { mb = chat + oz * nobs; ms = 1; }
  // initial broadcast source and chain base
  const double* pv_src = (prow && col < NS) ? chat + row * nobs + col
                         : (srow && col < NS) ? recl + P.off_f + col
                         : wlane ? wl + NY + kw : zero_p;
  const double* base_src = (srow && col < NS) ? recl + P.off_f + col
                           : slane ? kap + oz : zero_p;
  const double* ad_src = (srow && col < NS) ? recl + P.off_B + col * NUT : zero_p;
  // hand-off: writers store their chain value of step r, gather lanes read
  // the QP column values of row r (one masked LDS write + read per step)
  // (delay-line pointers advance one entry per step, z slots are reused)
  double* wp = zl;  // (masked: lanes without a writer role do not store)
  int winc = 0, rinc = 0;
  if (mlane) { wp = lines + row * rowlen + coff[c_in] + M - 1; winc = 1; }
  else if (slane) wp = zl + oz * U;
  // Gather lane (k, c) reads line c at (m-1-k) + r - D_c once r >= D_c and the
  // zero slot before (the delay-line history); the loop is split at the
  // distinct delays.  Lanes without a gather role read the zero slot too (a
  // broadcast).
  const double* rp = zero_p;
  const double* rline = zero_p;  // line pointer taken at r = gdel
  int gdel = 0x7fffffff;
  double smask = 0.0;  // 1: running-sum column (move M-1)
  if (glane) {
    if (col < M * NUT) {
      const int k = col / NUT, c = col - k * NUT;
      rline = lines + row * rowlen + coff[c] + (M - 1 - k);
      gdel = P.delay[c];
      smask = (k == M - 1) ? 1.0 : 0.0;
      if (gdel == 0) { rp = rline; rinc = 1; }
    } else if (PRE) {
      rp = zl + row * P.zl_stride;  // z line of output row, one entry per step
      rinc = 1;
    } else {
      rp = zl + row * U;
    }
  }
  // one history entry of one delay line per lane (first m-1 entries of each)
  const bool zero_lane = M > 1 && lane < NY * NUT * (M - 1);
  int zero_at = 0;
  if (zero_lane) {
    const int o = lane / (NUT * (M - 1)), rem = lane - o * NUT * (M - 1);
    const int c = rem / (M > 1 ? M - 1 : 1), i = rem - c * (M > 1 ? M - 1 : 1);
#pragma unroll
    for (int cc = 0; cc < NUT; ++cc)
      if (cc == c) zero_at = o * rowlen + coff[cc] + i;
  }
  const bool red_lane = (row >= 1 && row < NY) && col < NG;
  double* red_w = red + ((row >= 1 ? row - 1 : 0) * NG + col) * NV;

  // ---- prefetch the first record (coalesced 16-byte loads) ----
  int q = blockIdx.x * QPG + wave;
  double2 chunk[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int ci = lane + 64 * i;
    chunk[i] = (wA && q < P.nqp && ci < nchunk)
                   ? reinterpret_cast<const double2*>(P.lin + (size_t)q * rec_len)[ci]
                   : make_double2(0.0, 0.0);
  }
  double uold_l = (q < P.nqp && lane < NUT) ? P.u_old[(size_t)q * NUT + lane] : 0.0;

  // fair progress of a SIMD's waves: priority drops per completed quarter of
  // the wave's share (the SIMD otherwise favours its oldest wave and the
  // kernel waits on the youngest; cf. build_rows.hip)
  const int share = (P.nqp + nwaves - 1) / nwaves;
  int done_qp = 0;
  __builtin_amdgcn_s_setprio(3);
#if CMPC_WAVE_TIMING
  uint64_t tsum[6] = {0, 0, 0, 0, 0, 0}, tlast = __builtin_amdgcn_s_memtime();
  const uint64_t t0c = tlast, t0r = __builtin_amdgcn_s_memrealtime();
#endif
  // (SPLIT: one QP per pair, the launcher's grid covers the batch: no
  // loop-carried state, so the fused solve has the registers of the build;
  // a pair past the batch runs once on the last QP, storing nothing, so that
  // the workgroup's barriers match)
  bool first_qp = true;
  for (; q < P.nqp || (SPLIT && first_qp); q = SPLIT ? P.nqp : q + nwaves) {
    const bool qv = q < P.nqp;
    if constexpr (SPLIT) {  // the previous QP's epilogue has read its LDS
      if (!first_qp) __syncthreads();
      first_qp = false;
      if (!qv) q = P.nqp - 1;
    }
    CMPC_WT(5)  // back-edge
    {
      const int level = 3 - (4 * done_qp) / share;
      if (level <= 0) __builtin_amdgcn_s_setprio(0);
      else if (level == 1) __builtin_amdgcn_s_setprio(1);
      else if (level == 2) __builtin_amdgcn_s_setprio(2);
      ++done_qp;
    }
    const int s = q % S;
    const double* yl = yl_all + s * P.yl_stride;
    const double* lwt = lw_all + s * NY * NY;
    // record -> LDS, then issue the next record's loads
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int ci = lane + 64 * i;
      if (wA && ci < nchunk) reinterpret_cast<double2*>(recl)[ci] = chunk[i];
    }
    if (wA && lane < NUT) uol[lane] = uold_l;
    {
      const int qn = SPLIT ? P.nqp : q + nwaves;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int ci = lane + 64 * i;
        chunk[i] = (wA && qn < P.nqp && ci < nchunk)
                       ? reinterpret_cast<const double2*>(P.lin + (size_t)qn * rec_len)[ci]
                       : make_double2(0.0, 0.0);
      }
      uold_l = (qn < P.nqp && lane < NUT) ? P.u_old[(size_t)qn * NUT + lane] : 0.0;
    }
    CMPC_WT(0)  // staging
    const double* Cs = recl + P.off_C;
    const double* xa = recl + P.off_x;
    // C_hat = L_W' C_sel (ny x nobs), one element per lane
    if (wA && prow && col < nobs) {
      double t = 0.0;
#pragma unroll
      for (int o2 = 0; o2 < NY; ++o2)
        if (o2 >= row) t += lwt[row * NY + o2] * Cs[o2 * nobs + col];
      chat[row * nobs + col] = t;
    }
    // delay-line inputs w_t (stride NY), AdjustAllDelayedStates applied
    // (include/aug_lin_sys.h:141-154); zero once the delay line has drained
    for (int e = lane; wA && e < (pp + 3) * NY; e += 64) {
      const int t = e / NY, k = e - t * NY;
      double v = 0.0;
      int dl = 0, bo = 0, di = 0;
#pragma unroll
      for (int kk = 0; kk < ND; ++kk)
        if (k == kk) { dl = wdl[kk]; bo = wbo[kk]; di = wdi[kk]; }
      if (t < dl) {
        const double x = (t == 0) ? xa[P.ndist + k] : xa[bo + t - 1];
        v = x - uol[di];
      }
      wl[e] = v;
    }
    // kappa = L_W'(dist + y_prev) = C_hat_dist xa_dist + L_W' y_prev
    if (wA && prow && col == 15) {
      const double* yp = recl + P.off_y;
      double t = 0.0;
      for (int d = 0; d < P.ndist; ++d) t += chat[row * nobs + NS + d] * xa[d];
#pragma unroll
      for (int o2 = 0; o2 < NY; ++o2)
        if (o2 >= row) t += lwt[row * NY + o2] * yp[o2];
      kap[row] = t;
    }
    if constexpr (PRE) if (wA) {
      // free-response pre-pass: the row-3 lane roles of the ny <= 3 layout in
      // every row (states j < ns, outputs ns + o, delayed-input carriers in
      // the top ND lanes); row 3's output lanes store z_r at zl[o][r]
      const bool s_st = col < NS, s_out = col >= NS && col < NS + NY, s_w = col >= 16 - ND;
      const int soz = s_out ? col - NS : 0, skw = s_w ? col - (16 - ND) : 0;
      const double sym = s_out ? 1.0 : s_w ? -1.0 : 0.0;
      const double* smb = s_st ? recl + P.off_A + col * NS : s_out ? chat + soz * nobs : zero_p;
      const int sms = (s_st || s_out) ? 1 : 0;
      const double* sad = s_st ? recl + P.off_B + col * NUT : zero_p;
      double sm[NS + NDW];
#pragma unroll
      for (int l = 0; l < NS; ++l) sm[l] = smb[l * sms];
#pragma unroll
      for (int k = 0; k < NDW; ++k) sm[NS + k] = (ND > 0) ? sad[s_st ? wdi[k] : 0] : 0.0;
      const double sbase = *(s_st ? recl + P.off_f + col : s_out ? kap + soz : zero_p);
      double spv = *(s_st ? recl + P.off_f + col : s_w ? wl + NY + skw : zero_p);
#pragma unroll
      for (int k = 0; k < ND; ++k) spv += sm[NS + k] * wl[k];  // x_1 = f + Adelay w_0
      // chain init of step r formed at the end of step r - 1 from an operand
      // read one step earlier still (the LDS latency hides behind a chain;
      // the last step reads one entry past the table, inside the block)
      double san = __builtin_fma(-sym, s_w ? wl[2 * NY + skw] : yl[soz], sbase);
      const double* sylp = s_w ? wl + 3 * NY + skw : yl + NY + soz;
      double syh = sylp[0];
      const bool zlane = row == 3 && s_out;
      double* zq = zl + soz * P.zl_stride;
#define CMPC_PRE_STEP(u)                          \
  {                                               \
    double a = san;                               \
    prop1w_dpp<NS, ND>(spv, sm, a);               \
    san = __builtin_fma(-sym, syh, sbase);        \
    syh = sylp[((u) + 1) * NY];                   \
    spv = a;                                      \
    if (zlane) zq[u] = a;                         \
  }
      int r = 0;
      for (; r + U <= pp; r += U) {
        CMPC_PRE_STEP(0)
        CMPC_PRE_STEP(1)
        CMPC_PRE_STEP(2)
        CMPC_PRE_STEP(3)
        zq += U;
        sylp += U * NY;
      }
      for (; r < pp; ++r) {
        CMPC_PRE_STEP(0)
        zq += 1;
        sylp += NY;
      }
#undef CMPC_PRE_STEP
    }
    // per-lane operands (branch-free gathers through the descriptors)
    // m[NS + k] = Adelay[j][k]: the sim row's state lanes pick up w_{r+1}
    // from the carrier lanes 16 - ND + k inside the DPP chain
    double m[NS + NDW];
#pragma unroll
    for (int l = 0; l < NS; ++l) m[l] = mb[l * ms];
#pragma unroll
    for (int k = 0; k < NDW; ++k) m[NS + k] = (ND > 0) ? ad_src[ms == 1 ? P.dinput[k] : 0] : 0.0;
    const double base = *base_src;
    double pv = *pv_src;
#pragma unroll
    for (int k = 0; k < ND; ++k) pv += m[NS + k] * wl[k];  // sim: x_1 = f + Adelay w_0

    // zero the first m-1 entries of every delay line (history before t = 0);
    // the record area the lines overlay is dead once the operands above are
    // in registers
    if (wA && zero_lane) lines[zero_at] = 0.0;
    double acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    double va = 0.0;  // gather lane: QP column value of the previous row
    double rd = 0.0;  // gather lane: raw value read at the end of the previous step
    // per-step operand: yhat_r (output lanes) / w_{r+2} (carrier lanes); the
    // chain init `an` of step r + 1 is formed at the end of step r from the
    // operand read during step r - 1 (two steps of LDS read-ahead; the last
    // step reads one entry past the table, inside the LDS block)
    double yh = wlane ? wl[2 * NY + kw] : yl[oz];
    const double* ylp = wlane ? wl + 3 * NY + kw : yl + NY + oz;
    double an = __builtin_fma(-ym, yh, base);
    if constexpr (!PRE) yh = ylp[0];
    double* wq = wp;
    const double* rq = rp;

    // one horizon step; u = position inside the unrolled group (immediate offsets)
#define CMPC_BUILD_STEP(u)                                                             \
  {                                                                                    \
    /* chain init: f (states), kappa - yhat_r (outputs), w_{r+2} (carriers) */         \
    double a = an;                                                                     \
    /* chain; accumulate row r-1: acc[a] += column_a * own column (gather lanes) */   \
    CMPC_EXP_STEP(pv, m, a, va, acc);                                                  \
    if constexpr (!PRE) an = __builtin_fma(-ym, yh, base);                             \
    CMPC_EXP_YH(if constexpr (!PRE) yh = ylp[((u) + 1) * NY]);                         \
    /* a: P rows -> P_{r+1} / raw Markov of step r; sim lanes -> x_{r+2} / z_r */      \
    pv = a;                                                                            \
    CMPC_EXP_HAND(if (mlane || slane) wq[u] = a; rd = rq[u];)                          \
  }

    CMPC_WT(2)  // prologue compute
    if constexpr (SPLIT) {
      // wave 0: block b of the chain; wave 1: block b - 1 of the gather; one
      // barrier per block.  z goes through a ring of two blocks (the delay
      // lines hold the whole horizon).
      double* zring = recl + P.lds_per_wave;  // NY x 2U
      const bool zg = !PRE && glane && col == M * NUT;  // (PRE: z lines, read as the delay lines)
      int rinc_q = rinc, rB = 0, plen = 0, blk = 0;
#define CMPC_SPLIT_A(u)                                         \
  {                                                             \
    double a = an;                                              \
    CMPC_SPLIT_CHAIN(pv, m, a);                                 \
    if constexpr (!PRE) {                                       \
      an = __builtin_fma(-ym, yh, base);                        \
      yh = ylp[((u) + 1) * NY];                                 \
    }                                                           \
    pv = a;                                                     \
    if (mlane || slane) wa[u] = a;                              \
  }
#define CMPC_SPLIT_B(u)                                         \
  {                                                             \
    const double rd_ = rb[u];                                   \
    va = __builtin_fma(smask, va, rd_);                         \
    CMPC_EXP_GACC(va, acc);                                     \
  }
#define CMPC_SPLIT_BLOCK(L)                                                        \
  {                                                                                \
    if (wA) {                                                                      \
      if ((L) > 0) {                                                               \
        double* wa = slane ? zring + oz * (2 * U) + (blk & 1) * U : wq;           \
        CMPC_SPLIT_A(0)                                                            \
        if ((L) == U) {                                                            \
          CMPC_SPLIT_A(1)                                                          \
          CMPC_SPLIT_A(2)                                                          \
          CMPC_SPLIT_A(3)                                                          \
        }                                                                          \
        wq += (L) * winc;                                                          \
        ylp += (L) * NY;                                                           \
      }                                                                            \
    } else if (plen > 0) {                                                         \
      const double* rb = zg ? zring + row * (2 * U) + ((blk - 1) & 1) * U : rq;   \
      CMPC_SPLIT_B(0)                                                              \
      if (plen == U) {                                                             \
        CMPC_SPLIT_B(1)                                                            \
        CMPC_SPLIT_B(2)                                                            \
        CMPC_SPLIT_B(3)                                                            \
      }                                                                            \
      rq += plen * rinc_q;                                                         \
      rB += plen;                                                                  \
      if (gdel == rB) { /* delayed input's history is over: its line */            \
        rq = rline;                                                                \
        rinc_q = 1;                                                                \
      }                                                                            \
    }                                                                              \
    __syncthreads();                                                               \
    plen = (L);                                                                    \
    ++blk;                                                                         \
  }
      static_assert(U == 4, "the split block macros unroll four steps");
      int r = 0;
      for (int seg = 0; seg <= nbound; ++seg) {
        int r_end = pp;
#pragma unroll
        for (int c = 0; c < NUT; ++c)
          if (c == seg && seg < nbound) r_end = bnd[c];
        for (; r + U <= r_end; r += U) CMPC_SPLIT_BLOCK(U)
        for (; r < r_end; ++r) CMPC_SPLIT_BLOCK(1)
      }
      CMPC_SPLIT_BLOCK(0)  // the gather's last block
#undef CMPC_SPLIT_BLOCK
#undef CMPC_SPLIT_B
#undef CMPC_SPLIT_A
      if (!wB) continue;  // the chain wave waits at the next QP's barrier
    } else {
    int r = 0;
    int rinc_q = rinc;
    for (int seg = 0; seg <= nbound; ++seg) {
      int r_end = pp;
#pragma unroll
      for (int c = 0; c < NUT; ++c)
        if (c == seg && seg < nbound) r_end = bnd[c];
      for (; r + U <= r_end; r += U) {
        CMPC_BUILD_STEP(0)
        CMPC_BUILD_STEP(1)
        CMPC_BUILD_STEP(2)
        CMPC_BUILD_STEP(3)
        wq += U * winc;
        rq += U * rinc_q;
        ylp += U * NY;
      }
      for (; r < r_end; ++r) {
        CMPC_BUILD_STEP(0)
        wq += winc;
        rq += rinc_q;
        ylp += NY;
      }
      if (gdel == r) {  // delayed input's history is over: start reading its line
        rq = rline;
        rinc_q = 1;
      }
    }
#undef CMPC_BUILD_STEP
    va = __builtin_fma(smask, va, rd);
    gacc_dpp<NUT, NU, M>(va, acc);  // row p-1
    // (the accumulation at r = 0 adds products of the zero initial va)
    }
    CMPC_WT(3)  // horizon loop

    // reduce over the ny rows through LDS; row 0 of the gather lanes stores
    if (red_lane) {
#pragma unroll
      for (int k = 0; k < NV; ++k) red_w[k] = acc[k];
    }
    if constexpr (FUSE == 1 || FUSE == 2) {
      // every row forms the totals (row 0's partial through LDS as well), in
      // the order row 0 uses below: the solver's four rows see the same H
      if (row == 0 && col < NG) {
#pragma unroll
        for (int k = 0; k < NV; ++k) red[((NY - 1) * NG + col) * NV + k] = acc[k];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      double tot[NV];
      const int cg = col < NG ? col : 0;
#pragma unroll
      for (int k = 0; k < NV; ++k) tot[k] = red[((NY - 1) * NG + cg) * NV + k];
#pragma unroll
      for (int o = 1; o < NY; ++o) {
        const double* rr = red + ((o - 1) * NG + cg) * NV;
#pragma unroll
        for (int k = 0; k < NV; ++k) tot[k] += rr[k];
      }
      if (qv && row == 0 && col < NG) {
        double* out = P.qp + (size_t)q * P.qp_len;
        const double* uwt = uw_all + s * NU * NU;
        const int k2 = col / NUT, c2 = col - k2 * NUT;
        if (col == M * NUT) {
#pragma unroll
          for (int a = 0; a < NV; ++a) out[NV * NV + a] = tot[a];  // f
        } else {
#pragma unroll
          for (int a = 0; a < NV; ++a) {  // H = Su' W Su + blkdiag_m(uwt) (S = 1: no G)
            const double rw = (a / NU == k2) ? uwt[(a % NU) * NU + c2] : 0.0;
            out[a * NV + k2 * NU + c2] = tot[a] + rw;
          }
        }
      }
      // the solver's layout in every row (cf. build_rows.hip): lane l < NV
      // holds row l of H (the column of gather lane (l / NU, l % NU), H is
      // exactly symmetric) and f[l]
      constexpr int N = NV;
      const int rb = lane & ~15;
      const int lcol = (col < N) ? (col / NU) * NUT + (col % NU) : 0;
      const double* uwt = uw_all + s * NU * NU;
      double Hl[N], Fv[N], Gl[1] = {0.0};
#pragma unroll
      for (int c = 0; c < N; ++c) {
        const double a = __shfl(tot[c], rb + lcol, 64);
        const double rw = (col < N && c / NU == col / NU) ? uwt[(col % NU) * NU + (c % NU)] : 0.0;
        Hl[c] = (col < N) ? a + rw : 0.0;
      }
      static_for<N>([&](auto A) {
        constexpr int a = decltype(A)::value;
        Fv[a] = rbc<M * NUT>(tot[a]);
      });
      const double f_l = (col < N) ? sel<N>(Fv, col) : 0.0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // the totals are read before the scratch is written
      CMPC_WT(4)  // epilogue
      if constexpr (SPLIT && SW == 2) {  // the factor in LDS (registers: two waves per SIMD)
        double* lsh = recl + P.lds_per_wave + (NY * 8 + 31) / 32 * 32 + row * N * N;
        rows_solve_qp<N, NU, 0, FUSE == 2, false, true>(P.sv, q, qv && row == 0, 0, col, rb, Hl, f_l, Gl,
                                                        red + NY * NG * NV + row * N * N, lsh);
      } else {
        rows_solve_qp<N, NU, 0, FUSE == 2, false>(P.sv, q, qv && row == 0, 0, col, rb, Hl, f_l, Gl,
                                                  red + NY * NG * NV + row * N * N);
      }
      __builtin_amdgcn_wave_barrier();
      CMPC_WT(1)  // fused solve
      continue;
    }
    if (qv && row == 0 && col < NG) {
      double tot[NV];
#pragma unroll
      for (int k = 0; k < NV; ++k) tot[k] = acc[k];
#pragma unroll
      for (int o = 1; o < NY; ++o) {
        const double* rr = red + ((o - 1) * NG + col) * NV;
#pragma unroll
        for (int k = 0; k < NV; ++k) tot[k] += rr[k];
      }
      double* out = P.qp + (size_t)q * P.qp_len;
      constexpr int nuo = NUT - NU, nVo = M * nuo;
      const double* uwt = uw_all + s * NU * NU;
      const int k2 = col / NUT, c2 = col - k2 * NUT;
      if (col == M * NUT) {
#pragma unroll
        for (int a = 0; a < NV; ++a) out[NV * NV + a] = tot[a];  // f
      } else if (c2 < NU) {
#pragma unroll
        for (int a = 0; a < NV; ++a) {  // H = Su' W Su + blkdiag_m(uwt)
          const double rw = (a / NU == k2) ? uwt[(a % NU) * NU + c2] : 0.0;
          out[a * NV + k2 * NU + c2] = tot[a] + rw;
        }
      } else {
#pragma unroll
        for (int a = 0; a < NV; ++a) out[NV * NV + NV + a * nVo + k2 * nuo + (c2 - NU)] = tot[a];  // G
      }
    }
    __builtin_amdgcn_wave_barrier();
    CMPC_WT(4)  // epilogue
  }
  if constexpr (FUSE >= 3) {
    // every wave has stored its QP (one per wave: the launcher's grid covers
    // the batch); the barrier's workgroup-scope release/acquire makes the
    // stores of the other waves visible to wave 0 (one CU, write-through L0)
    __syncthreads();
    constexpr int NVO = M * (NUT - NU);
    if constexpr (FUSE == 5) {
      // the row solver: wave 0's DPP row r solves the workgroup's QP r (a
      // scenario's sub-controllers in adjacent rows), as the row iterate
      // kernel does (solve_rows.hip), in the build's LDS (its N x N scratch
      // per row after the lines, which are dead)
      static_assert(QPG <= 4, "one QP per DPP row of wave 0");
      if ((threadIdx.x >> 6) == 0) {
        constexpr int NVOA = NVO > 0 ? NVO : 1;
        const int l = col;
        const int ql = blockIdx.x * QPG + row;
        const bool al = row < QPG && ql < P.nqp;
        const int qc = ql < P.nqp ? ql : P.nqp - 1;
        const int sl = qc % S;
        const bool own = l < NV;
        const int lr = own ? l : NV - 1;
        const double* qr = P.qp + (size_t)qc * P.qp_len;
        double Hl[NV], Gl[NVOA];
#pragma unroll
        for (int c = 0; c < NV; ++c) Hl[c] = own ? qr[lr * NV + c] : 0.0;
        const double f_l = own ? qr[NV * NV + lr] : 0.0;
#pragma unroll
        for (int c = 0; c < NVOA; ++c) Gl[c] = (NVO > 0 && own) ? qr[NV * NV + NV + lr * NVO + c] : 0.0;
        rows_solve_qp<NV, NU, NVO, false, false>(P.sv, qc, al, sl, l, (lane & ~15) - 16 * sl, Hl, f_l, Gl,
                                                 smem + P.lds_block + row * NV * NV);
      }
    } else if ((threadIdx.x >> 6) == 0 && lane < QPG) {
      const int ql = blockIdx.x * QPG + lane;
      const bool al = ql < P.nqp;
      const int qc = al ? ql : P.nqp - 1;
      const int sl = qc % S;
      const double* qr = P.qp + (size_t)qc * P.qp_len;
      lane_solve_qp<NV, NU, NVO, FUSE == 4, false, 1>(P.sv, qc, al, sl, lane - sl, qr, qr + NV * NV + NV);
    }
  }
#if CMPC_WAVE_TIMING
  // slots as CMPC_ROWS_TIMING: 0 staging, 1 fused solve, 2 prologue, 3 loop,
  // 4 epilogue, 5 back-edge; 6 QPs, 7 marker, 8-11 clocks, 12-14 placement
  if (lane == 0) {
    const uint64_t t1c = __builtin_amdgcn_s_memtime(), t1r = __builtin_amdgcn_s_memrealtime();
    // (the hardware wave: SPLIT's two waves of a QP slot write their own)
    double* dbg = P.qp + (size_t)(blockIdx.x * CMPC_BUILD_WAVES + (threadIdx.x >> 6)) * 16;
    for (int i = 0; i < 6; ++i) dbg[i] = (double)tsum[i];
    dbg[6] = done_qp;
    dbg[7] = 1.0;
    dbg[8] = (double)(t1c - t0c);
    dbg[9] = (double)(t1r - t0r);
    dbg[10] = (double)t0r;
    dbg[11] = (double)t1r;
    dbg[12] = (double)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    dbg[13] = (double)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);
    dbg[14] = (double)(blockIdx.x * CMPC_BUILD_WAVES + wave);
  }
#endif
}

template <int NS, int NY, int NUT, int NU, int M, int ND, int FUSE = 0>
__global__ __launch_bounds__(64 * CMPC_BUILD_WAVES)
__attribute__((amdgpu_waves_per_eu(FUSE ? 1 : 4, FUSE ? 1 : 4)))
void cmpc_build_kernel(BuildParams P) {
  build_wave_body<NS, NY, NUT, NU, M, ND, FUSE>(P);
}

// the role split (build_wave_body SPLIT): a two-wave workgroup per QP, two
// waves per SIMD
template <int NS, int NY, int NUT, int NU, int M, int ND, int FUSE = 0>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2)))
void cmpc_build_split_kernel(BuildParams P) {
  build_wave_body<NS, NY, NUT, NU, M, ND, FUSE, true>(P);
}

#ifndef CMPC_STEP_SPLIT_BUILD
// 1: fused centralized steps on the role-split kernel, the row solver's
// factor in LDS to fit 256 VGPRs (5 VGPRs of spills left).  Measured slower
// at config 5 (35.0 vs 32.5 us per step, 43.2 vs 37.2 us with the move: the
// solve runs on one wave of the pair with its factor behind LDS latency),
// profiles/r5g_build_split_ab.txt
#define CMPC_STEP_SPLIT_BUILD 0
#endif
static size_t split_lds_bytes(const BuildParams& P, int ny) {
  // + the z ring (ny x 2U) + four N x N factor areas of the fused row solver
  return sizeof(double) * ((size_t)P.lds_block + (size_t)P.lds_per_wave + (size_t)((ny * 8 + 31) / 32 * 32) + 256);
}

// ---------------------------------------------------------------------------
// One-launch control step (cmpc_control_step): NerveCenter::GetNextInput for
// a small batch on the device in one kernel, the workgroup's four QP slots
// (one per wave):
//   1. ObserveAPosteriori + Update (linearise, discretise, the lin record):
//      the producer body (produce_body.h), wave 0, one slot per DPP row;
//   2. GenerateInitialQP + the K Jacobi iterations: the fused build + solve
//      (build_wave_body, FUSE 1: row solver of each wave; FUSE 3: the lane
//      solver of wave 0);
//   3. UpdateU (ObserveAPriori, u_old += du): observer_body.h, wave 0.
// Workgroup barriers between the phases order the global stores of one
// phase before the next phase's loads (one CU, write-through L0).  The
// producer's table and rows overlay the build's dynamic LDS before the build
// starts.
// ---------------------------------------------------------------------------
// SPLIT: the build as two role-split pairs (two QP slots per workgroup)
template <int NS, int NY, int NUT, int NU, int M, int ND, int FUSE, bool SPLIT = false>
__global__ __launch_bounds__(64 * CMPC_BUILD_WAVES) __attribute__((amdgpu_waves_per_eu(1, 1)))
void cmpc_control_step_kernel(ControlStepParams C) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int PLANT = NS == 11 ? CMPC_PLANT_PARALLEL : CMPC_PLANT_SERIAL;
  constexpr int QPG = SPLIT ? CMPC_BUILD_WAVES / 2 : CMPC_BUILD_WAVES;  // QP slots per workgroup
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // the unit of this lane's DPP row in the producer and a-priori phases
  // (rows past the workgroup's slots idle: an index past the batch)
  const int unit = (lane >> 4) < QPG ? blockIdx.x * QPG + (lane >> 4) : 0x3fffffff;
  int* src = reinterpret_cast<int*>(smem);
  int* dmap = src + C.pr.S * C.pr.rec_len;
  cmpc_prod::produce_table<PLANT>(C.pr, src, dmap, threadIdx.x, 64 * CMPC_BUILD_WAVES);
  __syncthreads();
  if (wave == 0)
    cmpc_prod::produce_row<PLANT>(C.pr, smem + C.pr_off + (lane >> 4) * cmpc_prod::kScnLds, src, dmap,
                                  unit, lane);
  __syncthreads();
  build_wave_body<NS, NY, NUT, NU, M, ND, FUSE, SPLIT, CMPC_BUILD_WAVES>(C.b);
  // polled completion: each wave's result stores (du, status, nWSR in
  // page-locked host memory; waves 1-3 store theirs when the block has 2-4
  // centralized QPs) are released at system scope by the wave itself, before
  // the barrier that orders them ahead of wave 0's done store (a workgroup
  // barrier does not wait for other waves' outstanding global stores)
  if (C.done) __threadfence_system();
  __syncthreads();
  if (wave == 0) {
    obs_prior_row<NS, NUT>(C.ob, unit, lane);
    // wave 0's a-priori stores before this release (a vector store, system
    // scope)
    if (C.done && lane == 0) __hip_atomic_store(C.done, C.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// FUSE_: the solve after the build; FUSES_: the same with the role-split
// build (up to one QP per CU: the coop row solver, faster there)
#define CONTROL_CASE(NS_, NY_, NU_, M_, FUSE_, FUSES_)                                      \
  if (ns == NS_ && ny == NY_ && nu == NU_ && m == M_ && P.nd == 2 && P.nu_tot == 4) {        \
    auto k_ = P.split ? cmpc_control_step_kernel<NS_, NY_, 4, NU_, M_, 2, FUSES_, true>       \
                      : cmpc_control_step_kernel<NS_, NY_, 4, NU_, M_, 2, FUSE_>;            \
    if (lds > 64 * 1024)                                                                      \
      cmpc_allow_lds(reinterpret_cast<const void*>(k_), lds);        \
    const int f_ = P.split ? FUSES_ : FUSE_;                                                  \
    *solver = (f_ == 1 || f_ == 5) ? CMPC_SOLVE_ROWS : CMPC_SOLVE_LANE;                       \
    cmpc_launch(k_, dim3(std::max(1, P.grid)), dim3(64 * CMPC_BUILD_WAVES), lds, s, C);      \
    return 0;                                                                                 \
  }

int cmpc_launch_control_step(const ControlStepParams& C, int ns, int ny, int nu, int m, void* stream,
                             int* solver) {
  hipStream_t s = (hipStream_t)stream;
  const BuildParams& P = C.b;
  // (P.split: two QP slots per workgroup, the role-split build)
  if (P.grid * (P.split ? CMPC_BUILD_WAVES / 2 : CMPC_BUILD_WAVES) < P.nqp || P.sv.trace) return -1;
  if (C.pr.S != P.S || !C.pr.per_qp || !C.pr.obs_M) return -1;
  size_t lds = sizeof(double) * ((size_t)P.lds_block + (size_t)P.lds_per_wave * CMPC_BUILD_WAVES);
  lds = std::max(lds, sizeof(double) * ((size_t)C.pr_off + 4 * cmpc_prod::kScnLds));
  if (lds > 160 * 1024) return -1;
  if (P.S == 1) {
    if (P.lds_per_wave < ny * (m * 4 + 1) * (nu * m) + 4 * (nu * m) * (nu * m)) return -1;
    CONTROL_CASE(11, 3, 4, 2, 1, 1)  // parallel centralized
    CONTROL_CASE(10, 4, 4, 2, 1, 1)  // serial centralized
    return -1;
  }
  if ((P.split ? CMPC_BUILD_WAVES / 2 : CMPC_BUILD_WAVES) % P.S) return -1;
  CONTROL_CASE(11, 3, 2, 2, 3, 5)  // parallel coop
  CONTROL_CASE(11, 2, 2, 2, 3, 5)  // parallel ncoop
  CONTROL_CASE(10, 2, 2, 2, 3, 5)  // serial ncoop
  CONTROL_CASE(10, 4, 2, 2, 3, 5)  // serial coop
  return -1;
}

#ifndef CMPC_SOLVE_WPE_SMALL
#define CMPC_SOLVE_WPE_SMALL 2  // waves per SIMD of the nV < 6 iterate kernel
#endif
#ifndef CMPC_SOLVE_WPE
#define CMPC_SOLVE_WPE(N) ((N) >= 6 ? 1 : CMPC_SOLVE_WPE_SMALL)
#endif

// H^-1 of one lane as column `base` of a [N*N][T] lane-contiguous LDS array
template <int N, int T>
struct HinvLds {
  double* base;
  __device__ __forceinline__ double operator()(int r, int c) const { return base[(r * N + c) * T]; }
  __device__ __forceinline__ void set(int r, int c, double v) { base[(r * N + c) * T] = v; }
};

// ---------------------------------------------------------------------------
// Jacobi iterate kernel (lane per QP)
// ---------------------------------------------------------------------------
// EXT: the other controllers' plans come from P.du_other (one GetInput call of
// a stand-alone sub-controller, cmpc_get_input) instead of the lanes of the
// scenario's other slots.
template <int N, int NU, int NVO, bool TRACE, bool EXT = false>
__global__ __launch_bounds__(CMPC_SOLVE_THREADS)
__attribute__((amdgpu_waves_per_eu(CMPC_SOLVE_WPE(N), CMPC_SOLVE_WPE(N))))
void cmpc_solve_kernel(SolveParams P) {
  // One wave per SIMD with the AGPR half of the register file open for
  // spills (an AGPR clobber keeps the compiler from inferring "no AGPRs"):
  // nV = 8 scratch 1480 -> 464 B per lane, iterate (K = 1, 65 536
  // centralized QPs) 0.131 -> 0.049 ms.  nV = 4 too since the map form (its
  // map of 40 doubles per lane beside the solver): K = 9 at 131 072 QPs
  // 32.1 us against 69.6 us at two waves per SIMD with 308 B of spills
  // (profiles/r5b_small_batch.txt)
  if constexpr (CMPC_SOLVE_WPE(N) == 1) asm volatile("" ::: "a0");
  constexpr int NVOA = NVO > 0 ? NVO : 1;
  const int q_raw = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = q_raw < P.nqp;
  const int q = active ? q_raw : P.nqp - 1;
  const int s = q % P.S;
  const int lane = threadIdx.x & 63;
  const int base_lane = lane - s;
  const double* rec = P.qp + (size_t)q * P.qp_len;

  // G = Su' W Su_other is read once per Jacobi iteration: it lives in LDS
  // (transposed, lane-contiguous) rather than in 2*N*NVO registers.  (Staging
  // the workgroup's contiguous H/f/G block through LDS with coalesced loads
  // measured 2-4 % slower: round 2)
  __shared__ double gsh[N * NVOA][CMPC_SOLVE_THREADS];
#pragma unroll
  for (int a = 0; a < N; ++a)
#pragma unroll
    for (int c = 0; c < NVOA; ++c)
      gsh[a * NVOA + c][threadIdx.x] = (NVO > 0) ? rec[N * N + N + a * NVO + c] : 0.0;

  if constexpr (CMPC_SOLVE_WPE(N) == 2) {
    // two waves per SIMD: H^-1 (used to build a working set's map and off the
    // map form's common path) in LDS as well, beside the map in registers
    __shared__ double hsh[N * N][CMPC_SOLVE_THREADS];
    lane_solve_qp<N, NU, NVO, TRACE, EXT, CMPC_SOLVE_THREADS, HinvStrided<N, CMPC_SOLVE_THREADS>>(
        P, q, active, s, base_lane, rec, &gsh[0][threadIdx.x], &hsh[0][threadIdx.x]);
  } else {
    lane_solve_qp<N, NU, NVO, TRACE, EXT, CMPC_SOLVE_THREADS>(P, q, active, s, base_lane, rec,
                                                             &gsh[0][threadIdx.x]);
  }
}

// standalone batched solve (parity and KKT tests)
template <int N, int NU>
__global__ __launch_bounds__(CMPC_SOLVE_THREADS) void cmpc_qp_batch_kernel(QpBatchParams P) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P.nqp) return;
  double H[N][N], g[N];
  Qp<N, NU> qp;
#pragma unroll
  for (int a = 0; a < N; ++a) {
#pragma unroll
    for (int b = 0; b < N; ++b) H[a][b] = P.H[(size_t)q * N * N + a * N + b];
    g[a] = P.g[(size_t)q * N + a];
    qp.lb[a] = P.lb[(size_t)q * N + a];
    qp.ub[a] = P.ub[(size_t)q * N + a];
    qp.lbA[a] = P.lbA[(size_t)q * N + a];
    qp.ubA[a] = P.ubA[(size_t)q * N + a];
  }
  qp.tolerances();
  const bool pd = hinv_of<N>(H, qp.Hinv);
  double hmax = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) hmax = fabs(H[i][i]) > hmax ? fabs(H[i][i]) : hmax;
  double x[N];
  QpOut o;
  qp_solve<N, NU>(qp, pd, TOL_D * (1.0 + hmax), g, P.ws_in[q], P.max_chg, x, o);
#pragma unroll
  for (int a = 0; a < N; ++a) P.x[(size_t)q * N + a] = x[a];
  P.status[q] = o.status;
  P.nchg[q] = o.nchg;
  P.ws_out[q] = o.ws;
  P.ntrace[q] = o.ntrace;
  uint32_t* tr = reinterpret_cast<uint32_t*>(P.trace + (size_t)q * 16);
#pragma unroll
  for (int t = 0; t < 4; ++t) tr[t] = o.tr[t];
}

// ---------------------------------------------------------------------------
// launchers — explicit instantiation list (cf. the reference's *_list.h)
// ---------------------------------------------------------------------------
#define BUILD_CASE(NS_, NY_, NU_, M_)                                                  \
  if (ns == NS_ && ny == NY_ && nu == NU_ && m == M_ && P.nd == 2 && P.nu_tot == 4) {                   \
    {                                                                                  \
      if (P.split) {                                                                   \
        const size_t lds2 = split_lds_bytes(P, NY_);                                   \
        auto k2_ = cmpc_build_split_kernel<NS_, NY_, 4, NU_, M_, 2>;                   \
        if (lds2 > 64 * 1024) cmpc_allow_lds(reinterpret_cast<const void*>(k2_), lds2); \
        cmpc_launch(k2_, dim3(P.nqp), dim3(128), lds2, s, P);                          \
        return 0;                                                                      \
      }                                                                                \
    }                                                                                  \
    const size_t lds = sizeof(double) * ((size_t)P.lds_block +                         \
                                         (size_t)P.lds_per_wave * CMPC_BUILD_WAVES);  \
    if (lds > 64 * 1024)                                                               \
      cmpc_allow_lds(reinterpret_cast<const void*>(cmpc_build_kernel<NS_, NY_, 4, NU_, M_, 2>), lds);                       \
    int per_cu = cmpc_blocks_per_cu(cmpc_build_kernel<NS_, NY_, 4, NU_, M_, 2>,        \
                                    64 * CMPC_BUILD_WAVES, lds);                       \
    if (per_cu < 1) per_cu = std::max<int>(1, (int)((160 * 1024) / lds));             \
    const int grid = std::max(1, std::min(P.grid, P.cus * per_cu));                   \
    cmpc_launch((cmpc_build_kernel<NS_, NY_, 4, NU_, M_, 2>), dim3(grid),                  \
                dim3(64 * CMPC_BUILD_WAVES), lds, s, P);                               \
    return 0;                                                                          \
  }

// fused build + K iterations on the one-QP-per-wave kernel, row solver in
// the QP's own wave (S = 1)
#define STEP_WAVE_CASE(NS_, NY_, NU_, M_)                                                \
  if (ns == NS_ && ny == NY_ && nu == NU_ && m == M_ && P.nd == 2 && P.nu_tot == 4) {   \
    if (P.lds_per_wave < NY_ * (M_ * 4 + 1) * (NU_ * M_) + 4 * (NU_ * M_) * (NU_ * M_)) \
      return -1;                                                                         \
    const size_t lds = sizeof(double) * ((size_t)P.lds_block +                           \
                                         (size_t)P.lds_per_wave * CMPC_BUILD_WAVES);    \
    if constexpr (NY_ < 4 && CMPC_STEP_SPLIT_BUILD) {                                    \
      if (P.nqp <= 4 * P.cus) {                                                          \
        const size_t lds2 = split_lds_bytes(P, NY_);                                     \
        auto k2_ = P.sv.trace ? cmpc_build_split_kernel<NS_, NY_, 4, NU_, M_, 2, 2>      \
                              : cmpc_build_split_kernel<NS_, NY_, 4, NU_, M_, 2, 1>;     \
        if (lds2 > 64 * 1024) cmpc_allow_lds(reinterpret_cast<const void*>(k2_), lds2);  \
        cmpc_launch(k2_, dim3(P.nqp), dim3(128), lds2, s, P);                            \
        return 0;                                                                        \
      }                                                                                  \
    }                                                                                    \
    if (P.sv.trace) {                                                                    \
      auto k_ = cmpc_build_kernel<NS_, NY_, 4, NU_, M_, 2, 2>;                           \
      if (lds > 64 * 1024)                                                               \
        cmpc_allow_lds(reinterpret_cast<const void*>(k_), lds); \
      cmpc_launch(k_, dim3(std::max(1, P.grid)), dim3(64 * CMPC_BUILD_WAVES), lds, s, P); \
    } else {                                                                             \
      auto k_ = cmpc_build_kernel<NS_, NY_, 4, NU_, M_, 2, 1>;                           \
      if (lds > 64 * 1024)                                                               \
        cmpc_allow_lds(reinterpret_cast<const void*>(k_), lds); \
      cmpc_launch(k_, dim3(std::max(1, P.grid)), dim3(64 * CMPC_BUILD_WAVES), lds, s, P); \
    }                                                                                    \
    return 0;                                                                            \
  }

// the same with the lane solver after a workgroup barrier (S divides 4, the
// scenario's sub-controllers in adjacent waves of one workgroup)
#define STEP_WAVE_LANE_CASE(NS_, NY_, NU_, M_)                                           \
  if (ns == NS_ && ny == NY_ && nu == NU_ && m == M_ && P.nd == 2 && P.nu_tot == 4) {   \
    const size_t lds = sizeof(double) * ((size_t)P.lds_block +                           \
                                         (size_t)P.lds_per_wave * CMPC_BUILD_WAVES);    \
    auto k_ = P.sv.trace ? cmpc_build_kernel<NS_, NY_, 4, NU_, M_, 2, 4>                 \
                         : cmpc_build_kernel<NS_, NY_, 4, NU_, M_, 2, 3>;                \
    if (lds > 64 * 1024)                                                                 \
      cmpc_allow_lds(reinterpret_cast<const void*>(k_), lds);   \
    *solver = CMPC_SOLVE_LANE;                                                           \
    cmpc_launch(k_, dim3(std::max(1, P.grid)), dim3(64 * CMPC_BUILD_WAVES), lds, s, P);   \
    return 0;                                                                            \
  }

// one workgroup per four QPs (no persistent loop: the fused path is for
// batches that give fewer waves than the GPU holds, each wave one QP)
int cmpc_launch_step_wave(const BuildParams& P, int ns, int ny, int nu, int m, void* stream, int* solver) {
  hipStream_t s = (hipStream_t)stream;
  if (P.grid * CMPC_BUILD_WAVES < P.nqp) return -1;
  if (P.S == 1) {
    *solver = CMPC_SOLVE_ROWS;
    STEP_WAVE_CASE(11, 3, 4, 2)  // parallel centralized
    STEP_WAVE_CASE(10, 4, 4, 2)  // serial centralized
    return -1;
  }
  if (CMPC_BUILD_WAVES % P.S) return -1;
  STEP_WAVE_LANE_CASE(11, 3, 2, 2)  // parallel coop
  STEP_WAVE_LANE_CASE(11, 2, 2, 2)  // parallel ncoop
  STEP_WAVE_LANE_CASE(10, 2, 2, 2)  // serial ncoop
  STEP_WAVE_LANE_CASE(10, 4, 2, 2)  // serial coop
  return -1;
}

int cmpc_launch_build(const BuildParams& P, int ns, int ny, int nu, int m, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  BUILD_CASE(11, 3, 2, 2)  // parallel coop        (ControlledOutputIndices <0,1,3>)
  BUILD_CASE(11, 2, 2, 2)  // parallel ncoop       (NCControlledOutputIndices)
  BUILD_CASE(11, 3, 4, 2)  // parallel centralized
  BUILD_CASE(10, 2, 2, 2)  // serial ncoop
  BUILD_CASE(10, 4, 2, 2)  // serial coop          (NullIndexArray<4>: all four outputs)
  BUILD_CASE(10, 4, 4, 2)  // serial centralized
  BUILD_CASE(11, 3, 2, 1)
  BUILD_CASE(11, 3, 2, 3)
  return -1;
}

#define SOLVE_CASE(N_, NU_, NVO_)                                                      \
  if (nV == N_ && nu == NU_ && nVo == NVO_) {                                          \
    if (P.qp_len != N_ * N_ + N_ + N_ * NVO_) return -1;                               \
    const int grid = (P.nqp + CMPC_SOLVE_THREADS - 1) / CMPC_SOLVE_THREADS;            \
    if (P.du_other) {                                                                  \
      if (NVO_ == 0 || P.trace) return -1;                                             \
      cmpc_launch((cmpc_solve_kernel<N_, NU_, NVO_, false, (NVO_ > 0)>), dim3(grid),   \
                  dim3(CMPC_SOLVE_THREADS), 0, s, P);                                  \
      return 0;                                                                        \
    }                                                                                  \
    if (P.trace)                                                                       \
      cmpc_launch((cmpc_solve_kernel<N_, NU_, NVO_, true>), dim3(grid),                \
                  dim3(CMPC_SOLVE_THREADS), 0, s, P);                                  \
    else                                                                               \
      cmpc_launch((cmpc_solve_kernel<N_, NU_, NVO_, false>), dim3(grid),               \
                  dim3(CMPC_SOLVE_THREADS), 0, s, P);                                  \
    return 0;                                                                          \
  }

int cmpc_launch_solve(const SolveParams& P, int nV, int nu, int nVo, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  SOLVE_CASE(4, 2, 4)   // coop / ncoop, S = 2, m = 2
  SOLVE_CASE(8, 4, 0)   // centralized, m = 2
  SOLVE_CASE(2, 2, 2)   // m = 1
  SOLVE_CASE(6, 2, 6)   // m = 3
  return -1;
}

// the map-form solve of one Jacobi iteration (g = f + G d) on standalone
// QPs: qp_solve_map with a map built for the QP (cmpc_qp_solve_batch_map;
// DistributedSolver::UpdateAndSolveQP)
template <int N, int NU, int NVO>
__global__ __launch_bounds__(CMPC_SOLVE_THREADS) void cmpc_qp_batch_map_kernel(QpBatchParams P) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P.nqp) return;
  double H[N][N], f[N], d[NVO];
  Qp<N, NU> qp;
#pragma unroll
  for (int a = 0; a < N; ++a) {
#pragma unroll
    for (int b = 0; b < N; ++b) H[a][b] = P.H[(size_t)q * N * N + a * N + b];
    f[a] = P.g[(size_t)q * N + a];
    qp.lb[a] = P.lb[(size_t)q * N + a];
    qp.ub[a] = P.ub[(size_t)q * N + a];
    qp.lbA[a] = P.lbA[(size_t)q * N + a];
    qp.ubA[a] = P.ubA[(size_t)q * N + a];
  }
#pragma unroll
  for (int c = 0; c < NVO; ++c) d[c] = P.d[(size_t)q * NVO + c];
  qp.tolerances();
  const bool pd = hinv_of<N>(H, qp.Hinv);
  double hmax = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) hmax = fabs(H[i][i]) > hmax ? fabs(H[i][i]) : hmax;
  double xu0[N], U[N][NVO];
  jmap_terms<N, NVO, 1>(qp.Hinv, f, P.G + (size_t)q * N * NVO, xu0, U);
  JMap<N, NVO> mp;
  mp.ws = kWsInvalid;
  double x[N];
  QpOut o;
  qp_solve_map<true, N, NVO>(qp, pd, TOL_D * (1.0 + hmax), xu0, URegs<N, NVO>{U}, d, P.ws_in[q], P.max_chg, x, o,
                             mp);
#pragma unroll
  for (int a = 0; a < N; ++a) P.x[(size_t)q * N + a] = x[a];
  P.status[q] = o.status;
  P.nchg[q] = o.nchg;
  P.ws_out[q] = o.ws;
  P.ntrace[q] = o.ntrace;
  uint32_t* tr = reinterpret_cast<uint32_t*>(P.trace + (size_t)q * 16);
#pragma unroll
  for (int t = 0; t < 4; ++t) tr[t] = o.tr[t];
}

int cmpc_launch_qp_batch_map(const QpBatchParams& P, int n, int nu, int nvo, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int grid = (P.nqp + CMPC_SOLVE_THREADS - 1) / CMPC_SOLVE_THREADS;
#define CMPC_QPMAP_CASE(N_, NU_, NVO_)                                                              \
  if (n == N_ && nu == NU_ && nvo == NVO_) {                                                        \
    hipLaunchKernelGGL((cmpc_qp_batch_map_kernel<N_, NU_, NVO_>), dim3(grid), dim3(CMPC_SOLVE_THREADS), 0, s, P); \
    return 0;                                                                                       \
  }
  CMPC_QPMAP_CASE(4, 2, 4)
  CMPC_QPMAP_CASE(6, 2, 6)
  CMPC_QPMAP_CASE(2, 2, 2)
#undef CMPC_QPMAP_CASE
  return -1;
}

bool cmpc_qp_batch_map_supported(int n, int nu, int nvo) {
  return (n == 4 && nu == 2 && nvo == 4) || (n == 6 && nu == 2 && nvo == 6) || (n == 2 && nu == 2 && nvo == 2);
}

bool cmpc_qp_batch_supported(int n, int nu) { return (n == 4 && nu == 2) || (n == 8 && nu == 4); }

int cmpc_launch_qp_batch(const QpBatchParams& P, int n, int nu, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int grid = (P.nqp + CMPC_SOLVE_THREADS - 1) / CMPC_SOLVE_THREADS;
  if (n == 4 && nu == 2) {
    hipLaunchKernelGGL((cmpc_qp_batch_kernel<4, 2>), dim3(grid), dim3(CMPC_SOLVE_THREADS), 0, s, P);
    return 0;
  }
  if (n == 8 && nu == 4) {
    hipLaunchKernelGGL((cmpc_qp_batch_kernel<8, 4>), dim3(grid), dim3(CMPC_SOLVE_THREADS), 0, s, P);
    return 0;
  }
  return -1;
}
