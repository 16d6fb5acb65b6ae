// Row-layout build kernel: condensation + QP build for FOUR QPs per wave64,
// one QP per 16-lane DPP row.
//
// Same computation as cmpc_build_kernel (cmpc_kernels.hip; reference
// AdjustAllDelayedStates + GeneratePrediction + GenerateDistributedQP +
// GenerateQP, include/aug_lin_sys.h:141-154, libs/aug_lin_sys.cc:260-334,
// include/distributed_solver.h:83-94, libs/mpc_qp_solver.cc:16-40), with the
// roles moved from rows to registers:
//
//   lane j of row R (QP q = 4 g + R), registers
//     pP[o], o < ny : row o of P_r = L_W' C A^r   (lanes j < ns: column j)
//     aP[o]         : chain result -> P_{r+1} (lanes j < ns), raw Markov value
//                     P_r . B_c (Markov lanes ns + c)
//     pS / aS       : free-response simulation: lanes j < ns state x, lanes
//                     ns + o the output z_r[o], lanes 16 - nd + k the
//                     delayed-input values w (carriers)
//     cv[o], acc[a] : gather lane b < m nu_tot + 1 holds QP column b of output
//                     row o (move k = b / nu_tot, input c = b % nu_tot; the
//                     last lane holds z) and accumulates acc[a] = sum_{r,o}
//                     column_a column_b
//
// One horizon step is ny*ns + ns + nd DPP broadcast FMAs (four independent
// chains interleaved link by link) plus ny*nV gather FMAs, for four QPs at
// once: 16.25 VALU per QP-step at ny = 3, nV = 4, against 19.75 in the
// one-QP-per-wave layout, and the sum over outputs stays inside the lane, so
// no cross-row reduction is needed at the end.
//
// Hand-off of Markov / free-response values to the gather lanes through LDS.
// Every hand-off entry holds the ny outputs side by side ([entry][o]), so the
// per-output accesses of a step differ by compile-time immediates.
//   undelayed input : a ring of U + 1 entries [-1, 0 .. U-1]; step u of an
//                     unrolled group writes entry u, the move-0 lane reads
//                     entry u and the move-1 lane entry u - 1; after the
//                     group's last step (and after every single step) the
//                     value is copied to entry -1, which therefore always
//                     holds the previous step.
//   delayed input   : a line of (m - 1) zero entries + (p - D) values written
//                     at steps r < p - D (then the writer switches to a dump
//                     area); the gather lanes read a zero area until r = D
//                     and the line from there on (the delay shifts out of the
//                     index, as in the one-QP-per-wave kernel).
//   z               : U entries, written and read in the same step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "cmpc_internal.h"
#include "rows_blocks.inc"
#include "lane_solve.h"
#include "solve_rows.h"

// Timing-only ablation switches (tools/ablate_rows.sh); the product build
// uses CMPC_RX = 0.  1: no LDS hand-off in the loop, 3: no gather
// accumulation, 4: no hand-off writes (reads kept).
#ifndef CMPC_RX
#define CMPC_RX 0
#endif
// Timing-only prologue/epilogue ablations (results invalid; tools/build_variant.sh):
// 1: no record staging (the region keeps the previous group's tables),
// 2: staging without the wait (the compiler still waits before the first LDS
//    read: only the explicit wait goes), 3: no QP stores.  At the steady
//    clock, 1 is 9-11 % faster; the same bytes through plain vector loads
//    instead of LDS-DMA are as slow as the product, and issuing the DMA
//    without any wait (asm-issued, round 2) too: the cost is the HBM read
//    itself, not its latency or the DMA issue.
#ifndef CMPC_PX
#define CMPC_PX 0
#endif
#ifndef CMPC_ROWS_PF
#define CMPC_ROWS_PF 0  // L2 prefetch of the next group's records (2% slower with LDS staging)
#endif
#ifndef CMPC_ROWS_FUSE
#define CMPC_ROWS_FUSE 1  // chain and gather FMAs of a step in one interleaved block
#endif
#ifndef CMPC_ROWS_AS0
#define CMPC_ROWS_AS0 1  // 0: no software-pipelined LDS consumption (PIPE) in any instantiation
#endif
#ifndef CMPC_ROWS_SPLIT
#define CMPC_ROWS_SPLIT 5  // chain link groups before the gather columns' running sums (0: none)
#endif
#ifndef CMPC_ROWS_ZL
#define CMPC_ROWS_ZL 1  // the P chain's accumulators zeroed by LDS reads (the parallel plant's kernels)
#endif
#ifndef CMPC_ROWS_PRIO
#define CMPC_ROWS_PRIO 1  // 1: priority by progress; 2: + prologue at top priority
#endif
// Diagnostic build (tools/rows_timing.py): per-wave s_memtime cycle totals of
// the group phases, written over the QP output (results invalid).
#ifndef CMPC_ROWS_TIMING
#define CMPC_ROWS_TIMING 0
#endif
#if CMPC_ROWS_TIMING
#define CMPC_T(i)                                          \
  {                                                        \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();    \
    tsum[i] += now_ - tlast;                               \
    tlast = now_;                                          \
  }
#else
#define CMPC_T(i)
#endif

#ifndef CMPC_FUSED_LANE_SOLVE
#define CMPC_FUSED_LANE_SOLVE 1  // fused nV = 4 steps solve one QP per lane (0: per 16-lane row)
#endif
#ifndef CMPC_ROWS_WPE
#define CMPC_ROWS_WPE 3  // waves per SIMD the kernel is compiled and launched for
#endif

// RING: some delayed input's hand-off line is a ring (RowsLayout::ring; p > 2 D + 1):
// the wrap bookkeeping and the longer segment list only where needed, so the
// bench kernel (p = 50) keeps its registers (167 VGPRs, no scratch).
// WPE: waves per SIMD the register allocation targets (CMPC_ROWS_WPE = 3, 168
// registers; 2 for layouts whose LDS admits no more than two waves per SIMD
// anyway: 256 registers, no spills for ny = 4 / nV = 8 at long horizons)
// FUSE (cmpc_step on small batches): after its QPs are built, the wave runs
// their K Jacobi iterations itself (solve_rows.h), H, f and G handed from the
// gather lanes to the solver's rows by lane shuffles; 1 plain, 2 with the
// working-set trace.  The QPs are still stored (cmpc_download_qp).
template <int NS, int NY, int NUT, int NU, int M, int ND, int WPG, bool RING, int WPE = CMPC_ROWS_WPE,
          int FUSE = 0>
__global__ __launch_bounds__(64 * WPG) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
void cmpc_build_rows_kernel(BuildParams P) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int NV = NU * M;
  constexpr int NG = M * NUT + 1;  // gather lanes: QP columns (move k, input c), then z
  constexpr int NDW = ND > 0 ? ND : 1;
  constexpr int U = cmpc_rows_unroll(NY);  // horizon-loop unroll (immediate LDS offsets)
  static_assert(U == 4 || U == 5 || U == 10, "the unrolled block has 4, 5 or 10 steps");
  static_assert(M == 1 || M == 2, "the ring hand-off holds one step of history");
  // software-pipelined LDS consumption (CMPC_ROWS_SPLIT, CMPC_ROWS_AS0; round
  // 3) where the registers allow it without scratch: the parallel plant's
  // coop / ncoop kernels with plain lines (the bench kernel among them)
  // (round 4: also every instantiation compiled for two or fewer waves per
  // SIMD -- the 256-register ring, ny = 4 and nV = 8 kernels of long
  // horizons: bit-identical, ser-coop p = 100 -1.2 %, par-cent p = 200
  // -0.5 %, profiles/r3_pipe_wpe2_ab.txt)
  constexpr bool PIPE = CMPC_ROWS_SPLIT > 0 && CMPC_ROWS_AS0 && ((NY <= 3 && NV <= 4 && !RING) || WPE <= 2);
  constexpr bool ZL = CMPC_ROWS_ZL && PIPE && NY <= 3 && NV <= 4 && !RING && FUSE == 0;
  static_assert(NG <= 16 && NS + NUT <= 16 && NS + NY + ND <= 16, "lane budget");
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int R = lane >> 4, j = lane & 15;
  const int pp = P.p, S = P.S, nobs = P.nobs, rec_len = P.rec_len, ndist = P.ndist;
  const int LQ = P.rows.LQ, WL = P.rows.WL, yls = P.rows.yls;
  const int nqp = P.nqp;
  const int ngroups = (nqp + 3) / 4;
  const int nwaves = gridDim.x * WPG;  // WPG waves per workgroup (launcher: 4, 2 or 1)

  double* zeros = smem;
  double* ylT = smem + P.rows.yl_off;  // [S][NY][yls]  L_W' y_ref, output-major
  double* lw_all = smem + P.rows.lw_off;
  double* uw_all = smem + P.rows.uw_off;
  double* wreg = smem + P.rows.lds_block + wave * P.rows.per_wave;
  double* lines = wreg;                 // [4][LQ]: per QP, hand-off entries of NY doubles
  double* chs = wreg + P.rows.ch_off;   // [4][NY][16]  C_hat rows
  double* wtab = wreg + P.rows.w_off;   // [4][ND][WL]  delay-line inputs w_t

  const int nthr = 64 * WPG;
  for (int e = threadIdx.x; e < S * NY * yls; e += nthr) {
    const int ss = e / (NY * yls), rem = e - ss * NY * yls;
    const int o = rem / yls, r = rem - o * yls;
    // stored negated: the free-response chain starts at kappa + (-yhat_r)
    ylT[e] = (r < pp) ? -P.cfg[(size_t)ss * P.co.len + P.co.yhat + r * NY + o] : 0.0;
  }
  for (int e = threadIdx.x; e < S * NY * NY; e += nthr)
    lw_all[e] = P.cfg[(size_t)(e / (NY * NY)) * P.co.len + P.co.lwt + e % (NY * NY)];
  for (int e = threadIdx.x; e < S * NU * NU; e += nthr)
    uw_all[e] = P.cfg[(size_t)(e / (NU * NU)) * P.co.len + P.co.uwt + e % (NU * NU)];
  if (threadIdx.x < 16) zeros[threadIdx.x] = 0.0;
  for (int e = lane; e < P.rows.per_wave; e += 64) wreg[e] = 0.0;  // line heads, dump, slots
  __syncthreads();

  // ---- per-lane roles (identical for every group) ----
  const bool st = j < NS;                          // state lane
  const bool mk = j >= NS && j < NS + NUT;         // Markov writer of input cm
  const int cm = mk ? j - NS : 0;
  const bool ol = j >= NS && j < NS + NY;          // free-response output lane
  const int oo = ol ? j - NS : 0;
  const bool cl = ND > 0 && j >= 16 - ND;          // delayed-input carrier lane
  const int kc = cl ? j - (16 - ND) : 0;
  const bool gl = j < NG;                          // gather lane
  const bool zlane = j == NG - 1;
  const int gk = (gl && !zlane) ? j / NUT : 0;
  const int gc = (gl && !zlane) ? j - gk * NUT : 0;
  const double smask = (gl && !zlane && gk == M - 1) ? 1.0 : 0.0;  // running-sum column
  int dg = 0, dm = 0, log_ = 0, lom = 0, dinp[NDW], dlen[NDW], boff[NDW];
#pragma unroll
  for (int c = 0; c < NUT; ++c) {
    if (c == gc) { dg = P.delay[c]; log_ = P.rows.lo[c]; }
    if (c == cm) { dm = P.delay[c]; lom = P.rows.lo[c]; }
  }
#pragma unroll
  for (int k = 0; k < NDW; ++k) {
    dinp[k] = (k < ND) ? P.dinput[k] : 0;
    dlen[k] = (k < ND) ? P.dlen[k] : 0;
    boff[k] = (k < ND) ? P.boff[k] : 0;
  }
  // a carrier's w line is zero from t = D on: at the loop segment r = D its
  // reads move to the zero slots, so the w table holds D + 3 entries, not p + 6
  int ysw = -1;
#pragma unroll
  for (int k = 0; k < NDW; ++k)
    if (cl && k == kc && dlen[k] < pp) ysw = dlen[k];
  const int nseg = P.rows.nseg;
  // segment bounds: the delayed inputs' D and p - D (and the ring wraps)
  constexpr int NSEG = RING ? CMPC_ROWS_NSEG : 2 * NDW;
  int segb[NSEG];
#pragma unroll
  for (int i = 0; i < NSEG; ++i) segb[i] = P.rows.seg[i];
  double* const qlines = lines + R * LQ;  // this row's QP
  // readers (entry pointers; output o at +o, step u of a group at +u*NY)
  const bool rdel = gl && !zlane && dg > 0;
  const int rsw = (rdel && dg < pp) ? dg : -1;  // step at which a delayed reader starts its line
  double* const zrow = qlines + P.rows.zr_off;  // never written
  double* const r_start = !gl ? zrow
                          : zlane ? qlines + P.rows.z_off
                          : (dg == 0) ? qlines + log_ + (1 - gk) * NY
                                      : zrow;
  double* const r_line = qlines + log_ + (M - 1 - gk) * NY;
  // writers
  const bool wdel = mk && dm > 0;
  double* const dump = qlines + P.rows.dump_off;
  double* const w_start = !mk ? dump
                          : (dm == 0) ? qlines + lom + NY
                          : (pp - dm > 0) ? qlines + lom + (M - 1) * NY
                                          : dump;
  const int winc0 = (wdel && pp - dm > 0) ? NY : 0;
  const int wsw = (wdel && pp - dm > 0) ? pp - dm : -1;
  // ring lines (RowsLayout::ring): the writer and each gather reader step back
  // by the ring at their wrap steps (rows_layout.cpp, rows_ring_*_wrap)
  int ringw = 0, ringr = 0;
  if constexpr (RING) {
#pragma unroll
    for (int c = 0; c < NUT; ++c) {
      if (c == cm) ringw = P.rows.ring[c];
      if (c == gc) ringr = P.rows.ring[c];
    }
  }
  const int wwr0 = (wdel && ringw) ? ringw - (M - 1) : -1;  // first wraps; then every ring steps
  const int rwr0 = (rdel && ringr) ? ringr + dg - (M - 1 - gk) : -1;
  const bool tl = M > 1 && mk && dm == 0;  // ring writer: copies each group's last value to entry -1
  double* const tq = qlines + lom;
  // every lane stores each step (no exec-mask branches in the loop): lanes
  // without a Markov or free-response role store into the dump area
  double* const zq = ol ? qlines + P.rows.z_off + oo : dump;

#if CMPC_ROWS_TIMING
  uint64_t tsum[6] = {0, 0, 0, 0, 0, 0}, tlast = __builtin_amdgcn_s_memtime();
  const uint64_t t0c = tlast, t0r = __builtin_amdgcn_s_memrealtime();
  int ngrp = 0;
#endif
  // Fair progress.  The SIMD issues from its oldest ready wave first, so with
  // a static group assignment the oldest wave finished early and the youngest
  // ran alone at the end (wave lifetimes 0.19-0.35 ms for a 0.35 ms kernel,
  // tools/rows_timing.py).  Each wave lowers its issue priority as it
  // completes quarters of its share, so waves that are behind win arbitration.
  const int share = (ngroups + nwaves - 1) / nwaves;
  // The oldest waves take the groups left over when nwaves does not divide
  // ngroups (round 3: giving them to the youngest instead, or priority by
  // quarters of the wave's own share, measured slower)
  const int g_first = blockIdx.x * WPG + wave;
  int done_groups = 0;
  __builtin_amdgcn_s_setprio(3);
  for (int g = g_first; g < ngroups; g += nwaves) {
    CMPC_T(5)  // loop back-edge / tail of the previous group
#if CMPC_ROWS_PRIO == 2
    __builtin_amdgcn_s_setprio(3);  // latency-bound prologue first
#else
    {
      const int level = 3 - (4 * done_groups) / share;  // 3 .. 0
      if (level <= 0) __builtin_amdgcn_s_setprio(0);
      else if (level == 1) __builtin_amdgcn_s_setprio(1);
      else if (level == 2) __builtin_amdgcn_s_setprio(2);
      ++done_groups;
    }
#endif
    const int q = 4 * g + R;
    const bool qv = q < nqp;
    const int qq = qv ? q : nqp - 1;
    const int s = qq & (S - 1);  // S divides 64 (cmpc_create), a power of two
    const double* lwt = lw_all + s * NY * NY;
    double* chq = chs + R * NY * 16;

    // ---- the group's four records -> LDS in one round trip ----
    // Consecutive QPs' records are contiguous, so the group's 4 rec_len
    // doubles are one coalesced block, copied with 16-byte LDS-DMA loads
    // (global_load_lds_dwordx4: no VGPRs) into the wave's region, which the
    // tables below overwrite once the records are read.  (Reading the records
    // with per-lane global loads took ~15 dependent round trips per group, and
    // L2 evicted records in between: 2.5x the algorithmic HBM bytes.)
    if (CMPC_PX != 1) {
      const int nq = min(4, nqp - 4 * g);
      const int nchunk = nq * rec_len / 2;
      // Whole 64-lane chunks in blocks of four sharing one global address
      // and one LDS base (M0): the instruction offset advances both by the
      // chunk's 1 KiB (offset field < 4 KiB), so a block costs one 64-bit
      // address add instead of an address, a readfirstlane and an exec mask
      // per chunk; the partial chunk last, lane-masked.
      const int nfull = nchunk >> 6;
      const double* gsrc = P.lin + (size_t)4 * g * rec_len + 2 * lane;
      int c = 0;
      for (; c + 4 <= nfull; c += 4) {
        auto* gp = (__attribute__((address_space(1))) void*)(gsrc + 128 * c);
        auto* lp = (__attribute__((address_space(3))) void*)(wreg + 128 * c);
        __builtin_amdgcn_global_load_lds(gp, lp, 16, 0, 0);
        __builtin_amdgcn_global_load_lds(gp, lp, 16, 1024, 0);
        __builtin_amdgcn_global_load_lds(gp, lp, 16, 2048, 0);
        __builtin_amdgcn_global_load_lds(gp, lp, 16, 3072, 0);
      }
      for (; c < nfull; ++c)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(gsrc + 128 * c),
                                         (__attribute__((address_space(3))) void*)(wreg + 128 * c), 16, 0, 0);
      if (lane < (nchunk & 63))
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(gsrc + 128 * nfull),
                                         (__attribute__((address_space(3))) void*)(wreg + 128 * nfull), 16, 0,
                                         0);
    }
    double uo[NDW];
#pragma unroll
    for (int k = 0; k < NDW; ++k) uo[k] = (k < ND) ? P.u_old[(size_t)qq * NUT + dinp[k]] : 0.0;
    CMPC_T(0)  // staging issue
    if (CMPC_PX != 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CMPC_T(1)  // staging wait
    const double* srec = wreg + R * rec_len;  // this row's record (staged)
    const double* xa = srec + P.off_x;
    double xw[NDW][4];  // delay-line sources of w_t, t = j + 16 i < 64
#pragma unroll
    for (int k = 0; k < ND; ++k) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = j + 16 * i;
        xw[k][i] = (t < dlen[k]) ? ((t == 0) ? xa[ndist + k] : xa[boff[k] + t - 1]) : 0.0;
      }
    }
    double cs[NY];  // controlled rows of C, column j
#pragma unroll
    for (int o2 = 0; o2 < NY; ++o2) cs[o2] = (j < nobs) ? srec[P.off_C + o2 * nobs + j] : 0.0;
    constexpr int KX = 16 - NS;  // >= disturbance states (nobs = ns + ndist <= 16)
    double kx[KX], ky[NY];
#pragma unroll
    for (int d = 0; d < KX; ++d) kx[d] = (d < ndist) ? xa[d] : 0.0;
#pragma unroll
    for (int o2 = 0; o2 < NY; ++o2) ky[o2] = srec[P.off_y + o2];
    // P-chain multipliers: A column j (state lanes), B column c (Markov lanes)
    double mP[NS];
    if (st) {
      const double* src = srec + P.off_A + j;
#pragma unroll
      for (int l = 0; l < NS; ++l) mP[l] = src[l * NS];
    } else if (mk) {
      const double* src = srec + P.off_B + cm;
#pragma unroll
      for (int l = 0; l < NS; ++l) mP[l] = src[l * NUT];
    } else {
#pragma unroll
      for (int l = 0; l < NS; ++l) mP[l] = 0.0;
    }
    // simulation multipliers of the state lanes: A row j, Adelay columns
    double mS[NS + NDW], fj = 0.0;
    if (st) {
      const double* arow = srec + P.off_A + j * NS;
      const double* brow = srec + P.off_B + j * NUT;
#pragma unroll
      for (int l = 0; l < NS; ++l) mS[l] = arow[l];
#pragma unroll
      for (int k = 0; k < NDW; ++k) mS[NS + k] = (ND > 0) ? brow[dinp[k]] : 0.0;
      fj = srec[P.off_f + j];
    } else {
#pragma unroll
      for (int l = 0; l < NS + NDW; ++l) mS[l] = 0.0;
    }
    // every staged read is issued before the first table write below (LDS
    // operations of a wave execute in order)
    __builtin_amdgcn_sched_barrier(0);

    // C_hat = L_W' C_sel (ny x nobs): lane j computes column j of its QP
    double pP[NY];
#pragma unroll
    for (int o = 0; o < NY; ++o) {
      double t = 0.0;
#pragma unroll
      for (int o2 = 0; o2 < NY; ++o2)
        if (o2 >= o) t = __builtin_fma(lwt[o * NY + o2], cs[o2], t);  // one VALU per term
      if (j < nobs) chq[o * 16 + j] = t;
      pP[o] = st ? t : 0.0;  // P_0 = C_hat[:, :ns]
    }
    // delay-line inputs of the QP, AdjustAllDelayedStates applied
    // (include/aug_lin_sys.h:141-154); zero once the line has drained
#pragma unroll
    for (int k = 0; k < ND; ++k) {
      double* wk = wtab + (R * ND + k) * WL;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = j + 16 * i;
        if (t < WL) wk[t] = (t < dlen[k]) ? xw[k][i] - uo[k] : 0.0;
      }
      if (WL > 64) {  // long horizons only (a uniform branch: no per-lane loop set-up)
        const double* gxa = P.lin + (size_t)qq * rec_len + P.off_x;
        for (int t = j + 64; t < WL; t += 16) wk[t] = (t < dlen[k]) ? gxa[boff[k] + t - 1] - uo[k] : 0.0;
      }
    }
    // simulation chain initialisation
    double base = 0.0, pS = 0.0, yh = 0.0;
    const double* yp = zeros;
    int yinc = 0;
    if (st) {
      base = fj;
      pS = base;
#pragma unroll
      for (int k = 0; k < ND; ++k) pS = __builtin_fma(mS[NS + k], wtab[(R * ND + k) * WL], pS);  // x_1 = f + Adelay w_0
    } else if (ol) {
#pragma unroll
      for (int l = 0; l < NS; ++l) mS[l] = chq[oo * 16 + l];
      // kappa = L_W'(dist + y_prev) = C_hat_dist xa_dist + L_W' y_prev
      double t = 0.0;
#pragma unroll
      for (int d = 0; d < KX; ++d)
        if (d < ndist) t = __builtin_fma(chq[oo * 16 + NS + d], kx[d], t);
#pragma unroll
      for (int o2 = 0; o2 < NY; ++o2)
        if (o2 >= oo) t = __builtin_fma(lwt[oo * NY + o2], ky[o2], t);
      base = t;
      const double* yl = ylT + (s * NY + oo) * yls;
      yh = yl[0];
      yp = yl + 1;
      yinc = 1;
    } else if (cl) {
      const double* wk = wtab + (R * ND + kc) * WL;
      pS = wk[1];
      yh = wk[2];
      yp = wk + 3;
      yinc = 1;
    }
    // restore the zero areas the staging (and the C_hat rows, which overlay
    // the hand-off areas and were read above) overwrote: the m - 1 history
    // entries at the head of each delayed input's line, and the zero slots
#pragma unroll
    for (int c = 0; c < NUT; ++c)
      if (P.delay[c] > 0 && j < (M - 1) * NY) qlines[P.rows.lo[c] + j] = 0.0;
    for (int e = j; e < U * NY; e += 16) qlines[P.rows.zr_off + e] = 0.0;
    // ring history before t = 0
    if (tl) {
#pragma unroll
      for (int o = 0; o < NY; ++o) tq[o] = 0.0;
    }
    double cv[NY], rd[NY], acc[NV];
#pragma unroll
    for (int o = 0; o < NY; ++o) cv[o] = rd[o] = 0.0;
#pragma unroll
    for (int a = 0; a < NV; ++a) acc[a] = 0.0;
    double* wq = w_start;
    double* rq = r_start;
    int winc = winc0, rinc = 0;
    int wwr = wwr0, rwr = rwr0;

    // Optional L2 prefetch of this wave's next group of records (one dword
    // per 128-byte line, consumed after the horizon loop).  Off: since the
    // records are staged with one LDS-DMA round trip, it only added HBM
    // re-fetches (A/B: 0.328 vs 0.322 ms).
    float pf0 = 0.f, pf1 = 0.f;
    if (CMPC_ROWS_PF) {
      const int gn = g + nwaves;
      if (gn < ngroups) {
        const char* nb = reinterpret_cast<const char*>(P.lin + (size_t)4 * gn * rec_len);
        const int nbytes = min(4, nqp - 4 * gn) * rec_len * (int)sizeof(double);
        if (lane * 128 < nbytes) pf0 = *reinterpret_cast<const float*>(nb + lane * 128);
        if ((lane + 64) * 128 < nbytes) pf1 = *reinterpret_cast<const float*>(nb + (lane + 64) * 128);
      }
    }

// one horizon step; u = position inside the unrolled group (immediate LDS
// offsets).  The LDS reads of a step are consumed one step later (yh at the
// chain start, rd after the chain), and the scheduling barrier keeps the
// compiler from sinking them next to their use.
#if CMPC_ROWS_FUSE && CMPC_RX != 3
// PIPE (kernels without register headroom excepted): the first
// CMPC_ROWS_SPLIT link groups of the chain, then the running sums of the
// gather columns (they consume the LDS reads at the end of the previous step:
// placed here, the wave does not wait on that round trip at the top of every
// step), then the other link groups with the gather FMAs interleaved.  The
// same FMA order per accumulator as the single block.
#define CMPC_ROWS_CG()                                                      \
    if constexpr (PIPE) {                                                   \
      rows_chain_head<NS, NY, ND, CMPC_ROWS_SPLIT>(pP, pS, mP, mS, aP, aS); \
      __builtin_amdgcn_sched_barrier(0);                                    \
      _Pragma("unroll") for (int o = 0; o < NY; ++o)                        \
          cv[o] = __builtin_fma(smask, cv[o], rd[o]);                       \
      __builtin_amdgcn_sched_barrier(0);                                    \
      rows_chain_gacc_tail<NS, NY, ND, NUT, NU, M, CMPC_ROWS_SPLIT>(pP, pS, mP, mS, aP, aS, cv, acc); \
    } else {                                                                \
      _Pragma("unroll") for (int o = 0; o < NY; ++o)                        \
          cv[o] = __builtin_fma(smask, cv[o], rd[o]);                       \
      rows_chain_gacc<NS, NY, ND, NUT, NU, M>(pP, pS, mP, mS, aP, aS, cv, acc); \
    }                                                                       \
    __builtin_amdgcn_sched_barrier(0);
#else
#define CMPC_ROWS_CG()                                                      \
    rows_chain<NS, NY, ND>(pP, pS, mP, mS, aP, aS);                         \
    __builtin_amdgcn_sched_barrier(0);                                      \
    _Pragma("unroll") for (int o = 0; o < NY; ++o)                          \
        cv[o] = __builtin_fma(smask, cv[o], rd[o]);                         \
    if (CMPC_RX != 3) rows_gacc<NY, NUT, NU, M>(cv, acc);
#endif
// PIPE: the free-response chain's start value base + y_hat of the next step
// is formed at the end of this step (its y_hat was read at the top of this
// step), so the first instructions of a step need no LDS value: at the head
// of an unrolled block the wave no longer waits on the previous block's LDS
// reads before its first FMA (the same addition, bit-identical)
#define CMPC_ROWS_AS_BEGIN() double aS = PIPE ? aS0 : base + yh;
#define CMPC_ROWS_AS_END() \
  if constexpr (PIPE) aS0 = base + yh;
// ZL: the P chain's accumulators start from zeros read from LDS (issued at
// the end of the previous step) instead of a v_mov_b64 each: CDNA4 has no
// non-accumulating FP64 DPP multiply, so every step needs NY zeroed
// accumulators, and the LDS pipe has the issue slots the VALU lacks
#define CMPC_ROWS_STEP(u)                                                   \
  {                                                                         \
    CMPC_ROWS_AS_BEGIN()                                                    \
    yh = yp[u];                                                             \
    double aP[NY];                                                          \
    _Pragma("unroll") for (int o = 0; o < NY; ++o) aP[o] = ZL ? zn[o] : 0.0; \
    CMPC_ROWS_CG()                                                          \
    _Pragma("unroll") for (int o = 0; o < NY; ++o) pP[o] = aP[o];           \
    pS = aS;                                                                \
    if constexpr (ZL) {                                                     \
      _Pragma("unroll") for (int o = 0; o < NY; ++o) zn[o] = zeros[o];      \
    }                                                                       \
    if (CMPC_RX != 1 && CMPC_RX != 4) {                                     \
      _Pragma("unroll") for (int o = 0; o < NY; ++o) wq[(u) * NY + o] = aP[o]; \
      zq[(u) * NY] = aS;                                                    \
    }                                                                       \
    if (CMPC_RX != 1) {                                                     \
      _Pragma("unroll") for (int o = 0; o < NY; ++o) rd[o] = rq[(u) * NY + o]; \
    }                                                                       \
    CMPC_ROWS_AS_END()                                                      \
    __builtin_amdgcn_sched_barrier(0);                                      \
  }
#define CMPC_ROWS_TAIL()                                                    \
  if (tl) {                                                                 \
    _Pragma("unroll") for (int o = 0; o < NY; ++o) tq[o] = pP[o];           \
  }

    CMPC_T(2)  // prologue compute
#if CMPC_ROWS_PRIO == 2
    {
      const int level = 2 - (3 * done_groups) / share;  // 2 .. 0
      if (level <= 0) __builtin_amdgcn_s_setprio(0);
      else if (level == 1) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(2);
      ++done_groups;
    }
#endif
    int r = 0;
    double aS0 = base + yh;  // CMPC_ROWS_AS0: start value of the next step's free-response chain
    (void)aS0;
    double zn[NY];  // ZL: the next step's zeroed P accumulators
#pragma unroll
    for (int o = 0; o < NY; ++o) zn[o] = ZL ? zeros[o] : 0.0;
    for (int sg = 0; sg <= nseg; ++sg) {
      int r_end = pp;
#pragma unroll
      for (int i = 0; i < NSEG; ++i)
        if (i == sg && sg < nseg) r_end = segb[i];
      for (; r + U <= r_end; r += U) {
        CMPC_ROWS_STEP(0)
        CMPC_ROWS_STEP(1)
        CMPC_ROWS_STEP(2)
        CMPC_ROWS_STEP(3)
        if constexpr (U >= 5) CMPC_ROWS_STEP(4)
        if constexpr (U >= 10) {
          CMPC_ROWS_STEP(5)
          CMPC_ROWS_STEP(6)
          CMPC_ROWS_STEP(7)
          CMPC_ROWS_STEP(8)
          CMPC_ROWS_STEP(9)
        }
        CMPC_ROWS_TAIL()
        wq += U * winc;
        rq += U * rinc;
        yp += U * yinc;
      }
      // a remainder of two or more steps runs as two-step blocks: their
      // chain registers alternate as in the unrolled loop (a one-step loop
      // copies them back, 11 moves a step)
      while (U > 2 && r + 2 <= r_end) {
        CMPC_ROWS_STEP(0)
        CMPC_ROWS_STEP(1)
        CMPC_ROWS_TAIL()
        wq += 2 * winc;
        rq += 2 * rinc;
        yp += 2 * yinc;
        r += 2;
      }
      for (; r < r_end; ++r) {
        CMPC_ROWS_STEP(0)
        CMPC_ROWS_TAIL()
        wq += winc;
        rq += rinc;
        yp += yinc;
      }
      if (r == rsw) { rq = r_line; rinc = NY; }
      if constexpr (RING) {
        if (r == rwr) { rq -= ringr * NY; rwr += ringr; }
        if (r == wwr) { wq -= ringw * NY; wwr += ringw; }
      }
      if (r == wsw) { wq = dump; winc = 0; wwr = -1; }
      if (r == ysw) { yp = zeros; yinc = 0; }
    }
#undef CMPC_ROWS_STEP
#undef CMPC_ROWS_TAIL
#undef CMPC_ROWS_AS_BEGIN
#undef CMPC_ROWS_AS_END
#undef CMPC_ROWS_CG
#pragma unroll
    for (int o = 0; o < NY; ++o) cv[o] = __builtin_fma(smask, cv[o], rd[o]);
    rows_gacc<NY, NUT, NU, M>(cv, acc);  // row p - 1
    asm volatile("" ::"v"(pf0), "v"(pf1));
    CMPC_T(3)  // horizon loop

    if (qv && gl && !CMPC_ROWS_TIMING && CMPC_PX != 3) {
      double* out = P.qp + (size_t)q * P.qp_len;
      constexpr int nuo = NUT - NU, nVo = M * nuo;
      const double* uwt = uw_all + s * NU * NU;
      const int k2 = j / NUT, c2 = j - k2 * NUT;
      if (zlane) {
#pragma unroll
        for (int a = 0; a < NV; ++a) out[NV * NV + a] = acc[a];  // f
      } else if (c2 < NU) {
#pragma unroll
        for (int a = 0; a < NV; ++a) {  // H = Su' W Su + blkdiag_m(uwt)
          const double rw = (a / NU == k2) ? uwt[(a % NU) * NU + c2] : 0.0;
          out[a * NV + k2 * NU + c2] = acc[a] + rw;
        }
      } else {
#pragma unroll
        for (int a = 0; a < NV; ++a) out[NV * NV + NV + a * nVo + k2 * nuo + (c2 - NU)] = acc[a];  // G
      }
    }
    if constexpr (FUSE > 0 && FUSE < 3) {
      // the row solver's layout: lane l < NV holds row l of H and of G and
      // f[l].  Gather lane b = (k, c) holds column (k, c) of H, G or f (its
      // acc[a] = entry a); H is exactly symmetric (acc_b[a] == acc_a[b]), so
      // row l of H is the column the gather lane of column l holds, and
      // H[l][c] = that lane's acc[c] + the R block entry, as stored above
      constexpr int N = NV, NVO = M * (NUT - NU), NVOA = NVO > 0 ? NVO : 1, nuo = NUT - NU;
      const int rb = lane & ~15;
      const int lcol = (j < N) ? (j / NU) * NUT + (j % NU) : 0;
      const double* uwt = uw_all + s * NU * NU;
      double Hl[N], Fv[N], Gl[NVOA];
#pragma unroll
      for (int c = 0; c < N; ++c) {
        const double a = __shfl(acc[c], rb + lcol, 64);
        const double rw = (j < N && c / NU == j / NU) ? uwt[(j % NU) * NU + (c % NU)] : 0.0;
        Hl[c] = (j < N) ? a + rw : 0.0;
      }
      static_for<N>([&](auto A) {
        constexpr int a = decltype(A)::value;
        Fv[a] = rbc<NG - 1>(acc[a]);  // f from the z lane
      });
#pragma unroll
      for (int c = 0; c < NVOA; ++c) Gl[c] = 0.0;
      if constexpr (NVO > 0) {
        static_for<NVO>([&](auto C) {
          constexpr int c = decltype(C)::value;
          constexpr int lg = (c / nuo) * NUT + NU + (c % nuo);  // gather lane of G's column c
          double col[N];
          static_for<N>([&](auto A) {
            constexpr int a = decltype(A)::value;
            col[a] = rbc<lg>(acc[a]);
          });
          Gl[c] = (j < N) ? sel<N>(col, j) : 0.0;
        });
      }
      const double f_l = (j < N) ? sel<N>(Fv, j) : 0.0;
      // the wave's region is dead until the next group's staging: H^-1 scratch
      rows_solve_qp<N, NU, NVO, FUSE == 2, false>(P.sv, qq, qv, s, j, rb - 16 * s, Hl, f_l, Gl,
                                                  wreg + R * N * N);
    }
    __builtin_amdgcn_wave_barrier();
    CMPC_T(4)  // epilogue
#if CMPC_ROWS_TIMING
    ++ngrp;
#endif
  }
  if constexpr (FUSE >= 3) {
    // the wave's QPs, built above and stored, are solved one per lane (the
    // iterate kernel's solver, lane_solve.h) once the build's registers are
    // dead: lane 4 i + r takes QP r of the wave's i-th group; a scenario's
    // sub-controllers share a quad (S divides 4), their plans exchanged by
    // lane shuffles.  The wave reads back its own QP stores once they have
    // completed (vmcnt(0)): the vector L0 is invalidated at kernel start and
    // is write-through, and no lane of the kernel reads a QP before its
    // group's wave has stored it, so the loads see the stores.  (An
    // agent-scope fence instead writes back the whole L2: 85 us a step at
    // SURVEY config 2, tools/time_small.py.)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    constexpr int NVO = M * (NUT - NU);
    constexpr int NVOA = NVO > 0 ? NVO : 1;
    const int gi = g_first + (lane >> 2) * nwaves;
    if (gi < ngroups) {
      const int ql = 4 * gi + (lane & 3);
      const bool al = ql < nqp;
      const int qc = al ? ql : nqp - 1;
      const int sl = qc & (S - 1);
      const double* qr = P.qp + (size_t)qc * P.qp_len;
      // G of the lane's QP into the wave's own LDS region (free once its
      // groups are built; the launcher checks its size), lane-contiguous, where
      // the map form replaces it by U = H^-1 G (registers: the solve's map)
      double* gl = wreg + lane;
#pragma unroll
      for (int a = 0; a < NV; ++a)
#pragma unroll
        for (int c = 0; c < NVOA; ++c) gl[(a * NVOA + c) * 64] = NVO > 0 ? qr[NV * NV + NV + a * NVO + c] : 0.0;
      lane_solve_qp<NV, NU, NVO, FUSE == 4, false, 64>(P.sv, qc, al, sl, lane - sl, qr, gl);
    }
  }
#if CMPC_ROWS_TIMING
  if (lane == 0) {
    const uint64_t t1c = __builtin_amdgcn_s_memtime(), t1r = __builtin_amdgcn_s_memrealtime();
    double* dbg = P.qp + (size_t)(blockIdx.x * WPG + wave) * 16;
    for (int i = 0; i < 6; ++i) dbg[i] = (double)tsum[i];
    dbg[6] = ngrp;
    dbg[7] = 1.0;
    dbg[8] = (double)(t1c - t0c);  // shader cycles of the wave's lifetime
    dbg[9] = (double)(t1r - t0r);  // 100 MHz ticks of the same span
    dbg[10] = (double)t0r;
    dbg[11] = (double)t1r;
    // placement: HW_ID (wave, simd, pipe, cu, sh, se, ...) and XCC_ID
    dbg[12] = (double)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    dbg[13] = (double)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);
    dbg[14] = (double)(blockIdx.x * WPG + wave);
  }
#endif
}

// ---------------------------------------------------------------------------
// launcher — explicit instantiation list (cf. the reference's *_list.h)
// ---------------------------------------------------------------------------
// Waves per workgroup (4, or 2 where that holds 1.5x the resident waves;
// cmpc_rows_waves_per_group in rows_layout.cpp).
template <int NS, int NY, int NU, int M, int WPG, bool RING, int WPE = CMPC_ROWS_WPE, int FUSE = 0>
static int rows_launch(const BuildParams& P, hipStream_t s) {
  auto kern = cmpc_build_rows_kernel<NS, NY, 4, NU, M, 2, WPG, RING, WPE, FUSE>;
  const size_t lds = sizeof(double) * ((size_t)P.rows.lds_block + (size_t)P.rows.per_wave * WPG);
  if (lds > 160 * 1024) return -1;
  if (lds > 64 * 1024)
    cmpc_allow_lds(reinterpret_cast<const void*>(kern), lds);
  int per_cu = cmpc_blocks_per_cu(kern, 64 * WPG, lds);
  if (per_cu < 1) per_cu = std::max<int>(1, (int)((160 * 1024) / lds));
  per_cu = std::min(per_cu, std::max(1, 4 * WPE / WPG));  // the register budget's waves per SIMD
  // the occupancy query counts the requested LDS only; the measured
  // allocation model (rows_layout.cpp) can allow fewer
  per_cu = std::max(1, std::min(per_cu, cmpc_rows_resident_groups(P.rows, WPG)));
  const int need = std::max(1, ((P.nqp + 3) / 4 + WPG - 1) / WPG);
  const int grid = std::max(1, std::min(need, P.cus * per_cu));
  // the lane solver after the groups (FUSE 3/4) solves one QP per lane: every
  // wave's groups must fit its 64 lanes (16 groups of four QPs)
  if (FUSE >= 3 && ((P.nqp + 3) / 4 + grid * WPG - 1) / (grid * WPG) > 16) return -1;
  cmpc_launch(kern, dim3(grid), dim3(64 * WPG), lds, s, P);
  return 0;
}

