#pragma once
// Device record producer body, shared by the producer
// kernel (produce.hip) and the one-launch control step (cmpc_kernels.hip):
// AugmentedLinearizedSystem::Update for every scenario of the batch, written
// straight into the lin records the build kernel reads.
//
//   continuous linearisation   plant_model.h (shared with the host producer)
//   DiscretizeRK4 (Taylor-4)   libs/aug_lin_sys.cc:232-255
//   record assembly            cmpc_plant_lin_record (plant.cpp) + the
//                              observer tail dx_aug and the controlled y
//
// Four scenarios per wave, one per 16-lane DPP row.  Lane 0 of each row runs
// the scalar plant model into LDS (the four side by side); the 11x11 products
// of the discretisation are DPP broadcast-FMA chains (v_fmac_f64_dpp
// row_newbcast, as the build kernel), and the S records of the scenario are
// written through a per-workgroup element -> source table.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_internal.h"
#include "plant_model.h"
#include "dpp_blocks.inc"

namespace cmpc_prod {


// LDS hand-offs inside one wave: order the stores before the other lanes'
// loads (compiler and hardware, wavefront scope)
#define WAVE_SYNC()                                           \
  do {                                                        \
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");    \
    __builtin_amdgcn_wave_barrier();                          \
  } while (0)

constexpr int kWaves = 4;          // waves per workgroup
constexpr int kSpw = 4;            // scenarios per wave: one per 16-lane row
constexpr int kLanes = 64 / kSpw;  // lanes per scenario
constexpr int kMat = 121;          // ns x ns, ns <= 11
// per scenario: A|Ad, Bc|Bd, Cc, fc|fd, x, u.  The discretised Ad, Bd, fd
// overwrite A, Bc, fc: every lane holds its column of [A | B | f] in
// registers before the first store, and one wave's LDS operations complete
// in order.  (Separate arrays: 2 waves/SIMD by LDS, 0.140 ms at 65 536
// scenarios; aliased, with the table sized by S: 4 waves/SIMD.)
constexpr int kScnLds = kMat + 2 * 44 + 11 + 2 * 11 + 3 + 4 + 2;
// the last two entries of a scenario's region hold 0.0 and 1.0, so that every
// record element before the observer tail is one table-indexed LDS read
constexpr int kZeroSlot = kScnLds - 2, kOneSlot = kScnLds - 1;

// Source of record element e of sub-controller s (same for every scenario):
// >= 0: offset in the scenario's LDS region (Ad, Bd, Cc, fd, or the 0.0 and
// 1.0 slots); kDx + i: observer tail element i; kY + o: plant output o;
// kZero: padding after y.
constexpr int kZero = -1, kDx = -1000, kY = -100;


// LDS bytes of the element -> source table (S x rec_len, then naug entries)
__host__ __device__ inline int table_ints(const ProduceParams& P) { return P.S * P.rec_len + P.naug; }

// The element -> source table of the workgroup (src) and the ring map of the
// observer tail (dmap = src + S * rec_len); threads tid of nthreads share the
// loops.  Barrier before produce_row reads them.
template <int PLANT>
__device__ __forceinline__ void produce_table(const ProduceParams& P, int* src, int* dmap, int tid, int nthreads) {
  constexpr int ns = PLANT == CMPC_PLANT_PARALLEL ? 11 : 10;
  // element -> source table (built once per workgroup)
  for (int t = tid; t < P.S * P.rec_len; t += nthreads) {
    const int s = t / P.rec_len, e = t - s * P.rec_len;
    int v = e < P.off_x ? kZeroSlot : kZero;
    constexpr int oAd = 0, oBd = kMat, oCc = kMat + 44, ofd = kMat + 88;  // Ad, Bd, Cc, fd in a unit region
    if (e >= P.off_A && e < P.off_A + ns * ns) {
      v = oAd + (e - P.off_A);
    } else if (e >= P.off_B && e < P.off_B + ns * P.nu_tot) {
      const int r = (e - P.off_B) / P.nu_tot, c = e - P.off_B - r * P.nu_tot;
      v = oBd + r * 4 + P.input_order[s][c];
    } else if (e >= P.off_C && e < P.off_C + P.ny * P.nobs) {
      const int o = (e - P.off_C) / P.nobs, k = e - P.off_C - o * P.nobs;
      const int oi = P.out_idx[s][o];
      v = (k < ns) ? oCc + oi * ns + k : ((oi == k - ns) ? kOneSlot : kZeroSlot);
    } else if (e >= P.off_f && e < P.off_f + ns) {
      v = ofd + (e - P.off_f);
    } else if (e >= P.off_x && e < P.off_x + P.naug) {
      v = kDx - (e - P.off_x);
    } else if (e >= P.off_y && e < P.off_y + P.ny) {
      v = kY - P.out_idx[s][e - P.off_y];
    }
    src[t] = v;
  }
  // logical entry e of a ring-stored delay block (observer state,
  // cmpc_obs_prior_kernel) -> its position in the row; the same for every unit
  for (int e = tid; e < P.naug; e += nthreads) {
    int pe = e;
    for (int k = 0; k < P.nring; ++k)
      if (e >= P.rb[k] && e < P.rb[k] + P.rlen[k]) {
        const int i = e - P.rb[k] + P.rot[k];
        pe = P.rb[k] + (i >= P.rlen[k] ? i - P.rlen[k] : i);
      }
    dmap[e] = pe;
  }
}

// One unit (scenario, or QP slot in per-QP mode) on one 16-lane DPP row of
// this wave: w = the row's kScnLds-double LDS region, lane = lane in the wave.
// Every lane of the wave calls it (wave barriers inside).
template <int PLANT>
__device__ __forceinline__ void produce_row(const ProduceParams& P, double* w, const int* src, const int* dmap,
                                            int unit, int lane) {
  const int g = lane / kLanes, l = lane - g * kLanes;  // unit row, lane in row
  const bool valid = unit < (P.per_qp ? P.B * P.S : P.B);  // (rows past the batch idle
                                                           //  but keep the wave's syncs)
  const int b = P.per_qp ? unit / P.S : unit;
  constexpr int ns = PLANT == CMPC_PLANT_PARALLEL ? 11 : 10;
  constexpr int ni = PLANT == CMPC_PLANT_PARALLEL ? 9 : 8;
  double *A = w, *Ad = A;
  double *Bc = A + kMat, *Bd = Bc, *Cc = Bc + 44, *fc = Cc + 44, *fd = fc;
  double *xs = fc + 11, *us = xs + 11, *tk = us + 14;  // tk: 4 (parallel plant)
  (void)g;
  if (l == 0) {  // the region's 0.0 and 1.0 slots (read through the table)
    w[kZeroSlot] = 0.0;
    w[kOneSlot] = 1.0;
  }

  // cmpc_observe_step: ObserveAPosteriori of the slot first (libs/observer.cc:
  // 27-44; the arithmetic order of oracle/or_observer.c or_observe_post),
  // then the linearisation at the updated x_hat.  The updated disturbance
  // states of dx reach the record's observer tail from registers (dnd).
  const bool post = P.per_qp && P.obs_M;
  double xq = 0.0, dnd = 0.0;
  if (post) {
    constexpr int NO = 4, NOBS = ns + NO;  // disturbance states = outputs (C = [C_plant | I])
    const int base = lane & ~(kLanes - 1);
    const int qq = valid ? unit : P.B * P.S - 1;
    const int bq = qq / P.S, sq = qq - bq * P.S;
    double* st = P.obs + (size_t)qq * P.x_stride;
    double* dxo = st + ns;
    double* yo = dxo + P.obs_ntot;
    const double* Cq = yo + NO;
    const double* yq = P.y + (size_t)bq * NO;
    const double* Mq = P.obs_M + (size_t)sq * NOBS * NO;
    const double dxl = (l < NOBS) ? dxo[l] : 0.0;
    const double xl = (l < ns) ? st[l] : 0.0;
    double mrow[NO], crow[ns];
#pragma unroll
    for (int o = 0; o < NO; ++o) mrow[o] = (l < NOBS) ? Mq[l * NO + o] : 0.0;
    const int lc = l < NO ? l : 0;
#pragma unroll
    for (int j = 0; j < ns; ++j) crow[j] = Cq[lc * ns + j];
    const double yl = yq[lc], yol = yo[lc];
    double t = 0.0;
#pragma unroll
    for (int j = 0; j < ns; ++j) t += crow[j] * __shfl(dxl, base + j, 64);
    t = t + __shfl(dxl, base + ns + lc, 64);
    const double v = (yl - yol) - t;
    double acc = 0.0;
#pragma unroll
    for (int o = 0; o < NO; ++o) acc += mrow[o] * __shfl(v, base + o, 64);
    const double dn = dxl + acc;
    xq = xl + dn;
    dnd = __shfl(dn, base + ns + lc, 64);
    if (valid) {
      if (l < NOBS) dxo[l] = dn;
      if (l < ns) st[l] = xq;
      if (l < NO) yo[l] = yl;
    }
  }
  if (valid && l < ns)
    xs[l] = post ? xq : P.per_qp ? P.x[(size_t)unit * P.x_stride + l] : P.x[(size_t)b * ns + l];
  if (valid && l < ni) us[l] = P.u_full[(size_t)b * ni + l];
  for (int e = l; e < ns * ns; e += kLanes) A[e] = 0.0;  // the row clears, its lane 0
  for (int e = l; e < ns * 4; e += kLanes) {             // writes the nonzeros
    Bc[e] = 0.0;
    Cc[e] = 0.0;
  }
  WAVE_SYNC();
#ifndef PRODUCE_EXP
#define PRODUCE_EXP 0
#endif
  // the scalar plant model, four scenarios side by side: the parallel
  // plant's two compressors on lanes 0 and 1 of the row, then its tank
  if (PLANT == CMPC_PLANT_PARALLEL) {
    if (PRODUCE_EXP != 1 && valid && l < 2)
      cmpc_plant::parallel_linearize_part(l, P.p_in, xs, us, A, Bc, Cc, fc, tk);
    WAVE_SYNC();
    if (PRODUCE_EXP != 1 && valid && l == 0)
      cmpc_plant::parallel_linearize_tank(P.p_out, xs, us, A, Cc, fc, tk);
  } else if (PRODUCE_EXP != 1 && valid && l == 0) {
    cmpc_plant::serial_linearize(P.p_in, P.p_out, xs, us, A, Bc, Cc, fc, false);
  }
  WAVE_SYNC();

  // DiscretizeRK4: Ac = Ts I + Ts^2/2 A + Ts^3/6 A^2 + Ts^4/24 A^3,
  // Ad = I + Ac A, Bd = Ac B, fd = Ac f.  Lane j of a row holds column j of
  // [A | B | f] (j < ns: A, then the 4 B columns, then f) and, for every
  // product row i, lane k holds X[i][k]: one row of X Y is one chain of ns
  // DPP broadcast FMAs (k ascending, fused multiply-add like the host).
  const double Ts = P.Ts;
  if (PRODUCE_EXP != 2) {
    double ycol[ns], a2[ns], a3[ns];
#pragma unroll
    for (int k = 0; k < ns; ++k)
      ycol[k] = (l < ns) ? A[k * ns + l] : (l < ns + 4) ? Bc[k * 4 + (l - ns)]
              : (l == ns + 4) ? fc[k] : 0.0;
    // A^2 and A^3 (row i of X is column i of A held as ycol[i] in lane k)
#pragma unroll
    for (int i = 0; i < ns; ++i) {
      double z = 0.0;
      prop1_dpp<ns>(ycol[i], ycol, z);
      a2[i] = z;
    }
#pragma unroll
    for (int i = 0; i < ns; ++i) {
      double z = 0.0;
      prop1_dpp<ns>(a2[i], ycol, z);
      a3[i] = z;
    }
    // Ac (element-wise, lane j holds column j) and Ac [A | B | f]; lane j
    // stores row i of its column at a per-lane base and stride (Ad, Bd or fd)
    double* const dst = (l < ns) ? Ad + l : (l < ns + 4) ? Bd + (l - ns) : fd;
    const int dstride = (l < ns) ? ns : (l < ns + 4) ? 4 : 1;
    const bool dstore = l < ns + 5;
#pragma unroll
    for (int i = 0; i < ns; ++i) {
      const double ac = Ts * (i == l) + Ts * Ts / 2.0 * ycol[i] + Ts * Ts * Ts / 6.0 * a2[i] +
                        Ts * Ts * Ts * Ts / 24.0 * a3[i];
      double z = 0.0;
      prop1_dpp<ns>(ac, ycol, z);
      if (dstore) dst[i * dstride] = (i == l) ? z + 1.0 : z;
    }
    WAVE_SYNC();
  }
  if (!valid || PRODUCE_EXP == 3) return;

  // the observer's next a-posteriori step reads this linearisation's C
  if (P.per_qp)
    for (int e = l; e < P.n_outputs * ns; e += kLanes) P.c_out[(size_t)unit * P.c_stride + e] = Cc[e];
  // records of the S sub-controllers of scenario b (per-QP mode: of slot q)
  const int s0 = P.per_qp ? unit - b * P.S : 0, s1 = P.per_qp ? s0 + 1 : P.S;
  const int dxs = P.per_qp ? P.dx_stride : P.naug;
  // Record layout: [A B C f] from this scenario's LDS through the table,
  // then the observer tail dx_aug (a straight copy: its loads do not wait on
  // the table, and the loop has no branches), then y and the padding.
  // Each loop gathers kU values per lane into registers before storing them:
  // the compiler cannot move a load of dx (or the table) above a store to
  // rec it may alias, so a plain loop pays one load latency per element
  // (cmpc_observe_step at 131 072 QP slots 0.220 -> 0.187 ms; scenario mode
  // unchanged at 0.10 ms).
  constexpr int kU = 8;
  for (int s = s0; s < s1; ++s) {
    const size_t q = (size_t)b * P.S + s;
    double* rec = P.lin + q * P.rec_len;
    const int* srow = src + s * P.rec_len;
    for (int e0 = l; e0 < P.off_x; e0 += kU * kLanes) {
      double v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + u * kLanes;
        v[u] = w[e < P.off_x ? srow[e] : kZeroSlot];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (e0 + u * kLanes < P.off_x) rec[e0 + u * kLanes] = v[u];
    }
    const double* dx = P.dx_aug ? P.dx_aug + q * dxs : nullptr;
    for (int e0 = l; e0 < P.naug; e0 += kU * kLanes) {
      double v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + u * kLanes;
        v[u] = (post && e < 4) ? dnd : (dx && e < P.naug) ? dx[dmap[e]] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (e0 + u * kLanes < P.naug) rec[P.off_x + e0 + u * kLanes] = v[u];
    }
    for (int e = P.off_x + P.naug + l; e < P.rec_len; e += kLanes) {
      const int t = srow[e];  // y (kY - o) or padding (kZero)
      rec[e] = (t == kZero) ? 0.0 : P.y[(size_t)b * P.n_outputs + (kY - t)];
    }
  }
}

}  // namespace cmpc_prod
