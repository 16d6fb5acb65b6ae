// Microbenchmark: is an FP64-MFMA formulation of the build kernel's horizon
// loop faster than the DPP-VALU one on MI355X?  FP64 MFMA has the VALU's FMA
// rate per cycle (microbench_mfma64: 16 FMA/clk/SIMD both) but holds 2.4 GHz
// where a DPP-FMA stream drops to ~1.9 GHz, so the question is clock x cycles.
// Instruction mixes per block of 4 horizon steps, four QPs per wave, random
// data restarted from memory every 12 blocks (one QP group at p = 50):
//   V0 (the bench kernel): 4 x [33 P-chain + 13 free-response DPP FMAs on four
//        interleaved accumulators, 12 gather DPP FMAs, 3 running-sum FMAs,
//        3 accumulator zeroings]
//   V1 (hybrid): 27 chain + 9 Markov v_mfma_f64_4x4x4_4b (A^4-blocked P rows,
//        tiles in registers) + 4 x [13 free-response DPP FMAs (2 chains),
//        12 gather DPP FMAs, 3 running-sum FMAs]
//   V2 (MFMA-heavy): 27 + 9 + 6 (prefix sums) + 6 (gather) MFMA + 4 x [13
//        free-response DPP FMAs (2 chains), 4 misc VALU]
// Prints ns per wave-block per SIMD and the in-kernel clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define NBLK 12
#define NGRP 8
#define CTRL "row_mask:0xf bank_mask:0xf"
#define M4(a, b, c) __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0)

__device__ __forceinline__ void free_resp(double& s0, double& s1, double p, const double* m) {
  // 13 DPP FMAs on two accumulators (links alternate)
  asm volatile("s_nop 1\n\t"
               "v_fmac_f64_dpp %0, %2, %3 row_newbcast:0 " CTRL "\n\t"
               "v_fmac_f64_dpp %1, %2, %4 row_newbcast:1 " CTRL "\n\t"
               "v_fmac_f64_dpp %0, %2, %5 row_newbcast:2 " CTRL "\n\t"
               "v_fmac_f64_dpp %1, %2, %6 row_newbcast:3 " CTRL "\n\t"
               "v_fmac_f64_dpp %0, %2, %7 row_newbcast:4 " CTRL "\n\t"
               "v_fmac_f64_dpp %1, %2, %8 row_newbcast:5 " CTRL "\n\t"
               "v_fmac_f64_dpp %0, %2, %9 row_newbcast:6 " CTRL "\n\t"
               "v_fmac_f64_dpp %1, %2, %10 row_newbcast:7 " CTRL "\n\t"
               "v_fmac_f64_dpp %0, %2, %11 row_newbcast:8 " CTRL "\n\t"
               "v_fmac_f64_dpp %1, %2, %12 row_newbcast:9 " CTRL "\n\t"
               "v_fmac_f64_dpp %0, %2, %13 row_newbcast:10 " CTRL "\n\t"
               "v_fmac_f64_dpp %1, %2, %14 row_newbcast:14 " CTRL "\n\t"
               "v_fmac_f64_dpp %0, %2, %15 row_newbcast:15 " CTRL "\n\t"
               : "+v"(s0), "+v"(s1)
               : "v"(p), "v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]), "v"(m[4]), "v"(m[5]), "v"(m[6]),
                 "v"(m[7]), "v"(m[8]), "v"(m[9]), "v"(m[10]), "v"(m[11]), "v"(m[12]));
}

__device__ __forceinline__ void gather(double* acc, const double* cv) {
  asm volatile("s_nop 1\n\t"
#define G(a, o, l) "v_fmac_f64_dpp %" #a ", %" #o ", %" #o " row_newbcast:" #l " " CTRL "\n\t"
               G(0, 4, 0) G(1, 4, 1) G(2, 4, 4) G(3, 4, 5) G(0, 5, 0) G(1, 5, 1) G(2, 5, 4) G(3, 5, 5)
                   G(0, 6, 0) G(1, 6, 1) G(2, 6, 4) G(3, 6, 5)
#undef G
               : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
               : "v"(cv[0]), "v"(cv[1]), "v"(cv[2]));
}

__device__ __forceinline__ void chain33(double* aP, double& aS, const double* pP, double pS, const double* m,
                                        const double* n) {
  // 33 P-chain + 13 free-response DPP FMAs, four accumulators interleaved
  asm volatile("s_nop 1\n\t"
#define C(l, r, s)                                                   \
  "v_fmac_f64_dpp %0, %4, %" #r " row_newbcast:" #l " " CTRL "\n\t" \
  "v_fmac_f64_dpp %1, %5, %" #r " row_newbcast:" #l " " CTRL "\n\t" \
  "v_fmac_f64_dpp %2, %6, %" #r " row_newbcast:" #l " " CTRL "\n\t" \
  "v_fmac_f64_dpp %3, %7, %" #s " row_newbcast:" #l " " CTRL "\n\t"
               C(0, 8, 19) C(1, 9, 20) C(2, 10, 21) C(3, 11, 22) C(4, 12, 23) C(5, 13, 24) C(6, 14, 25)
                   C(7, 15, 26) C(8, 16, 27) C(9, 17, 28) C(10, 18, 29)
#undef C
               "v_fmac_f64_dpp %3, %7, %30 row_newbcast:14 " CTRL "\n\t"
               "v_fmac_f64_dpp %3, %7, %31 row_newbcast:15 " CTRL "\n\t"
               : "+v"(aP[0]), "+v"(aP[1]), "+v"(aP[2]), "+v"(aS)
               : "v"(pP[0]), "v"(pP[1]), "v"(pP[2]), "v"(pS), "v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]),
                 "v"(m[4]), "v"(m[5]), "v"(m[6]), "v"(m[7]), "v"(m[8]), "v"(m[9]), "v"(m[10]), "v"(n[0]),
                 "v"(n[1]), "v"(n[2]), "v"(n[3]), "v"(n[4]), "v"(n[5]), "v"(n[6]), "v"(n[7]), "v"(n[8]),
                 "v"(n[9]), "v"(n[10]), "v"(n[11]), "v"(n[12]));
}


// V3: the 46 chain links and the 12 gather FMAs of a step interleaved in one
// block (8 independent accumulators instead of 4, then 4)
__device__ __forceinline__ void chain_gather(double* aP, double& aS, const double* pP, double pS, const double* m,
                                             const double* n, double* acc, const double* cv) {
  asm volatile("s_nop 1\n\t"
#define C(l, r, s)                                                   \
  "v_fmac_f64_dpp %0, %8, %" #r " row_newbcast:" #l " " CTRL "\n\t" \
  "v_fmac_f64_dpp %1, %9, %" #r " row_newbcast:" #l " " CTRL "\n\t" \
  "v_fmac_f64_dpp %2, %10, %" #r " row_newbcast:" #l " " CTRL "\n\t" \
  "v_fmac_f64_dpp %3, %11, %" #s " row_newbcast:" #l " " CTRL "\n\t"
#define G(a, o, l) "v_fmac_f64_dpp %" #a ", %" #o ", %" #o " row_newbcast:" #l " " CTRL "\n\t"
               C(0, 12, 23) G(4, 36, 0) G(5, 36, 1) C(1, 13, 24) G(6, 36, 4) G(7, 36, 5) C(2, 14, 25)
               G(4, 37, 0) G(5, 37, 1) C(3, 15, 26) G(6, 37, 4) G(7, 37, 5) C(4, 16, 27) G(4, 38, 0)
               G(5, 38, 1) C(5, 17, 28) G(6, 38, 4) G(7, 38, 5) C(6, 18, 29) C(7, 19, 30) C(8, 20, 31)
               C(9, 21, 32) C(10, 22, 33)
#undef C
#undef G
               "v_fmac_f64_dpp %3, %11, %34 row_newbcast:14 " CTRL "\n\t"
               "v_fmac_f64_dpp %3, %11, %35 row_newbcast:15 " CTRL "\n\t"
               : "+v"(aP[0]), "+v"(aP[1]), "+v"(aP[2]), "+v"(aS), "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]),
                 "+v"(acc[3])
               : "v"(pP[0]), "v"(pP[1]), "v"(pP[2]), "v"(pS), "v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]),
                 "v"(m[4]), "v"(m[5]), "v"(m[6]), "v"(m[7]), "v"(m[8]), "v"(m[9]), "v"(m[10]), "v"(n[0]),
                 "v"(n[1]), "v"(n[2]), "v"(n[3]), "v"(n[4]), "v"(n[5]), "v"(n[6]), "v"(n[7]), "v"(n[8]),
                 "v"(n[9]), "v"(n[10]), "v"(n[11]), "v"(n[12]), "v"(cv[0]), "v"(cv[1]), "v"(cv[2]));
}

template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void kern(const double* __restrict__ in, double* out, long long* clk) {
  const int lane = threadIdx.x & 63;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double res = 0;
  for (int g = 0; g < NGRP; ++g) {
    const double* src = in + ((blockIdx.x * 4 + (threadIdx.x >> 6)) * NGRP + g) % 4096 * 64 * 64;
    auto ld = [&](int i) { return src[i * 64 + lane]; };
    if constexpr (V == 0 || V == 3) {
      double pP[3], pS, m[11], n[13], acc[4] = {0, 0, 0, 0}, cv[3] = {0, 0, 0};
      for (int i = 0; i < 3; ++i) pP[i] = ld(i);
      pS = ld(3);
      for (int i = 0; i < 11; ++i) m[i] = ld(4 + i) * 0.3;
      for (int i = 0; i < 13; ++i) n[i] = ld(15 + i) * 0.3;
      double sm = ld(28), rd0 = ld(29), rd1 = ld(30), rd2 = ld(31);
      for (int b = 0; b < NBLK; ++b) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          double aP[3] = {0.0, 0.0, 0.0}, aS = rd0;
          if constexpr (V == 0) {
            chain33(aP, aS, pP, pS, m, n);
            cv[0] = __builtin_fma(sm, cv[0], rd0);
            cv[1] = __builtin_fma(sm, cv[1], rd1);
            cv[2] = __builtin_fma(sm, cv[2], rd2);
            gather(acc, cv);
          } else {
            chain_gather(aP, aS, pP, pS, m, n, acc, cv);
            cv[0] = __builtin_fma(sm, cv[0], rd0);
            cv[1] = __builtin_fma(sm, cv[1], rd1);
            cv[2] = __builtin_fma(sm, cv[2], rd2);
          }
          pP[0] = aP[0]; pP[1] = aP[1]; pP[2] = aP[2]; pS = aS;
        }
      }
      res += acc[0] + acc[1] + acc[2] + acc[3] + pP[0] + pP[1] + pP[2] + pS;
    } else if constexpr (V == 4) {
      // V4 (round 3): P^T chain on MFMA with A^4 blocking: P^T_{r+4} = (A^4)^T P^T_r
      // (3 row tiles x 3 k = 9), Markov of the block's 4 steps from P^T_r and
      // (A^k B)^T (4 x 3 = 12), Gram over k = 4 steps x 3 outputs (3 col tiles
      // x 3 k-chunks = 9); free response on DPP (13 per step, 2 chains), the
      // running sums as 1 VALU add per step; the column hand-off through LDS
      // (8 writes + 12 reads per block per lane)
      __shared__ double lds[4][64 * 8];
      double* wl = lds[threadIdx.x >> 6];
      double A4T[9], PT[3], AkB[12], m[13], S = 0.0;
      for (int i = 0; i < 9; ++i) A4T[i] = ld(i) * 0.3;
      for (int i = 0; i < 3; ++i) PT[i] = ld(9 + i);
      for (int i = 0; i < 12; ++i) AkB[i] = ld(12 + i) * 0.3;
      for (int i = 0; i < 13; ++i) m[i] = ld(24 + i) * 0.3;
      double pS = ld(37);
      double G[3] = {0, 0, 0};
#pragma unroll 1
      for (int b = 0; b < NBLK; ++b) {
        double Mk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // Markov of step 4b + k: (A^k B)^T P^T_r
          double d = M4(AkB[k * 3 + 0], PT[0], 0.0);
          d = M4(AkB[k * 3 + 1], PT[1], d);
          Mk[k] = M4(AkB[k * 3 + 2], PT[2], d);
        }
        double Pn[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          double d = M4(A4T[i * 3 + 0], PT[0], 0.0);
          d = M4(A4T[i * 3 + 1], PT[1], d);
          Pn[i] = M4(A4T[i * 3 + 2], PT[2], d);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          S = S + Mk[k];                       // running sum (move-1 columns)
          wl[(k * 2 + 0) * 64 + lane] = Mk[k];  // hand-off writes
          wl[(k * 2 + 1) * 64 + lane] = S;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          double s0 = pS * 0.5, s1 = 0.0;
          free_resp(s0, s1, pS, m);
          pS = s0 + s1;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        // column reads (A: own columns over 3 k-chunks, B: 3 tiles x 3 chunks)
        double Ac[3], Bc[9];
#pragma unroll
        for (int c = 0; c < 3; ++c) Ac[c] = wl[((c * 5 + 1) & 7) * 64 + (lane ^ (c + 1))];
#pragma unroll
        for (int t = 0; t < 9; ++t) Bc[t] = wl[((t * 3 + 2) & 7) * 64 + (lane ^ (t + 5))];
#pragma unroll
        for (int t = 0; t < 3; ++t) {  // Gram: 3 column tiles x 3 k-chunks
          double d = M4(Ac[0], Bc[t * 3 + 0], G[t]);
          d = M4(Ac[1], Bc[t * 3 + 1], d);
          G[t] = M4(Ac[2], Bc[t * 3 + 2], d);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) PT[i] = Pn[i];
      }
      res += pS + S + G[0] + G[1] + G[2] + PT[0] + PT[1] + PT[2];
    } else {
      // MFMA tiles: A4T[9] constants, T[9] chain state, Bt[3] constants
      double A4T[9], T[9], Bt[3], m[13], acc[4] = {0, 0, 0, 0}, cv[3] = {0, 0, 0}, Mk[3] = {0, 0, 0};
      for (int i = 0; i < 9; ++i) A4T[i] = ld(i) * 0.3;
      for (int i = 0; i < 9; ++i) T[i] = ld(9 + i);
      for (int i = 0; i < 3; ++i) Bt[i] = ld(18 + i);
      for (int i = 0; i < 13; ++i) m[i] = ld(21 + i) * 0.3;
      double pS = ld(34), sm = ld(35), Lc = ld(36), Jc = ld(37);
      double G[6] = {0, 0, 0, 0, 0, 0}, Nt[3] = {0, 0, 0};
      for (int b = 0; b < NBLK; ++b) {
        double Tn[9];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            double d = M4(A4T[i * 3 + 0], T[0 * 3 + t], 0.0);
            d = M4(A4T[i * 3 + 1], T[1 * 3 + t], d);
            Tn[i * 3 + t] = M4(A4T[i * 3 + 2], T[2 * 3 + t], d);
          }
        double Mn[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          double d = M4(T[0 * 3 + t], Bt[0], 0.0);
          d = M4(T[1 * 3 + t], Bt[1], d);
          Mn[t] = M4(T[2 * 3 + t], Bt[2], d);
        }
        if constexpr (V == 2) {
#pragma unroll
          for (int t = 0; t < 3; ++t) {  // prefix sums (L Mk + J carry) and gather
            const double c = Nt[t] + Mk[t];
            double nn = M4(Lc, Mk[t], 0.0);
            Nt[t] = M4(Jc, c, nn);
            G[2 * t] = M4(Mk[t], Mk[t], G[2 * t]);
            G[2 * t + 1] = M4(Mk[t], Nt[t], G[2 * t + 1]);
          }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          double s0 = pS * 0.5, s1 = 0.0;
          free_resp(s0, s1, pS, m);
          pS = s0 + s1;
          if constexpr (V == 1) {
            cv[0] = __builtin_fma(sm, cv[0], Mk[0]);
            cv[1] = __builtin_fma(sm, cv[1], Mk[1]);
            cv[2] = __builtin_fma(sm, cv[2], Mk[2]);
            gather(acc, cv);
          } else {
            cv[s & 1] = __builtin_fma(sm, cv[s & 1], pS);
          }
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) T[i] = Tn[i];
#pragma unroll
        for (int t = 0; t < 3; ++t) Mk[t] = Mn[t];
      }
      res += acc[0] + acc[1] + acc[2] + acc[3] + pS + cv[0] + cv[1];
      for (int i = 0; i < 9; ++i) res += T[i];
      for (int i = 0; i < 6; ++i) res += G[i];
      for (int i = 0; i < 3; ++i) res += Mk[i] + Nt[i];
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = res;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int V>
void timeit(const char* name, int wps, const double* in, double* out, long long* clk) {
  const int grid = 256 * wps;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // settle: ~0.3 s of launches (the clock ramps over the first ~40 ms of load)
  for (int rep = 0; rep < 300 * 4 / wps; ++rep)
    hipLaunchKernelGGL(kern<V>, dim3(grid), dim3(256), 0, 0, in, out, clk);
  const int R = 10;
  (void)hipEventRecord(e0);
  for (int rep = 0; rep < R; ++rep) hipLaunchKernelGGL(kern<V>, dim3(grid), dim3(256), 0, 0, in, out, clk);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= R;
  std::vector<long long> h(2 * grid);
  (void)hipMemcpy(h.data(), clk, sizeof(long long) * 2 * grid, hipMemcpyDeviceToHost);
  double ghz = 0;
  for (int b = 0; b < grid; ++b) ghz += (double)h[2 * b] / ((double)h[2 * b + 1] * 10.0);
  ghz /= grid;
  const double blocks = (double)grid * 4 * NGRP * NBLK;        // wave-blocks
  const double ns_blk = ms * 1e6 / blocks * (256 * 4);          // per SIMD
  printf("%-12s w/SIMD=%d %7.3f ms  %7.1f ns/block  %6.1f SIMD-cyc/block  clk %.2f GHz\n", name, wps, ms, ns_blk,
         ns_blk * ghz, ghz);
}

int main() {
  double *out, *in;
  long long* clk;
  (void)hipMalloc(&out, sizeof(double) * 256 * 256 * 8);
  (void)hipMalloc(&clk, sizeof(long long) * 2 * 256 * 8);
  const size_t nin = (size_t)4096 * 64 * 64;
  (void)hipMalloc(&in, sizeof(double) * nin);
  std::vector<double> h(nin);
  srand(1);
  for (size_t i = 0; i < nin; ++i) h[i] = ((double)rand() / RAND_MAX - 0.5) * 0.94;
  (void)hipMemcpy(in, h.data(), sizeof(double) * nin, hipMemcpyHostToDevice);
  for (int w : {2, 3, 4}) {
    timeit<0>("V0 dpp", w, in, out, clk);
    timeit<3>("V3 dpp ilp", w, in, out, clk);
    timeit<1>("V1 hybrid", w, in, out, clk);
    timeit<2>("V2 mfma", w, in, out, clk);
    timeit<4>("V4 mfma-a4", w, in, out, clk);
  }
  return 0;
}
