// Probe: (1) lane layouts of the FP64 MFMA forms on gfx950 (A/B/D dumps of
// v_mfma_f64_4x4x4_4b_f64 and v_mfma_f64_16x16x4_f64 on integer data; the
// maps are solved on the host by tools/probe_mfma64_layout.py), and (2) the
// issue cost and held clock of a horizon-step-shaped loop: per step and four
// QPs, NM 4x4x4 MFMAs in four 3-deep accumulation chains whose state tiles
// feed the next step, plus NV VALU DPP FMAs, against a pure-VALU step of 65
// DPP FMAs (the row kernel's loop body).  Data are random, restarted every 50
// steps from memory (a QP group), as in the build kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void layout(double* out) {
  const int l = threadIdx.x;
  double a = (double)(l + 1), b = (double)(1000 * (l + 1));
  // 4x4x4_4b: D = A*B per block (C = 0)
  double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  out[l] = d;
  // with B = 1 at exactly lane 0 (others 0) to separate maps
  d4 z = {0, 0, 0, 0};
  d4 e = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, z, 0, 0, 0);
  for (int i = 0; i < 4; ++i) out[64 + l * 4 + i] = e[i];
}

#define NSTEP 50
#define NGRP 16

// pure-VALU reference step: 65 DPP broadcast FMAs on 16 accumulators
__global__ __launch_bounds__(256) void valu_step(const double* __restrict__ in, double* out, long long* clk) {
  const int lane = threadIdx.x & 63;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double res = 0;
  for (int g = 0; g < NGRP; ++g) {
    const double* src = in + ((blockIdx.x * 4 + (threadIdx.x >> 6)) * NGRP + g) % 4096 * 64 * 20;
    double acc[16], m[4];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = src[i * 64 + lane];
#pragma unroll
    for (int i = 0; i < 4; ++i) m[i] = src[(16 + i) * 64 + lane] * 0.1;
    for (int s = 0; s < NSTEP; ++s) {
      asm volatile(
          "s_nop 1\n\t"
#define F(a, b, c, k) "v_fmac_f64_dpp %" #a ", %" #b ", %" #c " row_newbcast:" #k " row_mask:0xf bank_mask:0xf\n\t"
          F(0, 1, 16, 0) F(2, 3, 17, 1) F(4, 5, 18, 2) F(6, 7, 19, 3) F(8, 9, 16, 4) F(10, 11, 17, 5)
          F(12, 13, 18, 6) F(14, 15, 19, 7) F(1, 0, 16, 8) F(3, 2, 17, 9) F(5, 4, 18, 10) F(7, 6, 19, 11)
          F(9, 8, 16, 12) F(11, 10, 17, 13) F(13, 12, 18, 14) F(15, 14, 19, 15)
          F(0, 1, 16, 0) F(2, 3, 17, 1) F(4, 5, 18, 2) F(6, 7, 19, 3) F(8, 9, 16, 4) F(10, 11, 17, 5)
          F(12, 13, 18, 6) F(14, 15, 19, 7) F(1, 0, 16, 8) F(3, 2, 17, 9) F(5, 4, 18, 10) F(7, 6, 19, 11)
          F(9, 8, 16, 12) F(11, 10, 17, 13) F(13, 12, 18, 14) F(15, 14, 19, 15)
          F(0, 1, 16, 0) F(2, 3, 17, 1) F(4, 5, 18, 2) F(6, 7, 19, 3) F(8, 9, 16, 4) F(10, 11, 17, 5)
          F(12, 13, 18, 6) F(14, 15, 19, 7) F(1, 0, 16, 8) F(3, 2, 17, 9) F(5, 4, 18, 10) F(7, 6, 19, 11)
          F(9, 8, 16, 12) F(11, 10, 17, 13) F(13, 12, 18, 14) F(15, 14, 19, 15)
          F(0, 1, 16, 0) F(2, 3, 17, 1) F(4, 5, 18, 2) F(6, 7, 19, 3) F(8, 9, 16, 4) F(10, 11, 17, 5)
          F(12, 13, 18, 6) F(14, 15, 19, 7) F(1, 0, 16, 8) F(3, 2, 17, 9) F(5, 4, 18, 10) F(7, 6, 19, 11)
          F(9, 8, 16, 12) F(11, 10, 17, 13) F(13, 12, 18, 14) F(15, 14, 19, 15) F(0, 1, 16, 0)
          : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
            "+v"(acc[6]), "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]),
            "+v"(acc[12]), "+v"(acc[13]), "+v"(acc[14]), "+v"(acc[15])
          : "v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]));
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) res += acc[i];
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = res;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
#undef F

// hybrid step: 3 state tiles x 3 k-tiles + 1 output tile x 3 k-tiles of
// 4x4x4_4b MFMAs (12), then NV DPP FMAs on independent accumulators.
template <int NV>
__global__ __launch_bounds__(256) void hybrid_step(const double* __restrict__ in, double* out, long long* clk) {
  const int lane = threadIdx.x & 63;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double res = 0;
  for (int g = 0; g < NGRP; ++g) {
    const double* src = in + ((blockIdx.x * 4 + (threadIdx.x >> 6)) * NGRP + g) % 4096 * 64 * 20;
    double A[9], Cc[3], x[3], acc[8];
#pragma unroll
    for (int i = 0; i < 9; ++i) A[i] = src[i * 64 + lane];
#pragma unroll
    for (int i = 0; i < 3; ++i) Cc[i] = src[(9 + i) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = src[(12 + i) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = src[(12 + i) * 64 + lane] * 0.01;
    double y = 0;
    for (int s = 0; s < NSTEP; ++s) {
      double nx[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        double d = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) d = __builtin_amdgcn_mfma_f64_4x4x4f64(A[t * 3 + k], x[k], d, 0, 0, 0);
        nx[t] = d;
      }
      double yo = 0.0;
#pragma unroll
      for (int k = 0; k < 3; ++k) yo = __builtin_amdgcn_mfma_f64_4x4x4f64(Cc[k], x[k], yo, 0, 0, 0);
      y = yo;
      if constexpr (NV > 0) {
        asm volatile("s_nop 1\n\t"
#define G(a, k) "v_fmac_f64_dpp %" #a ", %8, %9 row_newbcast:" #k " row_mask:0xf bank_mask:0xf\n\t"
                     G(0, 0) G(1, 1) G(2, 2) G(3, 3) G(4, 4) G(5, 5) G(6, 6) G(7, 7)
                     G(0, 8) G(1, 9) G(2, 10) G(3, 11) G(4, 12) G(5, 13) G(6, 14) G(7, 15)
                     G(0, 0) G(1, 1) G(2, 2) G(3, 3) G(4, 4) G(5, 5)
                     : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]),
                       "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7])
                     : "v"(y), "v"(nx[0]));
#undef G
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) x[t] = nx[t];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) res += acc[i];
    res += x[0] + x[1] + x[2] + y;
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = res;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <typename K>
void timeit(const char* name, K kern, int wps, const double* in, double* out, long long* clk, double fma_per_step) {
  const int grid = 256 * wps;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 30; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out, clk);
  const int R = 10;
  hipEventRecord(e0);
  for (int rep = 0; rep < R; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out, clk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= R;
  std::vector<long long> h(2 * grid);
  (void)hipMemcpy(h.data(), clk, sizeof(long long) * 2 * grid, hipMemcpyDeviceToHost);
  double ghz = 0;
  for (int b = 0; b < grid; ++b) ghz += (double)h[2 * b] / ((double)h[2 * b + 1] * 10.0);
  ghz /= grid;
  const double steps = (double)grid * 4 * NGRP * NSTEP;  // wave-steps
  const double ns_per_wstep = ms * 1e6 / steps * (256 * 4);  // per SIMD
  const double tf = fma_per_step * 2 * steps / (ms * 1e-3) / 1e12;
  printf("%-28s w/SIMD=%d %7.3f ms  %6.1f TF/s(issued)  clk %.2f GHz  %6.1f SIMD-cyc/step\n", name, wps, ms,
         tf, ghz, ns_per_wstep * ghz);
}

int main() {
  double *out, *in;
  long long* clk;
  (void)hipMalloc(&out, sizeof(double) * 256 * 256 * 8);
  (void)hipMalloc(&clk, sizeof(long long) * 2 * 256 * 8);
  const size_t nin = (size_t)4096 * 64 * 20;
  (void)hipMalloc(&in, sizeof(double) * nin);
  std::vector<double> h(nin);
  srand(1);
  for (size_t i = 0; i < nin; ++i) h[i] = ((double)rand() / RAND_MAX - 0.5) * 0.94;
  (void)hipMemcpy(in, h.data(), sizeof(double) * nin, hipMemcpyHostToDevice);

  hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, out);
  std::vector<double> d(64 + 256);
  (void)hipMemcpy(d.data(), out, sizeof(double) * d.size(), hipMemcpyDeviceToHost);
  printf("LAYOUT4");
  for (int l = 0; l < 64; ++l) printf(" %.0f", d[l]);
  printf("\nLAYOUT16");
  for (int l = 0; l < 256; ++l) printf(" %.0f", d[64 + l]);
  printf("\n");
  for (int w : {2, 3, 4}) {
    timeit("VALU 65 dpp/step", valu_step, w, in, out, clk, 65 * 64);
    timeit("hybrid 12 M4 + 0 VALU", hybrid_step<0>, w, in, out, clk, 12 * 256);
    timeit("hybrid 12 M4 + 22 dpp", hybrid_step<22>, w, in, out, clk, 12 * 256 + 22 * 64);
  }
  return 0;
}
