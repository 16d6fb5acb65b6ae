// Microbenchmark: FP64 matrix-core rates on MI355X (gfx950) and whether FP64
// MFMA work overlaps FP64 VALU work issued by the same SIMD.
//   M16  : v_mfma_f64_16x16x4_f64, NACC independent accumulators per wave
//   M4   : v_mfma_f64_4x4x4_4b_f64 (four 4x4x4 blocks per instruction)
//   MIX  : one 16x16x4 MFMA + NV independent v_fma_f64 per iteration
//   VALU : NV independent v_fma_f64 per iteration, no MFMA
// Operands are non-trivial (no zeros) so the clock is the one held under load.
// Prints TF/s counted as issued FMA lanes x 2, the in-kernel clock
// (s_memtime / s_memrealtime) and cycles per loop iteration per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));

#define ITER 2048

template <int KIND, int NV>
__global__ __launch_bounds__(256) void kern(double* out, long long* clk, double s) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + lane * 1e-7 + s;
  double b = 0.999999 - lane * 3e-8;
  d4 acc0 = {a, b, a * b, a - b}, acc1 = acc0 * 0.5, acc2 = acc0 * 0.25, acc3 = acc0 * 0.125;
  double v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = a + i * 1e-3;
  double s4 = a;
  long long t0 = __builtin_amdgcn_s_memtime();
  long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITER; ++it) {
    if constexpr (KIND == 0) {  // M16, 4 independent accumulators
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, acc3, 0, 0, 0);
    } else if constexpr (KIND == 1) {  // M4, 4 independent accumulators
      v[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, v[0], 0, 0, 0);
      v[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(b, a, v[1], 0, 0, 0);
      v[2] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, a, v[2], 0, 0, 0);
      v[3] = __builtin_amdgcn_mfma_f64_4x4x4f64(b, b, v[3], 0, 0, 0);
    } else if constexpr (KIND == 2) {  // MIX: 1 M16 + NV VALU FMAs
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < NV; ++i) v[i] = __builtin_fma(v[i], b, a);
      asm volatile("" ::: "memory");
    } else if constexpr (KIND == 3) {  // VALU only
#pragma unroll
      for (int i = 0; i < NV; ++i) v[i] = __builtin_fma(v[i], b, a);
      asm volatile("" ::: "memory");
    } else if constexpr (KIND == 4) {  // M16 dependent chain on one accumulator
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
    } else if constexpr (KIND == 5) {  // MIX with 4x4x4: 1 M4 + NV VALU FMAs
      s4 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, s4, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < NV; ++i) v[i] = __builtin_fma(v[i], b, a);
      asm volatile("" ::: "memory");
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  long long r1 = __builtin_amdgcn_s_memrealtime();
  double r = acc0[0] + acc0[1] + acc0[2] + acc0[3] + acc1[0] + acc2[1] + acc3[2] + s4;
#pragma unroll
  for (int i = 0; i < 16; ++i) r += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int KIND, int NV>
void run(const char* name, double* out, long long* clk, int wps, double mfma_fma, double valu_fma) {
  const int grid = 256 * wps;  // 4 waves per block -> wps waves per SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  // ~1 s of back-to-back launches so the clock settles, then time one.
  for (int rep = 0; rep < 40; ++rep)
    hipLaunchKernelGGL((kern<KIND, NV>), dim3(grid), dim3(256), 0, 0, out, clk, 1e-9 * rep);
  hipEventRecord(e0);
  const int R = 5;
  for (int rep = 0; rep < R; ++rep)
    hipLaunchKernelGGL((kern<KIND, NV>), dim3(grid), dim3(256), 0, 0, out, clk, 1e-9 * rep);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  ms /= R;
  long long h[2];
  hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  const double ghz = (double)h[0] / ((double)h[1] * 10.0);  // memrealtime = 100 MHz
  const double waves = (double)grid * 4;
  const double tf = 2.0 * (mfma_fma + valu_fma) * ITER * waves / (ms * 1e-3) / 1e12;
  const double cyc_it = (double)h[0] / ITER;
  printf("%-34s w/SIMD=%d %8.3f ms %7.1f TF/s  clk %.2f GHz  %6.1f cyc/iter/wave\n", name, wps, ms,
         tf, ghz, cyc_it);
}

int main() {
  double* out;
  long long* clk;
  hipMalloc(&out, sizeof(double) * 256 * 256 * 8);
  hipMalloc(&clk, sizeof(long long) * 2 * 256 * 8);
  for (int w : {1, 2, 4}) {
    run<0, 0>("M16 x4 indep (1024 FMA each)", out, clk, w, 4 * 1024, 0);
    run<4, 0>("M16 dependent chain", out, clk, w, 1024, 0);
    run<1, 0>("M4_4b x4 indep (256 FMA each)", out, clk, w, 4 * 256, 0);
    run<3, 16>("VALU 16 fma_f64", out, clk, w, 0, 16 * 64);
    run<2, 4>("MIX M16 + 4 VALU", out, clk, w, 1024, 4 * 64);
    run<2, 8>("MIX M16 + 8 VALU", out, clk, w, 1024, 8 * 64);
    run<2, 12>("MIX M16 + 12 VALU", out, clk, w, 1024, 12 * 64);
    run<2, 16>("MIX M16 + 16 VALU", out, clk, w, 1024, 16 * 64);
    run<5, 4>("MIX M4 + 4 VALU", out, clk, w, 256, 4 * 64);
    run<5, 8>("MIX M4 + 8 VALU", out, clk, w, 256, 8 * 64);
  }
  return 0;
}
