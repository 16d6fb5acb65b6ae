// Microbenchmark: issue cost of the build kernel's DPP FMA patterns at 4 and
// 8 waves/SIMD (clock: s_memtime per wave; reported as cycles per instruction
// per SIMD).
//   A: 16 independent accumulators, fixed src0/src1
//   B: one dependent chain a += bcast_l(p) * m[l], 13 distinct m registers (the prop)
//   C: 13 independent accumulators acc[l] += bcast_l(p) * m[l]
//   D: B with plain v_fma_f64 (no DPP)
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 2048
#define CTRL "row_mask:0xf bank_mask:0xf"

template <int MODE>
__global__ __launch_bounds__(256) void chain(double* out, long long* cyc, double seed) {
  double m[13], acc[16];
  for (int i = 0; i < 13; ++i) m[i] = seed * (1 + i * 1e-3) + threadIdx.x * 1e-9;
  for (int i = 0; i < 16; ++i) acc[i] = i * 1e-3;
  double p = seed * 0.5, a = 0.0;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
    if (MODE == 0) {
      asm volatile("s_nop 1\n\t"
#define F(i) "v_fmac_f64_dpp %" #i ", %16, %17 row_newbcast:1 " CTRL "\n\t"
                   F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7) F(8) F(9) F(10) F(11) F(12)
#undef F
                   : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]),
                     "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]),
                     "+v"(acc[10]), "+v"(acc[11]), "+v"(acc[12]), "+v"(acc[13]), "+v"(acc[14]),
                     "+v"(acc[15])
                   : "v"(p), "v"(m[0]));
    } else if (MODE == 1) {
      asm volatile("s_nop 1\n\t"
#define F(i, j) "v_fmac_f64_dpp %0, %1, %" #j " row_newbcast:" #i " " CTRL "\n\t"
                   F(0, 2) F(1, 3) F(2, 4) F(3, 5) F(4, 6) F(5, 7) F(6, 8) F(7, 9) F(8, 10)
                       F(9, 11) F(10, 12) F(14, 13) F(15, 14)
#undef F
                   : "+v"(a)
                   : "v"(p), "v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]), "v"(m[4]), "v"(m[5]),
                     "v"(m[6]), "v"(m[7]), "v"(m[8]), "v"(m[9]), "v"(m[10]), "v"(m[11]),
                     "v"(m[12]));
      p = a;
    } else if (MODE == 2) {
      asm volatile("s_nop 1\n\t"
#define F(i, j) "v_fmac_f64_dpp %" #i ", %13, %" #j " row_newbcast:" #i " " CTRL "\n\t"
                   F(0, 14) F(1, 15) F(2, 16) F(3, 17) F(4, 18) F(5, 19) F(6, 20) F(7, 21)
                       F(8, 22) F(9, 23) F(10, 24) F(11, 25) F(12, 26)
#undef F
                   : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]),
                     "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]),
                     "+v"(acc[10]), "+v"(acc[11]), "+v"(acc[12])
                   : "v"(p), "v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]), "v"(m[4]), "v"(m[5]),
                     "v"(m[6]), "v"(m[7]), "v"(m[8]), "v"(m[9]), "v"(m[10]), "v"(m[11]),
                     "v"(m[12]));
    } else {
      for (int l = 0; l < 13; ++l) a = __builtin_fma(p, m[l], a);
      asm volatile("" : "+v"(a));
      p = a * 1e-300;
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  double s = a + p;
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int MODE>
void run(const char* name, double* out, long long* cyc, int blocks_per_cu) {
  const int grid = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((chain<MODE>), dim3(grid), dim3(256), 0, 0, out, cyc, 1.0000001);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  const double flops = 2.0 * 64 * 13.0 * ITER * (double)grid * 4;  // 4 waves per block
  printf("%-40s waves/SIMD=%d  %.3f ms  %.1f TFLOP/s\n", name, blocks_per_cu, ms, flops / ms / 1e9);
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, sizeof(double) * 256 * 256 * 8);
  hipMalloc(&cyc, sizeof(long long));
  for (int bpc : {1, 2, 3, 4, 8}) {
    run<0>("A 13 indep acc, fixed operands", out, cyc, bpc);
    run<1>("B dependent chain, 13 distinct m (prop)", out, cyc, bpc);
    run<2>("C 13 indep acc, distinct m", out, cyc, bpc);
    run<3>("D dependent v_fma_f64 chain (no DPP)", out, cyc, bpc);
  }
  return 0;
}
