// Microbenchmark: FP64 FMA issue rate on MI355X — plain v_fma_f64 (VOP3) vs
// v_fmac_f64_dpp row_newbcast (the build kernel's broadcast FMA).
// Each wave runs ITER iterations of 16 independent accumulator chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 4096
__global__ __launch_bounds__(256) void fma_plain(double* out, double a) {
  double acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = threadIdx.x * 1e-3 + i;
  double b = a + threadIdx.x * 1e-9;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = __builtin_fma(acc[i], b, a);
  }
  double s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void fma_dpp(double* out, double a) {
  double acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = threadIdx.x * 1e-3 + i;
  double b = a + threadIdx.x * 1e-9;
  double src = b * 0.5;
  for (int it = 0; it < ITER; ++it) {
    asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %16, %17 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %16, %17 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, %16, %17 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, %16, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, %16, %17 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, %16, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %6, %16, %17 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %7, %16, %17 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %8, %16, %17 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %9, %16, %17 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %10, %16, %17 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %11, %16, %17 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %12, %16, %17 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %13, %16, %17 row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %14, %16, %17 row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %15, %16, %17 row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
      : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
        "+v"(acc[6]), "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]),
        "+v"(acc[12]), "+v"(acc[13]), "+v"(acc[14]), "+v"(acc[15])
      : "v"(src), "v"(b));
  }
  double s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// single-wave-per-SIMD dependent chain latency of v_fmac_f64_dpp
__global__ void lat_dpp(double* out, long long* cyc, double a) {
  double acc = threadIdx.x * 1e-3, src = a;
  long long t0 = clock64();
  for (int it = 0; it < ITER; ++it) {
    asm volatile("v_fmac_f64_dpp %0, %1, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                 "v_fmac_f64_dpp %0, %1, %0 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                 : "+v"(acc) : "v"(src));
  }
  long long t1 = clock64();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
__global__ void lat_plain(double* out, long long* cyc, double a) {
  double acc = threadIdx.x * 1e-3, b = a + threadIdx.x;
  long long t0 = clock64();
  for (int it = 0; it < ITER; ++it) {
    acc = __builtin_fma(acc, b, a);
    acc = __builtin_fma(acc, b, a);
    asm volatile("" : "+v"(acc));
  }
  long long t1 = clock64();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  int ncu = 256;
  double* out; long long* cyc;
  hipMalloc(&out, sizeof(double) * 1 << 24);
  hipMalloc(&cyc, sizeof(long long));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int blocksPerCU : {4, 8}) {
    int grid = ncu * blocksPerCU * 4;
    for (int v = 0; v < 2; ++v) {
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(fma_plain, dim3(grid), dim3(256), 0, 0, out, 1.0000001);
        else hipLaunchKernelGGL(fma_dpp, dim3(grid), dim3(256), 0, 0, out, 1.0000001);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double flops = 2.0 * 16 * ITER * (double)grid * 256;
        if (rep == 2) printf("%s blocks/CU=%d: %.3f ms  %.1f TFLOP/s\n", v ? "v_fmac_f64_dpp" : "v_fma_f64     ",
                             blocksPerCU * 4, ms, flops / ms / 1e9);
      }
    }
  }
  long long c;
  hipLaunchKernelGGL(lat_dpp, dim3(1), dim3(64), 0, 0, out, cyc, 1.0); hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("dependent v_fmac_f64_dpp chain: %.2f clock64 ticks/instr\n", (double)c / (2 * ITER));
  hipLaunchKernelGGL(lat_plain, dim3(1), dim3(64), 0, 0, out, cyc, 1.0); hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("dependent v_fma_f64 chain: %.2f clock64 ticks/instr\n", (double)c / (2 * ITER));
  return 0;
}
