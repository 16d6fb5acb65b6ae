// Microbenchmark: LDS throughput per CU of ds_read_b64 / ds_read2_b64 /
// ds_write_b64 under different exec masks and address patterns, to size the
// build kernel's per-step LDS traffic.  16 waves per CU, each issuing ITER
// LDS instructions; reports CU-clocks per instruction per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 4096

// mode: 0 = 64 lanes distinct addresses, 1 = 64 lanes same address (broadcast),
//       2 = 16 lanes active (one row), 3 = 1 lane active
template <int MODE, int OP>
__global__ __launch_bounds__(256) void lds_kernel(double* out, long long* cyc) {
  __shared__ double buf[4096];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4096; i += 256) buf[i] = i * 1e-3;
  __syncthreads();
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int addr = (MODE == 1) ? wave * 8 : wave * 512 + lane;
  bool act = (MODE == 2) ? (lane < 16) : (MODE == 3) ? (lane == 0) : true;
  long long t0 = clock64();
  if (act) {
    for (int it = 0; it < ITER / 8; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int a = (addr + j * 64 * ((MODE == 1) ? 0 : 1) + (MODE == 1 ? j : 0)) & 2047;
        if (OP == 0) {
          acc[j] += buf[a];
        } else if (OP == 1) {
          acc[j] += buf[a] + buf[a + 1];
        } else {
          buf[a + 2048] = acc[j];
          acc[j] += 1.0;
        }
      }
      asm volatile("" ::: "memory");
    }
  }
  long long t1 = clock64();
  double t = 0;
  for (int j = 0; j < 8; ++j) t += acc[j];
  out[blockIdx.x * 256 + threadIdx.x] = t;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int MODE, int OP>
void run(const char* name, double* out, long long* cyc, int grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((lds_kernel<MODE, OP>), dim3(grid), dim3(256), 0, 0, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep == 2) {
      // instructions per CU: grid/256 CUs ... report ns per (wave-instruction per CU)
      const double waves_per_cu = (double)grid * 4 / 256;
      const double instr_per_cu = waves_per_cu * ITER;
      printf("%-34s %.3f ms  %.2f ns per wave-instr per CU (%.2f clk @2.4GHz)\n", name, ms,
             ms * 1e6 / instr_per_cu, ms * 1e6 / instr_per_cu * 2.4);
    }
  }
}

int main() {
  double* out;
  long long* cyc;
  const int grid = 256 * 4;  // 4 blocks x 4 waves per CU = 16 waves/CU
  hipMalloc(&out, sizeof(double) * grid * 256);
  hipMalloc(&cyc, sizeof(long long));
  run<0, 0>("read_b64  64 lanes distinct", out, cyc, grid);
  run<1, 0>("read_b64  64 lanes broadcast", out, cyc, grid);
  run<2, 0>("read_b64  16 lanes", out, cyc, grid);
  run<3, 0>("read_b64  1 lane", out, cyc, grid);
  run<0, 1>("read2_b64 64 lanes distinct", out, cyc, grid);
  run<1, 1>("read2_b64 64 lanes broadcast", out, cyc, grid);
  run<2, 1>("read2_b64 16 lanes", out, cyc, grid);
  run<0, 2>("write_b64 64 lanes distinct", out, cyc, grid);
  run<2, 2>("write_b64 16 lanes", out, cyc, grid);
  run<3, 2>("write_b64 1 lane", out, cyc, grid);
  return 0;
}
