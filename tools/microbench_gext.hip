// Microbenchmark: read bandwidth of the coupled iterate's G_ext access
// pattern (config 4 at S_total = 64: 262 144 QPs x 1 008 elements, 2.11 GB)
// against a QP-blocked layout and a plain linear stream, at 2 waves/SIMD (the
// coupled kernel's occupancy) and unconstrained.  Each lane sums its QP's
// elements (the kernel's f_k loop without the solve); 16 loads per trip,
// unrolled 4 trips, as the kernel keeps 64 loads in flight.
//   A: element-major [e][q] (the kernel's layout: a wave reads 512 B rows
//      2 MiB apart)
//   B: QP-blocked [q / 64][e][q % 64] (a wave reads one contiguous 516 KB block)
//   C: linear stream of the same bytes, 16 B per lane per load
// build: hipcc --offload-arch=gfx950 -O3 tools/microbench_gext.hip -o /tmp/mb_gext
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));      \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

constexpr int E = 1008;  // nV * (S_total - 1) * nV at S_total = 64

template <int MODE>
__device__ __forceinline__ double body(const double* __restrict__ g, int q, int nqp) {
  double acc = 0.0;
  if (MODE == 0) {
    const double* p = g + q;
#pragma unroll 4
    for (int e = 0; e < E; e += 16) {
      double v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = p[(size_t)(e + k) * nqp];
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += v[k];
    }
  } else {
    const double* p = g + (size_t)(q >> 6) * E * 64 + (q & 63);
#pragma unroll 4
    for (int e = 0; e < E; e += 16) {
      double v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = p[(size_t)(e + k) * 64];
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += v[k];
    }
  }
  return acc;
}

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void read_w2(const double* g, double* out, int nqp) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q < nqp) out[q] = body<MODE>(g, q, nqp);
}

template <int MODE>
__global__ __launch_bounds__(256) void read_free(const double* g, double* out, int nqp) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q < nqp) out[q] = body<MODE>(g, q, nqp);
}

__global__ __launch_bounds__(256) void stream(const double2* g, double* out, size_t n2) {
  double acc = 0.0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
    const double2 v = g[i];
    acc += v.x + v.y;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const int nqp = 262144;
  const size_t n = (size_t)E * nqp;
  double *g, *out;
  CHECK(hipMalloc(&g, n * sizeof(double)));
  const int sgrid = 256 * 8;  // stream kernel: one output per thread
  CHECK(hipMalloc(&out, (size_t)(nqp > sgrid * 256 ? nqp : sgrid * 256) * sizeof(double)));
  CHECK(hipMemset(g, 0, n * sizeof(double)));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int grid = nqp / 256;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipDeviceSynchronize());
    const int reps = 20;
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double t = ms / reps * 1e-3;
    std::printf("%-28s %8.1f us  %6.2f TB/s  (%.3f of 8 TB/s)\n", name, t * 1e6, n * 8.0 / t / 1e12,
                n * 8.0 / t / 8e12);
  };
  for (int round = 0; round < 2; ++round) {
    run("A element-major, 2 w/SIMD", [&] { read_w2<0><<<grid, 256>>>(g, out, nqp); });
    run("B QP-blocked,    2 w/SIMD", [&] { read_w2<1><<<grid, 256>>>(g, out, nqp); });
    run("A element-major, free", [&] { read_free<0><<<grid, 256>>>(g, out, nqp); });
    run("B QP-blocked,    free", [&] { read_free<1><<<grid, 256>>>(g, out, nqp); });
    run("C linear stream", [&] { stream<<<sgrid, 256>>>(reinterpret_cast<const double2*>(g), out, n / 2); });
  }
  CHECK(hipFree(g));
  CHECK(hipFree(out));
  return 0;
}
