// Microbenchmark: host round trip of one tiny launch whose completion the
// host polls in page-locked memory (the B = 1 control step's pattern), with a
// small kernel argument against a ControlStepParams-sized one (1 592 B), and
// with the large block passed by pointer (device copy refreshed by one
// hipMemcpyAsync per launch, or read in place from page-locked memory).
// build: hipcc --offload-arch=gfx950 -O3 tools/microbench_kernarg.hip -o tools/bin/mb_kernarg
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                   \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

struct Big {
  double v[199];  // 1 592 B
  unsigned* done;
  unsigned seq;
};

__global__ void k_small(unsigned* done, unsigned seq, double a) {
  if (threadIdx.x == 0 && a >= 0.0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_big(Big b) {
  double s = 0.0;
  for (int i = threadIdx.x; i < 199; i += 64) s += b.v[i];
  if (threadIdx.x == 0 && s >= -1.0)
    __hip_atomic_store(b.done, b.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_ptr(const Big* __restrict__ b) {
  double s = 0.0;
  for (int i = threadIdx.x; i < 199; i += 64) s += b->v[i];
  if (threadIdx.x == 0 && s >= -1.0)
    __hip_atomic_store(b->done, b->seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned* done = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&done), 64, hipHostMallocCoherent));
  *done = 0;
  Big* hb = nullptr;  // page-locked copy of the block
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&hb), sizeof(Big), hipHostMallocCoherent));
  Big* db = nullptr;
  CHECK(hipMalloc(&db, sizeof(Big)));
  Big big{};
  for (int i = 0; i < 199; ++i) big.v[i] = i * 1e-3;
  big.done = done;
  unsigned seq = 0;
  auto wait = [&](unsigned want) {
    while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != want) {
    }
  };
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 200; ++i) {
      launch(++seq);
      wait(seq);
    }
    const int n = 2000;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {
      launch(++seq);
      wait(seq);
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
    std::printf("%-44s %7.2f us per launch + poll\n", name, us);
  };
  for (int r = 0; r < 2; ++r) {
    run("small argument (20 B)", [&](unsigned s) { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, st, done, s, 1.0); });
    run("ControlStepParams-sized argument (1 608 B)", [&](unsigned s) {
      big.seq = s;
      hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, st, big);
    });
    run("pointer to a page-locked block", [&](unsigned s) {
      big.seq = s;
      std::memcpy(hb, &big, sizeof(Big));
      hipLaunchKernelGGL(k_ptr, dim3(1), dim3(64), 0, st, static_cast<const Big*>(hb));
    });
    run("pointer to a device block (memcpy per launch)", [&](unsigned s) {
      big.seq = s;
      std::memcpy(hb, &big, sizeof(Big));
      hipMemcpyAsync(db, hb, sizeof(Big), hipMemcpyHostToDevice, st);
      hipLaunchKernelGGL(k_ptr, dim3(1), dim3(64), 0, st, static_cast<const Big*>(db));
    });
  }
  CHECK(hipStreamSynchronize(st));
  CHECK(hipHostFree(done));
  CHECK(hipHostFree(hb));
  CHECK(hipFree(db));
  CHECK(hipStreamDestroy(st));
  return 0;
}
