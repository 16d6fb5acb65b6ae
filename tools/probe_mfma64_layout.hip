// Lane layouts of the FP64 MFMA forms on gfx950, by unit vectors:
// block e of the grid sets B = (lane == e) (A = lane + 1) and, in the second
// half, A = (lane == e) (B = lane + 1).  D[l] then names the A (resp. B) lane
// that meets B (resp. A) lane e in output lane l.  Host prints the maps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void probe(double* out) {
  const int l = threadIdx.x, e = blockIdx.x & 63, half = blockIdx.x >> 6;
  double a = half ? (l == e ? 1.0 : 0.0) : (double)(l + 1);
  double b = half ? (double)(l + 1) : (l == e ? 1.0 : 0.0);
  double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  out[blockIdx.x * 320 + l] = d;
  d4 z = {0, 0, 0, 0};
  d4 r = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, z, 0, 0, 0);
  for (int i = 0; i < 4; ++i) out[blockIdx.x * 320 + 64 + l * 4 + i] = r[i];
}

int main() {
  double* d;
  (void)hipMalloc(&d, sizeof(double) * 128 * 320);
  hipLaunchKernelGGL(probe, dim3(128), dim3(64), 0, 0, d);
  std::vector<double> h(128 * 320);
  (void)hipMemcpy(h.data(), d, sizeof(double) * h.size(), hipMemcpyDeviceToHost);
  // 4x4x4_4b: for each output lane l, list (A lane, B lane) pairs
  for (int form = 0; form < 2; ++form) {
    const int nout = form ? 256 : 64;
    printf(form ? "M16\n" : "M4\n");
    for (int o = 0; o < nout; ++o) {
      printf("D%d:", o);
      for (int e = 0; e < 64; ++e) {  // B lane e
        double v = h[e * 320 + (form ? 64 + o : o)];
        if (v != 0.0) printf(" (A%d,B%d)", (int)v - 1, e);
      }
      printf("\n");
    }
  }
  return 0;
}
