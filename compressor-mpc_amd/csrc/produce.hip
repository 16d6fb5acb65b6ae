// Device record producer kernel: four units per
// wave, four waves per workgroup (produce_body.h holds the body).
#include "produce_body.h"

namespace {
using namespace cmpc_prod;

template <int PLANT>
__global__ __launch_bounds__(64 * kWaves) void cmpc_produce_kernel(ProduceParams P) {
  __shared__ double lds[kWaves * kSpw * kScnLds];
  extern __shared__ int src[];  // S x rec_len, then naug (dynamic, cmpc_launch_produce)
  int* dmap = src + P.S * P.rec_len;  // observer tail entry -> its position in the dx row
  produce_table<PLANT>(P, src, dmap, threadIdx.x, 64 * kWaves);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane / kLanes;
  // unit: scenario b (S records), or in per-QP mode QP slot q (its record)
  const int unit = (blockIdx.x * kWaves + wave) * kSpw + g;
  produce_row<PLANT>(P, lds + (wave * kSpw + g) * kScnLds, src, dmap, unit, lane);
}

}  // namespace

int cmpc_launch_produce(const ProduceParams& P, int plant, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int units = P.per_qp ? P.B * P.S : P.B;
  const int grid = (units + kWaves * kSpw - 1) / (kWaves * kSpw);
  if (P.S < 1 || P.S > CMPC_MAX_S_PRODUCE || P.rec_len > 2 * 64 * CMPC_REC_CHUNKS) return -1;
  if (P.obs_M) {
    // the fused a-posteriori update assumes four outputs, four disturbance
    // states (C = [C_plant | I]) and the first four dx entries the
    // disturbances (ring blocks start after them): refuse anything else
    // rather than produce wrong records
    const int ns = plant == CMPC_PLANT_PARALLEL ? 11 : 10;
    if (!P.per_qp || P.n_outputs != 4 || P.nobs - ns != 4 || P.naug < 4) return -1;
    for (int k = 0; k < P.nring; ++k)
      if (P.rb[k] < 4) return -1;
  }
  const size_t table = sizeof(int) * ((size_t)P.S * P.rec_len + (size_t)P.naug);
  if (plant == CMPC_PLANT_PARALLEL)
    cmpc_launch(cmpc_produce_kernel<CMPC_PLANT_PARALLEL>, dim3(grid), dim3(64 * kWaves), table, s, P);
  else if (plant == CMPC_PLANT_SERIAL)
    cmpc_launch(cmpc_produce_kernel<CMPC_PLANT_SERIAL>, dim3(grid), dim3(64 * kWaves), table, s, P);
  else
    return -1;
  return 0;
}
