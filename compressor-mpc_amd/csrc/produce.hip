// Device record producer kernel: four units per
// wave, four waves per workgroup (produce_body.h holds the body).
#include "produce_body.h"

namespace {
using namespace cmpc_prod;

#ifndef CMPC_PRODUCE_LOOP
#define CMPC_PRODUCE_LOOP 1  // resident workgroups loop over the units (0: one group per wave)
#endif

// Each wave produces groups of kSpw units, striding over the batch with the
// grid's waves: its record stores drain while it computes the next group.
// (One group per wave, the phases of the resident waves stayed in step: the
// compute (53 us at 65 536 scenarios) and the record stores (51 us, near the
// write bandwidth) added up, profiles/r5u_produce_loop_ab/.)
#ifndef CMPC_PRODUCE_WPE
#define CMPC_PRODUCE_WPE 0  // waves per SIMD the registers are allocated for (0: the compiler's choice, 2)
#endif
#if CMPC_PRODUCE_WPE
#define CMPC_PRODUCE_ATTR __attribute__((amdgpu_waves_per_eu(CMPC_PRODUCE_WPE, CMPC_PRODUCE_WPE)))
#else
#define CMPC_PRODUCE_ATTR
#endif
template <int PLANT>
__global__ __launch_bounds__(64 * kWaves) CMPC_PRODUCE_ATTR void cmpc_produce_kernel(ProduceParams P) {
  __shared__ double lds[kWaves * kSpw * kScnLds];
  extern __shared__ int src[];  // S x rec_len, then naug (dynamic, cmpc_launch_produce)
  int* dmap = src + P.S * P.rec_len;  // observer tail entry -> its position in the dx row
  produce_table<PLANT>(P, src, dmap, threadIdx.x, 64 * kWaves);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane / kLanes;
  const int units = P.per_qp ? P.B * P.S : P.B;
  double* const w = lds + (wave * kSpw + g) * kScnLds;
  // unit: scenario b (S records), or in per-QP mode QP slot q (its record);
  // the loop bound is the wave's (every lane runs produce_row's wave syncs)
  const int stride = gridDim.x * kWaves;
  int gw = blockIdx.x * kWaves + wave;
  ProduceInputs in = produce_inputs<PLANT>(P, gw * kSpw + g, lane);
  for (; gw * kSpw < units; gw += stride) {
    ProduceInputs next;
    produce_row<PLANT>(P, w, src, dmap, gw * kSpw + g, lane, &in, &next, (gw + stride) * kSpw + g);
    in = next;
    WAVE_SYNC();  // this group's LDS reads before the next group's stores
  }
}

}  // namespace

int cmpc_launch_produce(const ProduceParams& P, int plant, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int units = P.per_qp ? P.B * P.S : P.B;
  int grid = (units + kWaves * kSpw - 1) / (kWaves * kSpw);
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
  if (CMPC_PRODUCE_LOOP) {
    // the resident workgroups only (occupancy of this kernel at this table
    // size, once per device, plant and table size)
    struct Occ {
      int dev, plant;
      size_t table;
      int wgs;
    };
    static thread_local Occ occ[8];
    static thread_local int nocc = 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    int wgs = 0;
    for (int i = 0; i < nocc && i < 8; ++i)
      if (occ[i].dev == dev && occ[i].plant == plant && occ[i].table == table) wgs = occ[i].wgs;
    if (!wgs) {
      int per_cu = 0, cus = 0;
      const void* k = plant == CMPC_PLANT_PARALLEL
                          ? reinterpret_cast<const void*>(cmpc_produce_kernel<CMPC_PLANT_PARALLEL>)
                          : reinterpret_cast<const void*>(cmpc_produce_kernel<CMPC_PLANT_SERIAL>);
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 64 * kWaves, table) != hipSuccess) per_cu = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
      wgs = std::max(1, per_cu) * std::max(1, cus);
      occ[nocc % 8] = Occ{dev, plant, table, wgs};
      ++nocc;
    }
    grid = std::max(1, std::min(grid, wgs));
  }
  if (plant == CMPC_PLANT_PARALLEL)
    cmpc_launch(cmpc_produce_kernel<CMPC_PLANT_PARALLEL>, dim3(grid), dim3(64 * kWaves), table, s, P);
  else if (plant == CMPC_PLANT_SERIAL)
    cmpc_launch(cmpc_produce_kernel<CMPC_PLANT_SERIAL>, dim3(grid), dim3(64 * kWaves), table, s, P);
  else
    return -1;
  return 0;
}
