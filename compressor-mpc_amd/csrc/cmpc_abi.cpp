// Host implementation of the C ABI declared in include/cmpc.h.
//
// The context owns every batched device buffer (HBM-resident between steps):
//   lin    B*S lin records (inputs of the build kernel)
//   qp     B*S condensed QPs [H | f | G]      (build -> iterate hand-off)
//   cfg    S per-sub-controller blocks          (weights, reference, bounds)
//   state  u_old, du_old, ws                   (persist across steps, as the
//                                               reference's member state)
//   out    du, status, nwsr, trace
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <chrono>
#include <vector>

#include "cmpc_internal.h"

namespace {

thread_local std::string g_err;

int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess)                                                          \
      return fail(std::string(#expr) + ": " + hipGetErrorString(e_));             \
  } while (0)

int layout_of(const cmpc_dims* d, cmpc_layout* L) {
  if (!d || !L) return fail("null argument");
  if (d->ns < 1 || d->ns > CMPC_MAX_NS || d->nu_tot < 1 || d->nu_tot > CMPC_MAX_INPUTS ||
      d->nu < 1 || d->nu > d->nu_tot || d->ny < 1 || d->p < 1 || d->m < 1 || d->m > d->p ||
      d->m * d->nu > CMPC_MAX_NV || d->ndist < 0 || d->S < 1 || d->B < 1)
    return fail("invalid dimensions");
  std::memset(L, 0, sizeof *L);
  for (int i = 0; i < d->nu_tot; ++i) {
    if (d->delay[i] < 0) return fail("negative delay");
    if (d->delay[i]) L->nd++;
    L->n_delay_states += d->delay[i];
  }
  L->naug = d->ndist + L->n_delay_states;
  L->nobs = d->ns + d->ndist;
  L->ntot = L->nobs + L->n_delay_states;
  L->nV = d->m * d->nu;
  L->nuo = d->nu_tot - d->nu;
  L->nVo = d->m * L->nuo;
  L->off_A = 0;
  L->off_B = d->ns * d->ns;
  L->off_C = L->off_B + d->ns * d->nu_tot;
  L->off_f = L->off_C + d->ny * L->nobs;
  L->off_x = L->off_f + d->ns;
  L->off_y = L->off_x + L->naug;
  L->rec_len = ((L->off_y + d->ny) + 7) / 8 * 8;
  return 0;
}

}  // namespace

thread_local LaunchEvents cmpc_launch_events;

namespace {

// Page-locked host buffer for the host-array entry points.  A hipMemcpy from or
// to pageable memory costs ~17 us per call here: the runtime stages it through
// its own bounce buffer (rocprofv3 --hip-trace of the B = 1 harness,
// DESIGN.md §3.6).  From pinned memory it is one DMA.  `busy` is recorded after
// the copies that read the buffer, and the next writer waits on it.
struct PinnedIO {
  char* buf = nullptr;
  char* dev = nullptr;  // the device's address of buf (kernels read it in place)
  size_t cap = 0;
  hipEvent_t busy = nullptr;
  bool pending = false;
};

int pinned_acquire(PinnedIO& p, size_t bytes) {
  if (p.pending) {
    HIP_TRY(hipEventSynchronize(p.busy));
    p.pending = false;
  }
  if (bytes > p.cap) {
    if (p.buf) HIP_TRY(hipHostFree(p.buf));
    p.buf = nullptr;
    p.cap = 0;
    const size_t cap = std::max<size_t>(bytes, 4096);
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&p.buf), cap, hipHostMallocCoherent));
    p.cap = cap;
    void* dv = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dv, p.buf, 0));
    p.dev = reinterpret_cast<char*>(dv);
  }
  return 0;
}

int pinned_release(PinnedIO& p, hipStream_t s) {
  if (!p.busy) HIP_TRY(hipEventCreateWithFlags(&p.busy, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(p.busy, s));
  p.pending = true;
  return 0;
}

void pinned_free(PinnedIO& p) {
  if (p.pending) (void)hipEventSynchronize(p.busy);
  if (p.buf) (void)hipHostFree(p.buf);
  if (p.busy) (void)hipEventDestroy(p.busy);
  p = PinnedIO{};
}

// host -> device: the k arrays (nullptr skipped) are packed into `pin` and
// copied by one DMA to `dev_base`; dev[i] receives each array's device address.
// dev_base == nullptr: no copy, the kernels read the page-locked buffer in
// place (dev[i] = its device address) and the caller calls pinned_release
// after the launch that reads it.
constexpr size_t kPad = 2;  // keep every array 16-byte aligned
int pinned_upload(PinnedIO& pin, hipStream_t s, double* dev_base, const double* const* host,
                  const size_t* n, int k, const double** dev) {
  size_t tot = 0;
  for (int i = 0; i < k; ++i) tot += host[i] ? (n[i] + kPad - 1) / kPad * kPad : 0;
  if (pinned_acquire(pin, sizeof(double) * std::max<size_t>(tot, 1))) return -1;
  double* h = reinterpret_cast<double*>(pin.buf);
  size_t off = 0;
  for (int i = 0; i < k; ++i) {
    if (dev) dev[i] = nullptr;
    if (!host[i]) continue;
    std::memcpy(h + off, host[i], sizeof(double) * n[i]);
    if (dev) dev[i] = (dev_base ? dev_base : reinterpret_cast<double*>(pin.dev)) + off;
    off += (n[i] + kPad - 1) / kPad * kPad;
  }
  if (!dev_base) return 0;
  if (off) HIP_TRY(hipMemcpyAsync(dev_base, h, sizeof(double) * off, hipMemcpyHostToDevice, s));
  return pinned_release(pin, s);
}

}  // namespace

struct cmpc_ctx {
  cmpc_dims d{};
  cmpc_layout L{};
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int nqp = 0, qp_len = 0;
  CfgOffsets co{};
  // host mirror of the configuration
  std::vector<double> ywt, uwt, yref, lower, upper, rlower, rupper;  // per s
  std::vector<double> h_cfg;
  std::vector<int> have_w, have_c, have_r;
  bool cfg_dirty = true;
  // device buffers
  const double* lin_bound = nullptr;  // external records (cmpc_bind_lin)
  double *lin = nullptr, *qp = nullptr, *cfg = nullptr, *u_old = nullptr, *du_old = nullptr,
         *du = nullptr;
  uint32_t* ws = nullptr;
  // the context's own state buffers; u_old/du_old/ws above point at them
  // unless cmpc_bind_state bound external ones
  double *own_u_old = nullptr, *own_du_old = nullptr;
  uint32_t* own_ws = nullptr;
  int32_t *status = nullptr, *nwsr = nullptr, *ntrace = nullptr;
  char* out_block = nullptr;  // du | status | nwsr in one allocation: one D2H for cmpc_download
  bool out_host = false;      // out_block is page-locked host memory the kernels write in place
  uint32_t* done_host = nullptr;  // out_host: the control step's completion word (after the block)
  uint32_t* done_dev = nullptr;   // its device address
  uint32_t done_seq = 0;
  size_t out_st = 0, out_nw = 0, out_len = 0;  // byte offsets of status, nwsr; block length
  uint8_t* trace = nullptr;
  size_t trace_cap = 0;
  int trace_K = 0;
  // observer (cmpc_set_observer / cmpc_observer_init)
  int obs_nout = 0, obs_len = 0, obs_plant = -1;
  double obs_pin = 0, obs_pout = 0, obs_Ts = 0;
  std::vector<double> obsM;  // S x nobs x n_out
  std::vector<int> have_M;
  bool obsM_dirty = true;
  double *d_obsM = nullptr, *obs = nullptr;
  double* stage = nullptr;  // host-pointer observer calls: device staging
  size_t stage_cap = 0;
  PinnedIO pin_in, pin_out;  // host-array calls: page-locked staging
  int64_t obs_steps = 0;  // a-priori steps since cmpc_observer_init: the delay blocks' ring phase
  int obs_io[CMPC_MAX_S_PRODUCE][CMPC_MAX_INPUTS] = {};
  int obs_oi[CMPC_MAX_S_PRODUCE][4] = {};
  // build kernel selection (cmpc_set_build_variant)
  int build_variant = CMPC_BUILD_AUTO;
  int last_build = 0;  // kernel launched by the last cmpc_build
  int solve_variant = CMPC_SOLVE_AUTO;  // cmpc_set_solve_variant
  int last_solve = 0;                   // kernel launched by the last solve
  int step_variant = CMPC_STEP_AUTO;    // cmpc_set_step_variant
  int cus = 0;                          // compute units of the device (0: not yet queried)
  std::vector<std::pair<const void*, size_t>> bound_ok;  // (device pointer, bytes) cmpc_bind_* validated before
  bool lds_layout_ok = false;           // lds_layout holds build_lds_layout(d, L)
  BuildParams lds_layout{};             // (a function of the dimensions only)
  int last_step_fused = 0;
  // timing
  int timing = 0;  // bit k: kernel k (CMPC_KERNEL_*) is timed
  int timing_stride = 1;                        // time every stride-th launch
  int64_t timing_seq[CMPC_KERNEL_COUNT] = {};  // launches since cmpc_enable_timing
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending[CMPC_KERNEL_COUNT];
  std::vector<hipEvent_t> event_pool;  // reused so timing stays cheap in a timed loop
  double tot_ms[CMPC_KERNEL_COUNT] = {};
  int64_t launches[CMPC_KERNEL_COUNT] = {};
};

namespace {

int rebuild_cfg(cmpc_ctx* c) {
  const cmpc_dims& d = c->d;
  const int S = d.S, ny = d.ny, nu = d.nu, p = d.p;
  for (int s = 0; s < S; ++s)
    if (!c->have_w[s] || !c->have_c[s] || !c->have_r[s])
      return fail("sub-controller " + std::to_string(s) +
                  ": weights, constraints and reference must all be set before the step");
  c->h_cfg.assign((size_t)S * c->co.len, 0.0);
  for (int s = 0; s < S; ++s) {
    double* b = c->h_cfg.data() + (size_t)s * c->co.len;
    // ywt = L_W L_W' (Cholesky; zero pivots allowed for PSD weights)
    const double* W = c->ywt.data() + (size_t)s * ny * ny;
    std::vector<double> Lw(ny * ny, 0.0);
    double scale = 0;
    for (int i = 0; i < ny * ny; ++i) scale = std::max(scale, std::fabs(W[i]));
    for (int i = 0; i < ny; ++i)
      for (int j = 0; j < ny; ++j)
        if (std::fabs(W[i * ny + j] - W[j * ny + i]) > 1e-12 * (1 + scale))
          return fail("ywt must be symmetric");
    for (int j = 0; j < ny; ++j) {
      double dd = W[j * ny + j];
      for (int k = 0; k < j; ++k) dd -= Lw[j * ny + k] * Lw[j * ny + k];
      if (dd < -1e-12 * (1 + scale)) return fail("ywt must be positive semi-definite");
      if (dd <= 1e-14 * (1 + scale)) continue;  // zero column
      const double ljj = std::sqrt(dd);
      Lw[j * ny + j] = ljj;
      for (int i = j + 1; i < ny; ++i) {
        double v = W[i * ny + j];
        for (int k = 0; k < j; ++k) v -= Lw[i * ny + k] * Lw[j * ny + k];
        Lw[i * ny + j] = v / ljj;
      }
    }
    for (int o = 0; o < ny; ++o)  // lwt = L_W' (upper triangular)
      for (int o2 = 0; o2 < ny; ++o2) b[c->co.lwt + o * ny + o2] = Lw[o2 * ny + o];
    const double* yr = c->yref.data() + (size_t)s * p * ny;
    for (int r = 0; r < p; ++r)
      for (int o = 0; o < ny; ++o) {
        double v = 0;
        for (int o2 = o; o2 < ny; ++o2) v += Lw[o2 * ny + o] * yr[r * ny + o2];
        b[c->co.yhat + r * ny + o] = v;
      }
    std::memcpy(b + c->co.uwt, c->uwt.data() + (size_t)s * nu * nu, sizeof(double) * nu * nu);
    std::memcpy(b + c->co.lower, c->lower.data() + (size_t)s * nu, sizeof(double) * nu);
    std::memcpy(b + c->co.upper, c->upper.data() + (size_t)s * nu, sizeof(double) * nu);
    std::memcpy(b + c->co.rlower, c->rlower.data() + (size_t)s * nu, sizeof(double) * nu);
    std::memcpy(b + c->co.rupper, c->rupper.data() + (size_t)s * nu, sizeof(double) * nu);
  }
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpyAsync(c->cfg, c->h_cfg.data(), sizeof(double) * c->h_cfg.size(),
                         hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->cfg_dirty = false;
  return 0;
}

int ensure_cfg(cmpc_ctx* c) { return c->cfg_dirty ? rebuild_cfg(c) : 0; }

hipError_t pooled_event(cmpc_ctx* c, hipEvent_t* e) {
  if (!c->event_pool.empty()) {
    *e = c->event_pool.back();
    c->event_pool.pop_back();
    return hipSuccess;
  }
  return hipEventCreate(e);
}

// A timed launch: the launcher (cmpc_launch, cmpc_internal.h) passes both
// events to hipExtLaunchKernelGGL, which writes the kernel's start and end
// into them; no marker packets go into the stream.  The guard hands the events
// to the context's pending list on end() and, on any early return (a failed
// launch), clears cmpc_launch_events and gives them back to the pool.
class TimedLaunch {
 public:
  TimedLaunch(cmpc_ctx* c, int k) : c_(c), k_(k) {}
  TimedLaunch(const TimedLaunch&) = delete;
  TimedLaunch& operator=(const TimedLaunch&) = delete;
  int begin() {
    cmpc_launch_events = LaunchEvents{};
    if (!((c_->timing >> k_) & 1)) return 0;
    if (c_->timing_seq[k_]++ % c_->timing_stride) return 0;  // a sampled launch only
    HIP_TRY(pooled_event(c_, &e0_));
    HIP_TRY(pooled_event(c_, &e1_));
    cmpc_launch_events.start = e0_;
    cmpc_launch_events.stop = e1_;
    return 0;
  }
  int end() {
    cmpc_launch_events = LaunchEvents{};
    if (e0_ && e1_) {
      c_->pending[k_].push_back({e0_, e1_});
      c_->launches[k_]++;
    }
    e0_ = e1_ = nullptr;
    return 0;
  }
  ~TimedLaunch() {
    if (!e0_ && !e1_) return;
    cmpc_launch_events = LaunchEvents{};
    if (e0_) c_->event_pool.push_back(e0_);
    if (e1_) c_->event_pool.push_back(e1_);
  }

 private:
  cmpc_ctx* c_;
  int k_;
  hipEvent_t e0_ = nullptr, e1_ = nullptr;
};

int resolve_timing(cmpc_ctx* c) {
  for (int k = 0; k < CMPC_KERNEL_COUNT; ++k) {
    for (auto& pr : c->pending[k]) {
      HIP_TRY(hipEventSynchronize(pr.second));
      float ms = 0;
      HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
      c->tot_ms[k] += ms;
      c->event_pool.push_back(pr.first);
      c->event_pool.push_back(pr.second);
    }
    c->pending[k].clear();
  }
  return 0;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(std::string(what) + ": " + hipGetErrorString(e));
  return 0;
}

int solve_params(cmpc_ctx* c, SolveParams* P) {
  std::memset(P, 0, sizeof *P);
  P->qp = c->qp;
  P->cfg = c->cfg;
  P->u_old = c->u_old;
  P->du_old = c->du_old;
  P->ws = c->ws;
  P->du = c->du;
  P->status = c->status;
  P->nwsr = c->nwsr;
  P->nqp = c->nqp;
  P->S = c->d.S;
  P->nu_tot = c->d.nu_tot;
  P->qp_len = c->qp_len;
  P->co = c->co;
  return 0;
}

}  // namespace

extern "C" {

int cmpc_layout_of(const cmpc_dims* d, cmpc_layout* L) { return layout_of(d, L); }

const char* cmpc_last_error(void) { return g_err.c_str(); }

int cmpc_create(cmpc_ctx** out, const cmpc_dims* dims, int device) {
  if (!out || !dims) return fail("null argument");
  *out = nullptr;
  cmpc_layout L;
  if (layout_of(dims, &L)) return -1;
  const cmpc_dims& d = *dims;
  if (64 % d.S != 0) return fail("S must divide the wavefront size (64)");
  // S sub-controllers share the inputs (nu_tot = S nu), or S = 1 with
  // nu < nu_tot: one stand-alone sub-controller whose other controllers'
  // plans come with every cmpc_get_input (DistributedController::GetInput)
  if (L.nuo != (d.S - 1) * d.nu && d.S != 1)
    return fail("nu_tot must equal S * nu (each sub-controller owns nu inputs), or S = 1");
  if (L.nd > CMPC_ND_MAX) return fail("more than 4 delayed inputs");
  // A one-step delay with several delayed inputs: the reference's BComposite
  // (libs/aug_lin_sys.cc:189-197) places such an input at index
  // n_delayed_inputs + (sum of the earlier blocks' D - 1) - 1 of the
  // augmented state, which is another input's delay state (only a single
  // delayed input gets its own slot).  That mapping is not reproduced.
  for (int i = 0; i < d.nu_tot; ++i)
    if (d.delay[i] == 1 && L.nd > 1)
      return fail("a delay of one step with several delayed inputs: the reference's BComposite "
                  "maps it onto another input's delay state (aug_lin_sys.cc:189-197); not supported");
  if (d.ns + d.nu_tot > 15) return fail("ns + nu_tot must be <= 15 (16-lane DPP rows)");
  if (d.m * d.nu_tot + 1 > 16) return fail("m * nu_tot + 1 must be <= 16 (gather lanes of a DPP row)");
  if (d.ny > 4) return fail("ny > 4 is not instantiated in the build kernel (one DPP row per output)");
  if (d.ns + d.ny + L.nd > 16)
    return fail("ns + ny + (delayed inputs) must be <= 16 (free-response DPP row)");
  const long long nqp = (long long)d.B * d.S;
  if (nqp > (1LL << 30)) return fail("batch too large");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail("no such HIP device");
  cmpc_ctx* c = new cmpc_ctx();
  c->d = d;
  c->L = L;
  c->device = device;
  c->nqp = (int)nqp;
  c->qp_len = (L.nV * L.nV + L.nV + L.nV * L.nVo + 1) / 2 * 2;
  int off = 0;
  c->co.lwt = off; off += d.ny * d.ny;
  c->co.yhat = off; off += d.p * d.ny;
  c->co.uwt = off; off += d.nu * d.nu;
  c->co.lower = off; off += d.nu;
  c->co.upper = off; off += d.nu;
  c->co.rlower = off; off += d.nu;
  c->co.rupper = off; off += d.nu;
  c->co.len = (off + 1) / 2 * 2;
  const int S = d.S;
  c->ywt.assign((size_t)S * d.ny * d.ny, 0);
  c->uwt.assign((size_t)S * d.nu * d.nu, 0);
  c->yref.assign((size_t)S * d.p * d.ny, 0);
  c->lower.assign((size_t)S * d.nu, 0);
  c->upper.assign((size_t)S * d.nu, 0);
  c->rlower.assign((size_t)S * d.nu, 0);
  c->rupper.assign((size_t)S * d.nu, 0);
  c->have_w.assign(S, 0);
  c->have_c.assign(S, 0);
  c->have_r.assign(S, 0);
  auto cleanup = [&](int rc) {
    cmpc_destroy(c);
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) return cleanup(fail("hipSetDevice failed"));
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail("hipStreamCreate failed"));
  c->own_stream = true;
  const size_t n = (size_t)c->nqp;
  if (hipMalloc(&c->lin, sizeof(double) * n * L.rec_len) != hipSuccess ||
      hipMalloc(&c->qp, sizeof(double) * n * c->qp_len) != hipSuccess ||
      hipMalloc(&c->cfg, sizeof(double) * (size_t)S * c->co.len) != hipSuccess ||
      hipMalloc(&c->u_old, sizeof(double) * n * d.nu_tot) != hipSuccess ||
      hipMalloc(&c->du_old, sizeof(double) * n * L.nV) != hipSuccess ||
      hipMalloc(&c->ws, sizeof(uint32_t) * n) != hipSuccess)
    return cleanup(fail("hipMalloc failed (batch too large for device memory?)"));
  c->own_u_old = c->u_old;
  c->own_du_old = c->du_old;
  c->own_ws = c->ws;
  {
    auto up16 = [](size_t v) { return (v + 15) / 16 * 16; };
    c->out_st = up16(sizeof(double) * n * L.nV);
    c->out_nw = c->out_st + up16(sizeof(int32_t) * n);
    c->out_len = c->out_nw + sizeof(int32_t) * n;
    // a few QPs (the reference's own B = 1 call pattern): the kernels write
    // du, status and nWSR straight into page-locked host memory, so
    // cmpc_download is a stream sync, no copy (a hipMemcpyAsync cost ~7 us of
    // host time and a copy kernel per step, profiles/r4e_b1_hip_api_stats.csv)
    char* dev_out = nullptr;
    if (n <= CMPC_HOST_OUT_MAX_QP) {
      void* dv = nullptr;
      const size_t done_off = up16(c->out_len);
      if (hipHostMalloc(reinterpret_cast<void**>(&c->out_block), done_off + 16, hipHostMallocCoherent) != hipSuccess ||
          hipHostGetDevicePointer(&dv, c->out_block, 0) != hipSuccess)
        return cleanup(fail("hipHostMalloc failed"));
      c->out_host = true;
      std::memset(c->out_block, 0, done_off + 16);
      dev_out = reinterpret_cast<char*>(dv);
      c->done_host = reinterpret_cast<uint32_t*>(c->out_block + done_off);
      c->done_dev = reinterpret_cast<uint32_t*>(dev_out + done_off);
    } else {
      if (hipMalloc(&c->out_block, c->out_len) != hipSuccess)
        return cleanup(fail("hipMalloc failed (batch too large for device memory?)"));
      dev_out = c->out_block;
    }
    c->du = reinterpret_cast<double*>(dev_out);
    c->status = reinterpret_cast<int32_t*>(dev_out + c->out_st);
    c->nwsr = reinterpret_cast<int32_t*>(dev_out + c->out_nw);
  }
  if (hipMemsetAsync(c->lin, 0, sizeof(double) * n * L.rec_len, c->stream) != hipSuccess ||
      hipMemsetAsync(c->qp, 0, sizeof(double) * n * c->qp_len, c->stream) != hipSuccess ||
      hipMemsetAsync(c->u_old, 0, sizeof(double) * n * d.nu_tot, c->stream) != hipSuccess ||
      hipMemsetAsync(c->du_old, 0, sizeof(double) * n * L.nV, c->stream) != hipSuccess ||
      (!c->out_host && hipMemsetAsync(c->out_block, 0, c->out_len, c->stream) != hipSuccess) ||
      hipMemsetAsync(c->ws, 0, sizeof(uint32_t) * n, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return cleanup(fail("device initialisation failed"));
  *out = c;
  return 0;
}

int cmpc_destroy(cmpc_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (int k = 0; k < CMPC_KERNEL_COUNT; ++k)
    for (auto& pr : c->pending[k]) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
  for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
  pinned_free(c->pin_in);
  pinned_free(c->pin_out);
  // own state buffers (bound external ones belong to the caller); before they
  // are recorded (a failed create) the active pointers are the own ones
  if (c->out_host && c->out_block) (void)hipHostFree(c->out_block);
  void* bufs[] = {c->lin, c->qp, c->cfg,
                  c->own_u_old ? c->own_u_old : c->u_old,
                  c->own_du_old ? c->own_du_old : c->du_old,
                  c->out_host ? nullptr : c->out_block,
                  c->own_ws ? c->own_ws : c->ws,
                  c->trace, c->ntrace, c->obs, c->d_obsM,
                  c->stage};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int cmpc_set_stream(cmpc_ctx* c, void* stream) {
  if (!c) return fail("null context");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  c->stream = (hipStream_t)stream;
  c->own_stream = false;
  return 0;
}

int cmpc_get_layout(const cmpc_ctx* c, cmpc_layout* L) {
  if (!c || !L) return fail("null argument");
  *L = c->L;
  return 0;
}

int cmpc_set_weights(cmpc_ctx* c, int s, const double* uwt, const double* ywt) {
  if (!c || !uwt || !ywt) return fail("null argument");
  if (s < 0 || s >= c->d.S) return fail("sub-controller index out of range");
  const int ny = c->d.ny, nu = c->d.nu;
  std::memcpy(c->ywt.data() + (size_t)s * ny * ny, ywt, sizeof(double) * ny * ny);
  std::memcpy(c->uwt.data() + (size_t)s * nu * nu, uwt, sizeof(double) * nu * nu);
  c->have_w[s] = 1;
  c->cfg_dirty = true;
  return 0;
}

int cmpc_set_constraints(cmpc_ctx* c, int s, const double* lo, const double* up,
                         const double* rlo, const double* rup) {
  if (!c || !lo || !up || !rlo || !rup) return fail("null argument");
  if (s < 0 || s >= c->d.S) return fail("sub-controller index out of range");
  const int nu = c->d.nu;
  for (int i = 0; i < nu; ++i)
    if (!(lo[i] <= up[i]) || !(rlo[i] <= rup[i]))
      return fail("constraints must satisfy lower <= upper (NaN bounds are unset)");
  std::memcpy(c->lower.data() + (size_t)s * nu, lo, sizeof(double) * nu);
  std::memcpy(c->upper.data() + (size_t)s * nu, up, sizeof(double) * nu);
  std::memcpy(c->rlower.data() + (size_t)s * nu, rlo, sizeof(double) * nu);
  std::memcpy(c->rupper.data() + (size_t)s * nu, rup, sizeof(double) * nu);
  c->have_c[s] = 1;
  c->cfg_dirty = true;
  return 0;
}

int cmpc_set_reference(cmpc_ctx* c, int s, const double* y_ref) {
  if (!c || !y_ref) return fail("null argument");
  if (s < 0 || s >= c->d.S) return fail("sub-controller index out of range");
  const size_t n = (size_t)c->d.p * c->d.ny;
  std::memcpy(c->yref.data() + s * n, y_ref, sizeof(double) * n);
  c->have_r[s] = 1;
  c->cfg_dirty = true;
  return 0;
}

int cmpc_set_state(cmpc_ctx* c, const double* u_old, const double* du_old, const uint32_t* ws) {
  if (!c) return fail("null context");
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)c->nqp;
  if (u_old)
    HIP_TRY(hipMemcpyAsync(c->u_old, u_old, sizeof(double) * n * c->d.nu_tot,
                           hipMemcpyHostToDevice, c->stream));
  if (du_old)
    HIP_TRY(hipMemcpyAsync(c->du_old, du_old, sizeof(double) * n * c->L.nV,
                           hipMemcpyHostToDevice, c->stream));
  if (ws) HIP_TRY(hipMemcpyAsync(c->ws, ws, sizeof(uint32_t) * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int cmpc_get_state(cmpc_ctx* c, double* u_old, double* du_old, uint32_t* ws) {
  if (!c) return fail("null context");
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)c->nqp;
  if (u_old)
    HIP_TRY(hipMemcpyAsync(u_old, c->u_old, sizeof(double) * n * c->d.nu_tot,
                           hipMemcpyDeviceToHost, c->stream));
  if (du_old)
    HIP_TRY(hipMemcpyAsync(du_old, c->du_old, sizeof(double) * n * c->L.nV,
                           hipMemcpyDeviceToHost, c->stream));
  if (ws) HIP_TRY(hipMemcpyAsync(ws, c->ws, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int cmpc_upload_lin(cmpc_ctx* c, const double* lin) {
  if (!c || !lin) return fail("null argument");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpyAsync(c->lin, lin, sizeof(double) * (size_t)c->nqp * c->L.rec_len,
                         hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int cmpc_download_lin(cmpc_ctx* c, double* lin) {
  if (!c || !lin) return fail("null argument");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpyAsync(lin, c->lin, sizeof(double) * (size_t)c->nqp * c->L.rec_len,
                         hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

void* cmpc_lin_device(cmpc_ctx* c) { return c ? (void*)c->lin : nullptr; }

// p is device memory of the context's device and [p, p + bytes) lies inside
// its allocation.  A rotation over a few bound buffers (the bench binds four
// per step) queries each (pointer, size) once: the runtime's lookups are
// several microseconds of host time per call, more than a small batch's
// kernels take.  A pointer is therefore validated the first time it is bound
// to this context (include/cmpc.h, cmpc_bind_lin): a caller that frees a
// bound buffer and binds another allocation at the same address must make
// it at least as large.
static bool device_ptr_ok(cmpc_ctx* c, const void* p, size_t bytes) {
  for (const auto& v : c->bound_ok)
    if (v.first == p && v.second >= bytes) return true;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeDevice || a.device != c->device)
    return false;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess && base &&
      (uintptr_t)p + bytes > (uintptr_t)base + size)
    return false;
  if (c->bound_ok.size() >= 64) c->bound_ok.erase(c->bound_ok.begin());
  c->bound_ok.emplace_back(p, bytes);
  return true;
}

int cmpc_bind_lin(cmpc_ctx* c, const double* lin_device) {
  if (!c) return fail("null context");
  if (lin_device) {
    if (!device_ptr_ok(c, lin_device, sizeof(double) * (size_t)c->nqp * c->L.rec_len))
      return fail("cmpc_bind_lin: not a device allocation of nqp * rec_len doubles on the context's device");
    // the build kernels read records with 16-byte loads (LDS-DMA / double2)
    if (reinterpret_cast<uintptr_t>(lin_device) % 16 != 0)
      return fail("cmpc_bind_lin: records must be 16-byte aligned");
  }
  c->lin_bound = lin_device;
  return 0;
}

int cmpc_bind_state(cmpc_ctx* c, double* u_old, double* du_old, uint32_t* ws) {
  if (!c) return fail("null context");
  const int nnull = !u_old + !du_old + !ws;
  if (nnull == 3) {
    c->u_old = c->own_u_old;
    c->du_old = c->own_du_old;
    c->ws = c->own_ws;
    return 0;
  }
  if (nnull != 0) return fail("cmpc_bind_state: bind all three state arrays or none");
  const size_t n = (size_t)c->nqp;
  if (!device_ptr_ok(c, u_old, sizeof(double) * n * c->d.nu_tot) ||
      !device_ptr_ok(c, du_old, sizeof(double) * n * c->L.nV) || !device_ptr_ok(c, ws, sizeof(uint32_t) * n))
    return fail("cmpc_bind_state: not device allocations of the state's size on the context's device");
  if (reinterpret_cast<uintptr_t>(u_old) % 8 || reinterpret_cast<uintptr_t>(du_old) % 8 ||
      reinterpret_cast<uintptr_t>(ws) % 4)
    return fail("cmpc_bind_state: misaligned state array");
  c->u_old = u_old;
  c->du_old = du_old;
  c->ws = ws;
  return 0;
}

static int fill_produce(cmpc_ctx* c, const char* who, int plant, double p_in, double p_out,
                        double Ts, const int32_t* input_order, const int32_t* out_idx,
                        ProduceParams* P, int* n_outputs) {
  const cmpc_dims& d = c->d;
  const cmpc_layout& L = c->L;
  int ns = 0, ni = 0, no = 0, nci = 0;
  if (cmpc_plant_dims(plant, &ns, &ni, &no, &nci)) return fail(std::string(who) + ": unknown plant");
  if (d.ns != ns || d.nu_tot != nci || d.ndist > no || d.ny > 4)
    return fail(std::string(who) + ": context dimensions do not match the plant");
  if (d.S > CMPC_MAX_S_PRODUCE) return fail(std::string(who) + ": too many sub-controllers");
  if (L.rec_len > 2 * 64 * CMPC_REC_CHUNKS)
    return fail(std::string(who) + ": lin record of " + std::to_string(L.rec_len) +
                " doubles exceeds the producer's " + std::to_string(2 * 64 * CMPC_REC_CHUNKS) +
                " (too many delay states)");
  std::memset(P, 0, sizeof *P);
  P->lin = c->lin;
  P->B = d.B;
  P->S = d.S;
  P->rec_len = L.rec_len;
  P->nu_tot = d.nu_tot;
  P->ny = d.ny;
  P->nobs = L.nobs;
  P->naug = L.naug;
  P->n_outputs = no;
  P->off_A = L.off_A; P->off_B = L.off_B; P->off_C = L.off_C;
  P->off_f = L.off_f; P->off_x = L.off_x; P->off_y = L.off_y;
  P->p_in = p_in;
  P->p_out = p_out;
  P->Ts = Ts;
  for (int s = 0; s < d.S; ++s) {
    for (int k = 0; k < d.nu_tot; ++k) {
      const int v = input_order[s * d.nu_tot + k];
      if (v < 0 || v >= nci) return fail(std::string(who) + ": bad input_order");
      P->input_order[s][k] = v;
    }
    for (int o = 0; o < d.ny; ++o) {
      const int v = out_idx[s * d.ny + o];
      if (v < 0 || v >= no) return fail(std::string(who) + ": bad out_idx");
      P->out_idx[s][o] = v;
    }
  }
  if (n_outputs) *n_outputs = no;
  return 0;
}

int cmpc_produce_lin(cmpc_ctx* c, int plant, double p_in, double p_out, double Ts,
                     const int32_t* input_order, const int32_t* out_idx, const double* x,
                     const double* u_full, const double* dx_aug, const double* y) {
  if (!c) return fail("null context");
  if (!input_order || !out_idx || !x || !u_full || !y) return fail("cmpc_produce_lin: null argument");
  ProduceParams P;
  if (fill_produce(c, "cmpc_produce_lin", plant, p_in, p_out, Ts, input_order, out_idx, &P, nullptr))
    return -1;
  P.x = x;
  P.u_full = u_full;
  P.dx_aug = dx_aug;
  P.y = y;
  HIP_TRY(hipSetDevice(c->device));
  c->lin_bound = nullptr;  // the build reads the produced records
  TimedLaunch tl(c, CMPC_KERNEL_PRODUCE);
  if (tl.begin()) return -1;
  if (cmpc_launch_produce(P, plant, c->stream)) return fail("cmpc_produce_lin: launch failed");
  if (check_launch("produce kernel")) return -1;
  return tl.end();
}

// ---- observer ----
static void observer_params(cmpc_ctx* c, ObserverParams* P) {
  const cmpc_dims& d = c->d;
  const cmpc_layout& L = c->L;
  std::memset(P, 0, sizeof *P);
  P->obs = c->obs;
  P->M = c->d_obsM;
  P->lin = c->lin;
  P->du_old = c->du_old;
  P->u_old = c->u_old;
  P->nqp = c->nqp;
  P->S = d.S;
  P->ns = d.ns;
  P->ndist = d.ndist;
  P->nobs = L.nobs;
  P->ntot = L.ntot;
  P->n_out = c->obs_nout;
  P->obs_len = c->obs_len;
  P->nu = d.nu;
  P->nu_tot = d.nu_tot;
  P->nV = L.nV;
  P->rec_len = L.rec_len;
  P->off_B = L.off_B;
  P->off_f = L.off_f;
  int blk = L.nobs + L.nd;
  for (int i = 0; i < d.nu_tot; ++i) {
    P->delay[i] = d.delay[i];
    if (d.delay[i]) {
      P->dinput[P->nd] = i;
      P->blk[P->nd] = blk;
      P->rot[P->nd] = d.delay[i] > 1 ? (int)(c->obs_steps % (d.delay[i] - 1)) : 0;
      blk += d.delay[i] - 1;
      P->nd++;
    }
  }
}

static int observer_upload_M(cmpc_ctx* c) {
  for (int s = 0; s < c->d.S; ++s)
    if (!c->have_M[s]) return fail("observer gain of sub-controller " + std::to_string(s) + " not set");
  if (c->obsM_dirty) {
    HIP_TRY(hipMemcpyAsync(c->d_obsM, c->obsM.data(), sizeof(double) * c->obsM.size(),
                           hipMemcpyHostToDevice, c->stream));
    c->obsM_dirty = false;
  }
  return 0;
}

int cmpc_set_observer(cmpc_ctx* c, int s, int n_outputs, const double* M) {
  if (!c || !M) return fail("null argument");
  const cmpc_dims& d = c->d;
  if (s < 0 || s >= d.S) return fail("cmpc_set_observer: bad sub-controller index");
  if (n_outputs < 1 || n_outputs > 8 || n_outputs < d.ndist)
    return fail("cmpc_set_observer: n_outputs must be in [ndist, 8]");
  if (c->obs_nout && c->obs_nout != n_outputs)
    return fail("cmpc_set_observer: n_outputs differs between sub-controllers");
  if (c->L.nobs > 32) return fail("cmpc_set_observer: ns + ndist > 32");
  if (!cmpc_obs_supported(d.ns, n_outputs, d.ndist, c->L.ntot - c->L.nobs, c->L.nd, d.nu_tot))
    return fail("cmpc_set_observer: no observer kernel for these dimensions (instantiated: ns 10 or 11, "
                "4 outputs, 4 disturbance states, 4 inputs)");
  for (int i = 0; i < d.nu_tot; ++i)
    if (d.delay[i] == 1) return fail("cmpc_set_observer: a one-step input delay has no delay block");
  HIP_TRY(hipSetDevice(c->device));
  if (!c->obs) {
    c->obs_nout = n_outputs;
    // rows padded to 128 B (16 doubles): every row starts on a cache line, so
    // the observer kernels' field reads touch no line shared with a neighbour
    c->obs_len = (d.ns + c->L.ntot + n_outputs + n_outputs * d.ns + 15) / 16 * 16;
    c->obsM.assign((size_t)d.S * c->L.nobs * n_outputs, 0.0);
    c->have_M.assign(d.S, 0);
    HIP_TRY(hipMalloc(&c->d_obsM, sizeof(double) * c->obsM.size()));
    HIP_TRY(hipMalloc(&c->obs, sizeof(double) * (size_t)c->nqp * c->obs_len));
    HIP_TRY(hipMemsetAsync(c->obs, 0, sizeof(double) * (size_t)c->nqp * c->obs_len, c->stream));
  }
  std::memcpy(c->obsM.data() + (size_t)s * c->L.nobs * n_outputs, M,
              sizeof(double) * c->L.nobs * n_outputs);
  c->have_M[s] = 1;
  c->obsM_dirty = true;
  return 0;
}

int cmpc_observer_len(const cmpc_ctx* c) { return c ? c->obs_len : 0; }

// the producer's per-QP parameters: every QP slot linearised at its own
// x_hat (observer state), C stored; with_post: the a-posteriori update of
// each slot first, in the same kernel
static int observer_produce_params(cmpc_ctx* c, const double* u_full, const double* y, bool with_post,
                                   ProduceParams& P) {
  int no = 0;
  int io[CMPC_MAX_S_PRODUCE * CMPC_MAX_INPUTS], oi[CMPC_MAX_S_PRODUCE * 4];
  for (int s = 0; s < c->d.S; ++s) {
    for (int k = 0; k < c->d.nu_tot; ++k) io[s * c->d.nu_tot + k] = c->obs_io[s][k];
    for (int o = 0; o < c->d.ny; ++o) oi[s * c->d.ny + o] = c->obs_oi[s][o];
  }
  if (fill_produce(c, "observer", c->obs_plant, c->obs_pin, c->obs_pout, c->obs_Ts, io, oi, &P, &no))
    return -1;
  P.per_qp = 1;
  {  // the observer rows' delay blocks are rings (cmpc_obs_prior_kernel)
    ObserverParams O;
    observer_params(c, &O);
    P.nring = O.nd;
    for (int k = 0; k < O.nd && k < CMPC_ND_MAX; ++k) {
      P.rb[k] = O.blk[k] - c->d.ns;  // dx index -> dx_aug tail index
      P.rlen[k] = O.delay[O.dinput[k]] - 1;
      P.rot[k] = O.rot[k];
    }
  }
  P.x = c->obs;
  P.x_stride = c->obs_len;
  P.dx_aug = c->obs + c->d.ns + c->d.ns;  // dx_aug tail (aug states) of slot 0
  P.dx_stride = c->obs_len;
  P.c_out = c->obs + c->d.ns + c->L.ntot + c->obs_nout;
  P.c_stride = c->obs_len;
  P.u_full = u_full;
  P.y = y;
  if (with_post) {
    P.obs_M = c->d_obsM;
    P.obs = c->obs;
    P.obs_ntot = c->L.ntot;
  }
  return 0;
}

static int observer_produce(cmpc_ctx* c, const double* u_full, const double* y, bool with_post) {
  ProduceParams P;
  if (observer_produce_params(c, u_full, y, with_post, P)) return -1;
  c->lin_bound = nullptr;
  TimedLaunch tl(c, CMPC_KERNEL_PRODUCE);
  if (tl.begin()) return -1;
  if (cmpc_launch_produce(P, c->obs_plant, c->stream)) return fail("observer: produce launch failed");
  if (check_launch("produce kernel (per QP)")) return -1;
  return tl.end();
}

int cmpc_observer_init(cmpc_ctx* c, int plant, double p_in, double p_out, double Ts,
                       const int32_t* input_order, const int32_t* out_idx, const double* x_init,
                       const double* u_full, const double* y_init, const double* dx_init) {
  if (!c) return fail("null context");
  if (!input_order || !out_idx || !x_init || !u_full || !y_init)
    return fail("cmpc_observer_init: null argument");
  if (!c->obs) return fail("cmpc_observer_init: set the observer gains first (cmpc_set_observer)");
  ProduceParams chk;
  int no = 0;
  if (fill_produce(c, "cmpc_observer_init", plant, p_in, p_out, Ts, input_order, out_idx, &chk, &no))
    return -1;
  if (no != c->obs_nout) return fail("cmpc_observer_init: plant outputs differ from the observer gains' n_outputs");
  c->obs_plant = plant;
  c->obs_pin = p_in;
  c->obs_pout = p_out;
  c->obs_Ts = Ts;
  for (int s = 0; s < c->d.S; ++s) {
    for (int k = 0; k < c->d.nu_tot; ++k) c->obs_io[s][k] = chk.input_order[s][k];
    for (int o = 0; o < c->d.ny; ++o) c->obs_oi[s][o] = chk.out_idx[s][o];
  }
  HIP_TRY(hipSetDevice(c->device));
  if (observer_upload_M(c)) return -1;
  c->obs_steps = 0;  // the rings start in logical order
  ObserverParams P;
  observer_params(c, &P);
  P.x_init = x_init;
  P.dx_init = dx_init;
  P.y = y_init;
  if (cmpc_launch_observer(P, CMPC_OBS_INIT, c->stream)) return fail("observer init launch failed");
  if (check_launch("observer init kernel")) return -1;
  return observer_produce(c, u_full, y_init, false);  // Initialize: Update(x_init, full_u_old)
}

int cmpc_observe_step(cmpc_ctx* c, const double* u_full, const double* y) {
  if (!c) return fail("null context");
  if (!u_full || !y) return fail("cmpc_observe_step: null argument");
  if (c->obs_plant < 0) return fail("cmpc_observe_step: call cmpc_observer_init first");
  HIP_TRY(hipSetDevice(c->device));
  if (observer_upload_M(c)) return -1;
  // ObserveAPosteriori + Update: one kernel (the producer runs the
  // a-posteriori update of its slot first, in or_observe_post's order)
  return observer_produce(c, u_full, y, true);
}

int cmpc_observe_apply(cmpc_ctx* c) {
  if (!c) return fail("null context");
  if (c->obs_plant < 0) return fail("cmpc_observe_apply: call cmpc_observer_init first");
  if (c->lin_bound) return fail("cmpc_observe_apply: records are bound externally");
  HIP_TRY(hipSetDevice(c->device));
  ObserverParams P;
  observer_params(c, &P);
  TimedLaunch tl(c, CMPC_KERNEL_OBSERVE_PRIOR);
  if (tl.begin()) return -1;
  if (cmpc_launch_observer(P, CMPC_OBS_PRIOR, c->stream))
    return fail("cmpc_observe_apply: no a-priori kernel instantiation for these dimensions");
  if (check_launch("observer a-priori kernel")) return -1;
  c->obs_steps++;  // the delay-block rings advance by one
  return tl.end();
}

static int build_params(cmpc_ctx* c, BuildParams& P);

// NerveCenter::GetNextInput on the device: cmpc_observe_step + cmpc_step(K,
// 0) + cmpc_observe_apply, as one kernel where the batch takes the
// one-QP-per-wave fused step (cmpc_control_step_kernel), else the three calls.
static int control_step(cmpc_ctx* c, const double* u_full, const double* y, int K, bool* flagged);

int cmpc_control_step(cmpc_ctx* c, const double* u_full, const double* y, int K) {
  return control_step(c, u_full, y, K, nullptr);
}

// flagged (optional): set when the launch stores c->done_seq into
// c->done_host once its results are in place
static int control_step(cmpc_ctx* c, const double* u_full, const double* y, int K, bool* flagged) {
  if (flagged) *flagged = false;
  if (!c) return fail("null context");
  if (!u_full || !y) return fail("cmpc_control_step: null argument");
  if (K < 0) return fail("K must be >= 0");
  if (c->obs_plant < 0) return fail("cmpc_control_step: call cmpc_observer_init first");
  HIP_TRY(hipSetDevice(c->device));
  if (observer_upload_M(c)) return -1;
  if (!c->cus) (void)hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device);
  const cmpc_dims& d = c->d;
  // one launch up to four QPs per CU: it wins there (config 5's cent-par
  // p = 200 at 1 024 QPs 50.7 vs 58.6 us, coop-par p = 50 at 512 QPs 48.5 vs
  // 49.5 us) and loses above (2 048 QPs: 75.2 vs 72.7 and 102.0 vs 73.0 us;
  // tools/control_step_ab.py, profiles/r6r_control_step_ab.txt)
  const bool fuse = K > 0 && c->step_variant != CMPC_STEP_SPLIT && c->build_variant == CMPC_BUILD_AUTO &&
                    c->solve_variant == CMPC_SOLVE_AUTO && c->nqp <= 4 * std::max(c->cus, 1) &&
                    c->L.nuo == (d.S - 1) * d.nu;
  if (fuse) {
    if (ensure_cfg(c)) return -1;
    ControlStepParams C;
    std::memset(&C, 0, sizeof C);
    if (observer_produce_params(c, u_full, y, true, C.pr)) return -1;
    c->lin_bound = nullptr;  // the build reads the produced records
    if (build_params(c, C.b)) return -1;
    // up to one QP per CU the build runs as role-split pairs, two QP slots
    // per workgroup (cent-ser B = 1 build 17.7 -> 15.7 us, §3.1)
#ifndef CMPC_CONTROL_SPLIT
#define CMPC_CONTROL_SPLIT 1
#endif
    C.b.split = CMPC_CONTROL_SPLIT && c->nqp <= std::max(c->cus, 1);
    if (C.b.split) C.b.grid = std::max(1, (c->nqp + 1) / 2);
    solve_params(c, &C.b.sv);
    C.b.sv.K = K;
    C.b.sv.flags = 0;  // u_old += du is the a-priori phase's
    observer_params(c, &C.ob);
    C.pr_off = ((C.pr.S * C.pr.rec_len + C.pr.naug + 3) / 4) * 2;  // doubles, 16-byte aligned
    const bool flag = flagged && c->done_dev && C.b.grid == 1;
    C.done = flag ? c->done_dev : nullptr;
    C.seq = flag ? ++c->done_seq : 0u;
    TimedLaunch tl(c, CMPC_KERNEL_STEP);
    if (tl.begin()) return -1;
    int solver = 0;
    if (cmpc_launch_control_step(C, d.ns, d.ny, d.nu, d.m, c->stream, &solver) == 0) {
      if (check_launch("control step kernel")) return -1;
      c->last_build = C.b.split ? CMPC_BUILD_SPLIT : CMPC_BUILD_WAVE;
      c->last_solve = solver;
      c->last_step_fused = 1;
      c->obs_steps++;  // the delay-block rings advance by one (cmpc_observe_apply)
      if (flagged) *flagged = flag;
      return tl.end();
    }
    cmpc_launch_events = LaunchEvents{};
  }
  if (cmpc_observe_step(c, u_full, y)) return -1;
  if (cmpc_step(c, K, 0)) return -1;
  return cmpc_observe_apply(c);
}

// copies host arrays (nullptr entries skipped) into the context's staging
// buffer on its stream; returns their device addresses
// host arrays of up to this many doubles are read by the kernels in place
static bool stage_in_place(size_t tot) { return tot <= 1024; }

static int stage_host(cmpc_ctx* c, const double* const* host, const size_t* n, int k,
                      const double** dev) {
  size_t tot = 0;
  for (int i = 0; i < k; ++i) tot += host[i] ? (n[i] + 1) / 2 * 2 : 0;
  if (!stage_in_place(tot) && tot > c->stage_cap) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->stage) HIP_TRY(hipFree(c->stage));
    c->stage = nullptr;
    HIP_TRY(hipMalloc(&c->stage, sizeof(double) * tot));
    c->stage_cap = tot;
  }
  // one DMA from page-locked memory (the device stage is read by kernels
  // queued after the copy on the same stream); small arrays are read by the
  // kernel in place (no copy: the caller releases the buffer after the launch)
  return pinned_upload(c->pin_in, c->stream, stage_in_place(tot) ? nullptr : c->stage, host, n, k, dev);
}

// after the launch that reads what stage_host staged
static int stage_done(cmpc_ctx* c) {
  return c->pin_in.pending ? 0 : pinned_release(c->pin_in, c->stream);
}

int cmpc_observer_init_host(cmpc_ctx* c, int plant, double p_in, double p_out, double Ts,
                            const int32_t* input_order, const int32_t* out_idx,
                            const double* x_init, const double* u_full, const double* y_init,
                            const double* dx_init) {
  if (!c) return fail("null context");
  int ns = 0, ni = 0, no = 0, nci = 0;
  if (cmpc_plant_dims(plant, &ns, &ni, &no, &nci)) return fail("cmpc_observer_init_host: unknown plant");
  HIP_TRY(hipSetDevice(c->device));
  const size_t B = c->d.B;
  const double* h[4] = {x_init, u_full, y_init, dx_init};
  const size_t n[4] = {B * ns, B * ni, B * no, (size_t)c->nqp * c->L.ntot};
  const double* d[4];
  if (stage_host(c, h, n, 4, d)) return -1;
  const int rc = cmpc_observer_init(c, plant, p_in, p_out, Ts, input_order, out_idx, d[0], d[1], d[2], d[3]);
  return stage_done(c) ? -1 : rc;
}

int cmpc_observe_step_host(cmpc_ctx* c, const double* u_full, const double* y) {
  if (!c) return fail("null context");
  if (c->obs_plant < 0) return fail("cmpc_observe_step_host: call cmpc_observer_init first");
  int ns = 0, ni = 0, no = 0, nci = 0;
  if (cmpc_plant_dims(c->obs_plant, &ns, &ni, &no, &nci)) return fail("unknown plant");
  HIP_TRY(hipSetDevice(c->device));
  const size_t B = c->d.B;
  const double* h[2] = {u_full, y};
  const size_t n[2] = {B * ni, B * no};
  const double* d[2];
  if (stage_host(c, h, n, 2, d)) return -1;
  const int rc = cmpc_observe_step(c, d[0], d[1]);
  return stage_done(c) ? -1 : rc;
}

// cmpc_control_step_host + cmpc_download: a one-workgroup launch signals its
// completion word, which the host polls (the results are in page-locked host
// memory already) instead of a stream synchronisation; anything else, and a
// poll that has not seen the word after a second, synchronises the stream.
int cmpc_control_step_download(cmpc_ctx* c, const double* u_full, const double* y, int K, double* du,
                               int32_t* status, int32_t* nwsr) {
  if (!c) return fail("null context");
  if (c->obs_plant < 0) return fail("cmpc_control_step_download: call cmpc_observer_init first");
  int ns = 0, ni = 0, no = 0, nci = 0;
  if (cmpc_plant_dims(c->obs_plant, &ns, &ni, &no, &nci)) return fail("unknown plant");
  HIP_TRY(hipSetDevice(c->device));
  const size_t B = c->d.B;
  const double* h[2] = {u_full, y};
  const size_t n[2] = {B * ni, B * no};
  const double* d[2];
  if (stage_host(c, h, n, 2, d)) return -1;
  bool flagged = false;
  const int rc = control_step(c, d[0], d[1], K, &flagged);
  if (rc) {
    (void)stage_done(c);
    return -1;
  }
  // (after cmpc_download's stream synchronisation the kernels have read the
  // staged inputs too: no event is needed on that path either)
  auto synced = [&]() {
    if (cmpc_download(c, du, status, nwsr) == 0) return 0;
    (void)stage_done(c);
    return -1;
  };
  if (!flagged || !c->out_host) return synced();
  // polled: the kernel stores the done word after its last read of the
  // staged inputs, so once the word is seen the staging buffer is free and
  // no event need guard it (its record and the next call's wait on it cost
  // ~5 us per B = 1 call: profiles/r6q_b1_noevent_ab.txt)
  const volatile uint32_t* w = c->done_host;
  const uint32_t want = c->done_seq;
  const auto t0 = std::chrono::steady_clock::now();
  long spins = 0;
  while (__atomic_load_n(const_cast<const uint32_t*>(w), __ATOMIC_ACQUIRE) != want) {
    if ((++spins & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1))
      return synced();  // (the stream synchronisation path)
  }
  const size_t nq = (size_t)c->nqp;
  if (du) std::memcpy(du, c->out_block, sizeof(double) * nq * c->L.nV);
  if (status) std::memcpy(status, c->out_block + c->out_st, sizeof(int32_t) * nq);
  if (nwsr) std::memcpy(nwsr, c->out_block + c->out_nw, sizeof(int32_t) * nq);
  return 0;
}

int cmpc_control_step_host(cmpc_ctx* c, const double* u_full, const double* y, int K) {
  if (!c) return fail("null context");
  if (c->obs_plant < 0) return fail("cmpc_control_step_host: call cmpc_observer_init first");
  int ns = 0, ni = 0, no = 0, nci = 0;
  if (cmpc_plant_dims(c->obs_plant, &ns, &ni, &no, &nci)) return fail("unknown plant");
  HIP_TRY(hipSetDevice(c->device));
  const size_t B = c->d.B;
  const double* h[2] = {u_full, y};
  const size_t n[2] = {B * ni, B * no};
  const double* d[2];
  if (stage_host(c, h, n, 2, d)) return -1;
  const int rc = cmpc_control_step(c, d[0], d[1], K);
  return stage_done(c) ? -1 : rc;
}

// ---- plant simulation ----
struct cmpc_sim {
  int plant = 0, B = 0, device = 0, ns = 0, ni = 0, no = 0, nc = 0, ring_len = 0;
  int cur[CMPC_MAX_INPUTS] = {};  // TimeDelay cursors (every scenario's are the same)
  double p_in = 1.0, p_out = 1.0;
  int delay[CMPC_MAX_INPUTS] = {}, cidx[CMPC_MAX_INPUTS] = {};
  hipStream_t stream = nullptr;
  bool own_stream = false;
  double *x = nullptr, *dt = nullptr, *u_full = nullptr, *u_offset = nullptr, *ring = nullptr,
         *scratch = nullptr, *stage = nullptr;  // stage: host-variant staging (B x max(ns, ni, no, nc))
  int32_t* status = nullptr;
  PinnedIO pin_in, pin_out;  // host-array calls: page-locked staging
};

int cmpc_sim_create(cmpc_sim** out, int plant, int B, int device, double p_in, double p_out,
                    int n_control, const int32_t* delays, const int32_t* control_index) {
  if (!out || !delays || !control_index) return fail("null argument");
  *out = nullptr;
  int ns = 0, ni = 0, no = 0, nci = 0;
  if (cmpc_plant_dims(plant, &ns, &ni, &no, &nci)) return fail("cmpc_sim_create: unknown plant");
  if (B < 1 || B > (1 << 28)) return fail("cmpc_sim_create: bad batch");
  if (n_control < 1 || n_control > CMPC_MAX_INPUTS) return fail("cmpc_sim_create: bad n_control");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail("no such HIP device");
  cmpc_sim* m = new cmpc_sim();
  m->plant = plant; m->B = B; m->device = device; m->ns = ns; m->ni = ni; m->no = no;
  m->nc = n_control; m->p_in = p_in; m->p_out = p_out;
  for (int i = 0; i < n_control; ++i) {
    if (delays[i] < 0 || control_index[i] < 0 || control_index[i] >= ni) {
      delete m;
      return fail("cmpc_sim_create: bad delay or control index");
    }
    m->delay[i] = delays[i];
    m->cidx[i] = control_index[i];
    m->ring_len += delays[i];
  }
  if (m->ring_len == 0) m->ring_len = 1;
  auto bail = [&](hipError_t e) {
    (void)e;
    void* bufs[] = {m->x, m->dt, m->u_full, m->u_offset, m->ring, m->scratch, m->stage, m->status};
    for (void* b : bufs)
      if (b) (void)hipFree(b);
    delete m;
    return fail("cmpc_sim_create: device allocation failed");
  };
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return bail(e);
  if ((e = hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking)) != hipSuccess) return bail(e);
  m->own_stream = true;
  const size_t Bz = (size_t)B;
  if ((e = hipMalloc(&m->x, sizeof(double) * Bz * ns)) != hipSuccess ||
      (e = hipMalloc(&m->dt, sizeof(double) * Bz)) != hipSuccess ||
      (e = hipMalloc(&m->u_full, sizeof(double) * Bz * ni)) != hipSuccess ||
      (e = hipMalloc(&m->u_offset, sizeof(double) * Bz * ni)) != hipSuccess ||
      (e = hipMalloc(&m->ring, sizeof(double) * Bz * m->ring_len)) != hipSuccess ||
      (e = hipMalloc(&m->scratch, sizeof(double) * Bz * (ni > n_control ? ni : n_control))) != hipSuccess ||
      (e = hipMalloc(&m->stage, sizeof(double) * Bz * 2 * std::max(std::max(ns, ni), std::max(no, n_control)))) !=
          hipSuccess ||
      (e = hipMalloc(&m->status, sizeof(int32_t) * Bz)) != hipSuccess ||
      (e = hipMemsetAsync(m->status, 0, sizeof(int32_t) * Bz, m->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(m->stream)) != hipSuccess)
    return bail(e);
  *out = m;
  return 0;
}

int cmpc_sim_destroy(cmpc_sim* m) {
  if (!m) return 0;
  (void)hipSetDevice(m->device);
  if (m->stream) (void)hipStreamSynchronize(m->stream);
  pinned_free(m->pin_in);
  pinned_free(m->pin_out);
  void* bufs[] = {m->x, m->dt, m->u_full, m->u_offset, m->ring, m->scratch, m->stage, m->status};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (m->own_stream && m->stream) (void)hipStreamDestroy(m->stream);
  delete m;
  return 0;
}

int cmpc_sim_set_stream(cmpc_sim* m, void* stream) {
  if (!m) return fail("null simulator");
  HIP_TRY(hipSetDevice(m->device));
  HIP_TRY(hipStreamSynchronize(m->stream));
  if (m->own_stream) (void)hipStreamDestroy(m->stream);
  m->stream = (hipStream_t)stream;
  m->own_stream = false;
  return 0;
}

static SimInputParams sim_input_params(cmpc_sim* m, const double* u_control, int use_delay) {
  SimInputParams P;
  std::memset(&P, 0, sizeof P);
  P.u_control = u_control;
  P.u_offset = m->u_offset;
  P.u_full = m->u_full;
  P.ring = m->ring;
  P.B = m->B;
  P.nc = m->nc;
  P.ni = m->ni;
  P.ring_len = m->ring_len;
  P.use_delay = use_delay;
  for (int i = 0; i < m->nc; ++i) {
    P.delay[i] = m->delay[i];
    P.cidx[i] = m->cidx[i];
    P.cur[i] = m->cur[i];
  }
  return P;
}

int cmpc_sim_reset(cmpc_sim* m, const double* x0, const double* u_offset, double dt0) {
  if (!m || !x0 || !u_offset) return fail("null argument");
  if (!(dt0 > 0)) return fail("cmpc_sim_reset: dt0 must be positive");
  HIP_TRY(hipSetDevice(m->device));
  const size_t Bz = (size_t)m->B;
  HIP_TRY(hipMemcpyAsync(m->x, x0, sizeof(double) * Bz * m->ns, hipMemcpyDeviceToDevice, m->stream));
  HIP_TRY(hipMemcpyAsync(m->u_offset, u_offset, sizeof(double) * Bz * m->ni, hipMemcpyDeviceToDevice,
                         m->stream));
  std::vector<double> dts(Bz, dt0);
  HIP_TRY(hipMemcpyAsync(m->dt, dts.data(), sizeof(double) * Bz, hipMemcpyHostToDevice, m->stream));
  // TimeDelay(): zero memory, cursor of input i at the sum of the delays before it
  HIP_TRY(hipMemsetAsync(m->ring, 0, sizeof(double) * Bz * m->ring_len, m->stream));
  HIP_TRY(hipMemsetAsync(m->status, 0, sizeof(int32_t) * Bz, m->stream));  // failures are sticky until here
  for (int i = 0, sum = 0; i < m->nc; ++i) {
    m->cur[i] = sum;
    sum += m->delay[i];
  }
  // u_ = GetPlantInput(u_init = 0) = u_offset
  HIP_TRY(hipMemcpyAsync(m->u_full, u_offset, sizeof(double) * Bz * m->ni, hipMemcpyDeviceToDevice,
                         m->stream));
  HIP_TRY(hipStreamSynchronize(m->stream));  // (host staging buffers above)
  return 0;
}

int cmpc_sim_set_input(cmpc_sim* m, const double* u_control) {
  if (!m || !u_control) return fail("null argument");
  HIP_TRY(hipSetDevice(m->device));
  const SimInputParams P = sim_input_params(m, u_control, 1);
  if (cmpc_launch_sim_input(P, m->stream)) return fail("sim input launch failed");
  if (check_launch("sim input kernel")) return -1;
  // TimeDelay::GetDelayedInput's cursor step (time_delay.h:41-58), on the host
  for (int i = 0, end = 0; i < m->nc; ++i) {
    if (m->delay[i] == 0) continue;
    end += m->delay[i];
    if (++m->cur[i] == end) m->cur[i] -= m->delay[i];
  }
  return 0;
}

int cmpc_sim_set_offset(cmpc_sim* m, const double* u_offset) {
  if (!m || !u_offset) return fail("null argument");
  HIP_TRY(hipSetDevice(m->device));
  HIP_TRY(hipMemcpyAsync(m->u_offset, u_offset, sizeof(double) * (size_t)m->B * m->ni,
                         hipMemcpyDeviceToDevice, m->stream));
  return 0;
}

int cmpc_sim_plant_input_offset(cmpc_sim* m, const double* u_control, const double* u_offset,
                                double* u_full_out) {
  if (!m || !u_control || !u_offset || !u_full_out) return fail("null argument");
  HIP_TRY(hipSetDevice(m->device));
  SimInputParams P = sim_input_params(m, u_control, 0);
  P.u_offset = u_offset;
  P.u_full = u_full_out;
  if (cmpc_launch_sim_input(P, m->stream)) return fail("sim input launch failed");
  return check_launch("sim input kernel");
}

int cmpc_sim_restart(cmpc_sim* m, double dt0) {
  if (!m) return fail("null simulator");
  if (!(dt0 > 0)) return fail("cmpc_sim_restart: dt0 must be positive");
  HIP_TRY(hipSetDevice(m->device));
  std::vector<double> dts((size_t)m->B, dt0);
  HIP_TRY(hipMemcpyAsync(m->dt, dts.data(), sizeof(double) * dts.size(), hipMemcpyHostToDevice, m->stream));
  HIP_TRY(hipStreamSynchronize(m->stream));  // (host staging buffer)
  return 0;
}

int cmpc_sim_plant_input(cmpc_sim* m, const double* u_control, double* u_full_out) {
  if (!m || !u_control || !u_full_out) return fail("null argument");
  HIP_TRY(hipSetDevice(m->device));
  SimInputParams P = sim_input_params(m, u_control, 0);
  P.u_full = u_full_out;
  if (cmpc_launch_sim_input(P, m->stream)) return fail("sim input launch failed");
  return check_launch("sim input kernel");
}

int cmpc_sim_integrate(cmpc_sim* m, double t, double t_end, double eps_abs, double eps_rel) {
  if (!m) return fail("null simulator");
  if (!(t_end >= t)) return fail("cmpc_sim_integrate: t_end < t");
  HIP_TRY(hipSetDevice(m->device));
  SimParams P;
  std::memset(&P, 0, sizeof P);
  P.x = m->x;
  P.dt = m->dt;
  P.u_full = m->u_full;
  P.status = m->status;
  P.B = m->B;
  P.t = t;
  P.t_end = t_end;
  P.eps_abs = eps_abs;
  P.eps_rel = eps_rel;
  P.p_in = m->p_in;
  P.p_out = m->p_out;
  if (cmpc_launch_sim(P, m->plant, m->stream)) return fail("sim launch failed");
  return check_launch("sim kernel");
}

int cmpc_sim_output(cmpc_sim* m, double* y) {
  if (!m || !y) return fail("null argument");
  HIP_TRY(hipSetDevice(m->device));
  if (cmpc_launch_sim_output(m->plant, m->x, y, m->B, m->stream)) return fail("sim output launch failed");
  return check_launch("sim output kernel");
}

int cmpc_sim_download(cmpc_sim* m, double* x, double* u_full, double* dt, int32_t* status) {
  if (!m) return fail("null simulator");
  HIP_TRY(hipSetDevice(m->device));
  const size_t Bz = (size_t)m->B;
  const size_t bx = sizeof(double) * Bz * m->ns, bu = sizeof(double) * Bz * m->ni, bd = sizeof(double) * Bz,
               bs = sizeof(int32_t) * Bz;
  auto up = [](size_t v) { return (v + 15) / 16 * 16; };
  const size_t ou = up(bx), od = ou + up(bu), os = od + up(bd);
  // device -> page-locked buffer (DMA), then host copies after one sync
  if (pinned_acquire(m->pin_out, os + bs)) return -1;
  char* h = m->pin_out.buf;
  if (x) HIP_TRY(hipMemcpyAsync(h, m->x, bx, hipMemcpyDeviceToHost, m->stream));
  if (u_full) HIP_TRY(hipMemcpyAsync(h + ou, m->u_full, bu, hipMemcpyDeviceToHost, m->stream));
  if (dt) HIP_TRY(hipMemcpyAsync(h + od, m->dt, bd, hipMemcpyDeviceToHost, m->stream));
  if (status) HIP_TRY(hipMemcpyAsync(h + os, m->status, bs, hipMemcpyDeviceToHost, m->stream));
  HIP_TRY(hipStreamSynchronize(m->stream));
  if (x) std::memcpy(x, h, bx);
  if (u_full) std::memcpy(u_full, h + ou, bu);
  if (dt) std::memcpy(dt, h + od, bd);
  if (status) std::memcpy(status, h + os, bs);
  return 0;
}

// Host-array variants: stage through the simulator's device buffer; each
// returns once the call's work is done (the host arrays are free again).
static int sim_stage(cmpc_sim* m, const double* h0, size_t n0, const double* h1, size_t n1) {
  HIP_TRY(hipSetDevice(m->device));
  const size_t half = (size_t)m->B * std::max(std::max(m->ns, m->ni), std::max(m->no, m->nc));
  // one DMA from page-locked memory: h0 at stage, h1 at stage + half
  const size_t tot = n1 ? half + n1 : n0;
  if (pinned_acquire(m->pin_in, sizeof(double) * std::max<size_t>(tot, 1))) return -1;
  double* h = reinterpret_cast<double*>(m->pin_in.buf);
  if (n0) std::memcpy(h, h0, sizeof(double) * n0);
  if (n1) std::memcpy(h + half, h1, sizeof(double) * n1);
  if (tot) HIP_TRY(hipMemcpyAsync(m->stage, h, sizeof(double) * tot, hipMemcpyHostToDevice, m->stream));
  return pinned_release(m->pin_in, m->stream);
}

int cmpc_sim_reset_host(cmpc_sim* m, const double* x0, const double* u_offset, double dt0) {
  if (!m || !x0 || !u_offset) return fail("null argument");
  const size_t half = (size_t)m->B * std::max(std::max(m->ns, m->ni), std::max(m->no, m->nc));
  if (sim_stage(m, x0, (size_t)m->B * m->ns, u_offset, (size_t)m->B * m->ni)) return -1;
  return cmpc_sim_reset(m, m->stage, m->stage + half, dt0);  // (synchronises)
}

int cmpc_sim_set_input_host(cmpc_sim* m, const double* u_control) {
  if (!m || !u_control) return fail("null argument");
  if (sim_stage(m, u_control, (size_t)m->B * m->nc, nullptr, 0)) return -1;
  if (cmpc_sim_set_input(m, m->stage)) return -1;
  return cmpc_sim_synchronize(m);
}

int cmpc_sim_set_offset_host(cmpc_sim* m, const double* u_offset) {
  if (!m || !u_offset) return fail("null argument");
  if (sim_stage(m, u_offset, (size_t)m->B * m->ni, nullptr, 0)) return -1;
  if (cmpc_sim_set_offset(m, m->stage)) return -1;
  return cmpc_sim_synchronize(m);
}

int cmpc_sim_output_host(cmpc_sim* m, double* y) {
  if (!m || !y) return fail("null argument");
  HIP_TRY(hipSetDevice(m->device));
  const size_t by = sizeof(double) * (size_t)m->B * m->no;
  if (pinned_acquire(m->pin_out, by)) return -1;
  if (cmpc_sim_output(m, m->stage)) return -1;
  HIP_TRY(hipMemcpyAsync(m->pin_out.buf, m->stage, by, hipMemcpyDeviceToHost, m->stream));
  if (cmpc_sim_synchronize(m)) return -1;
  std::memcpy(y, m->pin_out.buf, by);
  return 0;
}

double* cmpc_sim_state(cmpc_sim* m) { return m ? m->x : nullptr; }
double* cmpc_sim_input(cmpc_sim* m) { return m ? m->u_full : nullptr; }
double* cmpc_sim_step_size(cmpc_sim* m) { return m ? m->dt : nullptr; }
int32_t* cmpc_sim_status(cmpc_sim* m) { return m ? m->status : nullptr; }

int cmpc_sim_synchronize(cmpc_sim* m) {
  if (!m) return fail("null simulator");
  HIP_TRY(hipSetDevice(m->device));
  HIP_TRY(hipStreamSynchronize(m->stream));
  return 0;
}

// NerveCenter::UpdateUOld at the nerve level (nerve_center.h:313-319): the
// control input u_old_ (B x nu_tot, plant control order) += every
// sub-controller's first move of its own inputs (ControlInputIndices order)
int cmpc_accumulate_moves(cmpc_ctx* c, const int32_t* input_order, double* u_control) {
  if (!c || !input_order || !u_control) return fail("null argument");
  const cmpc_dims& d = c->d;
  if (d.S > CMPC_MAX_S_PRODUCE) return fail("cmpc_accumulate_moves: too many sub-controllers");
  AccumParams P;
  std::memset(&P, 0, sizeof P);
  P.du = c->du_old;
  P.u_control = u_control;
  P.B = d.B;
  P.S = d.S;
  P.nu = d.nu;
  P.nu_tot = d.nu_tot;
  P.nV = c->L.nV;
  for (int s = 0; s < d.S; ++s)
    for (int k = 0; k < d.nu; ++k) {
      const int v = input_order[s * d.nu_tot + k];
      if (v < 0 || v >= d.nu_tot) return fail("cmpc_accumulate_moves: bad input_order");
      P.order[s][k] = v;
    }
  HIP_TRY(hipSetDevice(c->device));
  if (cmpc_launch_accumulate(P, c->stream)) return fail("accumulate launch failed");
  return check_launch("accumulate kernel");
}

// Rows between the device layout (delay blocks as rings, rotated by the
// a-priori step count, cmpc_obs_prior_kernel) and the logical layout of the
// ABI (observer.h's AugmentedState order).  to_logical: device -> logical.
static void observer_rows_rotate(cmpc_ctx* c, const double* in, double* out, bool to_logical) {
  ObserverParams O;
  observer_params(c, &O);
  const size_t n = (size_t)c->nqp, len = c->obs_len;
  std::memcpy(out, in, sizeof(double) * n * len);
  for (int k = 0; k < O.nd; ++k) {
    const int L = O.delay[O.dinput[k]] - 1, r = O.rot[k];
    if (L < 2 || r == 0) continue;
    const size_t b0 = (size_t)c->d.ns + O.blk[k];  // row offset of the block (after x_hat)
    for (size_t q = 0; q < n; ++q)
      for (int i = 0; i < L; ++i) {
        const size_t phys = b0 + (i + r) % L, logi = b0 + i;
        if (to_logical) out[q * len + logi] = in[q * len + phys];
        else out[q * len + phys] = in[q * len + logi];
      }
  }
}

int cmpc_get_observer_state(cmpc_ctx* c, double* host) {
  if (!c || !host) return fail("null argument");
  if (!c->obs) return fail("no observer state (cmpc_set_observer)");
  HIP_TRY(hipSetDevice(c->device));
  std::vector<double> dev((size_t)c->nqp * c->obs_len);
  HIP_TRY(hipMemcpyAsync(dev.data(), c->obs, sizeof(double) * dev.size(), hipMemcpyDeviceToHost,
                         c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  observer_rows_rotate(c, dev.data(), host, true);
  return 0;
}

int cmpc_set_observer_state(cmpc_ctx* c, const double* host) {
  if (!c || !host) return fail("null argument");
  if (!c->obs) return fail("no observer state (cmpc_set_observer)");
  HIP_TRY(hipSetDevice(c->device));
  std::vector<double> dev((size_t)c->nqp * c->obs_len);
  observer_rows_rotate(c, host, dev.data(), false);
  HIP_TRY(hipMemcpyAsync(c->obs, dev.data(), sizeof(double) * dev.size(), hipMemcpyHostToDevice,
                         c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

// LDS layout of the build kernel (doubles; must match cmpc_kernels.hip).
// Bank model (MI355X_MICROARCH.md §LDS): ds_read_b64 is serviced per 32-lane
// group with 32 double-wide banks, ds_write_b64 per 16-lane group with 16.
// Per step the gather lanes of rows 0/1 (one read group) read lines at
// line_off[c] + (m-1-k) + r - D_c and row o's Markov lanes write at
// line_off[c] + m - 1 + r.  Lines (length m - 1 + p) are placed so that input
// c's read window sits at residues [m*pi(c), m*pi(c) + m) mod 32 and the
// write residues are distinct mod 16; rows are 16 mod 32 apart so row 1's
// window is disjoint from row 0's.  All addresses advance together, so a
// layout that is conflict-free at one step is conflict-free at every step.
static void build_lds_layout(const cmpc_dims& d, const cmpc_layout& L, BuildParams* P) {
  const int nut = d.nu_tot, M = d.m, ng = M * nut + 1;
  auto up = [](int v, int a) { return (v + a - 1) / a * a; };
  auto place = [&](const int* perm, int* off) {  // returns total length
    int cur = 0;
    for (int c = 0; c < nut; ++c) {
      const int want = (((M * perm[c] + d.delay[c]) % 32) + 32) % 32;
      int o = cur;
      while (((o % 32) + 32) % 32 != want) ++o;
      off[c] = o;
      cur = o + M - 1 + d.p;
    }
    return cur;
  };
  int perm[CMPC_MAX_INPUTS], best[CMPC_MAX_INPUTS], off[CMPC_MAX_INPUTS];
  for (int c = 0; c < nut; ++c) perm[c] = best[c] = c;
  int best_len = -1;
  do {  // permutations of the read windows: first one whose writes are conflict-free
    const int len = place(perm, off);
    bool ok = true;
    for (int a = 0; a < nut && ok; ++a)
      for (int b = a + 1; b < nut && ok; ++b)
        ok = (off[a] - off[b]) % 16 != 0;
    if (ok && (best_len < 0 || len < best_len)) {
      best_len = len;
      for (int c = 0; c < nut; ++c) best[c] = perm[c];
    }
  } while (std::next_permutation(perm, perm + nut));
  const int len = place(best, off);
  for (int c = 0; c < nut; ++c) P->line_off[c] = off[c];
  int rs = up(len, 2);
  while (rs % 32 != 16) rs += 2;
  P->line_rs = rs;
  const int head = L.rec_len + 8 + d.ny * L.nobs + 4;  // record, u_old, C_hat, kappa
  int o = std::max(std::max(d.ny * rs, (d.ny - 1) * ng * L.nV), head);
  o = up(o, 32) + 16;                                   // w table at 16 mod 32
  P->w_off = o;
  o += up((d.p + 3) * d.ny, 2);
  while (o % 32 != (M * nut) % 32) o += 2;               // z slots next to row 0's window
  P->zs_off = o;
  if (d.ny == 4) {
    // pre-pass z lines: stride = 1 mod 32, so row o's z read sits at residue
    // m*nu_tot + o (between the line windows of rows o and o+1 at 0 / 16 mod 32)
    // and the four writes of a step hit distinct banks
    int zst = d.p;
    while (zst % 32 != 1) ++zst;
    P->zl_stride = zst;
    o += d.ny * zst;
  } else {
    P->zl_stride = 4;
    o += d.ny * 4;
  }
  P->lds_per_wave = up(o, 32);
  P->yl_stride = up((d.p + 1) * d.ny, 32);
  P->lds_block = up(d.S * P->yl_stride + d.S * d.ny * d.ny + d.S * d.nu * d.nu + 16, 32);
  // loop segments: the distinct delays inside the horizon, ascending
  P->nbound = 0;
  for (int c = 0; c < nut; ++c) {
    const int D = d.delay[c];
    if (D <= 0 || D >= d.p) continue;
    bool seen = false;
    for (int i = 0; i < P->nbound; ++i) seen = seen || P->bound[i] == D;
    if (!seen) P->bound[P->nbound++] = D;
  }
  std::sort(P->bound, P->bound + P->nbound);
}

int cmpc_set_build_variant(cmpc_ctx* c, int variant) {
  if (!c) return fail("null context");
  if (variant != CMPC_BUILD_AUTO && variant != CMPC_BUILD_WAVE && variant != CMPC_BUILD_ROWS &&
      variant != CMPC_BUILD_SPLIT)
    return fail("cmpc_set_build_variant: unknown variant");
  c->build_variant = variant;
  return 0;
}

int cmpc_last_build_kernel(cmpc_ctx* c) {
  if (!c) return fail("null context");
  return c->last_build;
}

static int build_params(cmpc_ctx* c, BuildParams& P);

int cmpc_build(cmpc_ctx* c) {
  if (!c) return fail("null context");
  if (ensure_cfg(c)) return -1;
  HIP_TRY(hipSetDevice(c->device));
  const cmpc_dims& d = c->d;
  BuildParams P;
  if (build_params(c, P)) return -1;
  TimedLaunch tl(c, CMPC_KERNEL_BUILD);
  if (tl.begin()) return -1;
  int rc = -1;
  // AUTO: the row kernel wherever its LDS fits (measured as fast or faster
  // than the one-QP-per-wave kernel for every plant/controller type at
  // p = 20, 50, 100, 200: tools/gpu_build_table.sh) and the
  // batch gives it at least one wave per SIMD; else
  // the one-QP-per-wave kernel, which has four times the waves for a small
  // batch (cent p = 200, 1 024 QPs: 0.026 vs 0.057 ms)
  // Below one QP per SIMD the role-split kernel: two waves per QP
  // (config 5: 28.1 -> 22.6 us, profiles/r5g_build_split_ab.txt).
  const bool rows_fill = (c->nqp + 3) / 4 >= 4 * P.cus;
  const bool split_fit = c->nqp <= 4 * P.cus;
  if (c->build_variant == CMPC_BUILD_ROWS || (c->build_variant == CMPC_BUILD_AUTO && rows_fill))
    rc = cmpc_launch_build_rows(P, d.ns, d.ny, d.nu, d.m, c->stream);
  if (rc && c->build_variant == CMPC_BUILD_ROWS)
    return fail("row-layout build kernel not available for these dimensions");
  c->last_build = CMPC_BUILD_ROWS;
  if (rc) {
    P.split = c->build_variant == CMPC_BUILD_SPLIT || (c->build_variant == CMPC_BUILD_AUTO && split_fit);
    if (cmpc_launch_build(P, d.ns, d.ny, d.nu, d.m, c->stream))
      return fail("build kernel not instantiated for these dimensions (ns, ny, nu, m)");
    c->last_build = P.split ? CMPC_BUILD_SPLIT : CMPC_BUILD_WAVE;
  }
  if (check_launch("build kernel")) return -1;
  return tl.end();
}

static int build_params(cmpc_ctx* c, BuildParams& P) {
  const cmpc_dims& d = c->d;
  const cmpc_layout& L = c->L;
  std::memset(&P, 0, sizeof P);
  P.lin = c->lin_bound ? c->lin_bound : c->lin;
  P.cfg = c->cfg;
  P.u_old = c->u_old;
  P.qp = c->qp;
  P.nqp = c->nqp;
  P.S = d.S;
  P.p = d.p;
  P.nu_tot = d.nu_tot;
  P.ndist = d.ndist;
  P.nd = L.nd;
  P.rec_len = L.rec_len;
  P.qp_len = c->qp_len;
  P.off_A = L.off_A; P.off_B = L.off_B; P.off_C = L.off_C;
  P.off_f = L.off_f; P.off_x = L.off_x; P.off_y = L.off_y;
  P.nobs = L.nobs;
  P.co = c->co;
  int kd = 0, boff = d.ndist + L.nd, dmax = 1;
  for (int i = 0; i < d.nu_tot; ++i) {
    P.delay[i] = d.delay[i];
    P.dindex[i] = -1;
    if (d.delay[i] > 0) {
      P.dindex[i] = kd;
      P.dinput[kd] = i;
      P.dlen[kd] = d.delay[i];
      P.boff[kd] = boff;
      boff += d.delay[i] - 1;
      dmax = std::max(dmax, d.delay[i]);
      ++kd;
    }
  }
  P.dmax = dmax;
  // the LDS layout and the device's CU count are fixed per context: computed
  // once (the layout search and the attribute query are host time on every
  // launch of a small batch, whose kernels take tens of microseconds)
  if (!c->lds_layout_ok) {
    build_lds_layout(d, L, &c->lds_layout);
    c->lds_layout_ok = true;
  }
  {
    const BuildParams& T = c->lds_layout;
    P.lds_block = T.lds_block;
    P.yl_stride = T.yl_stride;
    P.lds_per_wave = T.lds_per_wave;
    std::memcpy(P.line_off, T.line_off, sizeof P.line_off);
    P.line_rs = T.line_rs;
    P.w_off = T.w_off;
    P.zs_off = T.zs_off;
    P.zl_stride = T.zl_stride;
    P.nbound = T.nbound;
    std::memcpy(P.bound, T.bound, sizeof P.bound);
  }
  if (L.rec_len > 2 * 64 * CMPC_REC_CHUNKS) return fail("lin record too long for the build kernel");
  const size_t lds_bytes = sizeof(double) * ((size_t)P.lds_block + (size_t)P.lds_per_wave * CMPC_BUILD_WAVES);
  if (lds_bytes > 160 * 1024) return fail("horizon/delays too long for the build kernel's LDS");
  {
    // persistent grid: the launcher caps this at (resident workgroups per CU,
    // from the occupancy query: registers and LDS) x CUs, so no workgroup
    // waits for a second round
    if (!c->cus) (void)hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device);
    P.cus = c->cus > 0 ? c->cus : 256;
    P.grid = std::max(1, (c->nqp + CMPC_BUILD_WAVES - 1) / CMPC_BUILD_WAVES);
  }
  cmpc_rows_layout(d, L.nd, L.nobs, L.rec_len, &P.rows);  // cached per dimension set
  return 0;
}

// working-set trace buffers for K iterations of every QP (CMPC_TRACE)
static int trace_buffers(cmpc_ctx* c, int K) {
  const size_t need = (size_t)c->nqp * K * 16;
  if (need > c->trace_cap) {
    if (c->trace) HIP_TRY(hipFree(c->trace));
    if (c->ntrace) HIP_TRY(hipFree(c->ntrace));
    c->trace = nullptr;
    c->ntrace = nullptr;
    HIP_TRY(hipMalloc(&c->trace, need));
    HIP_TRY(hipMalloc(&c->ntrace, sizeof(int32_t) * (size_t)c->nqp * K));
    c->trace_cap = need;
  }
  c->trace_K = K;
  return 0;
}

int cmpc_set_solve_variant(cmpc_ctx* c, int variant) {
  if (!c) return fail("null context");
  if (variant != CMPC_SOLVE_AUTO && variant != CMPC_SOLVE_LANE && variant != CMPC_SOLVE_ROWS)
    return fail("cmpc_set_solve_variant: unknown variant");
  c->solve_variant = variant;
  return 0;
}

int cmpc_last_solve_kernel(cmpc_ctx* c) {
  if (!c) return fail("null context");
  return c->last_solve;
}

// the iterate / init / get-input launch through the selected solve kernel
static int launch_solve(cmpc_ctx* c, const SolveParams& P, const char* who) {
  const int nV = c->L.nV, nu = c->d.nu, nVo = c->L.nVo;
  // AUTO: the row kernel for small batches of nV >= 6 QPs (centralized: the
  // lane kernel's nV = 8 solve is one long dependency chain per lane, 17 us
  // for one solve of 1 024 QPs against 9 us in rows, tools/time_small.py);
  // at nV = 4 up to four QPs per SIMD (K = 9: 7.7-7.8 vs 9.7-9.9 us from 2
  // to 1 024 QPs, profiles/r5k_small_batch.txt; in the bench's step loop
  // with the move applied 9.6-10.2 vs 11.6-12.1 us at 2 048 and 4 096 QPs,
  // p = 20, profiles/r6r_solver_variant_sweep.txt), the lane kernel above
  // (8 192 QPs: 11.9 vs 17.5 us)
  if (!c->cus) (void)hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device);
  const bool rows_small = nV >= 6 ? c->nqp < CMPC_SOLVE_ROWS_MAX_QP : c->nqp <= 16 * std::max(c->cus, 1);
  const bool want_rows = c->solve_variant == CMPC_SOLVE_ROWS || (c->solve_variant == CMPC_SOLVE_AUTO && rows_small);
  if (want_rows && cmpc_launch_solve_rows(P, nV, nu, nVo, c->stream) == 0) {
    c->last_solve = CMPC_SOLVE_ROWS;
    return 0;
  }
  if (c->solve_variant == CMPC_SOLVE_ROWS)
    return fail(std::string(who) + ": row solve kernel not available for these dimensions (S must divide 4)");
  if (cmpc_launch_solve(P, nV, nu, nVo, c->stream))
    return fail(std::string(who) + ": solve kernel not instantiated for these dimensions");
  c->last_solve = CMPC_SOLVE_LANE;
  return 0;
}

int cmpc_init_warmstart(cmpc_ctx* c) {
  if (!c) return fail("null context");
  if (ensure_cfg(c)) return -1;
  HIP_TRY(hipSetDevice(c->device));
  SolveParams P;
  solve_params(c, &P);
  P.init = 1;
  cmpc_launch_events = LaunchEvents{};  // untimed (a failed timed launch may have left them set)
  if (launch_solve(c, P, "cmpc_init_warmstart")) return -1;
  return check_launch("init kernel");
}

int cmpc_iterate(cmpc_ctx* c, int K, uint32_t flags) {
  if (!c) return fail("null context");
  if (K < 0) return fail("K must be >= 0");
  if (c->L.nuo != (c->d.S - 1) * c->d.nu)
    return fail("cmpc_iterate: the other controllers' plans are not in this context (S = 1, nu < nu_tot): "
                "use cmpc_get_input");
  if (ensure_cfg(c)) return -1;
  HIP_TRY(hipSetDevice(c->device));
  SolveParams P;
  solve_params(c, &P);
  P.K = K;
  P.flags = flags;
  if ((flags & CMPC_TRACE) && K > 0) {
    if (trace_buffers(c, K)) return -1;
    P.trace = c->trace;
    P.ntrace = c->ntrace;
  }
  TimedLaunch tl(c, CMPC_KERNEL_ITERATE);
  if (tl.begin()) return -1;
  if (launch_solve(c, P, "cmpc_iterate")) return -1;
  if (check_launch("iterate kernel")) return -1;
  return tl.end();
}

// DistributedController::GetInput (include/distributed_controller.h:206-226):
// one warm-started solve per slot with the other controllers' plans given.
int cmpc_get_input(cmpc_ctx* c, const double* du_last, uint32_t flags) {
  if (!c) return fail("null context");
  if (flags & CMPC_TRACE) return fail("cmpc_get_input: no trace");
  if (ensure_cfg(c)) return -1;
  if (c->L.nVo > 0 && !du_last) return fail("cmpc_get_input: du_last is needed (nu < nu_tot)");
  if (c->L.nVo == 0) return cmpc_iterate(c, 1, flags);  // full controller: SolveQP(qp_, u_old_)
  HIP_TRY(hipSetDevice(c->device));
  SolveParams P;
  solve_params(c, &P);
  P.K = 1;
  P.flags = flags;
  P.du_other = du_last;
  TimedLaunch tl(c, CMPC_KERNEL_ITERATE);
  if (tl.begin()) return -1;
  if (launch_solve(c, P, "cmpc_get_input")) return -1;
  if (check_launch("get-input kernel")) return -1;
  return tl.end();
}

int cmpc_get_input_host(cmpc_ctx* c, const double* du_last, uint32_t flags) {
  if (!c) return fail("null context");
  if (c->L.nVo == 0 || !du_last) return cmpc_get_input(c, nullptr, flags);
  HIP_TRY(hipSetDevice(c->device));
  const double* h[1] = {du_last};
  const size_t n[1] = {(size_t)c->nqp * c->L.nVo};
  const double* d[1];
  if (stage_host(c, h, n, 1, d)) return -1;
  const int rc = cmpc_get_input(c, d[0], flags);
  return stage_done(c) ? -1 : rc;
}

// DistributedController::UpdateU(du) (include/distributed_controller.h:145-152)
// with the caller's full input change: ObserveAPriori(du, u_old_), u_old_ += du.
int cmpc_update_u(cmpc_ctx* c, const double* du_full) {
  if (!c || !du_full) return fail("null argument");
  if (c->obs_plant < 0) return fail("cmpc_update_u: call cmpc_observer_init first");
  if (c->lin_bound) return fail("cmpc_update_u: records are bound externally");
  HIP_TRY(hipSetDevice(c->device));
  ObserverParams P;
  observer_params(c, &P);
  P.du_full = du_full;
  TimedLaunch tl(c, CMPC_KERNEL_OBSERVE_PRIOR);
  if (tl.begin()) return -1;
  if (cmpc_launch_observer(P, CMPC_OBS_PRIOR, c->stream))
    return fail("cmpc_update_u: no a-priori kernel instantiation for these dimensions");
  if (check_launch("observer a-priori kernel")) return -1;
  c->obs_steps++;  // the delay-block rings advance by one
  return tl.end();
}

int cmpc_update_u_host(cmpc_ctx* c, const double* du_full) {
  if (!c || !du_full) return fail("null argument");
  HIP_TRY(hipSetDevice(c->device));
  const double* h[1] = {du_full};
  const size_t n[1] = {(size_t)c->nqp * c->d.nu_tot};
  const double* d[1];
  if (stage_host(c, h, n, 1, d)) return -1;
  const int rc = cmpc_update_u(c, d[0]);
  return stage_done(c) ? -1 : rc;
}

int cmpc_coupled_validate(const cmpc_dims* d, int S_total, int S_local, int s_offset, size_t G_ext_len,
                          size_t du_all_len) {
  if (!d) return fail("cmpc_coupled_validate: null dims");
  cmpc_layout L;
  if (layout_of(d, &L)) return -1;
  const long long nqp_ll = (long long)d->B * d->S;
  if (S_local < 1 || nqp_ll % S_local || S_local % d->S)
    return fail("cmpc_coupled_iterate: S_local must divide B*S and be a multiple of S");
  if (S_total < S_local || S_total % S_local || s_offset < 0 || s_offset % S_local ||
      s_offset + S_local > S_total)
    return fail("cmpc_coupled_iterate: bad S_total / s_offset");
  // every read of the kernel must fall inside the caller's buffers: G_ext
  // holds nV x (S_total-1) nV per local QP, du_all the plans of all S_total
  // sub-controllers of the B scenarios (rank-major, S_total / S_local ranks)
  const size_t nV = (size_t)L.nV, nqp = (size_t)nqp_ll, B = nqp / (size_t)S_local;
  const size_t need_g = nV * (size_t)(S_total - 1) * nV * nqp;
  const size_t need_d = (size_t)S_total * B * nV;
  if (G_ext_len < need_g)
    return fail("cmpc_coupled_iterate: G_ext holds " + std::to_string(G_ext_len) + " doubles, the kernel reads " +
                std::to_string(need_g) + " (nV*(S_total-1)*nV per local QP)");
  if (du_all_len < need_d)
    return fail("cmpc_coupled_iterate: du_all holds " + std::to_string(du_all_len) + " doubles, the kernel reads " +
                std::to_string(need_d) + " (S_total x B x nV: every rank's plans; does S_local x world cover "
                "S_total?)");
  return 0;
}

int cmpc_coupled_iterate(cmpc_ctx* c, int S_total, int S_local, int s_offset, const double* G_ext,
                         size_t G_ext_len, const double* du_all, size_t du_all_len, double* du_out,
                         uint32_t flags) {
  if (!c) return fail("null context");
  if (!G_ext || !du_all) return fail("cmpc_coupled_iterate: null argument");
  if (cmpc_coupled_validate(&c->d, S_total, S_local, s_offset, G_ext_len, du_all_len)) return -1;
  if (ensure_cfg(c)) return -1;
  HIP_TRY(hipSetDevice(c->device));
  CoupledParams P;
  std::memset(&P, 0, sizeof P);
  P.qp = c->qp;
  P.cfg = c->cfg;
  P.co = c->co;
  P.u_old = c->u_old;
  P.du_old = c->du_old;
  P.ws = c->ws;
  P.du = c->du;
  P.du_out = du_out;
  P.status = c->status;
  P.nwsr = c->nwsr;
  P.G_ext = G_ext;
  P.du_all = du_all;
  P.nqp = c->nqp;
  P.qp_len = c->qp_len;
  P.nu_tot = c->d.nu_tot;
  P.S_cfg = c->d.S;
  P.S_total = S_total;
  P.S_local = S_local;
  P.s_offset = s_offset;
  P.B = c->nqp / S_local;
  P.flags = flags;
  TimedLaunch tl(c, CMPC_KERNEL_ITERATE);
  if (tl.begin()) return -1;
  if (cmpc_launch_coupled(P, c->L.nV, c->d.nu, c->stream))
    return fail("coupled kernel not instantiated for these dimensions (nV = 4, nu = 2)");
  if (check_launch("coupled kernel")) return -1;
  return tl.end();
}

int cmpc_set_step_variant(cmpc_ctx* c, int variant) {
  if (!c) return fail("null context");
  if (variant != CMPC_STEP_AUTO && variant != CMPC_STEP_SPLIT && variant != CMPC_STEP_FUSED)
    return fail("cmpc_set_step_variant: unknown variant");
  c->step_variant = variant;
  return 0;
}

int cmpc_last_step_fused(cmpc_ctx* c) {
  if (!c) return fail("null context");
  return c->last_step_fused;
}

// GetNextInputWithTiming's device part: the build, then K Jacobi iterations.
// On small batches one fused launch (the build kernel solves its own QPs:
// no launch gap, no HBM round trip of H, f, G); else cmpc_build + cmpc_iterate.
int cmpc_step(cmpc_ctx* c, int K, uint32_t flags) {
  if (!c) return fail("null context");
  if (K < 0) return fail("K must be >= 0");
  // AUTO fuses small batches on the build kernel AUTO would pick anyway: the
  // one-QP-per-wave kernel under one row group per SIMD (its own row solver
  // for centralized QPs, SURVEY config 5: 40.1 vs 44.8 us per step; the lane
  // solver of wave 0 after a workgroup barrier for S = 2, 4), the row kernel
  // from one row group per SIMD up to 16 384 QPs (config 2)
  if (!c->cus) (void)hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device);
  // (AUTO fuses nV >= 6 steps from one to four QPs per CU at p >= 50 only:
  // below one per CU the role-split build and the iterate kernel are faster
  // (cent-ser B = 1 21.8 vs 24.4 us); in that range fused wins by 2-3 %
  // (config 5: 37.3 vs 38.1 us with the move; ser-cent p = 100 512 QPs 37.6
  // vs 38.4 us) but loses at p = 20 (15.0 vs 13.9 us), and above it the split
  // steps win: 2 048 QPs 17.1 vs 28.3 us (par-cent p = 20) and 60.1 vs 73.0 us
  // (ser-cent p = 100), 8 192 QPs 112 vs 135 us (par-cent p = 200)
  // (tools/step_variant_ab.py, profiles/r6r_step_variant_sweep.txt; it costs
  // 3 % at 4 096 QPs for p = 50 and 200).  nV = 4 steps are two launches at
  // every size (coop-par 1 024 QPs 17.8 vs 18.6 us, config 2 26.4 vs
  // 54.1 us; profiles/r5j_split_step_ab.txt, profiles/r5k_small_batch.txt))
  const int cus1 = std::max(c->cus, 1);
  const bool auto_fuse = c->L.nV >= 6 && c->nqp > cus1 && c->nqp <= 4 * cus1 && c->d.p >= 50;
  const bool want = c->step_variant == CMPC_STEP_FUSED ||
                    (c->step_variant == CMPC_STEP_AUTO && auto_fuse &&
                     c->build_variant == CMPC_BUILD_AUTO && c->solve_variant == CMPC_SOLVE_AUTO);
  if (want && K > 0 && c->L.nuo == (c->d.S - 1) * c->d.nu) {
    if (ensure_cfg(c)) return -1;
    HIP_TRY(hipSetDevice(c->device));
    BuildParams P;
    if (build_params(c, P)) return -1;
    solve_params(c, &P.sv);
    P.sv.K = K;
    P.sv.flags = flags;
    if ((flags & CMPC_TRACE) && trace_buffers(c, K)) return -1;
    if (flags & CMPC_TRACE) {
      P.sv.trace = c->trace;
      P.sv.ntrace = c->ntrace;
    }
    TimedLaunch tl(c, CMPC_KERNEL_STEP);
    if (tl.begin()) return -1;
    const cmpc_dims& d = c->d;
    // the build kernel AUTO would pick: one QP per wave below one row group per
    // SIMD, else four QPs per wave
    const bool rows_fill = (c->nqp + 3) / 4 >= 4 * P.cus;
    int rc = -1, kind = CMPC_BUILD_ROWS, solver = CMPC_SOLVE_ROWS;
    if (!rows_fill) {
      rc = cmpc_launch_step_wave(P, d.ns, d.ny, d.nu, d.m, c->stream, &solver);
      kind = CMPC_BUILD_WAVE;
    }
    // AUTO leaves the row kernel's fused step with the lane solver (nV <= 4)
    // to the two launches, measured faster on every box this round (config 2:
    // 32.0-32.2 vs 33.7-33.9 us back to back, profiles/r4i_small_batch.txt)
    const bool rows_lane = c->L.nV <= 4 && c->step_variant == CMPC_STEP_AUTO;
    if (rc && !(rows_fill && rows_lane)) {
      rc = cmpc_launch_step_rows(P, d.ns, d.ny, d.nu, d.m, c->stream, &solver);
      kind = CMPC_BUILD_ROWS;
    }
    if (rc == 0) {
      if (check_launch("fused step kernel")) return -1;
      c->last_build = kind;
      c->last_solve = solver;
      c->last_step_fused = 1;
      return tl.end();
    }
    cmpc_launch_events = LaunchEvents{};
    if (c->step_variant == CMPC_STEP_FUSED)
      return fail("cmpc_step: no fused step kernel for these dimensions");
  }
  c->last_step_fused = 0;
  if (cmpc_build(c)) return -1;
  return cmpc_iterate(c, K, flags);
}

int cmpc_synchronize(cmpc_ctx* c) {
  if (!c) return fail("null context");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int cmpc_download(cmpc_ctx* c, double* du, int32_t* status, int32_t* nwsr) {
  if (!c) return fail("null context");
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)c->nqp;
  const size_t b_du = sizeof(double) * n * c->L.nV, b_i = sizeof(int32_t) * n;
  const size_t o_st = c->out_st, o_nw = c->out_nw;
  if (c->out_host) {  // the kernels wrote the block in place
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (du) std::memcpy(du, c->out_block, b_du);
    if (status) std::memcpy(status, c->out_block + o_st, b_i);
    if (nwsr) std::memcpy(nwsr, c->out_block + o_nw, b_i);
    return 0;
  }
  // device -> page-locked buffer (DMA; one copy of the du | status | nwsr
  // block when all are asked for), then host copies after one sync
  if (pinned_acquire(c->pin_out, c->out_len)) return -1;
  char* h = c->pin_out.buf;
  if (du && status && nwsr) {
    HIP_TRY(hipMemcpyAsync(h, c->out_block, c->out_len, hipMemcpyDeviceToHost, c->stream));
  } else {
    if (du) HIP_TRY(hipMemcpyAsync(h, c->du, b_du, hipMemcpyDeviceToHost, c->stream));
    if (status) HIP_TRY(hipMemcpyAsync(h + o_st, c->status, b_i, hipMemcpyDeviceToHost, c->stream));
    if (nwsr) HIP_TRY(hipMemcpyAsync(h + o_nw, c->nwsr, b_i, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (du) std::memcpy(du, h, b_du);
  if (status) std::memcpy(status, h + o_st, b_i);
  if (nwsr) std::memcpy(nwsr, h + o_nw, b_i);
  return 0;
}

int cmpc_download_qp(cmpc_ctx* c, double* H, double* f, double* G) {
  if (!c) return fail("null context");
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)c->nqp;
  const int nV = c->L.nV, nVo = c->L.nVo;
  std::vector<double> buf(n * c->qp_len);
  HIP_TRY(hipMemcpyAsync(buf.data(), c->qp, sizeof(double) * buf.size(), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (size_t q = 0; q < n; ++q) {
    const double* r = buf.data() + q * c->qp_len;
    if (H) std::memcpy(H + q * nV * nV, r, sizeof(double) * nV * nV);
    if (f) std::memcpy(f + q * nV, r + nV * nV, sizeof(double) * nV);
    if (G && nVo) std::memcpy(G + q * nV * nVo, r + nV * nV + nV, sizeof(double) * nV * nVo);
  }
  return 0;
}

int cmpc_download_trace(cmpc_ctx* c, uint8_t* trace, int32_t* ntrace) {
  if (!c) return fail("null context");
  if (!c->trace) return fail("no traced iterate (pass CMPC_TRACE to cmpc_iterate)");
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)c->nqp * c->trace_K;
  if (trace) HIP_TRY(hipMemcpyAsync(trace, c->trace, n * 16, hipMemcpyDeviceToHost, c->stream));
  if (ntrace) HIP_TRY(hipMemcpyAsync(ntrace, c->ntrace, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int cmpc_enable_timing(cmpc_ctx* c, int enable) {
  if (!c) return fail("null context");
  if (resolve_timing(c)) return -1;
  const int all = (1 << CMPC_KERNEL_COUNT) - 1;
  c->timing = enable == 0 ? 0 : enable == 1 ? all : (enable >> 1) & all;
  for (int k = 0; k < CMPC_KERNEL_COUNT; ++k) {
    c->tot_ms[k] = 0;
    c->launches[k] = 0;
    c->timing_seq[k] = 0;
  }
  return 0;
}

int cmpc_set_timing_stride(cmpc_ctx* c, int stride) {
  if (!c) return fail("null context");
  if (stride < 1) return fail("cmpc_set_timing_stride: stride must be >= 1");
  c->timing_stride = stride;
  return 0;
}

int cmpc_kernel_time(cmpc_ctx* c, int kernel, double* total_ms, int64_t* launches) {
  if (!c) return fail("null context");
  if (kernel < 0 || kernel >= CMPC_KERNEL_COUNT) return fail("unknown kernel id");
  HIP_TRY(hipSetDevice(c->device));
  if (resolve_timing(c)) return -1;
  if (total_ms) *total_ms = c->tot_ms[kernel];
  if (launches) *launches = c->launches[kernel];
  return 0;
}

int cmpc_qp_solve_batch(int device, int n, int nu, int nqp, const double* H, const double* g,
                        const double* lb, const double* ub, const double* lbA, const double* ubA,
                        const uint32_t* ws_in, int max_chg, double* x, int32_t* status,
                        int32_t* nchg, uint32_t* ws_out, uint8_t* trace, int32_t* ntrace) {
  return cmpc_qp_solve_batch_map(device, n, nu, 0, nqp, H, g, nullptr, nullptr, lb, ub, lbA, ubA, ws_in, max_chg, x,
                                 status, nchg, ws_out, trace, ntrace);
}

// cmpc_qp_solve_batch(_map): host arrays in, host arrays out.  The dimensions
// are checked against the kernel instances before anything is allocated, the
// device buffers are released on every exit path, and only the stream of the
// launch is waited for.
int cmpc_qp_solve_batch_map(int device, int n, int nu, int nvo, int nqp, const double* H, const double* f,
                            const double* G, const double* d, const double* lb, const double* ub,
                            const double* lbA, const double* ubA, const uint32_t* ws_in, int max_chg, double* x,
                            int32_t* status, int32_t* nchg, uint32_t* ws_out, uint8_t* trace, int32_t* ntrace) {
  if (nvo < 0) return fail("cmpc_qp_solve_batch_map: nvo < 0");
  if (nvo > 0 && (!G || !d)) return fail("cmpc_qp_solve_batch_map: G and d required for nvo > 0");
  if (nvo > 0 ? !cmpc_qp_batch_map_supported(n, nu, nvo) : !cmpc_qp_batch_supported(n, nu))
    return fail(nvo > 0 ? "map-form qp batch kernel not instantiated for (n, nu, nvo) = (" + std::to_string(n) +
                              ", " + std::to_string(nu) + ", " + std::to_string(nvo) + ")"
                        : "qp batch kernel not instantiated for (n, nu) = (" + std::to_string(n) + ", " +
                              std::to_string(nu) + ")");
  if (nqp <= 0) return 0;
  HIP_TRY(hipSetDevice(device));
  const size_t q = (size_t)nqp;
  struct Bufs {  // scope guard: every buffer allocated below is freed on return
    std::vector<void*> p;
    ~Bufs() {
      for (void* b : p) (void)hipFree(b);
    }
  } bufs;
  auto alloc = [&](auto** ptr, size_t bytes) -> hipError_t {
    void* v = nullptr;
    const hipError_t e = hipMalloc(&v, bytes ? bytes : 8);
    if (e == hipSuccess) bufs.p.push_back(v);
    *ptr = static_cast<std::remove_pointer_t<decltype(ptr)>>(v);
    return e;
  };
  double *dH, *dg, *dG = nullptr, *dd = nullptr, *dlb, *dub, *dlbA, *dubA, *dx;
  uint32_t *dws, *dwo;
  int32_t *dst, *dnc, *dnt;
  uint8_t* dtr;
  HIP_TRY(alloc(&dH, sizeof(double) * q * n * n));
  HIP_TRY(alloc(&dg, sizeof(double) * q * n));
  if (nvo > 0) {
    HIP_TRY(alloc(&dG, sizeof(double) * q * n * nvo));
    HIP_TRY(alloc(&dd, sizeof(double) * q * nvo));
  }
  HIP_TRY(alloc(&dlb, sizeof(double) * q * n));
  HIP_TRY(alloc(&dub, sizeof(double) * q * n));
  HIP_TRY(alloc(&dlbA, sizeof(double) * q * n));
  HIP_TRY(alloc(&dubA, sizeof(double) * q * n));
  HIP_TRY(alloc(&dx, sizeof(double) * q * n));
  HIP_TRY(alloc(&dws, sizeof(uint32_t) * q));
  HIP_TRY(alloc(&dwo, sizeof(uint32_t) * q));
  HIP_TRY(alloc(&dst, sizeof(int32_t) * q));
  HIP_TRY(alloc(&dnc, sizeof(int32_t) * q));
  HIP_TRY(alloc(&dnt, sizeof(int32_t) * q));
  HIP_TRY(alloc(&dtr, 16 * q));
  HIP_TRY(hipMemcpy(dH, H, sizeof(double) * q * n * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dg, f, sizeof(double) * q * n, hipMemcpyHostToDevice));
  if (nvo > 0) {
    HIP_TRY(hipMemcpy(dG, G, sizeof(double) * q * n * nvo, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dd, d, sizeof(double) * q * nvo, hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMemcpy(dlb, lb, sizeof(double) * q * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dub, ub, sizeof(double) * q * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dlbA, lbA, sizeof(double) * q * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dubA, ubA, sizeof(double) * q * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dws, ws_in, sizeof(uint32_t) * q, hipMemcpyHostToDevice));
  QpBatchParams P{dH, dg, dlb, dub, dlbA, dubA, dws, dx, dst, dnc, dnt, dwo, dtr, nqp, max_chg, dG, dd, nvo};
  const int lr = nvo > 0 ? cmpc_launch_qp_batch_map(P, n, nu, nvo, nullptr) : cmpc_launch_qp_batch(P, n, nu, nullptr);
  if (lr) return fail("qp batch kernel not instantiated");
  if (check_launch("qp batch kernel")) return -1;
  HIP_TRY(hipStreamSynchronize(nullptr));
  HIP_TRY(hipMemcpy(x, dx, sizeof(double) * q * n, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(status, dst, sizeof(int32_t) * q, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(nchg, dnc, sizeof(int32_t) * q, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(ws_out, dwo, sizeof(uint32_t) * q, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(trace, dtr, 16 * q, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(ntrace, dnt, sizeof(int32_t) * q, hipMemcpyDeviceToHost));
  return 0;
}

}  // extern "C"
