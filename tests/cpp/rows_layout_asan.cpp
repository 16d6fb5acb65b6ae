// Host-side check of the row build kernel's LDS layout search
// (compressor-mpc_amd/csrc/rows_layout.cpp) under AddressSanitizer and
// UndefinedBehaviorSanitizer: random dimension sets (plants, controller
// types, horizons, move counts, delays), every layout the search returns
// checked for the invariants the kernel relies on.  Built by the Makefile's
// rows_layout_asan target with rows_layout.cpp instrumented; the other
// symbols come from libcmpc.so.  Prints "ok <n>" or the first violation.
#include <cstdio>
#include <random>

#include "../../compressor-mpc_amd/csrc/cmpc_internal.h"

static int fail(const char* what, const cmpc_dims& d) {
  std::printf("FAIL %s: ns %d ny %d nu %d m %d p %d S %d delays %d %d %d %d\n", what, d.ns, d.ny, d.nu,
              d.m, d.p, d.S, d.delay[0], d.delay[1], d.delay[2], d.delay[3]);
  return 1;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 400;
  std::mt19937 rng(12345);
  auto pick = [&](int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); };
  int checked = 0, usable = 0;
  for (int it = 0; it < n; ++it) {
    cmpc_dims d{};
    const bool par = pick(0, 1);
    d.ns = par ? 11 : 10;
    d.ndist = 4;
    d.nu_tot = 4;
    const int ct = pick(0, 2);  // cent, coop, ncoop
    d.nu = ct == 0 ? 4 : 2;
    d.S = ct == 0 ? 1 : 2;
    d.ny = ct == 2 ? 2 : (par ? 3 : 4);
    d.p = pick(2, 250);
    d.m = pick(1, 2);
    if (d.m > d.p) d.m = d.p;
    for (int c = 0; c < 4; ++c) d.delay[c] = 0;
    d.delay[1] = pick(2, 120);
    d.delay[3] = pick(2, 120);
    d.B = 64;
    cmpc_layout L;
    if (cmpc_layout_of(&d, &L)) continue;
    RowsLayout R;
    cmpc_rows_layout(d, L.nd, L.nobs, L.rec_len, &R);
    ++checked;
    if (!R.ok) continue;
    ++usable;
    const long lds = 8L * (R.lds_block + 4L * R.per_wave);
    if (lds > 160 * 1024) return fail("LDS over 160 KB", d);
    if (R.nseg < 0 || R.nseg > CMPC_ROWS_NSEG) return fail("segment count", d);
    for (int i = 0; i < R.nseg; ++i) {
      if (R.seg[i] <= 0 || R.seg[i] >= d.p) return fail("segment bound outside (0, p)", d);
      if (i && R.seg[i] <= R.seg[i - 1]) return fail("segments not ascending", d);
    }
    if (4 * R.LQ > R.per_wave || R.w_off + 4 * L.nd * R.WL > R.per_wave)
      return fail("regions outside the wave's LDS", d);
    if (R.U != cmpc_rows_unroll(d.ny) || R.dump_off + R.U * d.ny > R.LQ || R.zr_off + R.U * d.ny > R.LQ)
      return fail("dump / zero areas outside the line block", d);
    for (int c = 0; c < d.nu_tot; ++c)
      if (R.lo[c] < 0 || R.lo[c] >= R.LQ) return fail("line offset outside the line block", d);
    if (R.uw_off + d.S * d.nu * d.nu > R.lds_block) return fail("tables outside the block", d);
    const double cyc = cmpc_rows_layout_conflicts(d, L.nd, R, 0);
    if (!(cyc >= 0.0 && cyc < 1e6)) return fail("conflict model", d);
  }
  std::printf("ok %d checked, %d with a row layout\n", checked, usable);
  return 0;
}
