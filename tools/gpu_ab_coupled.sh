#!/bin/bash
# A/B of the coupled iterate (config 4's 64-sub-controller system at world 1)
# between the in-tree library and ab/<v>/libcmpc.so for each named variant,
# alternating, after the coupled GPU tests on the in-tree one.
#   usage: ROUNDS=3 tools/gpu_ab_coupled.sh TAG v1 [v2 ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=$1; shift; OUT=gpurun_out/abc_$TAG.txt; : > $OUT
timeout -k 10 300 python -u -m pytest tests/test_coupled.py tests/test_multirank.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/abc_tests.log 2>&1; rc=$?; tail -2 gpurun_out/abc_tests.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq ${ROUNDS:-3}); do
  for v in new "$@"; do
    if [ $v = new ]; then L=""; else L=ab/$v/libcmpc.so; fi
    CMPC_LIBRARY=$L timeout -k 10 300 python3 -c "
import sys, json; sys.path.insert(0, 'compressor-mpc_amd')
from cmpc.coupled import run_coupled_bench
r = run_coupled_bench(0, 1, 0, S_local=64, S_total=64, B=4096, steps=10, settle_seconds=0.25)
print(sys.argv[1], sys.argv[2], 'ms_per_step %.4f iterate_ms %.4f G_ext_hbm_frac %.3f ok %.3f' % (r['elapsed_s'] / r['steps'] * 1e3, r['iterate_kernel_ms'], r['G_ext_hbm_frac'], r['qp_status_ok_fraction']))
" $v $i >> $OUT 2> gpurun_out/abc_$v$i.err || exit $?
  done
done
cat $OUT
