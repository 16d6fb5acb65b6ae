cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_coupled.py tests/test_multirank.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cpl_tests.log 2>&1; rc=$?; tail -3 gpurun_out/cpl_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 300 python3 -c "
import sys, json; sys.path.insert(0, 'compressor-mpc_amd')
from cmpc.coupled import run_coupled_bench
r = run_coupled_bench(0, 1, 0, S_local=64, S_total=64, B=4096, steps=10, settle_seconds=0.25)
print('blocked', sys.argv[1], 'ms_per_step %.4f iterate_ms %.4f G_ext_hbm_frac %.3f ok %.3f' % (r['elapsed_s'] / r['steps'] * 1e3, r['iterate_kernel_ms'], r['G_ext_hbm_frac'], r['qp_status_ok_fraction']))
" $i >> gpurun_out/cpl_ab.txt 2> gpurun_out/cpl_$i.err || exit $?
done
cat gpurun_out/cpl_ab.txt
