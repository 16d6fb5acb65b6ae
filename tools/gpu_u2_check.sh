cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/u2_tests.log 2>&1; rc=$?; tail -2 gpurun_out/u2_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc_c3.sh
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --configs-only --no-cpu > gpurun_out/u2_cfg$i.json 2> gpurun_out/u2_cfg$i.err || exit $?
python3 -c "
import json,sys; c=json.loads(open(sys.argv[1]).read().splitlines()[-1])['configs']
print(' '.join('c%s build_us %.2f frac %.4f step_us %.2f' % (k, c[k]['build_ms']*1e3, c[k]['build_roofline']['frac'], c[k]['ms_per_step']*1e3) for k in ('2','3','5')))" gpurun_out/u2_cfg$i.json; done
