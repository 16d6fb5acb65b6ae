#!/bin/bash
# Full GPU suite, then a bench line (closed-loop observer timings).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tq.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tq.log; tail -4 gpurun_out/tq.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bq.json 2> gpurun_out/bq.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bq.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['kernels_ms_per_step']['iterate']); print(json.dumps(d['closed_loop_device_resident']))"
