#!/bin/bash
# Closed-loop driver timing (plant simulation + observer + build + K
# iterations + delay line, all on the device): the reference's single
# scenario and a 65 536-scenario batch, plus a kernel-trace summary.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 1 65536; do
  timeout -k 10 300 python tools/run_closed_loop.py par coop --batch $B --steps 100 --perturb 0.002 \
    > gpurun_out/cl_$B.json 2> gpurun_out/cl_$B.err || exit $?
  tail -1 gpurun_out/cl_$B.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/clprof -o run --output-format csv -- \
  python3 tools/run_closed_loop.py par coop --batch 65536 --steps 50 --perturb 0.002 > gpurun_out/clprof.json 2> gpurun_out/clprof.err || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/clprof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:9.1f} us  total% {float(r['Percentage']):5.1f}")
PY
