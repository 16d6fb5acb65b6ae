#!/bin/bash
# Launch-gap and iterate diagnostics: step time with/without timing events,
# a kernel trace of the bench step (GPU-side gaps between kernels), and the
# iterate kernel on the bench batch and with no active constraints.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/time_step_gaps.py > gpurun_out/gaps.log 2>&1 || exit $?
timeout -k 10 200 python tools/time_iterate.py 65536 9 >> gpurun_out/gaps.log 2>&1 || exit $?
CMPC_TI_UNCONSTRAINED=1 timeout -k 10 200 python tools/time_iterate.py 65536 9 >> gpurun_out/gaps.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gtrace -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 2 --no-cpu --settle-seconds 0.1 > gpurun_out/gtrace.json 2> gpurun_out/gtrace.err || exit $?
grep -v amdgpu.ids gpurun_out/gaps.log
