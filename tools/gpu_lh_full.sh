#!/bin/bash
# Full GPU suite, then the long-horizon timing (tools/gpu_long_horizon.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tq.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tq.log; tail -3 gpurun_out/tq.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_long_horizon.sh
