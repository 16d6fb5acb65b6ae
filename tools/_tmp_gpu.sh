#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --configs-only --no-cpu > gpurun_out/cs3_configs.json 2> gpurun_out/cs3_configs.err || exit $?
bash tools/gpu_b1_trace.sh cs3 || exit $?
echo ALLDONE
