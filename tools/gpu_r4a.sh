#!/bin/bash
# round-4 small-batch work: parity of the row solver / fused step, then timings
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-r4a}
timeout -k 10 900 python -u -m pytest tests/test_gpu_small_batch.py tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "small_batch or row_solver or fused or step_matches or step_other or solver_bitexact or survey" > gpurun_out/test_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/test_$TAG.log
[ $rc -ne 0 ] && exit $rc
tools/gpu_small_ab.sh $TAG "c5 c2 b1 c1b1" base ilp2 ilp4
