#!/bin/bash
# Round 3 build-kernel change check: all GPU tests, the bench A/B against
# ab/libcmpc_u4.so (the previous unroll), and DESIGN §3.0's build table.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-r3g}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/test_$TAG.log 2>&1 || exit $?
LIBS=ab/libcmpc_u4.so bash tools/gpu_bench_ab.sh || exit $?
cp gpurun_out/bab.log gpurun_out/bab_$TAG.log
bash tools/gpu_build_table.sh > gpurun_out/btab_$TAG.txt || exit $?
echo ALLDONE
