#!/bin/bash
# Round 3: GPU tests, the build table and the bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-r3c}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/test_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/test_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 bash tools/gpu_build_table.sh > gpurun_out/btab_$TAG.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
echo ALLDONE
