#!/bin/bash
# One GPU round: parity tests, smoke, bench, kernel-trace profile.
# Every GPU step has its own time limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/test_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/test_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/benchprof_$TAG.json 2> gpurun_out/benchprof_$TAG.err || exit $?
echo ALLDONE
