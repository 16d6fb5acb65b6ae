#!/bin/bash
# Coupled (config 4) kernel A/B: parity tests on the current library, then
# tools/bench_coupled.py with ab/libcmpc_old.so (if present) and the current one.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-cab}
timeout -k 10 300 python -u -m pytest tests/test_coupled.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/test_$TAG.log 2>&1 || exit $?
for lib in old new; do
  if [ $lib = old ]; then [ -f ab/libcmpc_old.so ] || continue; export CMPC_LIBRARY=$PWD/ab/libcmpc_old.so; else unset CMPC_LIBRARY; fi
  for sl in 64 8; do
    timeout -k 10 300 python tools/bench_coupled.py --s-local $sl --batch 4096 --steps 20 > gpurun_out/coupled_${TAG}_${lib}_$sl.json 2> gpurun_out/coupled_${TAG}_${lib}_$sl.err || exit $?
  done
done
unset CMPC_LIBRARY
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 tools/bench_coupled.py --s-local 64 --batch 4096 --steps 10 > gpurun_out/coupledprof_$TAG.json 2> gpurun_out/coupledprof_$TAG.err || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace -T --kernel-include-regex 'cmpc_coupled' --pmc FETCH_SIZE -d gpurun_out/pmc${TAG}_fetch -o run --output-format csv -- python3 tools/bench_coupled.py --s-local 64 --batch 4096 --steps 2 --warmup 1 --settle-seconds 0 > gpurun_out/pmc${TAG}_fetch.json 2>&1 || exit $?
echo ALLDONE
