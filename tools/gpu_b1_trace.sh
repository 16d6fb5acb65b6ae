#!/bin/bash
# B = 1 step latency through the C++ adapter: host clock per GetNextInput,
# then one kernel + HIP-API trace of the same loop (no counters) to split the
# step into kernels, copies and host-side gaps.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-b1}
export PYTHONPATH=$PWD/compressor-mpc_amd
for cfg in "par coop 50" "ser cent 100"; do
  set -- $cfg
  python3 -c "from cmpc.configs import reference_setup; open('gpurun_out/setup-$2-$1','w').write(reference_setup('$1','$2').text())" || exit 1
  echo "== $cfg" >> gpurun_out/b1_$TAG.txt
  timeout -k 10 120 tests/cpp/nerve_center_latency gpurun_out/setup-$2-$1 $1 $2 $3 400 >> gpurun_out/b1_$TAG.txt 2>&1 || exit $?
done
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --stats -d gpurun_out/b1trace_$TAG -o run --output-format csv -- \
  tests/cpp/nerve_center_latency gpurun_out/setup-coop-par par coop 50 200 >> gpurun_out/b1_$TAG.txt 2>&1 || exit $?
echo ALLDONE >> gpurun_out/b1_$TAG.txt
