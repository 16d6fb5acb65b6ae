#!/bin/bash
# B = 1 GetNextInput latency A/B through the C++ adapter
# (tests/cpp/nerve_center_latency): the in-tree libcmpc.so ("new") against
# ab/<base>/libcmpc.so (LD_LIBRARY_PATH overrides the harness's RUNPATH),
# alternating over ROUNDS rounds, coop-par p = 50 and cent-ser p = 100.
#   usage: ROUNDS=3 tools/gpu_ab_b1.sh TAG BASE
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=$1; BASE=$2
OUT=gpurun_out/abb1_$TAG.txt; : > $OUT
export PYTHONPATH=$PWD/compressor-mpc_amd
for cfg in "par coop" "ser cent"; do
  set -- $cfg
  python3 -c "from cmpc.configs import reference_setup; open('gpurun_out/setup-$2-$1','w').write(reference_setup('$1','$2').text())" || exit 1
done
for i in $(seq ${ROUNDS:-3}); do
  for v in new $BASE; do
    for cfg in "par coop 50" "ser cent 100"; do
      set -- $cfg
      if [ $v = new ]; then LP=""; else LP=$PWD/ab/$v; fi
      r=$(LD_LIBRARY_PATH=$LP timeout -k 10 120 tests/cpp/nerve_center_latency gpurun_out/setup-$2-$1 $1 $2 $3 400 2>&1 | tail -1) || exit 1
      echo "$v $i $cfg $r" >> $OUT
    done
  done
done
cat $OUT
