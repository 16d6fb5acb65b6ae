#!/bin/bash
# Headline A/B: `bench.py --headline-only --no-cpu` with the product library
# and each library in $LIBS, alternately, ${ROUNDS:-3} times; prints value,
# ms per step, build / iterate ms and the build roofline fraction per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/hab.log
for i in $(seq ${ROUNDS:-3}); do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so $LIBS; do
    CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python bench.py --headline-only --no-cpu --steps ${STEPS:-100} > gpurun_out/hab_one.json 2>/dev/null || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/hab_one.json')); k=d['kernels_ms_per_step']
print('$lib', round(d['value']/1e9,4), round(d['ms_per_step'],4), round(k['build'],4), round(k['iterate'],4), round(d['roofline']['frac'],4))" >> gpurun_out/hab.log
  done
done
cat gpurun_out/hab.log
