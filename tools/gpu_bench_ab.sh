#!/bin/bash
# Bench-line A/B: the product library and each library in $LIBS, alternately,
# twice, each a full `bench.py --no-cpu` run; prints value, build/iterate ms
# and the build roofline fraction per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/bab.log
for i in 1 2; do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so $LIBS; do
    CMPC_LIBRARY=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS:-100} > gpurun_out/bab_one.json 2>/dev/null || exit $?
    python -c "
import json,sys; d=json.load(open('gpurun_out/bab_one.json')); k=d['kernels_ms_per_step']
print('$lib', round(d['value']/1e9,4), round(d['ms_per_step'],4), round(k['build'],4), round(k['iterate'],4), round(d['roofline']['frac'],4))" >> gpurun_out/bab.log
  done
done
cat gpurun_out/bab.log
