#!/bin/bash
# Closed-loop kernel A/B: bench.py's closed-loop sections (scenario-mode and
# per-QP producer, observer kernels, build, iterate) with the product library
# and each library in $LIBS, alternately, twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/clab.log
for i in 1 2; do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so $LIBS; do
    CMPC_LIBRARY=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps 20 > gpurun_out/clab_one.json 2>/dev/null || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/clab_one.json'))['closed_loop_device_resident']
w=d['with_observer']; p=d['with_plant']
print('$lib', 'step', round(d['ms_per_step'],4), 'produce', round(d['kernels_ms']['produce'],4),
      '| obs step', round(w['ms_per_step'],4), {k: round(v,4) for k,v in w['kernels_ms'].items()},
      '| plant step', round(p['ms_per_step'],4))" >> gpurun_out/clab.log
  done
done
cat gpurun_out/clab.log
