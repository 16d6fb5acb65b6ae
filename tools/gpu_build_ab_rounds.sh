#!/bin/bash
# Build-kernel A/B at the bench configuration (coop-par p = 50, 65 536
# scenarios, tools/time_build.py settled, $N event-timed builds per run):
# the product library and each library in $LIBS alternately, ${ROUNDS:-4} rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/bab_rounds.log
for i in $(seq ${ROUNDS:-4}); do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so $LIBS; do
    r=$(CMPC_LIBRARY=$PWD/$lib CMPC_TB_VARIANT=rows CMPC_TB_N=${N:-400} timeout -k 10 120 python tools/time_build.py 65536 50 2>/dev/null | grep build) || exit $?
    echo "$lib $r" >> gpurun_out/bab_rounds.log
  done
done
cat gpurun_out/bab_rounds.log
