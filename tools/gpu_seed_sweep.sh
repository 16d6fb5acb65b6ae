#!/bin/bash
# Row-kernel LDS layout search seeds (CMPC_ROWS_SEED) at p = 50: build time per seed, twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/seed.log
for i in 1 2; do
  for sd in 0x5eed 1 2 3 4 5 6 7 8 9 10; do
    echo "seed $sd: $(CMPC_ROWS_SEED=$sd CMPC_TB_VARIANT=rows timeout -k 10 100 python tools/time_build.py 65536 50 2>&1 | grep -v amdgpu.ids)" >> gpurun_out/seed.log || exit 1
  done
done
cat gpurun_out/seed.log
