#!/bin/bash
# Build-kernel timing sweep over horizons (both variants).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 300 python tools/time_build.py 65536 ${@:-2 10 25 50 100} > gpurun_out/tb.log 2>&1
rc=$?; cat gpurun_out/tb.log; exit $rc
