#!/bin/bash
# rocprofv3 summaries of the closed loop: (1) B = 1 through the C++ adapter
# (tests/cpp/with_timing, 2 000 steps, HIP API + kernel trace), (2) 65 536
# scenarios through cmpc.driver.ClosedLoop (tools/run_closed_loop.py, 200 steps).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/clp_b1 -o run --output-format csv -- \
  tests/cpp/with_timing tools/setup-coop-par par coop gpurun_out/clp_wt 2000 > gpurun_out/clp_b1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/clp_big -o run --output-format csv -- \
  python3 tools/run_closed_loop.py par coop --p 50 --batch 65536 --steps 200 --perturb 0.002 > gpurun_out/clp_big.log 2>&1 || exit $?
tail -1 gpurun_out/clp_b1.log; tail -1 gpurun_out/clp_big.log
