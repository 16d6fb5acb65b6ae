#!/bin/bash
# The max-batch/large-batch GPU tests, then iterate timings of $LIBS (ablations).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "max_batch or large_batch" > gpurun_out/mb.log 2>&1
rc=$?; tail -3 gpurun_out/mb.log; [ $rc -eq 0 ] || exit $rc
LIBS="$LIBS" bash tools/gpu_iter_phases.sh
