#!/bin/bash
# Round 3 measurement call: SURVEY config table, the headline-size step parity
# with its near-tie counts printed, then the round's profile set
# (tools/gpu_round.sh: tests, smoke, bench, rocprofv3 stats and PMC passes).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-r3e}
timeout -k 10 400 python tools/time_survey_configs.py > gpurun_out/survey_$TAG.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -s --timeout 300 --timeout-method thread \
  -k "headline_size or step_matches_oracle" > gpurun_out/parity_$TAG.log 2>&1 || exit $?
bash tools/gpu_round.sh $TAG
