#!/bin/bash
# Bench line (no CPU leg) twice, then the SURVEY configuration table.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bq.json 2> gpurun_out/bq.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bq.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_ms_per_step'])"
done
timeout -k 10 300 python tools/time_survey_configs.py 2>&1 | grep -v amdgpu.ids
