#!/bin/bash
# The round's full GPU record: tools/gpu_round.sh (parity tests, smoke, bench,
# rocprofv3 stats, PMC passes), the B = 1 adapter latency and trace, the
# small-batch timings and the config-5 apply-move A/B.  usage: TAG (default r4i)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
bash tools/gpu_round.sh ${1:-r4i} || exit $?
bash tools/gpu_b1_trace.sh ${1:-r4i} || exit $?
CMPC_TS_REPS=40 timeout -k 10 300 python -u tools/time_small.py c5 c2 b1 c1b1 > gpurun_out/small_${1:-r4i}.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/time_apply_move.py > gpurun_out/apply_move_${1:-r4i}.txt 2>&1 || exit $?
echo ALLDONE
