#!/bin/bash
# A/B of several libraries: the in-tree one ("new") and ab/<v>/libcmpc.so for
# each named variant, alternating over ROUNDS rounds (the box's clock drifts):
# the headline (bench.py --headline-only) and, with CONFIGS=1, the SURVEY
# configs' build kernels (bench.py --configs-only).
#   usage: ROUNDS=2 CONFIGS=1 tools/gpu_ab_multi.sh TAG v1 v2 ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
OUT=gpurun_out/abm_$TAG.txt; : > $OUT
for i in $(seq ${ROUNDS:-2}); do
  for v in new "$@"; do
    if [ $v = new ]; then L=""; else L=ab/$v/libcmpc.so; fi
    CMPC_LIBRARY=$L timeout -k 10 200 python3 bench.py --headline-only --steps 50 --no-cpu > gpurun_out/abm_${TAG}_$v$i.json 2> gpurun_out/abm_${TAG}_$v$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('%-8s %d head step_ms %.4f build_us %.2f frac %.4f iterate_us %.2f' % (sys.argv[2], int(sys.argv[3]), d['ms_per_step'], d['roofline']['avg_launch_ms']*1e3, d['roofline']['frac'], d['kernels_ms_per_step']['iterate']*1e3))" gpurun_out/abm_${TAG}_$v$i.json $v $i >> $OUT
    if [ "${CONFIGS:-0}" = 1 ]; then
      CMPC_LIBRARY=$L timeout -k 10 300 python3 bench.py --configs-only --no-cpu > gpurun_out/abm_${TAG}_cfg_$v$i.json 2> gpurun_out/abm_${TAG}_cfg_$v$i.err || exit $?
      python3 -c "
import json,sys; c=json.loads(open(sys.argv[1]).read().splitlines()[-1])['configs']
print('%-8s %d cfgs ' % (sys.argv[2], int(sys.argv[3])) + ' '.join('c%s build_us %.2f frac %.4f step_us %.2f' % (k, c[k]['build_ms']*1e3, c[k]['build_roofline']['frac'], c[k]['ms_per_step']*1e3) for k in ('2','3','5') if 'error' not in c[k]))" gpurun_out/abm_${TAG}_cfg_$v$i.json $v $i >> $OUT
    fi
  done
done
cat $OUT
