#!/bin/bash
# The timed steps' build events: every launch (stride 1), every 5th, none
# (separate pass), alternating on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/evs_ab.txt; : > $OUT
for i in $(seq ${ROUNDS:-3}); do
  for m in s1 s5 s10 sep; do
    case $m in s1) A="--build-event-stride 1";; s5) A="--build-event-stride 5";; s10) A="--build-event-stride 10";; sep) A="--build-events separate";; esac
    timeout -k 10 200 python3 bench.py --headline-only --steps 50 --no-cpu $A > gpurun_out/evs_$m$i.json 2> gpurun_out/evs_$m$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], 'step_ms %.4f build_us %.2f (%d launches) frac %.4f iterate_us %.2f' % (d['ms_per_step'], r['avg_launch_ms']*1e3, r['launches'], r['frac'], d['kernels_ms_per_step']['iterate']*1e3))" gpurun_out/evs_$m$i.json $m $i >> $OUT
  done
done
cat $OUT
