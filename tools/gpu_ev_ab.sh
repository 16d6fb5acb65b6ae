cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/ev_ab.txt; : > $OUT
for i in 1 2 3; do
  for m in timed separate; do
    timeout -k 10 200 python3 bench.py --headline-only --steps 50 --no-cpu --build-events $m > gpurun_out/ev_$m$i.json 2> gpurun_out/ev_$m$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'step_ms %.4f build_us %.2f iterate_us %.2f' % (d['ms_per_step'], d['roofline']['avg_launch_ms']*1e3, d['kernels_ms_per_step']['iterate']*1e3))" gpurun_out/ev_$m$i.json $m $i >> $OUT
  done
done
cat $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_ev -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu --headline-only --markers --build-events separate > gpurun_out/benchprof_ev.json 2> gpurun_out/benchprof_ev.err || exit $?
python3 tools/headline_pass_stats.py gpurun_out/prof_ev/run_kernel_trace.csv gpurun_out/benchprof_ev.json gpurun_out/ev_separate3.json
python3 tools/headline_pass_stats.py gpurun_out/prof_ev/run_kernel_trace.csv gpurun_out/benchprof_ev.json gpurun_out/ev_timed3.json
