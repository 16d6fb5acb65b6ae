#!/bin/bash
# A/B of the headline build kernel: bench.py --headline-only with the in-tree
# library and with ab/<base>/libcmpc.so, alternating (the box's clock drifts),
# then the build parity tests and one PMC pass (VALU mix) on the in-tree one.
#   usage: tools/gpu_ab_build.sh TAG [BASE=base] [ROUNDS=3]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=$1; BASE=${2:-base}; N=${3:-3}
OUT=gpurun_out/ab_$TAG.txt; : > $OUT
for i in $(seq $N); do
  for v in new $BASE; do
    if [ $v = new ]; then L=""; else L=ab/$BASE/libcmpc.so; fi
    CMPC_LIBRARY=$L timeout -k 10 200 python3 bench.py --headline-only --steps 50 --no-cpu > gpurun_out/ab_${TAG}_$v$i.json 2> gpurun_out/ab_${TAG}_$v$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'step_ms %.4f build_us %.2f frac %.4f iterate_us %.2f' % (d['ms_per_step'], d['roofline']['avg_launch_ms']*1e3, d['roofline']['frac'], d['kernels_ms_per_step']['iterate']*1e3))" gpurun_out/ab_${TAG}_$v$i.json $v $i >> $OUT
  done
done
cat $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "build or step or headline or large" > gpurun_out/ab_${TAG}_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/ab_${TAG}_tests.log; tail -2 gpurun_out/ab_${TAG}_tests.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -T --kernel-include-regex 'cmpc_build' --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/ab_${TAG}_pmc -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --headline-only --settle-seconds 0 > /dev/null 2> gpurun_out/ab_${TAG}_pmc.err || exit $?
python3 - gpurun_out/ab_${TAG}_pmc/run_counter_collection.csv <<'PY'
import csv, sys, statistics
from collections import defaultdict
acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "build_rows" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: statistics.median(v) for k, v in acc.items()}
w = m["SQ_WAVES"]
print({k: round(v / w, 1) if k != "SQ_WAVES" else v for k, v in m.items()})
print("non-FMA VALU per wave %.0f" % ((m["SQ_INSTS_VALU"] - m["SQ_INSTS_VALU_FMA_F64"]) / w))
PY
