#!/bin/bash
# VALU mix of config 3's build kernel (ny = 2) and the headline's, one PMC pass
# each (tools/pmc_small.py: 20 build launches after a warm-up).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c3 head; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex 'cmpc_build' --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_c3_$c -o run --output-format csv -- python3 tools/pmc_small.py $c build 20 > gpurun_out/pmc_c3_$c.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, statistics
from collections import defaultdict
for c in ("c3", "head"):
    acc = defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/pmc_c3_{c}/run_counter_collection.csv")):
        if "build" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: statistics.median(v) for k, v in acc.items()}
    w = m["SQ_WAVES"]
    print(c, {k: round(v / w, 1) for k, v in m.items() if k != "SQ_WAVES"}, "waves", w,
          "non-FMA VALU/wave %.0f" % ((m["SQ_INSTS_VALU"] - m["SQ_INSTS_VALU_FMA_F64"]) / w),
          "VALU busy %.3f" % (3 * m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]))
PY
