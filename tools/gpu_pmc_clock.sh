#!/bin/bash
# In-kernel clock of the row build kernel per configuration: GRBM_GUI_ACTIVE
# (GPU busy cycles per dispatch) against the traced duration (time_build.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in ${CASES:-par-coop ser-coop}; do
  CMPC_TB_VARIANT=rows CMPC_TB_CASE=$c timeout -s KILL 120 rocprofv3 --kernel-trace \
    --kernel-include-regex 'cmpc_build_rows' --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
    -d gpurun_out/pmck_$c -o run --output-format csv -- python3 tools/time_build.py 65536 ${P:-50} > gpurun_out/pmck_$c.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, collections, os
for c in os.environ.get("CASES", "par-coop ser-coop").split():
    d = f"gpurun_out/pmck_{c}"
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv"))]
    g = sum(agg["GRBM_GUI_ACTIVE"]) / len(agg["GRBM_GUI_ACTIVE"])
    t = sorted(dur)[len(dur) // 2]
    print(c, "median ns", t, "GRBM_GUI_ACTIVE", round(g), "GHz", round(g / t, 3), "SQ_BUSY", round(sum(agg["SQ_BUSY_CYCLES"]) / len(agg["SQ_BUSY_CYCLES"])))
PY
