#!/bin/bash
# Round 4: does any gfx950 counter measure VALU issue time (a point
# estimate of VALU issue)?  The VALU microbenchmark (2.2- and 4.1-cycle instruction kinds)
# under SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU2 / SQ_BUSY_CU_CYCLES.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4b
mkdir -p $O
cd $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/ub -o run -- $R/tools/ubench/valu_rate > $O/ub.log 2>&1 || { echo "ubench pmc failed"; tail -5 $O/ub.log; exit 1; }
cat $O/ub.log | head -40
python3 - $O/ub/run_counter_collection.csv <<'PY'
import csv, sys
from collections import defaultdict
c = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    c[(r["Kernel_Name"][:24], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(c.items(), key=lambda kv: int(kv[0][1])):
    i = v["SQ_INSTS_VALU"] or 1
    print("%-26s insts %.3g  activeVALU/insts %.3f  threadcyc/insts %.2f  valu2/insts %.3f  busyCU %.3g  wave %.3g" % (
        k[0], i, v["SQ_ACTIVE_INST_VALU"] / i, v["SQ_THREAD_CYCLES_VALU"] / i, v["SQ_ACTIVE_INST_VALU2"] / i,
        v["SQ_BUSY_CU_CYCLES"], v["SQ_WAVE_CYCLES"]))
PY
