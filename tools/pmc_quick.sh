#!/bin/bash
# One SQ counter pass per variant library (A/B of instruction mix and waits).
# usage: tools/pmc_quick.sh "base nofast" [extra bench args]; 'base' = the default library
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
SET="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for v in $1; do
  if [ "$v" = base ]; then unset GS_LIB; else export GS_LIB=$R/grayshift_amd/variants/$v.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $R/gpurun_out/pmcq_$v -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu $2 > $R/gpurun_out/pmcq_$v.log 2>&1 || { echo "pmc $v failed"; tail -3 $R/gpurun_out/pmcq_$v.log; exit 1; }
  python3 - "$R/gpurun_out/pmcq_$v/run_counter_collection.csv" "$v" <<'PY'
import csv, sys
from collections import defaultdict
c = defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "gs_render_kernel" in r["Kernel_Name"]:
        c[r["Counter_Name"]] += float(r["Counter_Value"])
w = c["SQ_WAVE_CYCLES"] or 1
print("%s: VALU %.4g SALU %.4g LDS %.4g | wait %.3f active %.3f activeVALU %.3f | gui %.4g" % (
    sys.argv[2], c["SQ_INSTS_VALU"], c["SQ_INSTS_SALU"], c["SQ_INSTS_LDS"], c["SQ_WAIT_ANY"] / w,
    c["SQ_ACTIVE_INST_ANY"] / w, c["SQ_ACTIVE_INST_VALU"] / w, c["GRBM_GUI_ACTIVE"]))
PY
done
