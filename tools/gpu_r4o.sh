#!/bin/bash
# Round 4: the fixed-spp comparators of the adaptive lines (one batch of each scene's own
# settings: hdri 64 spp, cornell_box 32 spp) on the final code, and A2's per-launch trace.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4o
mkdir -p $O
timeout -k 10 300 python3 -u bench.py --config hdri --width 1920 --spp 64 --steps 3 --warmup 1 --no-cpu > $O/hdri_fixed64.json 2> $O/hdri.err || { echo "hdri failed"; tail -5 $O/hdri.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --config cornell_box --width 1024 --spp 32 --steps 3 --warmup 1 --no-cpu > $O/cornell_fixed32.json 2> $O/cornell.err || { echo "cornell failed"; tail -5 $O/cornell.err; exit 1; }
python3 -c "
import json
for f in ['hdri_fixed64','cornell_fixed32']:
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['config']['rays_per_frame'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/a2trace -o run -- python3 $R/bench.py --config A2 --steps 1 --warmup 0 --no-cpu > $O/a2trace.log 2>&1 || { echo "trace failed"; tail -5 $O/a2trace.log; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("$O/a2trace/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f))]
for r in rows:
    n = r["Kernel_Name"]
    if "gs_" in n:
        print("%-40s %8.3f ms" % (n[:40], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
PY
