#!/bin/bash
# Round 4: full-frame parity of the scenes whose leaf tests changed this round (every pixel at
# full spp against the oracle): C3, final_scene and cornell_smoke at 1440^2 x 64.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s
mkdir -p $O
timeout -k 10 400 python3 -u bench.py --config C3 --steps 1 --warmup 1 --cpu-stride 1 --cpu-runs 1 > $O/c3_full.json 2> $O/c3_full.err || { echo "C3 failed"; tail -5 $O/c3_full.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --config final_scene --width 1440 --spp 64 --steps 1 --warmup 1 --cpu-stride 1 --cpu-runs 1 > $O/fs_full.json 2> $O/fs_full.err || { echo "fs failed"; tail -5 $O/fs_full.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --config cornell_smoke --width 1440 --spp 64 --steps 1 --warmup 1 --cpu-stride 1 --cpu-runs 1 > $O/cs_full.json 2> $O/cs_full.err || { echo "cs failed"; tail -5 $O/cs_full.err; exit 1; }
python3 -c "
import json
for f in ['c3_full','fs_full','cs_full']:
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); p=d['parity']; print(f, d['value'], p['pixels'], p['max_abs_delta'], p['n_over_tol'], p['bit_identical_frac'], d['cpu_baseline']['value'])
"
