#!/bin/bash
# Round 4: the stamps-build hang (r03: -DGS_STAMPS never finishes on media scenes) -- which
# part of the stamps code is needed for it: each probe build on cornell_smoke 96x54x4 spp
# with a short limit; then the adaptive tests and lines on the product library.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4d
mkdir -p $O
for v in wdonly st_both st_notime st_nopass stamps; do
  GS_LIB=$R/grayshift_amd/variants/$v.so timeout -k 5 45 python3 -u $R/tools/stamps.py --config cornell_smoke --width 96 --spp 4 \
      > $O/probe_$v.txt 2>&1
  echo "probe $v rc=$?"; grep -v amdgpu.ids $O/probe_$v.txt | head -c 1500
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_adaptive.py tests/test_gpu_instancing_noise.py tests/test_gpu_volumes.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in A1 A2; do
timeout -k 10 300 python3 -u $R/bench.py --config $c --steps 3 --warmup 1 --cpu-runs 1 --cpu-stride 8 > $O/$c.json 2> $O/$c.err || { echo "$c failed"; tail -5 $O/$c.err; exit 1; }
done
timeout -k 10 300 python3 -u $R/bench.py --config final_scene --width 1440 --spp 64 --steps 2 --warmup 1 --cpu-stride 4 --cpu-runs 1 > $O/fs.json 2> $O/fs.err || { echo "fs failed"; tail -5 $O/fs.err; exit 1; }
python3 -c "
import json
for f in ['A1','A2','fs']:
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['config']['rays_per_frame'], d['parity']['max_abs_delta'], d['cpu_baseline']['value'])
"
