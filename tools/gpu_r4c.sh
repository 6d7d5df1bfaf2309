#!/bin/bash
# Round 4: adaptive batch rounds with whole-batch items (tests + A1/A2 lines), the nested-LDS
# variants on final_scene, and the stamps-build hang probe.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_adaptive.py tests/test_gpu_multi.py tests/test_gpu_robustness.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in 1 0; do
timeout -k 10 300 python3 -u $R/bench.py --config A1 --steps 3 --warmup 1 --cpu-runs 1 --adaptive-mode $m > $O/a1_m$m.json 2> $O/a1_m$m.err || { echo "A1 failed"; tail -5 $O/a1_m$m.err; exit 1; }
timeout -k 10 300 python3 -u $R/bench.py --config A2 --steps 3 --warmup 1 --cpu-runs 1 --cpu-stride 8 --adaptive-mode $m > $O/a2_m$m.json 2> $O/a2_m$m.err || { echo "A2 failed"; tail -5 $O/a2_m$m.err; exit 1; }
done
python3 -c "
import json
for f in ['a1_m1','a1_m0','a2_m1','a2_m0']:
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['config']['rays_per_frame'], d['parity']['max_abs_delta'], d['cpu_baseline']['value'])
"
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/nlds.so variants/nldsq.so --config final_scene --width 1440 --spp 64 --steps 2 > $O/ab_nlds.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_nlds.txt; exit 1; }
cat $O/ab_nlds.txt
