#!/bin/bash
# Round 4 GPU call: variant correctness (GS_LIB=variants/r4all.so: SALU visit counts, quad-run
# lists, nested records in LDS), then A/B against the product library, the stamps build's
# watchdog on the media scenes (the r03 hang), and the adaptive configs A1 / A2.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4a
mkdir -p $O
GS_LIB=$R/grayshift_amd/variants/r4all.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_volumes.py tests/test_gpu_instancing_noise.py tests/test_gpu_adaptive.py tests/test_gpu_multi.py tests/test_gpu_placement.py -x -q --timeout 120 --timeout-method thread > $O/tests_r4all.log 2>&1 || { echo "VARIANT TESTS FAILED"; tail -40 $O/tests_r4all.log; exit 1; }
tail -2 $O/tests_r4all.log
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/r4all.so variants/qrun.so variants/salu.so --config final_scene cornell_smoke cornell_box --width 1440 --spp 64 --steps 1 > $O/ab_scenes.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_scenes.txt; exit 1; }
cat $O/ab_scenes.txt
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/r4all.so variants/salu.so --config C4 C3 C5 --steps 2 --spp 512 > $O/ab_cfg.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_cfg.txt; exit 1; }
cat $O/ab_cfg.txt
for sc in cornell_smoke final_scene; do
  GS_LIB=$R/grayshift_amd/variants/stamps.so timeout -k 10 100 python3 -u $R/tools/stamps.py --config $sc --width 96 --spp 4 \
      > $O/stamps_$sc.txt 2> $O/stamps_$sc.err
  echo "stamps $sc rc=$?"; head -c 3000 $O/stamps_$sc.txt
done
for m in 1 0; do
timeout -k 10 300 python3 -u $R/bench.py --config A1 --steps 2 --warmup 1 --cpu-runs 1 --adaptive-mode $m > $O/a1_m$m.json 2> $O/a1_m$m.err || { echo "A1 failed"; tail -5 $O/a1_m$m.err; exit 1; }
cat $O/a1_m$m.json
timeout -k 10 300 python3 -u $R/bench.py --config A2 --steps 2 --warmup 1 --cpu-runs 1 --cpu-stride 8 --adaptive-mode $m > $O/a2_m$m.json 2> $O/a2_m$m.err || { echo "A2 failed"; tail -5 $O/a2_m$m.err; exit 1; }
cat $O/a2_m$m.json
done
timeout -k 10 200 python3 -u $R/bench.py --config hdri --width 1920 --spp 64 --no-cpu --steps 2 > $O/hdri_fixed64.json 2>&1 || exit 1
timeout -k 10 200 python3 -u $R/bench.py --config cornell_box --width 1024 --spp 32 --no-cpu --steps 2 > $O/cornell_fixed32.json 2>&1 || exit 1
python3 -c "
import json
for f in ['hdri_fixed64','cornell_fixed32']:
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['config']['rays_per_frame'])
"
