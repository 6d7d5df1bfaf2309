#!/bin/bash
# Round-end measurement of the final code object, in stages (STAGES="tests bench pmc stamps
# configs"), each step under its own time limit, results under gpurun_out/$TAG:
#   tests   the whole -m gpu suite
#   bench   the default bench line (C4: parity + CPU baseline) and its rocprofv3 kernel stats
#   pmc     tools/pmc.sh for every config named in PMC_CONFIGS (default C4 C3 C5 A2 final_scene;
#           final_scene at 1440^2 x 64 spp)
#   configs every BASELINE config at its stated size, with parity and the CPU baseline, plus
#           the adaptive A1 / A2 and final_scene at 1440^2 x 64 spp
#   stamps  the stamps build's phase split and lane-efficiency summary of every config
#   ranks   tools/rank_sim.py: every rank of 1/2/4/8-GPU planned frames of C4 and C5, alone
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TAG:-r05_final}
O=$R/gpurun_out/$T
mkdir -p $O
STAGES=${STAGES:-"tests bench pmc stamps configs"}
for st in $STAGES; do
case $st in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log ;;
bench)
  timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/stats_bench.json 2> $O/stats_bench.err || { echo "stats run failed"; tail -5 $O/stats_bench.err; exit 1; }
  cat $O/stats_bench.json
  find $O/stats -name "*kernel_stats.csv" -exec head -6 {} \; ;;
pmc)
  for c in ${PMC_CONFIGS:-C4 C3 C5 A2 final_scene}; do
    case $c in
      final_scene|cornell_smoke) BA="--width 1440 --spp 64"; PT=${c}_w1440_s64 ;;
      *) BA=""; PT=$c ;;
    esac
    CONFIG=$c BENCH_ARGS="$BA" PMC_TAG=$PT bash $R/tools/pmc.sh || exit 1
  done
  # (later stages' bench lines read them from the tree; gpurun_out/pmc_out comes back to commit)
  cp $R/gpurun_out/pmc_out/*.json $R/profiles/pmc/ ;;
configs)
  for spec in "C1 1 3" "C2 4 1" "C3 8 1" "C4 3 3" "C5 24 1" "A1 3 1" "A2 8 1"; do
    set -- $spec
    timeout -k 10 600 python -u bench.py --config $1 --steps 3 --warmup 1 --cpu-stride $2 --cpu-runs $3 > $O/cfg_$1.json 2> $O/cfg_$1.err || { echo "bench $1 failed"; tail -5 $O/cfg_$1.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/cfg_$1.json').read().strip().splitlines()[-1]); p=d['parity']; r=d['roofline']; print('$1', d['value'], 'Msamples/s', d['ms_per_step'], 'ms', 'parity max|d| %g over %d px' % (p['max_abs_delta'], p['pixels']), 'cpu', d['cpu_baseline']['value'], 'frac', r['frac'], 'lane_frac', r.get('lane_frac'), 'useful_frac', r.get('useful_frac'))"
  done
  timeout -k 10 300 python3 -u bench.py --config final_scene --width 1440 --spp 64 --steps 2 --warmup 1 --cpu-stride 4 --cpu-runs 1 > $O/final_scene_1440.json 2> $O/final_scene_1440.err || { echo "final_scene failed"; tail -5 $O/final_scene_1440.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/final_scene_1440.json').read().strip().splitlines()[-1]); print('final_scene', d['value'], d['ms_per_step'], d['parity']['max_abs_delta'], d['cpu_baseline']['value'], d['roofline']['frac'], d['roofline'].get('lane_frac'))"
  timeout -k 10 300 python3 -u bench.py --config cornell_smoke --width 1440 --spp 64 --steps 2 --warmup 1 --cpu-stride 4 --cpu-runs 1 > $O/cornell_smoke_1440.json 2> $O/cornell_smoke_1440.err || { echo "cornell_smoke failed"; tail -5 $O/cornell_smoke_1440.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/cornell_smoke_1440.json').read().strip().splitlines()[-1]); print('cornell_smoke', d['value'], d['ms_per_step'], d['parity']['max_abs_delta'], d['cpu_baseline']['value'])" ;;
stamps)
  # every config's lane-efficiency summary (bench.py's roofline lane_frac), at the config's own
  # size (final_scene / cornell_smoke at 1440^2 x 64 spp), into the tree and gpurun_out/stamps_out
  mkdir -p $R/gpurun_out/stamps_out
  for spec in ${STAMPS_SPECS:-"C1" "C2" "C3" "C4" "C5" "A1" "A2" "final_scene --width 1440 --spp 64" "cornell_smoke --width 1440 --spp 64"}; do
    set -- $spec
    GS_LIB=$R/grayshift_amd/variants/stamps.so timeout -k 10 300 python3 $R/tools/stamps.py --config $spec --json $R/profiles/stamps > $O/stamps_$1.txt 2> $O/stamps_$1.err || { echo "stamps $1 failed"; tail -5 $O/stamps_$1.err; exit 1; }
    echo "== stamps $1"; cat $O/stamps_$1.txt
  done
  cp $R/profiles/stamps/*.json $R/gpurun_out/stamps_out/ ;;
ranks)
  # projection of the N-GPU frame from one GPU: every rank's planned share rendered alone
  # (tools/rank_sim.py), C4 and C5 at their stated sizes
  timeout -k 10 300 python3 -u $R/tools/rank_sim.py --config C4 --worlds 1,2,4,8 --all-ranks --plan > $O/rank_sim_C4.txt 2> $O/rank_sim_C4.err || { echo "rank_sim C4 failed"; tail -5 $O/rank_sim_C4.err; exit 1; }
  grep projected $O/rank_sim_C4.txt
  timeout -k 10 900 python3 -u $R/tools/rank_sim.py --config C5 --worlds 1,2,4,8 --all-ranks --plan --reps 1 > $O/rank_sim_C5.txt 2> $O/rank_sim_C5.err || { echo "rank_sim C5 failed"; tail -5 $O/rank_sim_C5.err; exit 1; }
  grep projected $O/rank_sim_C5.txt ;;
esac
done
