#!/bin/bash
# The rest of a profile round after tools/gpu_round.sh, in two parts (each fits one call):
#   PART=1: every BASELINE config with parity and CPU rows, then final_scene at 1440^2 with
#           the oracle's CPU rate, parity and the PMC passes;
#   PART=2: every reference scene at 400 px and the four heavy ones at 1440^2 (rocprof of
#           final_scene), then the N-rank projection (tools/rank_sim.py).
# usage (on the GPU box): TAG=r03_x PART=1 bash tools/gpu_round_extra.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TAG:-extra}
if [ "${PART:-1}" = 1 ]; then
  bash $R/tools/bench_configs.sh ${T}_configs || exit 1
  TAG=${T}_fs PMC=1 CPU_RUNS=3 bash $R/tools/gpu_final_scene.sh || exit 1
else
  TAG=${T}_s400 WIDTH=400 NOPROF=1 SCENES="bouncing_spheres checkered_spheres cornell_box cornell_smoke earth earth_hdr final_scene hdri mixed perlin_spheres quads simple_light triangles" \
      bash $R/tools/gpu_scenes.sh || exit 1
  TAG=${T}_s1440 bash $R/tools/gpu_scenes.sh || exit 1
  mkdir -p $R/gpurun_out/$T
  timeout -k 10 400 python3 -u $R/tools/rank_sim.py --worlds 1,2,4,8 --ranks 0,1,2,3,4,5,6,7 --plan \
      > $R/gpurun_out/$T/rank_sim.txt 2> $R/gpurun_out/$T/rank_sim.err || { echo "rank_sim failed"; tail -5 $R/gpurun_out/$T/rank_sim.err; exit 1; }
  cat $R/gpurun_out/$T/rank_sim.txt
fi
