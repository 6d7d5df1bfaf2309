#!/bin/bash
# One reference scene at a chip-filling size (default final_scene, 1440x1440 x 64 spp): the
# bench line with the oracle's CPU rate and parity beside it, then (STAMPS=1) the phase split
# of the stamps build and (PMC=1) the hardware-counter passes of tools/pmc.sh.
# usage (on the GPU box): TAG=r03_fs STAMPS=1 PMC=1 bash tools/gpu_final_scene.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TAG:-fs}
O=$R/gpurun_out/$T
mkdir -p $O
SC=${SCENE:-final_scene}
W=${WIDTH:-1440}
S=${SPP:-64}
if [ "${BENCH:-1}" = 1 ]; then
timeout -k 10 400 python3 -u $R/bench.py --config $SC --width $W --spp $S --steps ${STEPS:-2} --warmup 1 \
    --cpu-stride ${CPU_STRIDE:-4} --cpu-runs ${CPU_RUNS:-3} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
fi
if [ "${STAMPS:-0}" = 1 ]; then
  GS_LIB=$R/grayshift_amd/variants/stamps.so timeout -k 10 150 python3 $R/tools/stamps.py --config $SC --width ${STAMPS_WIDTH:-$W} --spp ${STAMPS_SPP:-$S} \
      > $O/stamps.txt 2> $O/stamps.err || { echo "stamps failed"; tail -5 $O/stamps.err; exit 1; }
  cat $O/stamps.txt
fi
if [ "${PMC:-0}" = 1 ]; then
  CONFIG=$SC BENCH_ARGS="--width $W --spp $S" bash $R/tools/pmc.sh || exit 1
fi
