#!/bin/bash
# Every BASELINE config on one GPU at its stated size and spp, each frame checked against
# the CPU oracle on a pixel subset sized for ~10 s of CPU work (bench.py's parity block).
# usage (on the GPU box): bash tools/bench_configs.sh [tag]   -> gpurun_out/<tag>/cfg_<C>.json
set -o pipefail
T=${1:-configs}
O=gpurun_out/$T
mkdir -p $O
for spec in "C1 1 3" "C2 4 1" "C3 8 1" "C4 3 3" "C5 24 1"; do
  set -- $spec
  timeout -k 10 600 python -u bench.py --config $1 --steps 3 --warmup 1 --cpu-stride $2 --cpu-runs $3 > $O/cfg_$1.json 2> $O/cfg_$1.err || { echo "bench $1 failed"; tail -5 $O/cfg_$1.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/cfg_$1.json').read().strip().splitlines()[-1]); p=d['parity']; print('$1', d['value'], 'Msamples/s', d['ms_per_step'], 'ms', 'parity max|d| %g over %d px' % (p['max_abs_delta'], p['pixels']), 'cpu', d['cpu_baseline']['value'])"
done
