#!/bin/bash
# Sweep launch tuning on the C4 bench frame: tools/sweep_tuning.sh "<leaf batches>" "<shade batches>"
set -o pipefail
mkdir -p gpurun_out
for lb in $1; do for sb in $2; do
  timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu --leaf-batch $lb --shade-batch $sb > gpurun_out/sw.json 2>gpurun_out/sw.err || { echo "failed lb=$lb sb=$sb"; tail -3 gpurun_out/sw.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('leaf_batch $lb shade_batch $sb', d['value'], 'Msamples/s', d['ms_per_step'], 'ms')"
done; done
