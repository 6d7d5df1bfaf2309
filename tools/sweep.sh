#!/bin/bash
# Sweep bench tuning knobs on the default library: tools/sweep.sh "16 24 32 48" [blocks_per_cu]
mkdir -p gpurun_out
for sb in $1; do
  timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu --shade-batch $sb ${2:+--blocks-per-cu $2} $3 > gpurun_out/sw_$sb.json 2>gpurun_out/sw_$sb.err || { echo "sb $sb failed"; tail -5 gpurun_out/sw_$sb.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sw_$sb.json').read().strip().splitlines()[-1]); print('shade_batch $sb', d['value'], 'Msamples/s', d['ms_per_step'], 'ms frac', d['roofline']['frac'])"
done
