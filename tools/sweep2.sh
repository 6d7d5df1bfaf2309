#!/bin/bash
# tools/sweep2.sh "SB:LB SB:LB ..."  (shade batch : leaf batch) on the default library
mkdir -p gpurun_out
for p in $1; do
  sb=${p%%:*}; lb=${p##*:}
  timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu --shade-batch $sb --leaf-batch $lb $2 > gpurun_out/sw2_${sb}_${lb}.json 2>gpurun_out/sw2.err || { echo "$p failed"; tail -5 gpurun_out/sw2.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sw2_${sb}_${lb}.json').read().strip().splitlines()[-1]); print('sb $sb lb $lb', d['value'], 'Msamples/s', d['ms_per_step'], 'ms frac', d['roofline']['frac'])"
done
