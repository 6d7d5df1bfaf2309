#!/bin/bash
# tools/sweep3.sh "SB:LB:CHUNK ..." [extra bench args]  (shade batch : leaf batch : sample chunk)
mkdir -p gpurun_out
for p in $1; do
  IFS=: read sb lb ch <<< "$p"
  out=gpurun_out/sw3_${sb}_${lb}_${ch}.json
  timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu --shade-batch $sb --leaf-batch $lb --sample-chunk $ch $2 > $out 2>gpurun_out/sw3.err || { echo "$p failed"; tail -5 gpurun_out/sw3.err; exit 1; }
  python -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('sb $sb lb $lb ch $ch', d['value'], 'Msamples/s', d['ms_per_step'], 'ms frac', d['roofline']['frac'])"
done
