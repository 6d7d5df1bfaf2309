#!/bin/bash
# A/B the variant libraries on the C4 bench workload (one frame each).
# usage: tools/ab_variants.sh "n1 n4 i4" [extra bench args]
set -o pipefail
mkdir -p gpurun_out
for v in $1; do
  GS_LIB=$PWD/grayshift_amd/variants/$v.so timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu $2 > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || { echo "variant $v failed"; cat gpurun_out/ab_$v.err | tail -5; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], 'Msamples/s', d['ms_per_step'], 'ms', 'frac', d['roofline']['frac'])"
done
