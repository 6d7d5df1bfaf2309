#!/bin/bash
# Reference scenes at a chip-filling size (1440x1440 = 2.07 Mpx, like 1080p; 64 spp), one
# bench line each, then rocprofv3 kernel stats of the slowest (final_scene).
# usage (on the GPU box): TAG=r03_x SCENES="final_scene cornell_smoke" bash tools/gpu_scenes.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TAG:-scenes}
O=$R/gpurun_out/$T
mkdir -p $O
W=${WIDTH:-1440}
S=${SPP:-64}
for sc in ${SCENES:-final_scene cornell_smoke perlin_spheres simple_light}; do
  timeout -k 10 240 python3 -u $R/bench.py --config $sc --width $W --spp $S --steps ${STEPS:-1} --warmup 1 --no-cpu \
      > $O/$sc.json 2> $O/$sc.err || { echo "$sc failed"; tail -5 $O/$sc.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-16s %9.1f Msamples/s %9.1f ms kernel %9.1f ms rays %d' % (sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['rays_per_frame']))" $O/$sc.json $sc
done
if [ "${NOPROF:-0}" != 1 ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${PROF:-final_scene} -o run -- \
      python3 $R/bench.py --config ${PROF:-final_scene} --width $W --spp $S --steps 1 --warmup 1 --no-cpu \
      > $O/prof.json 2> $O/prof.err || { echo "prof failed"; tail -5 $O/prof.err; exit 1; }
  find $O/prof_${PROF:-final_scene} -name "*kernel_stats.csv" -exec head -4 {} \;
fi
