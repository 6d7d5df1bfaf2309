# whole-frame parity of the final code object: every pixel against the oracle (C4, A2, final_scene)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/fullframe2; mkdir -p $O
for spec in "C4" "A2" "final_scene --width 1440 --spp 64"; do set -- $spec
  timeout -k 10 400 python -u bench.py --config $spec --steps 1 --warmup 1 --cpu-stride 1 --cpu-runs 1 > $O/$1.json 2> $O/$1.err || { echo "$1 failed"; tail -5 $O/$1.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); p=d['parity']; print('$1', d['roofline']['code_object'], json.dumps(p))"
done
