set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r06s2_check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for spec in "A2 1" "A1 1" "A1 2" "C3 1"; do set -- $spec
timeout -k 10 200 python bench.py --config $1 --steps 3 --warmup 1 --no-cpu --adaptive-mode $2 > $O/$1_$2.json 2>$O/$1_$2.err || exit 1
python -c "import json; d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); print('$1 mode $2', d['value'], d['ms_per_step'])"
done
