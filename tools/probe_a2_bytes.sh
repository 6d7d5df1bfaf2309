# A2 fabric bytes per round launch by per-sample layout (FETCH_SIZE / WRITE_SIZE passes), and A1 in
# batch rounds vs the per-lane loop
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/a2bytes; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_adaptive.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in base sm; do
  if [ $lib = base ]; then export -n GS_LIB; unset GS_LIB; else export GS_LIB=$GRAFT_REPO_ROOT/grayshift_amd/variants/$lib.so; fi
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/${lib}_$c -o run -- python3 bench.py --config A2 --steps 1 --warmup 0 --no-cpu > $O/${lib}_$c.log 2>&1 || { echo "pmc $lib $c failed"; tail -3 $O/${lib}_$c.log; exit 1; }
  done
done
unset GS_LIB
for m in 1 2 0; do timeout -k 10 120 python bench.py --config A1 --steps 3 --warmup 1 --no-cpu --adaptive-mode $m > $O/A1_mode$m.json 2>$O/A1_mode$m.err || exit 1; python -c "import json; d=json.loads(open('$O/A1_mode$m.json').read().strip().splitlines()[-1]); print('A1 mode $m', d['value'], d['ms_per_step'])"; done
timeout -k 10 120 python bench.py --config A2 --steps 3 --warmup 1 --no-cpu > $O/A2.json 2>$O/A2.err && python -c "import json; d=json.loads(open('$O/A2.json').read().strip().splitlines()[-1]); print('A2', d['value'], d['ms_per_step'])"
