# Round 5: bench.py's timed loop without per-frame Python conversions (host-side only).
export TMPDIR=/tmp
O=gpurun_out/r05_s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_multiprocess.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 -u tools/sweep.py --config C1 --steps 30 > $O/c1.txt 2>&1 || { echo "c1 failed"; tail -5 $O/c1.txt; exit 1; }
timeout -k 10 300 python3 -u tools/sweep.py --config C1 --steps 200 >> $O/c1.txt 2>&1 || { echo "c1 failed"; tail -5 $O/c1.txt; exit 1; }
cat $O/c1.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
