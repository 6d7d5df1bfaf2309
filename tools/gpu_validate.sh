set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
