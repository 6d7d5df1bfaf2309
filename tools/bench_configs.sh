set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instancing_noise.py tests/test_gpu_volumes.py -m "gpu and not slow" -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for c in C1 C2 C3 C4 C5; do
  timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu > gpurun_out/cfg_$c.json 2>gpurun_out/cfg_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/cfg_$c.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/cfg_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
