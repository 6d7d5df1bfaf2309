# Round 5: the sticky long-sample flag (host side, code object c557a991): multi tests, the 400-px scenes, C1.
export TMPDIR=/tmp
O=gpurun_out/r05_y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 900 python3 -u tools/sweep.py --config checkered_spheres perlin_spheres simple_light earth quads cornell_box C1 --steps 5 > $O/rule.txt 2>&1 || { echo "rule failed"; tail -5 $O/rule.txt; exit 1; }
cat $O/rule.txt
