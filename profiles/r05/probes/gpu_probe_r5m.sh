# Round 5: claim divisor 4, the small-frame rule for simple scenes only: GPU suite, C1, final_scene 400, C4.
export TMPDIR=/tmp
O=gpurun_out/r05_m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python3 -u tools/sweep.py --config C1 --steps 30 > $O/c1.txt 2>&1 || { echo "c1 failed"; tail -5 $O/c1.txt; exit 1; }
timeout -k 10 600 python3 -u tools/sweep.py --config final_scene cornell_smoke perlin_spheres --steps 3 >> $O/c1.txt 2>&1 || { echo "small failed"; tail -5 $O/c1.txt; exit 1; }
timeout -k 10 600 python3 -u tools/sweep.py --config C4 C2 --steps 2 >> $O/c1.txt 2>&1 || { echo "big failed"; tail -5 $O/c1.txt; exit 1; }
cat $O/c1.txt
