# Round 5: counters zeroed by the params kernel, no unpack event in direct mode; fine-chunk
# rule sweep (C1, final_scene, cornell_smoke at 1440^2 x 64).
export TMPDIR=/tmp
O=gpurun_out/r05_j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python3 -u tools/sweep.py --config C1 --steps 30 --fine-chunk 3 4 5 6 --tail-pct 0 300 > $O/c1.txt 2>&1 || { echo "c1 failed"; tail -5 $O/c1.txt; exit 1; }
cat $O/c1.txt
timeout -k 10 600 python3 -u tools/sweep.py --config final_scene cornell_smoke --width 1440 --spp 64 --steps 2 --fine-chunk 0 2 4 > $O/fs.txt 2>&1 || { echo "fs failed"; tail -5 $O/fs.txt; exit 1; }
cat $O/fs.txt
timeout -k 10 600 python3 -u tools/sweep.py --config C2 --steps 3 --fine-chunk 0 8 > $O/c2.txt 2>&1 || { echo "c2 failed"; tail -5 $O/c2.txt; exit 1; }
cat $O/c2.txt
