# Round 5: the nested walk with the single camera-ray site and the reused medium boundary
# transform (both now unconditional): GPU suite, final_scene leaf-batch sweep, C4 check,
# final_scene full-frame parity at 1440^2 x 64 spp.
export TMPDIR=/tmp
O=gpurun_out/r05_h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python3 -u tools/sweep.py --config final_scene --width 1440 --spp 64 --steps 2 --leaf-batch 16 24 32 > $O/fs.txt 2>&1 || { echo "fs failed"; tail -5 $O/fs.txt; exit 1; }
cat $O/fs.txt
timeout -k 10 300 python3 -u tools/sweep.py --config C4 --steps 2 > $O/c4.txt 2>&1 || { echo "c4 failed"; tail -5 $O/c4.txt; exit 1; }
cat $O/c4.txt
timeout -k 10 900 python3 -u bench.py --config final_scene --width 1440 --spp 64 --steps 1 --warmup 1 --cpu-stride 1 --cpu-runs 1 > $O/fs_fullframe.json 2> $O/fs_fullframe.err || { echo "fullframe failed"; tail -5 $O/fs_fullframe.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/fs_fullframe.json').read().strip().splitlines()[-1]); print(d['value'], d['parity'])"
