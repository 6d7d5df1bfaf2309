#!/bin/bash
# Round 4: 16-step node passes for nested-sphere kernels -- the -m gpu suite, A/B on final_scene
# against 8 (nsu8), two runs each; then the default bench + rocprof stats and PMC on the new code.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/nsu8.so base variants/nsu8.so --config final_scene --width 1440 --spp 64 --steps 2 > $O/ab_fs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_fs.txt; exit 1; }
cat $O/ab_fs.txt
STAGES="bench pmc" TAG=r04_final5 bash $R/tools/gpu_final.sh || exit 1
