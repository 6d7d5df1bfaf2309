#!/bin/bash
# Round 4: nested walk counters in registers (once per walk) -- A/B against per-visit LDS
# atomics (nlc0) and a leaf batch of 56 for nested scenes (lb56), two runs each; GPU tests.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/nlc0.so variants/lb56.so base variants/nlc0.so variants/lb56.so --config final_scene --width 1440 --spp 64 --steps 2 > $O/ab_fs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_fs.txt; exit 1; }
cat $O/ab_fs.txt
