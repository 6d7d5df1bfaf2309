#!/bin/bash
# Round 4: cube records ordered by box size for the LDS mirror's prefix (host only: the device
# code object is unchanged) -- the -m gpu suite, A/B on final_scene against list order (two runs each).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/corder0.so base variants/corder0.so --config final_scene --width 1440 --spp 64 --steps 2 > $O/ab_fs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_fs.txt; exit 1; }
cat $O/ab_fs.txt
