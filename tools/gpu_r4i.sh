#!/bin/bash
# Round 4: cube records read from LDS by a wave-uniform choice; A/B against no cube mirror,
# and the leaf-batch / node-step knobs re-swept on the scenes whose leaf tests changed.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/cnolds.so --config final_scene cornell_smoke --width 1440 --spp 64 --steps 2 > $O/ab_fs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_fs.txt; exit 1; }
cat $O/ab_fs.txt
timeout -k 10 900 python3 -u tools/sweep.py --config final_scene --width 1440 --spp 64 --steps 2 --leaf-batch 32 48 64 --node-steps 3 8 > $O/sweep_fs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/sweep_fs.txt; exit 1; }
cat $O/sweep_fs.txt
timeout -k 10 900 python3 -u tools/sweep.py --config C3 --steps 1 --leaf-batch 8 12 16 > $O/sweep_c3.txt 2>&1 || { echo "sweep failed"; tail -5 $O/sweep_c3.txt; exit 1; }
cat $O/sweep_c3.txt
timeout -k 10 900 python3 -u tools/sweep.py --config cornell_smoke --width 1440 --spp 64 --steps 2 --leaf-batch 8 12 16 > $O/sweep_cs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/sweep_cs.txt; exit 1; }
cat $O/sweep_cs.txt
timeout -k 10 900 python3 -u tools/sweep.py --config C5 --spp 256 --steps 1 --leaf-batch 8 12 16 > $O/sweep_c5.txt 2>&1 || { echo "sweep failed"; tail -5 $O/sweep_c5.txt; exit 1; }
cat $O/sweep_c5.txt
