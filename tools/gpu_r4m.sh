#!/bin/bash
# Round 4: final_scene's leaf batch / node steps re-swept after the nested-leaf changes.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4m
mkdir -p $O
timeout -k 10 900 python3 -u tools/sweep.py --config final_scene --width 1440 --spp 64 --steps 2 --leaf-batch 24 32 40 48 56 --node-steps 8 > $O/sweep_fs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/sweep_fs.txt; exit 1; }
cat $O/sweep_fs.txt
timeout -k 10 900 python3 -u tools/sweep.py --config final_scene --width 1440 --spp 64 --steps 2 --leaf-batch 48 --node-steps 4 6 --shade-batch 44 52 60 > $O/sweep_fs2.txt 2>&1 || { echo "sweep failed"; tail -5 $O/sweep_fs2.txt; exit 1; }
cat $O/sweep_fs2.txt
