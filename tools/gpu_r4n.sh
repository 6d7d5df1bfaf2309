#!/bin/bash
# Round 4: final_scene leaf batch x shade batch at 8 node steps, twice.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4n
mkdir -p $O
for rep in 1 2; do
timeout -k 10 900 python3 -u tools/sweep.py --config final_scene --width 1440 --spp 64 --steps 2 --leaf-batch 48 56 64 --node-steps 8 --shade-batch 44 52 > $O/sweep_fs_$rep.txt 2>&1 || { echo "sweep failed"; tail -5 $O/sweep_fs_$rep.txt; exit 1; }
cat $O/sweep_fs_$rep.txt
done
