#!/bin/bash
# Round 4: node steps per unrolled node pass, 8 (base) / 12 / 16, on final_scene and C4.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4u
mkdir -p $O
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/ns12.so variants/ns16.so base variants/ns12.so variants/ns16.so --config final_scene --width 1440 --spp 64 --steps 2 > $O/ab_fs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_fs.txt; exit 1; }
cat $O/ab_fs.txt
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/ns12.so variants/ns16.so --config C4 C5 --steps 2 --spp 128 > $O/ab_c4.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
