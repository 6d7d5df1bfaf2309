#!/bin/bash
# Round 4: 96-B cube records with an LDS mirror: cube tests and the -m gpu suite, A/B against
# the list loop (cube0), lazy face loads (clazy), no cube mirror (cnolds); stamps.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cube.py -x -v --timeout 120 --timeout-method thread > $O/cube_tests.log 2>&1 || { echo "CUBE TESTS FAILED"; tail -40 $O/cube_tests.log; exit 1; }
tail -3 $O/cube_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/cube0.so variants/clazy.so variants/cnolds.so variants/nww.so --config final_scene cornell_smoke --width 1440 --spp 64 --steps 2 > $O/ab_fs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_fs.txt; exit 1; }
cat $O/ab_fs.txt
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/cube0.so variants/clazy.so variants/cnolds.so --config C3 --steps 2 > $O/ab_c3.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/cube0.so variants/clazy.so variants/cnolds.so --config C5 --spp 256 --steps 2 > $O/ab_c5.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
for spec in "final_scene 1440 64" "cornell_smoke 1440 64"; do
  set -- $spec
  GS_LIB=$R/grayshift_amd/variants/stamps.so timeout -k 10 150 python3 $R/tools/stamps.py --config $1 --width $2 --spp $3 > $O/stamps_$1.txt 2> $O/stamps_$1.err || { echo "stamps $1 failed rc=$?"; tail -3 $O/stamps_$1.err; exit 1; }
  echo "== stamps $1"; cat $O/stamps_$1.txt
done
