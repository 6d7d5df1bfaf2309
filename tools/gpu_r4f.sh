#!/bin/bash
# Round 4: axis-aligned quad test (GS_AQUAD) -- the -m gpu suite on the product library,
# A/B against the full test (aq0) and the wave-uniform copies (aqu), leaf-kind stamps.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/aq0.so variants/aqu.so --config final_scene cornell_smoke --width 1440 --spp 64 --steps 2 > $O/ab_fs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_fs.txt; exit 1; }
cat $O/ab_fs.txt
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/aq0.so variants/aqu.so --config C3 C4 --steps 2 > $O/ab_c3.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_c3.txt; exit 1; }
cat $O/ab_c3.txt
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/aq0.so --config C5 --spp 256 --steps 2 > $O/ab_c5.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
for spec in "final_scene 1440 64" "cornell_smoke 1440 64" "C3 1024 256"; do
  set -- $spec
  GS_LIB=$R/grayshift_amd/variants/stamps.so timeout -k 10 150 python3 $R/tools/stamps.py --config $1 --width $2 --spp $3 > $O/stamps_$1.txt 2> $O/stamps_$1.err || { echo "stamps $1 failed rc=$?"; tail -3 $O/stamps_$1.err; exit 1; }
  echo "== stamps $1"; cat $O/stamps_$1.txt
done
