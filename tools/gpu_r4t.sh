#!/bin/bash
# Round 4: the stamps build on the adaptive configs (A1: the per-lane loop; A2: batch rounds).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4t
mkdir -p $O
for c in A1 A2; do
  GS_LIB=$R/grayshift_amd/variants/stamps.so timeout -k 10 200 python3 $R/tools/stamps.py --config $c > $O/stamps_$c.txt 2> $O/stamps_$c.err || { echo "stamps $c failed"; tail -5 $O/stamps_$c.err; exit 1; }
  echo "== stamps $c"; cat $O/stamps_$c.txt
done
