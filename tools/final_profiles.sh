#!/bin/bash
# Evidence for one kernel version under profiles/: rocprof kernel stats + the bench line of
# the same command, PMC passes (tools/pmc.sh), and the stamps phase split.
# usage (on the GPU box): bash tools/final_profiles.sh <tag>     -> gpurun_out/prof_<tag>/...
set -o pipefail
export TMPDIR=/tmp
T=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$T
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --steps 3 --warmup 1 > $O/bench.log 2>&1 || { echo "stats run failed"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
bash $R/tools/pmc.sh || exit 1
python3 $R/tools/pmc_summary.py $R/gpurun_out $O/pmc.json || exit 1
GS_LIB=$R/grayshift_amd/variants/stamps.so timeout -k 10 200 python3 $R/tools/stamps.py > $O/stamps.txt 2>$O/stamps.err || { echo "stamps failed"; tail -5 $O/stamps.err; exit 1; }
cat $O/stamps.txt
