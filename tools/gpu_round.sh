#!/bin/bash
# One GPU call: the -m gpu suite, the default bench line (C4, parity + CPU baseline),
# the rocprofv3 kernel stats of the same command, and (PMC=1) the PMC passes.
# usage (on the GPU box): TAG=r02_x PMC=1 bash tools/gpu_round.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TAG:-run}
O=$R/gpurun_out/$T
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 > $O/stats_bench.json 2> $O/stats_bench.err || { echo "stats run failed"; tail -5 $O/stats_bench.err; exit 1; }
cat $O/stats_bench.json
find $O/stats -name "*kernel_stats.csv" -exec head -4 {} \;
if [ "${PMC:-0}" = 1 ]; then
  CONFIG=C4 bash $R/tools/pmc.sh || exit 1
fi
if [ "${STAMPS:-0}" = 1 ]; then
  GS_LIB=$R/grayshift_amd/variants/stamps.so timeout -k 10 200 python3 $R/tools/stamps.py > $O/stamps.txt 2> $O/stamps.err || { echo "stamps failed"; tail -5 $O/stamps.err; exit 1; }
  cat $O/stamps.txt
fi
