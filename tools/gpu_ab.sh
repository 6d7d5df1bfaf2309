#!/bin/bash
# A/B of library builds on one GPU: the -m gpu suite on the product library, then
# tools/sweep.py over the given builds and configs.
# usage (on the GPU box): LIBS="base variants/x.so" CONFIGS="C4 C3" bash tools/gpu_ab.sh [tag]
set -o pipefail
export TMPDIR=/tmp
T=${1:-ab}
O=gpurun_out/$T
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
timeout -k 10 900 python -u tools/sweep.py --lib ${LIBS:-base} --config ${CONFIGS:-C4} --steps ${STEPS:-2} ${SWEEP_ARGS} 2>&1 | tee $O/sweep.txt
