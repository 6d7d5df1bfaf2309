#!/bin/bash
# Round 4: nested-tree variants (inline sphere records with 1 / 16 radii, the generic test with
# 17, cubes, triangles) against the oracle.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_instancing_noise.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -15 $O/tests.log
