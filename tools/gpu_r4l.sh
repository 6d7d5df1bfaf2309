#!/bin/bash
# Round 4: the nested spheres' radius by a scalar load when a wave shares it -- A/B on
# final_scene (two runs each), GPU tests of the nested scenes, stamps of final_scene.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instancing_noise.py tests/test_gpu_cube.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/nrad0.so base variants/nrad0.so --config final_scene --width 1440 --spp 64 --steps 2 > $O/ab_fs.txt 2>&1 || { echo "sweep failed"; tail -5 $O/ab_fs.txt; exit 1; }
cat $O/ab_fs.txt
GS_LIB=$R/grayshift_amd/variants/stamps.so timeout -k 10 150 python3 $R/tools/stamps.py --config final_scene --width 1440 --spp 64 > $O/stamps_final_scene.txt 2> $O/stamps_final_scene.err || { echo "stamps failed"; tail -3 $O/stamps_final_scene.err; exit 1; }
cat $O/stamps_final_scene.txt
