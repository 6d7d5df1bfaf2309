# Round 5: returns from nested trees taken at the start of the leaf pass (variant retmerge):
# its nested / media parity tests, then final_scene A/B at 1440^2 x 64.
export TMPDIR=/tmp
O=gpurun_out/r05_v; mkdir -p $O
GS_LIB=$PWD/grayshift_amd/variants/retmerge.so timeout -k 10 600 python -u -m pytest tests/test_gpu_instancing_noise.py tests/test_gpu_volumes.py tests/test_gpu_cube.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/variant_tests.log 2>&1 || { echo "VARIANT TESTS FAILED"; tail -30 $O/variant_tests.log; exit 1; }
tail -2 $O/variant_tests.log
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/retmerge.so base variants/retmerge.so --config final_scene --width 1440 --spp 64 --steps 2 > $O/ab.txt 2>&1 || { echo "ab failed"; tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
