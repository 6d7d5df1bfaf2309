# Round 5: the small-frame rule with the learned per-sample cost (host-side; code object
# c557a991 unchanged): GPU suite, every 400-px reference scene, C1.
export TMPDIR=/tmp
O=gpurun_out/r05_r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
S="checkered_spheres perlin_spheres simple_light earth earth_hdr hdri quads triangles cornell_box bouncing_spheres"
timeout -k 10 900 python3 -u tools/sweep.py --config $S --steps 3 > $O/rule.txt 2>&1 || { echo "rule failed"; tail -5 $O/rule.txt; exit 1; }
cat $O/rule.txt
timeout -k 10 300 python3 -u tools/sweep.py --config C1 --steps 30 > $O/c1.txt 2>&1 || { echo "c1 failed"; tail -5 $O/c1.txt; exit 1; }
cat $O/c1.txt
