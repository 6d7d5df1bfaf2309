# wave-priority defaults: the GPU suite on the product build, then A/B against leaf priority off
# (l0) and no priority (p0) on the configs the first sweeps did not cover
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/prio3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u tools/sweep.py --config final_scene cornell_smoke --width 1440 --spp 64 --steps 2 --lib base variants/l0.so variants/p0.so || exit 1
timeout -k 10 300 python -u tools/sweep.py --config A2 C4 C3 --steps 2 --lib base variants/p0.so || exit 1
timeout -k 10 400 python -u tools/sweep.py --config C5 --steps 1 --timeout 300 --lib base variants/l0.so variants/p0.so || exit 1
