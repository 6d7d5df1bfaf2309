#!/bin/bash
# Round 5 probes: the -m gpu suite, then final_scene (1440^2 x 64 spp) over leaf batch / node
# steps / shade batch, and the C1 chunk sweep + kernel gaps.  usage: STAGES="tests fs c1" bash tools/gpu_probe_r5.sh
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_f}; mkdir -p $O
for st in ${STAGES:-tests fs}; do
case $st in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log ;;
fs)
  timeout -k 10 900 python3 -u tools/sweep.py --config final_scene --width 1440 --spp 64 --steps 2 ${FS_ARGS:---leaf-batch 12 24 48 --node-steps 8 3} > $O/fs.txt 2>&1 || { echo "fs sweep failed"; tail -5 $O/fs.txt; exit 1; }
  cat $O/fs.txt ;;
c1)
  bash tools/gpu_probe_c1.sh ;;
esac
done
