# A2 (adaptive batch rounds) probes: the adaptive GPU tests, then A/B builds on A2 (tools/sweep.py)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/${TAG:-a2probe}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_adaptive.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u tools/sweep.py --config A2 --steps 2 --lib ${LIBS:-base} > $O/sweep.txt 2>&1 || { echo SWEEP FAILED; tail -20 $O/sweep.txt; exit 1; }
cat $O/sweep.txt
# per-launch kernel times of one A2 frame (rocprofv3 kernel trace)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config A2 --steps 1 --warmup 1 --no-cpu > $O/trace.json 2>$O/trace.err || { echo TRACE FAILED; tail -5 $O/trace.err; exit 1; }
python3 - $O <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/trace/run_kernel_trace.csv")))
by = {}
for r in rows:
    by.setdefault(r["Kernel_Name"].split("(")[0][:40], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in by.items():
    print("%-40s %4d launches %9.2f ms total (2 frames)" % (k, len(v), sum(v)))
PY
