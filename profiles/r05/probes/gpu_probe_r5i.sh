# Round 5: C1 frame overheads (queue reset in the params kernel, chunk-major sums, pinned
# counters copy, one event fewer) and the guided tail's knobs.
export TMPDIR=/tmp
O=gpurun_out/r05_i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python3 -u tools/sweep.py --config C1 --steps 30 --fine-chunk 0 4 8 --tail-pct 0 50 100 > $O/c1_tail.txt 2>&1 || { echo "c1 failed"; tail -5 $O/c1_tail.txt; exit 1; }
cat $O/c1_tail.txt
timeout -k 10 600 python3 -u tools/sweep.py --config C1 --steps 30 --sample-chunk 8 --fine-chunk 0 2 4 --tail-pct 0 25 100 > $O/c1_tail8.txt 2>&1 || { echo "c1 8 failed"; tail -5 $O/c1_tail8.txt; exit 1; }
cat $O/c1_tail8.txt
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --config C1 --steps 10 --warmup 2 --no-cpu > $O/c1_trace.json 2> $O/c1_trace.err || { echo trace failed; tail -5 $O/c1_trace.err; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r05_i/tr/**/run_kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
prev = None
for r in rows[-14:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev else 0
    print('%-60s %9.1f us  gap %8.1f us' % (r['Kernel_Name'][:60], (e - s) / 1e3, gap))
    prev = e
PY
timeout -k 10 300 python3 -u tools/sweep.py --config C4 C3 --steps 2 > $O/c4.txt 2>&1 || { echo "c4 failed"; tail -5 $O/c4.txt; exit 1; }
cat $O/c4.txt
