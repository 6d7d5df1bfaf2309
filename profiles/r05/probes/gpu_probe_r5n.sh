# Round 5: media inside instanced BVHs (GPU parity), C1 frame timeline (host gaps?), then PMC C5 A1 A2.
export TMPDIR=/tmp
O=gpurun_out/r05_n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_volumes.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/vol_tests.log 2>&1 || { echo "VOLUME TESTS FAILED"; tail -40 $O/vol_tests.log; exit 1; }
tail -2 $O/vol_tests.log
timeout -k 10 300 python3 -u tools/sweep.py --config C1 --steps 30 > $O/c1.txt 2>&1 || { echo "c1 failed"; tail -5 $O/c1.txt; exit 1; }
timeout -k 10 300 python3 -u tools/sweep.py --config C1 --steps 200 >> $O/c1.txt 2>&1 || { echo "c1 failed"; tail -5 $O/c1.txt; exit 1; }
cat $O/c1.txt
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --config C1 --steps 10 --warmup 2 --no-cpu > $O/c1_trace.json 2> $O/c1_trace.err || { echo trace failed; tail -5 $O/c1_trace.err; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r05_n/tr/**/run_kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
prev = None
for r in rows[-12:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev else 0
    print('%-60s %9.1f us  gap %8.1f us' % (r['Kernel_Name'][:60], (e - s) / 1e3, gap))
    prev = e
PY
STAGES=pmc PMC_CONFIGS="C5 A1 A2" TAG=r05_final bash tools/gpu_final.sh
