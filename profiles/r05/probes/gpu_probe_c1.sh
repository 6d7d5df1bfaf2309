export TMPDIR=/tmp
O=gpurun_out/r05_e; mkdir -p $O
timeout -k 10 300 python3 -u tools/sweep.py --config C1 --steps 20 --sample-chunk -1 2 4 8 25 100 > $O/c1_chunk.txt 2>&1; cat $O/c1_chunk.txt
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --config C1 --steps 10 --warmup 2 --no-cpu > $O/c1_trace.json 2> $O/c1_trace.err || { echo trace failed; tail -5 $O/c1_trace.err; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r05_e/tr/**/run_kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
prev = None
for r in rows[-40:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev else 0
    print('%-60s %9.1f us  gap %8.1f us' % (r['Kernel_Name'][:60], (e - s) / 1e3, gap))
    prev = e
PY
