# Round 5: is A2's tail (the last ~15 rounds, ~2-3 ms each) bound by one sample path's
# latency?  Kernel traces of one A2 frame at node steps 1 (the scene's choice) and 8, leaf
# batch 12 and 1.
export TMPDIR=/tmp
O=gpurun_out/r05_k; mkdir -p $O
for spec in "1 0" "8 0" "8 1" "2 1"; do
  set -- $spec
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr_ns$1_lb$2 -o run -- python3 bench.py --config A2 --steps 1 --warmup 1 --no-cpu --node-steps $1 --leaf-batch $2 > $O/a2_ns$1_lb$2.json 2> $O/a2_ns$1_lb$2.err || { echo "trace $spec failed"; tail -5 $O/a2_ns$1_lb$2.err; exit 1; }
  python3 - $O/tr_ns$1_lb$2 "$spec" <<'PY'
import csv, glob, sys, json
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
ks = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows if 'gs_render_kernel' in r['Kernel_Name']]
last = ks[-32:]
print("node_steps/leaf_batch", sys.argv[2], "rounds", len(last), "total %.1f ms" % sum(last), "last 16: %.1f ms" % sum(last[-16:]), " ".join("%.2f" % x for x in last))
PY
done
