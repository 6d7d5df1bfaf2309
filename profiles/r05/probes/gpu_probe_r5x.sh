# Round 5: every BASELINE config checked against the CPU oracle over its full frame (C5 every
# 4th row and column: its full frame is ~40 min of CPU), at the config's spp, code object c557a991.
export TMPDIR=/tmp
O=gpurun_out/r05_x; mkdir -p $O
for spec in "C1 1" "C2 1" "A1 1" "A2 1" "C4 1" "C3 1" "C5 4"; do
  set -- $spec
  timeout -k 10 900 python3 -u bench.py --config $1 --steps 1 --warmup 1 --cpu-stride $2 --cpu-runs 1 > $O/full_$1.json 2> $O/full_$1.err || { echo "$1 failed"; tail -5 $O/full_$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/full_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['parity'])"
done
