# Round 5: adaptive A1 / A2 under each mode (1 auto, 2 batch rounds, 0 the per-lane loop) on
# the final code object: does the auto rule still pick the faster one?
export TMPDIR=/tmp
O=gpurun_out/r05_z; mkdir -p $O
for m in 1 2 0; do
  for c in A1 A2; do
    timeout -k 10 300 python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu --adaptive-mode $m > $O/${c}_m$m.json 2> $O/${c}_m$m.err || { echo "$c m$m failed"; tail -5 $O/${c}_m$m.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${c}_m$m.json').read().strip().splitlines()[-1]); print('$c mode $m', d['value'], d['ms_per_step'])"
  done
done
