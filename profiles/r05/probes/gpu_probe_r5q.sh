# Round 5: the small-frame rule (every tile in 4-sample chunks) against the 1-sample tail
# (--tail-pct 200 = the rule off) on every 400-px reference scene it applies to.
export TMPDIR=/tmp
O=gpurun_out/r05_q; mkdir -p $O
S="checkered_spheres perlin_spheres simple_light earth earth_hdr hdri quads triangles cornell_box bouncing_spheres mixed"
timeout -k 10 900 python3 -u tools/sweep.py --config $S --steps 3 --tail-pct 0 200 > $O/rule.txt 2>&1 || { echo "rule failed"; tail -5 $O/rule.txt; exit 1; }
cat $O/rule.txt
