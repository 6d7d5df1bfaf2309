# Round 5: 8-rank projection of C4 by tile size (the cost-balanced plan packs finer tiles tighter?).
export TMPDIR=/tmp
O=gpurun_out/r05_t; mkdir -p $O
timeout -k 10 900 python3 -u tools/rank_sim.py --config C4 --worlds 8 --tiles 32,48,64 --all-ranks --plan > $O/rank_tiles.txt 2> $O/rank_tiles.err || { echo "rank_sim failed"; tail -5 $O/rank_tiles.err; exit 1; }
grep max_rank $O/rank_tiles.txt
