#!/usr/bin/env python3
"""Simulate one rank of an N-GPU run on one GPU: time rank r's share of the C4 frame
(gs_render_tiles_async over its round-robin tiles) for a given world size and sample
chunk, and report that rank's ray throughput.  Strong-scaling efficiency at N GPUs is
~ (rank throughput at N) / (throughput at 1), since every rank runs the same kind of
work.  Usage: python tools/rank_sim.py --worlds 1,8 --chunks -1,16 [--ranks 0,3 | --all-ranks]
[--config C5 --spp 4096] [--plan]; with --all-ranks the last line per world is the projection:
the slowest rank's time bounds the N-GPU frame before the gather.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,8")
    ap.add_argument("--chunks", default="-1")
    ap.add_argument("--ranks", default="0")
    ap.add_argument("--config", default="C4")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--tiles", default="64")
    ap.add_argument("--tile-h", type=int, default=0, help="tile height (default: square tiles)")
    ap.add_argument("--plan", action="store_true", help="cost-balanced tiles (gs_plan_tiles)")
    ap.add_argument("--all-ranks", action="store_true", help="every rank of each world size, and the projection")
    ap.add_argument("--spp", type=int, default=None, help="override the config's spp")
    a = ap.parse_args()
    import torch
    import grayshift_amd as g
    from grayshift_amd import scenes
    sc = scenes.config(a.config, spp=a.spp)
    one_ms = None
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    for world, tile, chunk in [(w, t, c) for w in [int(x) for x in a.worlds.split(",")]
                               for t in [int(x) for x in a.tiles.split(",")]
                               for c in [int(x) for x in a.chunks.split(",")]]:
        if True:
            g.set_tuning(0, 0, 0, chunk)
            worst = 0.0
            for rank in (range(world) if a.all_ranks else [int(x) for x in a.ranks.split(",")]):
                if rank >= world:
                    continue
                r = g.Renderer(sc, rank=rank, world_size=world, tile=tile, tile_h=a.tile_h or tile, plan=a.plan)
                out = torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev)
                cnt = torch.zeros(16, dtype=torch.int64, device=dev)
                r.render_async(out.data_ptr(), cnt.data_ptr(), stream.cuda_stream, seed=1)  # warm-up
                torch.cuda.synchronize()
                best = 1e30
                for _ in range(a.reps):
                    cnt.zero_()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    r.render_async(out.data_ptr(), cnt.data_ptr(), stream.cuda_stream, seed=1)
                    torch.cuda.synchronize()
                    best = min(best, time.perf_counter() - t0)
                rays = int(cnt[0].item())
                print(json.dumps({"config": a.config, "world": world, "tile": tile, "plan": a.plan, "rank": rank, "chunk": chunk,
                                  "ms": round(best * 1e3, 2), "Msamples_per_s": round(rays / best / 1e6, 1)}), flush=True)
                worst = max(worst, best)
                r.close()
            if a.all_ranks:
                if world == 1:
                    one_ms = worst * 1e3
                print(json.dumps({"config": a.config, "world": world, "max_rank_ms": round(worst * 1e3, 2),
                                  "projected_speedup": round(one_ms / (worst * 1e3), 3) if one_ms else None}), flush=True)


if __name__ == "__main__":
    main()
