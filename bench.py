#!/usr/bin/env python3
"""Benchmark: Msamples/s (primary + secondary rays) of the MI355X megakernel.

Contract:
    python bench.py --gpus N --steps K --warmup W
One step = one full frame of the configured workload (default C4: the 10k-sphere
BVH scene, 1920x1080, 512 spp, HDRI sky), tile-partitioned round-robin over the N
ranks (64x64 tiles), then one RCCL gather of the finished tiles to rank 0 and an
unpack into the frame.  The scene is resident in HBM before timing starts.
value = all rays traced by all ranks / wall time (max over ranks); a "ray" is one
world.hit call (camera.rs:177), counted on the device by the very launches timed.

Rank 0 prints ONE JSON line.  At N=1, rank 0 also times the CPU oracle (the
reference's algorithm restated in C++, oracle/) on a bounded subset of the same
frame (every --cpu-stride-th row and column, ~10 s): `cpu_baseline`.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic bytes per unit: what the reference
# algorithm reads for each counted event.
BYTES = {"node_visits": 56, "sphere_tests": 40, "msphere_tests": 64, "quad_tests": 136, "tri_tests": 104,
         "instance_tests": 32, "medium_tests": 16, "hits": 32, "image_texels": 3, "hdri_texels": 12, "pixels": 12,
         "noise_evals": 168}  # noise: 7 octaves x 8 corners x 3 permutation-table bytes
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def algorithmic_bytes(c):
    return sum(BYTES[k] * int(c[k]) for k in BYTES)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C4", help="BASELINE config C1..C5 (default C4)")
    ap.add_argument("--width", type=int, default=None, help="override (testing only; invalidates the metric)")
    ap.add_argument("--spp", type=int, default=None, help="override (testing only; invalidates the metric)")
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--no-plan", action="store_true",
                    help="N>1: round-robin tiles instead of the cost-balanced plan (gs_plan_tiles)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--shade-batch", type=int, default=None)
    ap.add_argument("--blocks-per-cu", type=int, default=None)
    ap.add_argument("--leaf-batch", type=int, default=None)
    ap.add_argument("--sample-chunk", type=int, default=None, help="samples per work item (-1 auto, 0 whole pixel)")
    ap.add_argument("--cpu-stride", type=int, default=3, help="CPU baseline: every Nth row and column")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_C4_latest.json"),
                    help="JSON with PMC-derived HBM bytes per launch (tools/pmc.sh -> profiles/)")
    ap.add_argument("--dump", default=None, help="write the frame (rank 0) as .npy")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collectives: nccl (= RCCL over xGMI, the measured path) or gloo (host-staged; testing)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="testing only: every rank uses cuda:0 (rehearse N>1 on a one-GPU box; use --backend gloo)")
    return ap.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus %d needs torch.distributed.run with %d ranks" % (a.gpus, a.gpus))
    if a.share_gpu:
        local = 0
    if local >= torch.cuda.device_count():
        raise SystemExit("rank %d: LOCAL_RANK %d but only %d GPUs visible (one GPU per rank)"
                         % (rank, local, torch.cuda.device_count()))
    torch.cuda.set_device(local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    host_coll = world > 1 and a.backend == "gloo"  # gloo collectives on host copies

    import grayshift_amd as g
    from grayshift_amd import scenes

    g.set_tuning(a.shade_batch or 52, a.blocks_per_cu or 0, 12 if a.leaf_batch is None else a.leaf_batch,
                 -1 if a.sample_chunk is None else a.sample_chunk)
    sc = scenes.config(a.config, width=a.width, spp=a.spp)
    # N > 1: tiles are assigned by a cost-balanced plan computed once at setup (a 1-spp pilot
    # of the frame, identical on every rank; outside the timed region, like the BVH build).
    plan = world > 1 and not a.no_plan
    r = g.Renderer(sc, rank=rank, world_size=world, tile=a.tile, plan=plan)
    # Every rank's packed buffer has rank 0's capacity (the most tiles any rank holds)
    p0 = g._native.gs_partition(0, world, a.tile, a.tile, r.part.d_tile_order, r.part.slots_per_rank, 0)
    cap0 = g._native.lib.gs_partition_capacity(__import__("ctypes").byref(r.cam), __import__("ctypes").byref(p0))
    dev = torch.device("cuda", local)
    packed = torch.zeros(cap0 * 3, dtype=torch.float32, device=dev)
    counters = torch.zeros(16, dtype=torch.int64, device=dev)
    frame = torch.zeros(r.height * r.width * 3, dtype=torch.float32, device=dev) if rank == 0 else None
    gathered = torch.empty(world * cap0 * 3, dtype=torch.float32, device=dev) if (rank == 0 and world > 1) else None
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    kernel_ms = []

    def step(timed):
        counters.zero_()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        r.render_async(packed.data_ptr(), counters.data_ptr(), sptr, seed=a.seed)
        ev1.record(stream)
        if world > 1 and host_coll:
            src = packed.cpu()
            if rank == 0:
                bufs = [torch.empty_like(src) for _ in range(world)]
                dist.gather(src, gather_list=bufs, dst=0)
                gathered.copy_(torch.cat(bufs))
                r.unpack_async(gathered.data_ptr(), frame.data_ptr(), world, sptr)
            else:
                dist.gather(src, dst=0)
        elif world > 1:
            if rank == 0:
                dist.gather(packed, gather_list=list(gathered.view(world, -1).unbind(0)), dst=0)
                r.unpack_async(gathered.data_ptr(), frame.data_ptr(), world, sptr)
            else:
                dist.gather(packed, dst=0)
        else:
            r.unpack_async(packed.data_ptr(), frame.data_ptr(), 1, sptr)
        if timed:
            kernel_ms.append((ev0, ev1))

    # The counter accumulation runs in the warm-up too: the first torch int64 add loads its
    # kernel (~13 ms), which must not land in the timed region.
    tot = torch.zeros(16, dtype=torch.int64, device=dev)
    for _ in range(a.warmup):
        step(False)
        tot += counters
    torch.cuda.synchronize()
    tot.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
        tot += counters
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kms = [e0.elapsed_time(e1) for e0, e1 in kernel_ms]
    if world > 1:
        cdev = torch.device("cpu") if host_coll else dev
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot_c = tot.to(cdev)
        dist.all_reduce(tot_c, op=dist.ReduceOp.SUM)
        tot = tot_c.to(dev)
        km = torch.tensor([sum(kms) / len(kms)], dtype=torch.float64, device=cdev)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kernel_avg_ms = float(km.item())
    else:
        kernel_avg_ms = sum(kms) / len(kms)

    from grayshift_amd._native import COUNTER_NAMES
    c = {n: int(tot[i].item()) // a.steps for i, n in enumerate(COUNTER_NAMES)}
    rays_per_frame = c["rays"]
    value = rays_per_frame * a.steps / elapsed / 1e6
    abytes = algorithmic_bytes(c) / max(1, world)  # per launch (per rank)
    achieved = abytes / (kernel_avg_ms / 1e3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(sc, a)

    traffic = None
    if a.traffic and os.path.exists(a.traffic) and world == 1:  # a 1-GPU whole-frame figure
        with open(a.traffic) as f:
            tj = json.load(f)
        if tj.get("config") == a.config and tj.get("hbm_bytes_per_launch") and a.width is None and a.spp is None:
            traffic = tj["hbm_bytes_per_launch"]

    if rank == 0:
        if a.dump:
            import numpy as np
            np.save(a.dump, frame.view(r.height, r.width, 3).cpu().numpy())
        invalid = a.width is not None or a.spp is not None
        out = {
            "metric": "Msamples/sec (primary+secondary rays)",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (deterministic scene generator, seed 'grayshif'; decoded reference assets)",
            "config": {
                "workload": "%s: %s %dx%d, %d spp%s" % (a.config, sc.name, r.width, r.height,
                                                      sc.settings.batch_size,
                                                      " (OVERRIDDEN: not the metric)" if invalid else ""),
                "tile": a.tile, "parallelism": "tiles%d" % world, "tile_plan": "cost-balanced" if plan else "round-robin",
                "seed": a.seed,
                "rays_per_frame": rays_per_frame, "paths_per_frame": c["paths"],
                "node_visits_per_ray": round(c["node_visits"] / max(1, rays_per_frame), 3),
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel_ms": round(kernel_avg_ms, 3), "algorithmic_bytes_per_launch": int(abytes),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    r.close()


def cpu_baseline(sc, a):
    """The CPU oracle on every cpu_stride-th row and column of the same frame."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test-infrastructure checker, used here only as the CPU baseline
    threads = a.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    W, H, s = sc.width, sc.height, a.cpu_stride
    sub = np.array([j * W + i for j in range(0, H, s) for i in range(0, W, s)], dtype=np.int32)
    t0 = time.perf_counter()
    _, c = oracle.render(sc, seed=a.seed, threads=threads, subset=sub)
    dt = time.perf_counter() - t0
    return {"value": round(c["rays"] / dt / 1e6, 3), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": "%d px (every %dth row/col of the frame) x %d spp = %d rays in %.1fs (incl. world/BVH build)"
                      % (len(sub), s, sc.settings.batch_size, c["rays"], dt)}


if __name__ == "__main__":
    main()
