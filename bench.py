#!/usr/bin/env python3
"""Benchmark: Msamples/s (primary + secondary rays) of the MI355X megakernel.

Contract:
    python bench.py --gpus N --steps K --warmup W
One step = one full frame of the configured workload (default C4: the 10k-sphere
BVH scene, 1920x1080, 512 spp, HDRI sky), tile-partitioned over N GPUs (64x64 tiles;
cost-balanced plan for N > 1), then one RCCL gather of the finished tiles to the first
GPU and an unpack into the frame.  The scene is resident in HBM before timing starts.
value = all rays traced on all GPUs / wall time; a "ray" is one world.hit call
(camera.rs:177), counted on the device by the very launches timed.

Two launch modes, one frame:
* no launcher (WORLD_SIZE unset): one process drives N devices through the C-ABI frame
  context (gs_multi_create once — scene upload, ncclCommInitAll — then gs_multi_render
  per frame: render on every device, ncclGather, unpack).  --gpus N above the visible
  device count fails with a message and a non-zero exit.
* under torch.distributed.run (WORLD_SIZE = N): one process per GPU; each rank renders
  its planned tiles (plan from rank 0, broadcast), one torch.distributed gather (backend
  nccl = RCCL over xGMI) to rank 0, which unpacks; the time is the max over ranks.

Rank 0 prints ONE JSON line with, beside the contract's fields:
* parity — the timed frame checked against the CPU oracle (the reference's algorithm
  restated, oracle/) on a deterministic pixel subset, at the full config;
* cpu_baseline — at N=1 the oracle's render time on that subset (median of 3, world and
  BVH build excluded), on this host's cores;
* roofline — the kernel's binding ceiling, VALU issue: the VALU busy cycles the PMC
  counters of this very code object measured (profiles/pmc/, keyed by the hash of the
  library's gfx950 code objects; 4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2), below)
  over the SIMDs' cycles of this run's kernel time, with the per-class pricing bracket
  beside it (frac_lower / frac_upper); the measured HBM fraction and the cache-served
  algorithmic byte rate beside those.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic bytes per unit: what the reference
# algorithm reads for each counted event.  Almost all of it is served from LDS / L1 / L2,
# so its rate is not an HBM figure.
BYTES = {"node_visits": 56, "sphere_tests": 40, "msphere_tests": 64, "quad_tests": 136, "tri_tests": 104,
         "instance_tests": 32, "medium_tests": 16, "hits": 32, "image_texels": 3, "hdri_texels": 12, "pixels": 12,
         "noise_evals": 168}  # noise: 7 octaves x 8 corners x 3 permutation-table bytes
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
SIMDS = 1024  # 256 CUs x 4 SIMDs
# Issue cycles per wave64 VALU instruction on one SIMD-32 at full occupancy, by the PMC
# instruction classes (SQ_INSTS_VALU_*; "OTHER" = SQ_INSTS_VALU minus the listed classes:
# moves, compares, selects, bit operations, f32 min/max).  MI355X_MICROARCH.md:54,473: a
# wave64 32-bit VALU instruction issues over 2 cycles on a SIMD-32; f64 runs at half the
# f32 vector rate (4).  tools/ubench/valu_rate.hip (profiles/r03/valu_rate_ubench.txt,
# 8 waves per SIMD, cycles at the in-kernel clock) measured: 2.2 for VOP1/VOP2 forms with
# VGPR operands, 4.1 for the 8-byte VOP3 forms (SGPR / constant operands, v_pk_fma_f32,
# 64-bit integer ops) and every f64 add / mul / fma, 8.1 for v_sqrt_f32, 16.1 for
# v_sqrt_f64 / v_rcp_f64.  VALU_CYCLES prices the classes at those costs with 32-bit
# non-transcendental work at the guide's 2 (a lower bound: the kernel's VOP3 share costs
# 4), so `frac` is the smallest defensible VALU-issue fraction.  (Pricing every
# non-transcendental instruction at the VOP3 cost of 4 instead gives 1.01 for the round-3
# kernel -- more issue cycles than the SIMDs had -- so that bound is no longer reported.)
VALU_CYCLES = {"ADD_F32": 2, "MUL_F32": 2, "FMA_F32": 2, "TRANS_F32": 8, "ADD_F64": 4, "MUL_F64": 4,
               "FMA_F64": 4, "TRANS_F64": 16, "INT32": 2, "INT64": 4, "CVT": 2, "OTHER": 2}
# ... and the upper end of that bracket: every non-transcendental instruction at the VOP3 cost.
VALU_CYCLES_UPPER = dict(VALU_CYCLES, ADD_F32=4, MUL_F32=4, FMA_F32=4, INT32=4, CVT=4, OTHER=4)
# The point estimate (round 4, profiles/r04/valu_dual_issue_ubench.txt): on gfx950 every VALU
# instruction holds its SIMD for SQ_ACTIVE_INST_VALU quad-cycles (1; 2 for v_sqrt_f32 class, 4
# for f64 transcendentals), and two VOP1/VOP2 instructions of different waves can issue in one
# quad-cycle, counted by SQ_ACTIVE_INST_VALU2.  On the microbenchmark 4 x (ACTIVE_INST_VALU -
# ACTIVE_INST_VALU2) / instructions reproduces every measured cost: v_add_f32_e32 2.16 (measured
# 2.20), v_fma_f32 with VGPRs 3.56 (3.65), v_fmac_f32_e32 3.65 (3.73), VOP3 / f64 4.0 (4.1-4.2),
# v_sqrt_f32 8 (8.1), f64 rcp / sqrt 16 (16.1).  So the kernel's VALU busy cycles are measured,
# not priced: busy = 4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) summed over the SIMDs.
PARITY_TOL = 1e-3  # north star: per-channel |delta| < 1e-3 vs the CPU path at a fixed seed


def settings_desc(ss):
    """'512 spp' for fixed-spp settings (one batch, camera.rs:158), else the adaptive ones."""
    if ss.tolerance == 0.0 and ss.max_samples < ss.batch_size:
        return "%d spp" % ss.batch_size
    return "adaptive (confidence %g, tolerance %g, batch %d, max %d)" % (ss.confidence, ss.tolerance, ss.batch_size,
                                                                        ss.max_samples)


def algorithmic_bytes(c):
    return sum(BYTES[k] * int(c[k]) for k in BYTES)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C4",
                    help="BASELINE config C1..C5 (default C4), or a scene name of grayshift_amd.scenes (testing only; "
                         "not the metric; --width / --spp default to 400 / 64)")
    ap.add_argument("--width", type=int, default=None, help="override (testing only; invalidates the metric)")
    ap.add_argument("--spp", type=int, default=None, help="override (testing only; invalidates the metric)")
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--no-plan", action="store_true",
                    help="N>1: round-robin tiles instead of the cost-balanced plan (gs_plan_tiles)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--shade-batch", type=int, default=None)
    ap.add_argument("--blocks-per-cu", type=int, default=None)
    ap.add_argument("--leaf-batch", type=int, default=None)
    ap.add_argument("--node-steps", type=int, default=0, help="node steps per node pass (0: the scene's choice)")
    ap.add_argument("--camera-batch", type=int, default=0,
                    help="lanes wanting a camera ray before a wave generates them (0: the scene's choice)")
    ap.add_argument("--sample-chunk", type=int, default=None, help="samples per work item (-1 auto, 0 whole pixel)")
    ap.add_argument("--fine-chunk", type=int, default=0, help="auto chunks' guided tail: samples per fine chunk (0: default)")
    ap.add_argument("--tail-pct", type=int, default=0,
                    help="auto chunks' guided tail: fine samples as %% of lanes x coarse chunk (0: default 200)")
    ap.add_argument("--adaptive-mode", type=int, default=1, choices=[0, 1, 2],
                    help="adaptive settings (gs_set_adaptive_mode): 1 auto (default), 2 batch rounds, 0 the per-lane loop")
    ap.add_argument("--cpu-stride", type=int, default=3,
                    help="CPU baseline / parity subset at N=1: every Nth row and column")
    ap.add_argument("--parity-stride", type=int, default=12, help="parity subset at N>1: every Nth row and column")
    ap.add_argument("--cpu-runs", type=int, default=3, help="CPU baseline: median of this many renders")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline and the parity check")
    ap.add_argument("--pmc-dir", default=os.path.join(ROOT, "profiles", "pmc"),
                    help="PMC summaries (tools/pmc_summary.py), matched by code-object hash and config")
    ap.add_argument("--dump", default=None, help="write the frame (rank 0) as .npy")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collectives: nccl (= RCCL over xGMI, the measured path) or gloo (host-staged; testing)")
    ap.add_argument("--gather", action="store_true",
                    help="run the gather path even at N=1 (a 1-rank process group; exercises RCCL on one GPU)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="testing only: every rank uses cuda:0 (rehearse N>1 on a one-GPU box; use --backend gloo)")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in os.environ and world != a.gpus:
        raise SystemExit("bench.py: --gpus %d under a launcher with WORLD_SIZE=%d (one rank per GPU)" % (a.gpus, world))
    if world > 1 or a.gather:
        return main_ranks(a, world)
    return main_context(a)


def load_scene(a):
    import grayshift_amd as g
    from grayshift_amd import scenes
    g.set_tuning(a.shade_batch or 0, a.blocks_per_cu or 0, 0 if a.leaf_batch is None else a.leaf_batch,
                 -1 if a.sample_chunk is None else a.sample_chunk)
    g._native.check(g._native.lib.gs_set_node_steps(a.node_steps))
    g._native.check(g._native.lib.gs_set_camera_batch(a.camera_batch))
    g._native.check(g._native.lib.gs_debug_set_guided_tail(a.fine_chunk, a.tail_pct))
    g._native.check(g._native.lib.gs_set_adaptive_mode(a.adaptive_mode))
    if a.config in scenes.CONFIGS:
        return scenes.config(a.config, width=a.width, spp=a.spp)
    a.width, a.spp = a.width or 400, a.spp or 64
    return scenes.SCENES[a.config](width=a.width, settings=scenes.fixed_spp(a.spp))


def main_context(a):
    """One process, N devices, through the C-ABI frame context (gs_multi_*)."""
    import ctypes as C
    import numpy as np
    import torch
    n_vis = torch.cuda.device_count()  # (counts devices without initialising HIP)
    if a.gpus < 1 or a.gpus > n_vis:
        print("bench.py: --gpus %d but %d GPU(s) visible" % (a.gpus, n_vis), file=sys.stderr, flush=True)
        raise SystemExit(2)
    import grayshift_amd as g
    from grayshift_amd import _native as N
    sc = load_scene(a)
    plan = a.gpus > 1 and not a.no_plan
    m = g.MultiRenderer(sc, num_gpus=a.gpus, tile=a.tile, plan=plan)

    def sync_all():
        for d in m.devices:
            torch.cuda.synchronize(d)

    for _ in range(a.warmup):
        m.render(seed=a.seed)
    sync_all()
    # every frame's gs_stats into its own preallocated struct; read after the timed loop
    stats = [N.gs_stats() for _ in range(a.steps)]
    t0 = time.perf_counter()
    for st in stats:
        m.render_stats(a.seed, st)  # synchronous: returns once the frame is in the device frame
    sync_all()
    elapsed = time.perf_counter() - t0
    kms = [st.kernel_ms_max for st in stats]
    tot = None
    for st in stats:
        cd = st.counters.as_dict()
        tot = cd if tot is None else {k: tot[k] + v for k, v in cd.items()}
    c = {k: v // a.steps for k, v in tot.items()}
    d_rgb, dev0 = m.frame_ptr()
    img = np.zeros((m.height, m.width, 3), dtype=np.float32)
    N.check(N.lib.gs_device_download(img.ctypes.data, C.c_void_p(d_rgb), img.nbytes))
    emit(a, sc, m, c, elapsed, sum(kms) / len(kms), img, a.gpus,
         {"tile_plan": "cost-balanced" if plan else "round-robin",
          "collective": "rccl" if a.gpus > 1 else "none",
          "launch": "one process, %d device(s): gs_multi_create once, gs_multi_render per frame" % a.gpus})
    m.close()


def main_ranks(a, world):
    """One process per GPU under torch.distributed.run (or --gather at N=1)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.share_gpu:
        local = 0
    if local >= torch.cuda.device_count():
        raise SystemExit("rank %d: LOCAL_RANK %d but only %d GPUs visible (one GPU per rank)"
                         % (rank, local, torch.cuda.device_count()))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if a.backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    host_coll = a.backend == "gloo"  # gloo collectives on host copies

    import grayshift_amd as g
    sc = load_scene(a)
    # N > 1: tiles are assigned by a cost-balanced plan (a 1-spp pilot of the frame),
    # computed once at setup on rank 0 and broadcast, so every rank uses the same one
    # (outside the timed region, like the BVH build).
    plan = world > 1 and not a.no_plan
    if plan:
        cam = g.camera(sc.camera)
        tiles = -(-cam.image_width // a.tile) * -(-cam.image_height // a.tile)
        slots = -(-tiles // world)  # gs_plan_tiles: at most ceil(tiles / world) per rank
        r = g.Renderer(sc, rank=rank, world_size=world, tile=a.tile, plan=True) if rank == 0 else None
        cdev = torch.device("cpu") if host_coll else dev
        t = torch.from_numpy(r.order).to(cdev) if rank == 0 else \
            torch.empty(slots * world, dtype=torch.int32, device=cdev)
        dist.broadcast(t, src=0)
        order = t.cpu().numpy()
        if rank != 0:
            r = g.Renderer(sc, rank=rank, world_size=world, tile=a.tile, order=order)
    else:
        r = g.Renderer(sc, rank=rank, world_size=world, tile=a.tile)
    # Every rank's packed buffer has rank 0's capacity (the most tiles any rank holds)
    import ctypes as C
    p0 = g._native.gs_partition(0, world, a.tile, a.tile, r.part.d_tile_order, r.part.slots_per_rank, 0)
    cap0 = g._native.lib.gs_partition_capacity(C.byref(r.cam), C.byref(p0))
    packed = torch.zeros(cap0 * 3, dtype=torch.float32, device=dev)
    counters = torch.zeros(16, dtype=torch.int64, device=dev)
    frame = torch.zeros(r.height * r.width * 3, dtype=torch.float32, device=dev) if rank == 0 else None
    gathered = torch.empty(world * cap0 * 3, dtype=torch.float32, device=dev) if rank == 0 else None
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
        if host_coll:
            src = packed.cpu()
            if rank == 0:
                bufs = [torch.empty_like(src) for _ in range(world)]
                dist.gather(src, gather_list=bufs, dst=0)
                gathered.copy_(torch.cat(bufs))
                r.unpack_async(gathered.data_ptr(), frame.data_ptr(), world, sptr)
            else:
                dist.gather(src, dst=0)
        else:  # RCCL over xGMI
            if rank == 0:
                dist.gather(packed, gather_list=list(gathered.view(world, -1).unbind(0)), dst=0)
                r.unpack_async(gathered.data_ptr(), frame.data_ptr(), world, sptr)
            else:
                dist.gather(packed, dst=0)
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
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
        tot += counters
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kms = [e0.elapsed_time(e1) for e0, e1 in kernel_ms]
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

    from grayshift_amd._native import COUNTER_NAMES
    c = {n: int(tot[i].item()) // a.steps for i, n in enumerate(COUNTER_NAMES)}
    if rank == 0:
        img = frame.view(r.height, r.width, 3).cpu().numpy()
        emit(a, sc, r, c, elapsed, kernel_avg_ms, img, world,
             {"tile_plan": "cost-balanced" if plan else "round-robin",
              "collective": "rccl" if a.backend == "nccl" else "gloo",
              "launch": "torch.distributed.run: %d process(es), one GPU each" % world})
    dist.destroy_process_group()
    r.close()


def emit(a, sc, r, c, elapsed, kernel_avg_ms, img, world, launch_info):
    """Rank 0's JSON line (kernel_avg_ms: the render launch of the slowest GPU, per frame)."""
    import numpy as np
    rays_per_frame = c["rays"]
    value = rays_per_frame * a.steps / elapsed / 1e6
    if a.dump:
        np.save(a.dump, img)
    cpu = parity = None
    if not a.no_cpu:
        stride = a.cpu_stride if world == 1 else a.parity_stride
        cpu, parity = cpu_check(sc, a, img, stride, runs=a.cpu_runs if world == 1 else 1)
        if world > 1:
            cpu = None  # the CPU baseline is an N=1 figure
    invalid = a.width is not None or a.spp is not None
    info = r.scene_info() if hasattr(r, "scene_info") else None
    cfg = {
        "workload": "%s: %s %dx%d, %s%s" % (a.config, sc.name, r.width, r.height, settings_desc(sc.settings),
                                          " (OVERRIDDEN: not the metric)" if invalid else ""),
        "tile": a.tile, "parallelism": "tiles%d" % world,
    }
    cfg.update(launch_info)
    cfg.update({"seed": a.seed, "rays_per_frame": rays_per_frame, "paths_per_frame": c["paths"],
                "node_visits_per_ray": round(c["node_visits"] / max(1, rays_per_frame), 3)})
    if info:
        cfg["scene"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in info.items()}
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
        "config": cfg,
        "roofline": roofline(a, c, world, kernel_avg_ms, invalid),
        "parity": parity,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)


def valu_cycles(k, cost=None):
    """Issue cycles of a launch's VALU instructions on their SIMDs: every PMC instruction
    class times its cost (VALU_CYCLES, or `cost`), the unclassified rest as "OTHER".
    Returns (cycles, {class: [count, cycles]})."""
    cost = cost or VALU_CYCLES
    classes = [c for c in cost if c != "OTHER"]
    mix = {}
    listed = 0.0
    for c in classes:
        n = float(k.get("SQ_INSTS_VALU_" + c, 0.0))
        listed += n
        mix[c] = [n, n * cost[c]]
    other = max(0.0, float(k["SQ_INSTS_VALU"]) - listed)
    mix["OTHER"] = [other, other * cost["OTHER"]]
    return sum(v[1] for v in mix.values()), mix


def roofline(a, c, world, kernel_ms, invalid):
    """The dominant kernel's ceiling.  The C4 working set (~3.5 MB: threaded BVH records
    and the RGBE sky) lives in LDS / L1 / L2, so HBM does not bound it (measured fabric
    traffic below); VALU issue does.  frac = the launch's VALU issue cycles (each PMC
    instruction class at its measured cycles per wave-instruction on a SIMD-32, VALU_CYCLES)
    over the SIMDs' cycles of this run's kernel time at the profiled effective clock, from
    the PMC summary of this very code object (same config).  What the rest of the SIMD
    time goes to is reported beside it: waves parked on s_waitcnt (SQ_WAIT_ANY) and
    issue-stalled (SQ_WAIT_INST_ANY) as shares of wave cycles."""
    from grayshift_amd import codeobj
    from grayshift_amd._native import LIB_PATH
    kernel_s = kernel_ms / 1e3
    abytes = algorithmic_bytes(c) / max(1, world)  # per launch (per rank)
    out = {"bound": "valu_issue", "achieved": None, "peak": None, "unit": "G VALU issue-cycles/s", "frac": None,
           "traffic": None, "hbm_frac": None, "kernel_ms": round(kernel_ms, 3),
           "cache_served_algorithmic_GBps": round(abytes / kernel_s / 1e9, 1),
           "cache_served_algorithmic_over_hbm_peak": round(abytes / kernel_s / 1e9 / HBM_PEAK_GBS, 4),
           "algorithmic_bytes_per_launch": int(abytes), "pmc": None}
    try:
        h = codeobj.code_object_hash(LIB_PATH)
    except Exception as e:  # noqa: BLE001
        out["pmc"] = "no code-object hash: %s" % e
        return out
    out["code_object"] = h
    if world != 1:
        return out  # the PMC summaries are 1-GPU whole-frame figures of one config
    # (an overridden size has its own summary: <config>_w<width>_s<spp>_<hash>.json, e.g.
    # final_scene at 1440^2 x 64 spp from tools/gpu_final.sh)
    key = a.config if not invalid else "%s_w%s_s%s" % (a.config, a.width, a.spp)
    # Lane efficiency: of the SIMD issue time `frac` counts, the share of
    # the 64 lanes that did work -- the stamps build's active lanes per phase, weighted by each
    # phase's wave clock (tools/stamps.py --json, profiles/stamps/<config>_<hash>.json); no
    # gfx950 counter counts active lanes per VALU instruction.  useful_frac = frac x lane_frac.
    spath = os.path.join(os.path.dirname(a.pmc_dir), "stamps", "%s_%s.json" % (key, h))
    lane = None
    if os.path.exists(spath):
        sj = json.load(open(spath))
        lane = sj["lane_frac"]
        out.update({"lane_frac": lane, "lane_frac_by_phase": {k: v["active_lanes"] for k, v in sj["phases"].items()},
                    "stamps": os.path.relpath(spath, ROOT)})
    else:
        out.update({"lane_frac": None, "stamps": "none for this code object (%s)" % os.path.relpath(spath, ROOT)})
    path = os.path.join(a.pmc_dir, "%s_%s.json" % (key, h))
    if not os.path.exists(path):
        out["pmc"] = "none for this code object (%s)" % os.path.relpath(path, ROOT)
        return out
    pj = json.load(open(path))
    k = pj["counters"]
    prof_s = pj["kernel_duration_ms_profiled"] / 1e3
    clock = k["GRBM_GUI_ACTIVE"] / 8.0 / prof_s  # effective shader clock of the profiled launch (Hz)
    cyc, mix = valu_cycles(k)
    cyc_hi, _ = valu_cycles(k, VALU_CYCLES_UPPER)
    n_disp0 = int(pj.get("dispatches_per_frame", 1) or 1)
    cyc1 = cyc
    cyc, cyc_hi = cyc * n_disp0, cyc_hi * n_disp0
    busy = None
    if "SQ_ACTIVE_INST_VALU2" in k and "SQ_ACTIVE_INST_VALU" in k:
        busy = 4.0 * (float(k["SQ_ACTIVE_INST_VALU"]) - float(k["SQ_ACTIVE_INST_VALU2"]))
    # the counters are per megakernel launch; a frame of batch rounds launches it once per
    # round (and segment): the frame's VALU work is that many launches' over the frame's time
    busy = None if busy is None else busy * n_disp0
    peak = SIMDS * clock
    achieved = (busy if busy is not None else cyc) / kernel_s  # VALU issue cycles per second, all SIMDs
    wc = float(k.get("SQ_WAVE_CYCLES", 0.0)) or 1.0
    out.update({"achieved": round(achieved / 1e9, 2), "peak": round(peak / 1e9, 2), "frac": round(achieved / peak, 4),
                "frac_method": ("measured: 4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) busy quad-cycles"
                                if busy is not None else "priced: VALU_CYCLES per PMC class"),
                "frac_lower": round(cyc / kernel_s / peak, 4), "frac_upper": round(cyc_hi / kernel_s / peak, 4),
                "traffic": pj["hbm_bytes_per_launch"],
                "hbm_frac": round(pj["hbm_bytes_per_launch"] / kernel_s / 1e9 / HBM_PEAK_GBS, 5),
                "effective_clock_ghz": round(clock / 1e9, 3),
                "valu_instructions": int(k["SQ_INSTS_VALU"]) * n_disp0,
                "launches_per_frame": n_disp0,
                "valu_cycle_mix": {c2: round(v[1] / cyc1, 4) for c2, v in mix.items()},
                "wave_cycles_waiting": round(float(k.get("SQ_WAIT_ANY", 0.0)) / wc, 4),
                "wave_cycles_issue_stalled": round(float(k.get("SQ_WAIT_INST_ANY", 0.0)) / wc, 4),
                "wave_cycles_issuing": round(float(k.get("SQ_ACTIVE_INST_ANY", 0.0)) / wc, 4),
                "pmc": os.path.relpath(path, ROOT)})
    if lane is not None:
        out["useful_frac"] = round(out["frac"] * lane, 4)
    return out


def cpu_check(sc, a, img, stride, runs):
    """The CPU oracle on every stride-th row and column of the same frame: its render time
    (median of `runs`; world/BVH build excluded) and the per-channel parity of the GPU
    frame at those pixels."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test-infrastructure checker, used here as the checker and the CPU baseline only
    threads = a.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    W, H = sc.width, sc.height
    sub = np.array([j * W + i for j in range(0, H, stride) for i in range(0, W, stride)], dtype=np.int32)
    times, ref, cnt = [], None, None
    for _ in range(max(1, runs)):
        tm = {}
        rgb, cc = oracle.render(sc, seed=a.seed, threads=threads, subset=sub, timing=tm)
        times.append(tm["render_s"])
        if ref is None:
            ref, cnt = rgb, cc
        elif not np.array_equal(ref, rgb):
            raise RuntimeError("CPU oracle is not deterministic across runs")
    med = statistics.median(times)
    gpu = img.reshape(-1, 3)[sub].astype(np.float64)
    d = np.abs(gpu - ref.astype(np.float64))
    parity = {"pixels": int(len(sub)), "subset": "every %dth row and column" % stride,
              "max_abs_delta": float(d.max()), "n_over_tol": int((d >= PARITY_TOL).sum()), "tolerance": PARITY_TOL,
              "bit_identical_frac": round(float((gpu == ref.astype(np.float64)).mean()), 6),
              "pass": bool(d.max() < PARITY_TOL)}
    cpu = {"value": round(cnt["rays"] / med / 1e6, 3), "unit": "Msamples/s", "cores": threads, "kind": "port",
           "sample": "%d px (every %dth row/col of the frame) x %s = %d rays; render only (world/BVH build "
                     "excluded), median of %d: %s s" % (len(sub), stride, settings_desc(sc.settings), cnt["rays"],
                                                        len(times), ", ".join("%.2f" % t for t in times))}
    return cpu, parity


if __name__ == "__main__":
    main()
