"""GPU parity: the HIP megakernel (through the C-ABI) against the CPU oracle.

Tolerance (north star): per-channel |delta| < 1e-3 on the linear f32 framebuffer at
a fixed seed.  Work counters: paths and pixels exactly, traversal work (rays, node
visits, primitive tests, texel fetches) within 1e-4 relative — the device walks
the reference's traversal order, and only ulp-level libm differences reroute a
grazing ray (see counters_match).  Small frames are compared in full; BASELINE-size frames through
size-independent properties plus an oracle spot-check of sampled pixels.
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import _native as N
from grayshift_amd import scenes
from grayshift_amd.scene import camera_spec, fixed_spp, sample_settings
import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = 1e-3  # per-channel absolute, BASELINE.json north star

GOLD = np.load(os.path.join(HERE, "golden", "frames.npz"), allow_pickle=False)
COUNTS = json.load(open(os.path.join(HERE, "golden", "counters.json")))


def maxdiff(a, b):
    return float(np.abs(a.astype(np.float64) - b.astype(np.float64)).max())


def counters_match(gpu, ref, rel=1e-4):
    """Paths and pixels exactly; traversal work within `rel`.  The device's OCML
    sin/cos/acos/atan2/asin can differ from glibc's by an ulp, and a grazing ray can
    then take another route through the BVH to the same hit (e.g. 18
    node visits in 1.3e8 on C5 256x144x32spp, frame bit-identical)."""
    if gpu["paths"] != ref["paths"] or gpu["pixels"] != ref["pixels"]:
        return False
    for k, v in ref.items():
        if abs(gpu[k] - v) > rel * max(v, 1) + 2:
            return False
    return True


@pytest.mark.parametrize("name", list(make_golden.GOLDEN))
def test_gpu_matches_golden(name):
    sc = make_golden.build(name)
    out, c = g.render(sc, seed=COUNTS["seed"])
    assert maxdiff(out, GOLD[name]) < TOL
    assert counters_match(c, COUNTS["counters"][name])


@pytest.mark.parametrize("name", ["C1", "C3", "C4", "C5"])
def test_gpu_vs_oracle_small_configs(name):
    sc = scenes.config(name, width=96, spp=16)
    out, gc = g.render(sc, seed=11)
    ref, rc = oracle.render(sc, seed=11)
    assert maxdiff(out, ref) < TOL
    assert counters_match(gc, rc)


@pytest.mark.parametrize("scene", ["hdri", "cornell_box", "earth", "checkered_spheres", "quads", "triangles"])
def test_gpu_vs_oracle_adaptive_sampling(scene):
    """The reference scenes with their own adaptive SampleSettings (variable spp per pixel)."""
    sc = scenes.SCENES[scene](width=40)
    out, gc = g.render(sc, seed=2)
    ref, rc = oracle.render(sc, seed=2)
    assert maxdiff(out, ref) < TOL
    assert counters_match(gc, rc)


def test_bouncing_spheres_adaptive():
    sc = scenes.bouncing_spheres(grid=11, width=48)
    out, gc = g.render(sc, seed=4)
    ref, rc = oracle.render(sc, seed=4)
    assert maxdiff(out, ref) < TOL and counters_match(gc, rc)


def test_determinism_and_seed_dependence():
    sc = scenes.config("C4", width=48, spp=4)
    a, ca = g.render(sc, seed=1)
    b, cb = g.render(sc, seed=1)
    c, _ = g.render(sc, seed=2)
    assert np.array_equal(a, b) and ca == cb
    assert not np.array_equal(a, c)


# ------------------------------------------------------------- edge cases
def _custom(width, aspect, spp=4, depth=50, batch=None, maxs=None, tol=0.0):
    b = g.SceneBuilder()
    m = b.lambertian((0.5, 0.6, 0.7))
    b.add(b.sphere((0, 0, 0), 1.0, m))
    b.add(b.sphere((0, -101, 0), 100.0, b.metal((0.8, 0.8, 0.8), 0.3)))
    b.add(b.quad((-2, -1, -2), (4, 0, 0), (0, 3, 0), b.dielectric(1.5)))
    b.background_solid((0.7, 0.8, 1.0))
    cam = camera_spec(aspect, width, depth, 40.0, (0, 1, 6), (0, 0, 0), (0, 1, 0), 0.0, 6.0)
    ss = sample_settings(0.95, tol, batch or spp, maxs if maxs is not None else spp - 1)
    return scenes.Scene("custom", b.build(), cam, ss)


@pytest.mark.parametrize("width,aspect", [(1, 1.0), (7, 7.0), (37, 1.6), (65, 1.0), (129, 2.0)])
def test_odd_image_sizes(width, aspect):
    sc = _custom(width, aspect)
    out, gc = g.render(sc, seed=9)
    ref, rc = oracle.render(sc, seed=9)
    assert out.shape == ref.shape and maxdiff(out, ref) < TOL and counters_match(gc, rc)


@pytest.mark.parametrize("depth", [0, 1, 2])
def test_shallow_max_depth(depth):
    sc = _custom(24, 1.0, depth=depth)
    out, gc = g.render(sc, seed=9)
    ref, rc = oracle.render(sc, seed=9)
    assert maxdiff(out, ref) < TOL and counters_match(gc, rc)
    if depth == 0:
        assert not out.any() and gc["rays"] == 0


@pytest.mark.parametrize("batch,maxs,tol", [(1, 0, 0.0), (1, 5, 0.5), (3, 17, 0.1), (2, 40, 1e-9)])
def test_adaptive_edge_settings(batch, maxs, tol):
    """batch 1 (variance 0/0 = NaN never converges), tiny/huge tolerances."""
    sc = _custom(20, 1.0, batch=batch, maxs=maxs, tol=tol)
    out, gc = g.render(sc, seed=5)
    ref, rc = oracle.render(sc, seed=5)
    assert maxdiff(out, ref) < TOL and counters_match(gc, rc)


def test_unsupported_scene_fails_cleanly():
    b = g.SceneBuilder()
    m = b.lambertian((1, 1, 1))
    # media three deep (one medium as another's boundary is supported since round 6)
    b.add(b.medium(b.medium(b.medium(b.sphere((0, 0, 0), 1, m), 0.5, m), 0.5, m), 0.5, m))
    sc = scenes.Scene("vol", b.build(), camera_spec(1.0, 8, 5, 40, (0, 0, 5), (0, 0, 0), (0, 1, 0), 0, 5),
                      fixed_spp(1))
    with pytest.raises(N.GrayshiftError) as e:
        g.render(sc)
    assert e.value.code == N.GS_ERR_UNSUPPORTED


# ------------------------------------------------ partition / multi-GPU path
def _render_partitioned(sc, world, tile, seed=3):
    import torch
    dev = torch.device("cuda", 0)
    cam = g.camera(sc.camera)
    cap0 = N.lib.gs_partition_capacity(C.byref(cam), C.byref(N.gs_partition(0, world, tile, tile)))
    gathered = torch.zeros(world * cap0 * 3, dtype=torch.float32, device=dev)
    counters = torch.zeros(16, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for r in range(world):
        rr = g.Renderer(sc, rank=r, world_size=world, tile=tile)
        rr.render_async(gathered.data_ptr() + r * cap0 * 12, counters.data_ptr(), stream, seed=seed)
        torch.cuda.synchronize()
        rr.close()
    frame = torch.zeros(cam.image_height * cam.image_width * 3, dtype=torch.float32, device=dev)
    rr = g.Renderer(sc, rank=0, world_size=world, tile=tile)
    rr.unpack_async(gathered.data_ptr(), frame.data_ptr(), world, stream)
    torch.cuda.synchronize()
    rr.close()
    c = counters.cpu().numpy()
    return frame.view(cam.image_height, cam.image_width, 3).cpu().numpy(), {
        n: int(c[i]) for i, n in enumerate(N.COUNTER_NAMES)}


def _render_planned(sc, world, tile, seed=3):
    """gs_plan_tiles partitions: every rank renders its planned tiles, the gathered
    buffers unpack through the plan's order."""
    import torch
    dev = torch.device("cuda", 0)
    rs = [g.Renderer(sc, rank=r, world_size=world, tile=tile, plan=True) for r in range(world)]
    cap = rs[0].capacity
    orders = [r.order for r in rs]
    for o in orders[1:]:
        assert np.array_equal(o, orders[0])  # the pilot is deterministic: every rank plans alike
    tiles = orders[0][orders[0] >= 0]
    cam = rs[0].cam
    nt = ((cam.image_width + tile - 1) // tile) * ((cam.image_height + tile - 1) // tile)
    assert sorted(tiles.tolist()) == list(range(nt))  # each tile exactly once
    gathered = torch.zeros(world * cap * 3, dtype=torch.float32, device=dev)
    counters = torch.zeros(16, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for r, rr in enumerate(rs):
        assert rr.capacity == cap
        rr.render_async(gathered.data_ptr() + r * cap * 12, counters.data_ptr(), stream, seed=seed)
    frame = torch.zeros(cam.image_height * cam.image_width * 3, dtype=torch.float32, device=dev)
    rs[0].unpack_async(gathered.data_ptr(), frame.data_ptr(), world, stream)
    torch.cuda.synchronize()
    for rr in rs:
        rr.close()
    c = counters.cpu().numpy()
    return frame.view(cam.image_height, cam.image_width, 3).cpu().numpy(), {
        n: int(c[i]) for i, n in enumerate(N.COUNTER_NAMES)}


@pytest.mark.parametrize("world,tile", [(2, 64), (3, 16), (8, 8)])
def test_planned_partition_invariance(world, tile):
    """Cost-balanced tile plans (gs_plan_tiles) change who renders what, never the frame."""
    sc = scenes.config("C5", width=80, spp=8)
    full, fc = g.render(sc, seed=3)
    part, pc = _render_planned(sc, world, tile, seed=3)
    assert np.array_equal(full, part)
    assert fc == pc


@pytest.mark.parametrize("world,tile", [(1, 64), (2, 64), (3, 16), (4, 24), (8, 8)])
def test_partition_invariance(world, tile):
    """G logical partitions rendered on one GPU, gathered and unpacked by the device
    kernel, are bit-identical to the full-frame render."""
    sc = scenes.config("C5", width=80, spp=8)
    full, fc = g.render(sc, seed=3)
    part, pc = _render_partitioned(sc, world, tile, seed=3)
    assert np.array_equal(full, part)
    assert fc == pc


# ------------------------------------------------------ sample chunking
class _chunk:
    """Force gs_set_tuning's sample_chunk for one render (restores auto)."""
    def __init__(self, n):
        self.n = n

    def __enter__(self):
        g.set_tuning(52, 0, 0, self.n)

    def __exit__(self, *a):
        g.set_tuning(0, 0, 0, -1)


@pytest.mark.parametrize("name", ["C4", "C3", "earth_fixed"])
@pytest.mark.parametrize("chunk", [1, 3, 5, 16, 0])
def test_sample_chunks_match_oracle(name, chunk):
    """Single-batch renders split into sample chunks (one work item each): every
    sample keeps its RNG stream, so counters are the oracle's and the colour differs
    only by the association of the f64 sum (tolerance as everywhere)."""
    if name == "earth_fixed":
        base = scenes.SCENES["earth"](width=48)
        sc = scenes.Scene("earth16", base.spec, base.camera, fixed_spp(16))
    else:
        sc = scenes.config(name, width=64, spp=16)
    with _chunk(chunk):
        out, gc = g.render(sc, seed=13)
    ref, rc = oracle.render(sc, seed=13)
    assert maxdiff(out, ref) < TOL and counters_match(gc, rc)
    with _chunk(0):
        whole, wc = g.render(sc, seed=13)
    assert wc == gc
    # same samples, re-associated sum: a few f32 ulps at most, mostly identical
    assert np.allclose(out, whole, rtol=4e-7, atol=1e-30)
    assert (out == whole).mean() > 0.98


def test_chunking_ignored_for_multi_batch_settings():
    sc = _custom(20, 1.0, batch=3, maxs=17, tol=0.1)
    with _chunk(1):
        a, ca = g.render(sc, seed=5)
    with _chunk(0):
        b, cb = g.render(sc, seed=5)
    assert np.array_equal(a, b) and ca == cb


@pytest.mark.parametrize("world,tile,chunk", [(3, 16, 3), (8, 8, 1), (2, 64, 7)])
def test_partition_invariance_chunked(world, tile, chunk):
    sc = scenes.config("C5", width=80, spp=8)
    with _chunk(chunk):
        full, fc = g.render(sc, seed=3)
        part, pc = _render_partitioned(sc, world, tile, seed=3)
    assert np.array_equal(full, part)
    assert fc == pc


# ----------------------------------------------- BASELINE-size properties
def _spot_check(sc, out, seed, n=96):
    rng = np.random.default_rng(123)
    ids = np.sort(rng.choice(sc.width * sc.height, size=n, replace=False)).astype(np.int32)
    ref, _ = oracle.render(sc, seed=seed, subset=ids)
    return maxdiff(out.reshape(-1, 3)[ids], ref)


@pytest.mark.slow
@pytest.mark.parametrize("name,spp", [("C1", None), ("C2", None), ("C4", None), ("C3", 64), ("C5", 16)])
def test_full_size_frames(name, spp):
    """BASELINE resolution (C3/C5 at reduced spp to bound test time): every pixel
    finite and >= 0, exact path/pixel counts, and an oracle spot-check of sampled pixels."""
    sc = scenes.config(name, spp=spp)
    out, c = g.render(sc, seed=1)
    W, H, s = sc.width, sc.height, sc.settings.batch_size
    assert out.shape == (H, W, 3)
    assert np.isfinite(out).all() and (out >= 0).all()
    assert c["pixels"] == W * H and c["paths"] == W * H * s
    assert c["rays"] >= c["paths"] * (1 if name != "C3" else 1) and c["rays"] <= c["paths"] * 50
    assert _spot_check(sc, out, seed=1, n=48 if name in ("C3", "C5") else 96) < TOL
    if name == "C1":  # small enough to check every pixel
        ref, rc = oracle.render(sc, seed=1)
        assert maxdiff(out, ref) < TOL and counters_match(c, rc)


# ------------------------------------- C3 / C5 at their stated spp (auto chunks)
@pytest.mark.parametrize("name,width,cpp", [("C3", 64, None), ("C5", 64, None), ("C5", 64, 16), ("C5", 48, 8)])
def test_stated_spp_configs_vs_oracle(name, width, cpp):
    """C3 at its full 1024 spp and C5 at its full 4096 spp (reduced width), rendered
    through the auto sample-chunk rule (render.hip: 16-sample chunks, or batch/64, then
    doubled while the chunk sums exceed the budget).  C3 at 1024 spp: 64 chunks of 16
    per pixel.  C5 at 3840x2160 takes the doubling branch (4096 spp: 256-sample chunks,
    16 per pixel); a test budget of capacity x cpp x 24 bytes makes this small frame
    take the same branch (cpp = 16: 256-sample chunks; cpp = 8: 512)."""
    sc = scenes.config(name, width=width)
    cam = g.camera(sc.camera)
    cap = N.lib.gs_partition_capacity(C.byref(cam), C.byref(N.gs_partition(0, 1, 64, 64)))
    if cpp:
        N.check(N.lib.gs_debug_set_partial_budget(cap * cpp * 24))
    try:
        out, gc = g.render(sc, seed=17)
    finally:
        N.check(N.lib.gs_debug_set_partial_budget(0))
    ref, rc = oracle.render(sc, seed=17)
    assert gc["paths"] == sc.width * sc.height * sc.settings.batch_size
    assert maxdiff(out, ref) < TOL and counters_match(gc, rc)


# ------------------------------------- the guided tail's knobs (gs_debug_set_guided_tail)
@pytest.mark.parametrize("chunk,fine,pct", [(-1, 1, 1), (-1, 1, 10), (8, 1, 5), (-1, 0, 0), (-1, 1, 400)])
def test_guided_tail_settings_vs_oracle(chunk, fine, pct):
    """C1's scene at 100 spp, 160x90 (six 64x64 tile slots) under other guided-tail settings:
    tails of 1 or 2 tiles (coarse and fine chunk sums both present: the chunk-major layout's
    two regions, render.hip KParams.partial), an explicit 8-sample coarse chunk with a tail,
    and the default and a 4x tail (every tile in 1-sample items) -- against the oracle,
    counters exact.  The tail is scheduling only (round 6): its 1-sample sums are regrouped
    into the coarse chunks, so the frame equals the same coarse chunking without a tail bit for
    bit (auto chunks with a tail_pct: the 16-sample chunks; explicit 8: 8 without a tail)."""
    sc = scenes.config("C1", width=160)
    g.set_tuning(0, 0, 0, chunk)
    N.check(N.lib.gs_debug_set_guided_tail(fine, pct))
    try:
        out, gc = g.render(sc, seed=23)
    finally:
        N.check(N.lib.gs_debug_set_guided_tail(0, 0))
        g.set_tuning(0, 0, 0, -1)
    ref, rc = oracle.render(sc, seed=23)
    assert gc["paths"] == sc.width * sc.height * sc.settings.batch_size
    assert maxdiff(out, ref) < TOL and counters_match(gc, rc)
    if pct:
        # the same coarse chunks with no tail at all (a 1-tile frame: a tail share of ~0)
        g.set_tuning(0, 0, 0, 16 if chunk < 0 else chunk)
        try:
            plain, pc = g.render(sc, seed=23)
        finally:
            g.set_tuning(0, 0, 0, -1)
        assert np.array_equal(out, plain) and pc == gc
