"""Adaptive sampling in batch rounds (render.hip gs_round_*_kernel): the
reference's per-pixel batch loop (camera.rs:135-165) restated as rounds -- round r renders
batch r of every pixel still active, spread over the lanes; a combine adds each pixel's
samples into its sums in sample order and takes the stop test.  Every stop decision and
every output must be bit-identical to the per-lane loop (gs_set_adaptive_mode(0)), and
within the north star's tolerance of the CPU oracle with its counters."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import _native as N
from grayshift_amd import scenes
from grayshift_amd.scene import camera_spec, sample_settings

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import oracle  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = 1e-3


class _mode:
    def __init__(self, mode, chunk=-1, budget=0, items=0):
        self.mode, self.chunk, self.budget, self.items = mode, chunk, budget, items

    def __enter__(self):
        N.check(N.lib.gs_set_adaptive_mode(self.mode))
        g.set_tuning(52, 0, 0, self.chunk)
        N.check(N.lib.gs_debug_set_partial_budget(self.budget))
        N.check(N.lib.gs_debug_set_round_items(self.items))

    def __exit__(self, *a):
        N.check(N.lib.gs_set_adaptive_mode(1))
        g.set_tuning(0, 0, 0, -1)
        N.check(N.lib.gs_debug_set_partial_budget(0))
        N.check(N.lib.gs_debug_set_round_items(0))


def _both(sc, seed, **kw):
    """Batch rounds (split items at these small sizes) and the per-lane loop; also asserts the
    whole-batch round items render the same frame."""
    with _mode(2, **kw):
        a, ca = g.render(sc, seed=seed)
    with _mode(0):
        b, cb = g.render(sc, seed=seed)
    with _mode(2, items=1):
        w, cw = g.render(sc, seed=seed)
    assert np.array_equal(w, b) and cw == cb
    return a, ca, b, cb


def _edge(width, batch, maxs, tol):
    b = g.SceneBuilder()
    m = b.lambertian((0.5, 0.6, 0.7))
    b.add(b.sphere((0, 0, 0), 1.0, m))
    b.add(b.sphere((0, -101, 0), 100.0, b.metal((0.8, 0.8, 0.8), 0.3)))
    b.add(b.quad((-2, -1, -2), (4, 0, 0), (0, 3, 0), b.dielectric(1.5)))
    b.background_solid((0.7, 0.8, 1.0))
    cam = camera_spec(1.0, width, 50, 40.0, (0, 1, 6), (0, 0, 0), (0, 1, 0), 0.0, 6.0)
    return scenes.Scene("edge", b.build(), cam, sample_settings(0.95, tol, batch, maxs))


@pytest.mark.parametrize("scene", ["hdri", "cornell_box", "cornell_smoke", "earth_hdr", "final_scene", "triangles"])
def test_rounds_equal_per_lane_and_oracle(scene):
    """The reference scenes with their own adaptive SampleSettings."""
    kw = {"final_scene": {"boxes_per_side": 4, "n_balls": 60}}.get(scene, {})
    sc = scenes.SCENES[scene](width=40, **kw)
    a, ca, b, cb = _both(sc, seed=2)
    assert np.array_equal(a, b) and ca == cb
    ref, rc = oracle.render(sc, seed=2)
    assert float(np.abs(a.astype(np.float64) - ref).max()) < TOL
    assert ca["paths"] == rc["paths"] and ca["pixels"] == rc["pixels"] == sc.width * sc.height


@pytest.mark.parametrize("batch,maxs,tol", [(1, 0, 0.0), (1, 5, 0.5), (3, 17, 0.1), (2, 40, 1e-9), (7, 7, 0.2),
                                            (64, 200, 0.05)])
def test_round_edge_settings(batch, maxs, tol):
    """batch 1 (variance 0/0 = NaN never converges: every round to the cap), max_samples equal
    to the batch (two rounds), tiny and huge tolerances."""
    sc = _edge(24, batch, maxs, tol)
    a, ca, b, cb = _both(sc, seed=5)
    assert np.array_equal(a, b) and ca == cb
    ref, rc = oracle.render(sc, seed=5)
    assert float(np.abs(a.astype(np.float64) - ref).max()) < TOL and ca["paths"] == rc["paths"]


@pytest.mark.parametrize("chunk", [1, 3, 32])
def test_round_chunks_and_segments(chunk):
    """Fixed sample chunks per work item, and a sample-buffer budget of 100 pixels' batches
    (the active list rendered in segments): the same frame."""
    sc = scenes.cornell_box(width=48)
    ref, rc = _both(sc, seed=7)[2:]
    with _mode(2, chunk=chunk):
        a, ca = g.render(sc, seed=7)
    assert np.array_equal(a, ref) and ca == rc
    with _mode(2, chunk=chunk, budget=100 * sc.settings.batch_size * 24):
        s, cs = g.render(sc, seed=7)
    assert np.array_equal(s, ref) and cs == rc


def test_round_ppm_bytes_equal_oracle():
    """write_color's bytes of the f64 colour (gs_render_ppm) in batch rounds: the oracle's text."""
    sc = scenes.hdri(width=48)
    text, _ = g.render_ppm(sc, seed=3)
    ref, _ = oracle.render_ppm(sc, seed=3)
    assert text == ref


@pytest.mark.parametrize("world,tile", [(2, 16), (3, 24)])
def test_round_partition_invariance(world, tile):
    """Ranks render their tiles in rounds of their own: the gathered frame equals the full one."""
    import torch
    sc = scenes.cornell_box(width=56)
    full, fc = g.render(sc, seed=3)
    dev = torch.device("cuda", 0)
    cam = g.camera(sc.camera)
    cap0 = N.lib.gs_partition_capacity(C.byref(cam), C.byref(N.gs_partition(0, world, tile, tile)))
    gathered = torch.zeros(world * cap0 * 3, dtype=torch.float32, device=dev)
    counters = torch.zeros(16, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for r in range(world):
        rr = g.Renderer(sc, rank=r, world_size=world, tile=tile)
        rr.render_async(gathered.data_ptr() + r * cap0 * 12, counters.data_ptr(), stream, seed=3)
        torch.cuda.synchronize()
        rr.close()
    frame = torch.zeros(cam.image_height * cam.image_width * 3, dtype=torch.float32, device=dev)
    rr = g.Renderer(sc, rank=0, world_size=world, tile=tile)
    rr.unpack_async(gathered.data_ptr(), frame.data_ptr(), world, stream)
    torch.cuda.synchronize()
    rr.close()
    part = frame.view(cam.image_height, cam.image_width, 3).cpu().numpy()
    c = counters.cpu().numpy()
    assert np.array_equal(full, part)
    assert {n: int(c[i]) for i, n in enumerate(N.COUNTER_NAMES)} == fc


def test_adaptive_mode_rejects_bad_values():
    assert N.lib.gs_set_adaptive_mode(3) == N.GS_ERR_ARG
    assert N.lib.gs_set_adaptive_mode(-1) == N.GS_ERR_ARG
    assert N.lib.gs_debug_set_round_items(2) == N.GS_ERR_ARG


@pytest.mark.parametrize("items", [0, 1, -1])
def test_round_items_at_a_chip_filling_size(items):
    """cornell_box at 768 x 768 (590 k pixels: above twice the device's 262 k lanes, so item
    rule -1 runs whole-batch items in the first round and split ones later), split (0) and
    whole (1) items, and the default auto mode: the per-lane loop's frame every time."""
    sc = scenes.cornell_box(width=768)
    with _mode(0):
        ref, rc = g.render(sc, seed=9)
    with _mode(2, items=items):
        a, ca = g.render(sc, seed=9)
    with _mode(1):
        auto, cauto = g.render(sc, seed=9)
    assert np.array_equal(a, ref) and ca == rc
    assert np.array_equal(auto, ref) and cauto == rc


def test_rounds_past_every_pixels_stop_are_empty_and_cheap():
    """settings whose pixels all stop after the first batch while max_samples
    allows hundreds of rounds (here 257 rounds of 4 samples).  Every round after the first
    has no active pixel, so its launches must return at once (render.hip: the megakernel's
    early return on an empty round, before the LDS mirror copy) -- and the frame is still
    the per-lane loop's, bit for bit, and the oracle's."""
    b = g.SceneBuilder()
    b.add(b.sphere((0, 0, 60), 1.0, b.lambertian((0.5, 0.5, 0.5))))  # behind the camera
    b.background_solid((0.7, 0.8, 1.0))
    cam = camera_spec(1.0, 48, 50, 20.0, (0, 0, 30), (0, 0, 0), (0, 1, 0), 0.0, 30.0)
    # every primary ray sees the solid sky: every sample of a pixel is the same colour, so
    # the variance is 0 and the first stop test passes (0 < mean^2 * tol^2)
    sc = scenes.Scene("sky", b.build(), cam, sample_settings(0.95, 0.05, 4, 1024))
    with _mode(2):
        st = {}
        a, ca = g.render(sc, seed=4, stats=st)
    with _mode(0):
        ref_loop, cl = g.render(sc, seed=4)
    assert np.array_equal(a, ref_loop) and ca == cl
    assert ca["paths"] == 48 * 48 * 4  # one batch per pixel
    ref, rc = oracle.render(sc, seed=4)
    assert float(np.abs(a.astype(np.float64) - ref.astype(np.float64)).max()) < TOL
    # 257 rounds x (parameters + megakernel + combine), 256 of them empty: launch overhead
    assert st["kernel_ms_max"] < 100.0, st
