"""A frame's bits depend on the frame, the settings and the seed only (VERDICT
r5 item 2): not on the device count, the tile assignment, the rank's capacity, the guided
tail's placement or a timing measured by an earlier frame.

The chunk association (render.hip `launch`): a pixel's colour is the in-order sum of its
chunks of c samples, c fixed by (W x H, spp, the scene's flags, the knobs).  The guided tail's
1-sample items are regrouped into those chunks by gs_combine_kernel, so how many tiles of a
rank run in the tail -- which depends on the rank's capacity, the device's lanes and, for small
frames, on the scene's measured cost per sample (gs_device_scene_note_frame) -- is scheduling
only.  These tests put the frame where those choices differ and compare with np.array_equal.
"""
import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import _native as N
from grayshift_amd import scenes
from tests.test_gpu_parity import _render_partitioned, _render_planned

pytestmark = pytest.mark.gpu


class _same_device:
    """gs_debug_set_multi_same_device: N frame-context ranks on the one device (test hook)."""
    def __enter__(self):
        N.check(N.lib.gs_debug_set_multi_same_device(1))

    def __exit__(self, *a):
        N.check(N.lib.gs_debug_set_multi_same_device(0))


@pytest.fixture(scope="module")
def c4_32():
    """C4 at its stated 1920x1080, 32 spp: 16-sample chunks, and a guided tail of 64 of the
    510 tiles on one GPU -- every tile of a rank at 8 ranks (the tail is sized per rank)."""
    sc = scenes.config("C4", spp=32)
    full, fc = g.render(sc, seed=3)
    return sc, full, fc


def test_c4_round_robin_ranks_equal_one_gpu(c4_32):
    sc, full, fc = c4_32
    part, pc = _render_partitioned(sc, 8, 64, seed=3)
    assert np.array_equal(full, part)
    assert fc == pc


def test_c4_planned_ranks_equal_one_gpu(c4_32):
    sc, full, fc = c4_32
    part, pc = _render_planned(sc, 8, 64, seed=3)
    assert np.array_equal(full, part)
    assert fc == pc


@pytest.mark.parametrize("plan", [False, True])
def test_c4_frame_context_of_eight_ranks_equals_one_gpu(c4_32, plan):
    """the frame context's N > 1 host loop on one GPU -- eight device scenes,
    streams and event sets on device 0, the tile plan (cost-balanced or round-robin), eight
    concurrent launches, the gather (device copies in place of ncclGather), the rank-major
    unpack, the counters summed over the ranks and each rank's frame note -- renders the N = 1
    frame bit for bit, frame after frame."""
    sc, full, fc = c4_32
    with _same_device():
        m = g.MultiRenderer(sc, devices=[0] * 8, tile=64, plan=plan)
    try:
        assert m.devices == [0] * 8
        for _ in range(2):
            res = m.render(seed=3, rgb=True, rgb8=True)
            assert np.array_equal(res["rgb"], full)
            assert res["counters"] == fc
            st = res["stats"]
            assert st["num_gpus"] == 8 and st["gathered_bytes"] > 0
            assert 0 < st["kernel_ms_min"] <= st["kernel_ms_max"] <= st["render_ms_max"]
        # every rank's scene is its own upload, placed by its own pilot, alike
        infos = [m.scene_info(r) for r in range(8)]
        assert all(i["placement"] == infos[0]["placement"] for i in infos)
        assert all(i["lds_nodes"] == infos[0]["lds_nodes"] for i in infos)
    finally:
        m.close()
    ppm_one, _ = g.render_ppm(sc, seed=3)
    with _same_device():
        res = g.render_multi(sc, devices=[0] * 8, seed=3, rgb=False, ppm=True)
    assert res["ppm"] == ppm_one


def test_same_device_lists_need_the_hook():
    sc = scenes.config("C4", width=32, spp=1)
    with pytest.raises(N.GrayshiftError) as e:
        g.MultiRenderer(sc, devices=[0, 0])
    assert e.value.code == N.GS_ERR_ARG


@pytest.mark.parametrize("name", ["checkered_spheres", "perlin_spheres"])
def test_small_frame_context_frames_equal_the_one_shot_render(name):
    """A small frame (400 px, 64 spp: 4-sample chunks) of a scene whose samples are long: the
    frame context times each frame, and once one measures more than 50 lane-us a sample the
    scene's later frames take the guided tail (1-sample items) -- perlin_spheres always
    (~390 lane-us), checkered_spheres near the threshold.  Three frames of one seed in one
    context and the one-shot gs_render (a fresh scene: never timed) are the same bits."""
    sc = scenes.config(name)
    one, oc = g.render(sc, seed=1)
    m = g.MultiRenderer(sc, num_gpus=1, tile=64, plan=False)
    try:
        frames = [m.render(seed=1, rgb=True) for _ in range(3)]
        info = m.scene_info()
    finally:
        m.close()
    for f in frames:
        assert np.array_equal(f["rgb"], one)
        assert f["counters"] == oc
    if name == "perlin_spheres":
        assert info["long_samples"] == 1  # frames 2 and 3 did run with the tail


def test_tail_share_does_not_change_the_frame():
    """The same C4 frame with the default tail, a 4x tail (every tile in 1-sample items) and
    none (an explicit 16-sample chunk): the same bits."""
    sc = scenes.config("C4", width=640, spp=48)
    base, bc = g.render(sc, seed=7)
    try:
        N.check(N.lib.gs_debug_set_guided_tail(1, 400))
        wide, wc = g.render(sc, seed=7)
    finally:
        N.check(N.lib.gs_debug_set_guided_tail(0, 0))
    g.set_tuning(0, 0, 0, 16)
    try:
        none, nc = g.render(sc, seed=7)
    finally:
        g.set_tuning(0, 0, 0, -1)
    assert np.array_equal(base, wide) and np.array_equal(base, none)
    assert bc == wc == nc


def test_capacity_zero_rank_counters_start_from_zero():
    """a rank with no tiles (more ranks than tiles) launches nothing; the frame
    context's summed counters must still be exactly the frame's, frame after frame."""
    sc = scenes.config("C4", width=96, spp=4)  # 2 x 1 tiles of 64: ranks 2..3 hold none
    one, oc = g.render(sc, seed=2)
    with _same_device():
        m = g.MultiRenderer(sc, devices=[0] * 4, tile=64, plan=False)
    try:
        for _ in range(2):
            res = m.render(seed=2, rgb=True)
            assert np.array_equal(res["rgb"], one) and res["counters"] == oc
    finally:
        m.close()
