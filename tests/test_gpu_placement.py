"""Placement of the threaded BVH records in the per-block LDS mirror (render.hip
place_records / run_pilot): the first launch of a scene whose records do not all fit
runs a pilot that counts every record's tests and re-places the records by measured
visits per byte.  Placement must never change a frame or a counter, the pilot's counts
must be the frame's own work counts, and the re-placed mirror must serve more of the
visits than the static estimate."""
import ctypes as C

import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import _native as N
from grayshift_amd import scenes

pytestmark = pytest.mark.gpu


class _placement:
    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        N.check(N.lib.gs_set_placement(self.mode))

    def __exit__(self, *a):
        N.check(N.lib.gs_set_placement(1))


def _visits(r, torch):
    dev = torch.device("cuda", 0)
    info = r.scene_info()
    nn, nl = info["node_records"], info["leaf_records"]
    packed = torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev)
    vm = torch.zeros(nn + nl, dtype=torch.int32, device=dev)
    N.check(N.lib.gs_debug_record_visits(r.dev, C.byref(r.cam), C.byref(r.settings), 3, C.byref(r.part),
                                         C.c_void_p(packed.data_ptr()), C.c_void_p(vm.data_ptr()), None))
    torch.cuda.synchronize()
    v = vm.cpu().numpy().astype(np.int64)
    return r.scene_info(), v[:nn], v[nn:], packed.cpu().numpy()


@pytest.mark.parametrize("config,width,spp", [("C4", 240, 8), ("C5", 160, 4), ("C2", 96, 8)])
def test_placement_never_changes_the_frame(config, width, spp):
    sc = scenes.config(config, width=width, spp=spp)
    with _placement(0):
        ref, rc = g.render(sc, seed=11)
    img, c = g.render(sc, seed=11)
    assert np.array_equal(img, ref)
    assert c == rc


def test_pilot_places_and_counts_the_frames_work():
    torch = pytest.importorskip("torch")
    # (a launch of >= 16x the pilot's pixel samples: smaller ones leave the pilot pending)
    sc = scenes.config("C4", width=160, spp=32)
    with _placement(0):
        r0 = g.Renderer(sc, 0, 1, 64)
        s_info, s_nodes, s_leaves, s_img = _visits(r0, torch)
        r0.close()
    r1 = g.Renderer(sc, 0, 1, 64)
    m_info, m_nodes, m_leaves, m_img = _visits(r1, torch)
    r1.close()
    assert s_info["placement"] == 1 and m_info["placement"] == 2 and m_info["pilot_ms"] > 0
    # the same frame and the same total work under either placement
    assert np.array_equal(s_img, m_img)
    assert s_nodes.sum() == m_nodes.sum() and s_leaves.sum() == m_leaves.sum()
    assert sorted(s_nodes.tolist()) == sorted(m_nodes.tolist())
    # the counts are the frame's own counters (C4: top-level nodes only, sphere leaves only)
    _, c = g.render(sc, seed=3)
    assert m_nodes.sum() == c["node_visits"] and m_leaves.sum() == c["sphere_tests"]
    # the measured placement's mirror serves at least as many visits as the static one
    served = lambda info, n, l: n[:info["lds_nodes"]].sum() + l[:info["lds_leaves"]].sum()
    assert served(m_info, m_nodes, m_leaves) >= served(s_info, s_nodes, s_leaves)
    assert m_nodes[:m_info["lds_nodes"]].sum() > 0.97 * m_nodes.sum()


def test_whole_tree_scenes_skip_the_pilot():
    torch = pytest.importorskip("torch")
    sc = scenes.config("C3", width=64, spp=2)
    r = g.Renderer(sc, 0, 1, 64)
    assert r.scene_info()["placement"] == 0  # pending until the first launch
    info, nodes, leaves, _ = _visits(r, torch)
    r.close()
    assert info["lds_nodes"] == info["node_records"] and info["lds_leaves"] == info["leaf_records"]
    assert info["placement"] == 1 and info["pilot_ms"] == 0.0
    assert nodes.sum() > 0


def test_small_launches_leave_the_pilot_pending():
    """A launch of fewer than 16x the pilot's samples does not pay for a pilot:
    the scene stays pending, and the next large launch runs it."""
    torch = pytest.importorskip("torch")
    small = scenes.config("C4", width=160, spp=4)
    r = g.Renderer(small, 0, 1, 64)
    dev = torch.device("cuda", 0)
    packed = torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev)
    r.render_async(packed.data_ptr(), 0, 0, seed=3)
    torch.cuda.synchronize()
    assert r.scene_info()["placement"] == 0
    big = scenes.config("C4", width=160, spp=32)
    N.check(N.lib.gs_render_tiles_async(r.dev, C.byref(r.cam), C.byref(big.settings), 3, C.byref(r.part),
                                        C.c_void_p(packed.data_ptr()), None, None))
    torch.cuda.synchronize()
    assert r.scene_info()["placement"] == 2
    r.close()


def test_pilot_waits_for_launches_in_flight():
    """the pilot rewrites the scene's records in place, and it is not always the
    scene's first launch (small launches leave it pending).  A small launch still queued on
    stream A (behind a spin kernel) when a large launch on stream B runs the pilot must
    render with the records it was launched with: pilot_end waits for every launch slot's
    event before the rewrite.  Both frames equal those of a scene that never pilots."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    small = scenes.config("C4", width=160, spp=4)
    big = scenes.config("C4", width=160, spp=32)

    def frames(r, sa, sb, spin):
        a = torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev)
        b = torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev)
        if spin:
            with torch.cuda.stream(sa):
                torch.cuda._sleep(200_000_000)  # ~0.1 s: the small launch waits behind it
        r.render_async(a.data_ptr(), 0, sa.cuda_stream, seed=3)
        N.check(N.lib.gs_render_tiles_async(r.dev, C.byref(r.cam), C.byref(big.settings), 5, C.byref(r.part),
                                            C.c_void_p(b.data_ptr()), None, C.c_void_p(sb.cuda_stream)))
        torch.cuda.synchronize()
        return a.cpu().numpy(), b.cpu().numpy()

    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    with _placement(0):
        r0 = g.Renderer(small, 0, 1, 64)
        ref_a, ref_b = frames(r0, sa, sb, False)
        r0.close()
    r = g.Renderer(small, 0, 1, 64)
    got_a, got_b = frames(r, sa, sb, True)
    assert r.scene_info()["placement"] == 2  # the large launch ran the pilot
    r.close()
    assert np.array_equal(got_a, ref_a)
    assert np.array_equal(got_b, ref_b)
