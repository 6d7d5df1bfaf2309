"""Malformed parts of a flat scene that the kernel never reads must stay harmless: the
upload (gs_device_scene_create) threads the BVHs under instances a reachable leaf walks,
and nothing else (an unreachable instance with a bad node child or a node cycle
must neither read past the node array nor loop).  And the frame context under two host
threads: the context's mutex serialises them, each frame the same."""
import ctypes as C
import threading

import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import _native as N
from grayshift_amd import scenes
from grayshift_amd.scene import SceneBuilder, camera_spec, fixed_spp

pytestmark = pytest.mark.gpu

GS_REF_SHIFT = 28
GS_REF_NODE, GS_REF_INSTANCE = 1, 7
GS_INST_TRANSLATE = 1


class gs_instance(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("child", C.c_uint32), ("p", C.c_double * 3)]


class gs_node(C.Structure):
    _fields_ = [("min", C.c_double * 3), ("max", C.c_double * 3), ("left", C.c_uint32), ("right", C.c_uint32),
                ("pad", C.c_uint32 * 2)]


def _nested_scene():
    """A BVH of 40 spheres under Translate(RotateY(..)) beside a ground sphere."""
    b = SceneBuilder()
    m = b.lambertian((0.7, 0.6, 0.5))
    inner = b.bvh([b.sphere((float(i % 8) - 4.0, float(i // 8) * 0.9, 0.0), 0.4, m) for i in range(40)])
    b.add(b.translate(b.rotate_y(inner, 15.0), (0.0, 0.5, 0.0)))
    b.add(b.sphere((0.0, -100.5, 0.0), 100.0, m))
    b.background_solid((0.7, 0.8, 1.0))
    cam = camera_spec(16.0 / 9.0, 64, 8, 30.0, (0.0, 2.0, 9.0), (0.0, 1.0, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    return b.build(), cam


def _render_flat(flat, cam_spec, spp=4):
    cam = g.camera(cam_spec)
    out = np.zeros((cam.image_height, cam.image_width, 3), dtype=np.float32)
    st = N.gs_stats()
    N.check(N.lib.gs_render(C.byref(flat), C.byref(cam), C.byref(fixed_spp(spp)), 5, out.ctypes.data, C.byref(st)))
    return out, st.counters.as_dict()


@pytest.mark.parametrize("bad", ["node_out_of_range", "node_cycle"])
def test_unreachable_instance_with_a_bad_tree_is_harmless(bad):
    spec, cam_spec = _nested_scene()
    hs = g.HostScene(spec)
    flat = N.gs_flat_scene.from_buffer_copy(hs.flat)
    ref, rc = _render_flat(flat, cam_spec)
    n = flat.n_instances
    old = (gs_instance * n).from_address(flat.instances)
    insts = (gs_instance * (n + 2))()
    for i in range(n):
        insts[i] = old[i]
    keep = []
    if bad == "node_out_of_range":
        child = (GS_REF_NODE << GS_REF_SHIFT) | (flat.n_nodes + 1000)
    else:
        # two extra nodes, each the other's left child: a cycle under an unreachable instance
        nn = flat.n_nodes
        nodes = (gs_node * (nn + 2))()
        C.memmove(nodes, flat.nodes, nn * C.sizeof(gs_node))
        for k in range(2):
            nodes[nn + k].left = (GS_REF_NODE << GS_REF_SHIFT) | (nn + 1 - k)
            nodes[nn + k].right = 0xFFFFFFFF
        keep.append(nodes)
        flat.nodes = C.cast(nodes, C.c_void_p).value
        flat.n_nodes = nn + 2
        child = (GS_REF_NODE << GS_REF_SHIFT) | nn
    insts[n] = gs_instance(GS_INST_TRANSLATE, child, (C.c_double * 3)(1.0, 0.0, 0.0))
    # and an unreachable instance chain that loops through itself
    insts[n + 1] = gs_instance(GS_INST_TRANSLATE, (GS_REF_INSTANCE << GS_REF_SHIFT) | (n + 1),
                               (C.c_double * 3)(0.0, 1.0, 0.0))
    flat.instances = C.cast(insts, C.c_void_p).value
    flat.n_instances = n + 2
    out = C.c_void_p()
    N.check(N.lib.gs_device_scene_create(C.byref(flat), C.byref(out)))
    N.check(N.lib.gs_device_scene_destroy(out))
    img, cnt = _render_flat(flat, cam_spec)
    assert np.array_equal(img, ref) and cnt == rc
    hs.close()


def test_frame_context_two_threads():
    """Two host threads rendering through one frame context: the context's mutex serialises
    whole frames, so both get the single-threaded frame."""
    sc = scenes.config("C4", width=96, spp=4)
    ref, _ = g.render(sc, seed=3)
    m = g.MultiRenderer(sc, num_gpus=1, tile=64, plan=False)
    res, errs = [None, None], []

    def work(k):
        try:
            for _ in range(3):
                r = m.render(seed=3, rgb=True)
            res[k] = r["rgb"]
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    m.close()
    assert not errs, errs
    for r in res:
        assert r is not None and np.array_equal(r.reshape(ref.shape), ref)
