"""Compositions the reference's `Box<dyn Hittable>` allows beyond the reference scenes' own
(VERDICT r5 item 8), rendered by the device and compared with the CPU oracle, which builds the
same world with the reference's recursive trait objects:

* Translate / RotateY chains deeper than 4 (hittable.rs:93-135 wrap any Hittable): the device
  walks up to GS_MAX_CHAIN = 16 and re-walks the chain for the hit record's back-transforms;
* a chain inside a BVH that is itself under a chain (Translate(BVH([.., Translate(RotateY(x)),
  ..]))): the device keeps both chains of such a hit and applies the inner one, then the outer
  one, innermost first -- for spheres, cube lists, quads and media at the end of the chain;
* a BVH as a ConstantMedium boundary (volume.rs:10-17 takes any Hittable): its pre-order walk
  with the f64 slab test, every node counted, both boundary hits;
* one medium as another's boundary: the inner medium's own free-flight draws inside the outer
  one's boundary hits, in the reference's order (volume.rs:36-48).
Scenes with these shapes run on one catch-all kernel instantiation (GS_FEAT_GENERAL).

Still GS_ERR_UNSUPPORTED (tests/test_host.py): two levels of BVHs under chains, media two deep
inside media, list members that are not primitives.
Tolerance as everywhere: per-channel |delta| < 1e-3; counters as tests/test_gpu_parity.py.
"""
import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import scenes
from grayshift_amd.scene import camera_spec, fixed_spp
import oracle

from tests.test_gpu_parity import TOL, counters_match, maxdiff

pytestmark = pytest.mark.gpu


def _camera(width, look_from=(0.0, 2.0, 10.0)):
    return camera_spec(1.0, width, 12, 35.0, look_from, (0.0, 0.5, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)


def _check(sc, seed=3):
    out, gc = g.render(sc, seed=seed)
    ref, rc = oracle.render(sc, seed=seed)
    assert maxdiff(out, ref) < TOL
    assert counters_match(gc, rc)
    return gc


def _deep_chain(b, obj, depth):
    """depth instances, alternating RotateY and Translate (innermost first)."""
    for k in range(depth):
        obj = b.rotate_y(obj, 7.0 + 11.0 * k) if k % 2 == 0 else b.translate(obj, (0.1 * k, 0.05, -0.07 * k))
    return obj


@pytest.mark.parametrize("depth", [5, 9, 16])
def test_chains_deeper_than_four(depth):
    b = g.SceneBuilder()
    red, white = b.lambertian((0.8, 0.2, 0.2)), b.lambertian((0.7, 0.7, 0.7))
    b.add(_deep_chain(b, b.cube((-0.5, 0.0, -0.5), (0.5, 1.0, 0.5), red), depth))
    b.add(_deep_chain(b, b.sphere((1.5, 0.5, 0.0), 0.5, b.metal((0.8, 0.8, 0.9), 0.1)), depth))
    b.add(b.sphere((0.0, -100.0, 0.0), 100.0, white))
    b.background_solid((0.6, 0.7, 0.9))
    gc = _check(scenes.Scene("deep%d" % depth, b.build(), _camera(40), fixed_spp(8)))
    assert gc["instance_tests"] > 0


def test_chain_of_seventeen_is_rejected():
    b = g.SceneBuilder()
    b.add(_deep_chain(b, b.sphere((0.0, 0.0, 0.0), 1.0, b.lambertian((1, 1, 1))), 17))
    b.add(b.sphere((0.0, -100.0, 0.0), 99.0, b.lambertian((1, 1, 1))))
    from grayshift_amd import _native as N
    with pytest.raises(N.GrayshiftError) as e:
        g.render(scenes.Scene("deep17", b.build(), _camera(8), fixed_spp(1)))
    assert e.value.code == N.GS_ERR_UNSUPPORTED


def _nested_scene(inner, width=40, spp=8):
    """A BVH under Translate(RotateY(.)) whose leaves include `inner(b)`'s chained objects."""
    b = g.SceneBuilder()
    white, blue = b.lambertian((0.7, 0.7, 0.7)), b.lambertian((0.2, 0.3, 0.8))
    members = [b.sphere((-1.5 + 0.6 * k, 0.3, 0.2 * k), 0.25, blue) for k in range(6)]
    members += inner(b)
    b.add(b.translate(b.rotate_y(b.bvh(members), 25.0), (0.2, 0.0, -0.3)))
    b.add(b.sphere((0.0, -100.0, 0.0), 100.0, white))
    b.add(b.quad((-3.0, 4.0, -3.0), (6.0, 0.0, 0.0), (0.0, 0.0, 6.0), b.diffuse_light((3.0, 3.0, 3.0))))
    b.background_solid((0.4, 0.5, 0.6))
    return scenes.Scene("nested_chain", b.build(), _camera(width), fixed_spp(spp))


@pytest.mark.parametrize("what", ["sphere", "cube", "quad", "medium", "deep"])
def test_chain_inside_a_bvh_under_a_chain(what):
    def inner(b):
        m = b.lambertian((0.9, 0.5, 0.1))
        if what == "sphere":
            return [b.translate(b.rotate_y(b.sphere((0.8, 0.6, 0.0), 0.5, b.metal((0.9, 0.9, 0.9), 0.0)), 30.0),
                                (0.0, 0.2, 0.5))]
        if what == "cube":
            return [b.translate(b.rotate_y(b.cube((0.0, 0.0, 0.0), (0.8, 1.2, 0.8), m), -20.0), (0.5, 0.0, 0.3)),
                    b.rotate_y(b.cube((-1.2, 0.0, -0.4), (-0.6, 0.6, 0.2), b.dielectric(1.5)), 45.0)]
        if what == "quad":
            return [b.translate(b.quad((0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.3), m), (0.3, 0.1, 0.6))]
        if what == "medium":
            med = b.medium(b.cube((0.0, 0.0, 0.0), (1.0, 1.0, 1.0), m), 1.2, b.isotropic((0.8, 0.8, 0.8)))
            return [b.translate(b.rotate_y(med, 15.0), (0.4, 0.0, 0.2))]
        return [_deep_chain(b, b.sphere((0.5, 0.5, 0.5), 0.4, m), 7)]  # inner chain of 7, outer of 2
    gc = _check(_nested_scene(inner))
    assert gc["instance_tests"] > 0
    if what == "medium":
        assert gc["medium_tests"] > 0


def test_chain_inside_a_bvh_under_a_chain_on_eight_ranks():
    """The two-chain hit record travels through the frame context's ranks unchanged."""
    sc = _nested_scene(lambda b: [b.translate(b.rotate_y(b.cube((0, 0, 0), (0.8, 1.2, 0.8),
                                                                 b.lambertian((0.9, 0.5, 0.1))), -20.0),
                                              (0.5, 0.0, 0.3))], width=96, spp=4)
    one, oc = g.render(sc, seed=4)
    from grayshift_amd import _native as N
    N.check(N.lib.gs_debug_set_multi_same_device(1))
    try:
        m = g.MultiRenderer(sc, devices=[0] * 8, tile=16, plan=True)
    finally:
        N.check(N.lib.gs_debug_set_multi_same_device(0))
    try:
        res = m.render(seed=4, rgb=True)
    finally:
        m.close()
    assert np.array_equal(res["rgb"], one) and res["counters"] == oc


def _fog_camera(width):
    return camera_spec(1.0, width, 16, 40.0, (0.0, 1.0, 8.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.0, 8.0)


@pytest.mark.parametrize("chain", [False, True])
def test_bvh_as_a_medium_boundary(chain):
    b = g.SceneBuilder()
    glass, white = b.dielectric(1.5), b.lambertian((0.7, 0.7, 0.7))
    blobs = b.bvh([b.sphere((0.6 * k - 1.2, 0.2 * (k % 2), 0.1 * k), 0.5, glass) for k in range(5)] +
                  [b.cube((-0.5, -0.6, -0.5), (0.5, -0.2, 0.5), white)])
    boundary = b.translate(b.rotate_y(blobs, 20.0), (0.1, 0.2, 0.0)) if chain else blobs
    b.add(b.medium(boundary, 0.8, b.isotropic((0.9, 0.6, 0.3))))
    b.add(b.sphere((0.0, -101.0, 0.0), 100.0, white))
    b.add(b.quad((-2.0, 3.0, -2.0), (4.0, 0.0, 0.0), (0.0, 0.0, 4.0), b.diffuse_light((4.0, 4.0, 4.0))))
    b.background_solid((0.3, 0.4, 0.5))
    gc = _check(scenes.Scene("bvh_boundary", b.build(), _fog_camera(40), fixed_spp(12)))
    assert gc["medium_tests"] > 0 and gc["node_visits"] > 0


def test_medium_as_a_medium_boundary():
    b = g.SceneBuilder()
    glass, white = b.dielectric(1.5), b.lambertian((0.7, 0.7, 0.7))
    inner = b.medium(b.sphere((0.0, 0.0, 0.0), 1.2, glass), 1.5, b.isotropic((0.3, 0.8, 0.4)))
    b.add(b.medium(inner, 0.7, b.lambertian((0.8, 0.3, 0.3))))
    b.add(b.medium(b.translate(b.medium(b.cube((0, 0, 0), (1, 1, 1), white), 2.0, b.isotropic((0.9, 0.9, 0.9))),
                               (1.4, -0.9, -0.8)), 0.9, b.isotropic((0.5, 0.5, 0.9))))
    b.add(b.sphere((0.0, -101.0, 0.0), 100.0, white))
    b.add(b.quad((-2.0, 3.0, -2.0), (4.0, 0.0, 0.0), (0.0, 0.0, 4.0), b.diffuse_light((4.0, 4.0, 4.0))))
    b.background_solid((0.3, 0.4, 0.5))
    gc = _check(scenes.Scene("nested_media", b.build(), _fog_camera(40), fixed_spp(12)))
    assert gc["medium_tests"] > 0


def test_general_compositions_together_on_eight_ranks():
    """A scene holding every shape at once: frame-context ranks change nothing."""
    b = g.SceneBuilder()
    m, white = b.lambertian((0.9, 0.5, 0.1)), b.lambertian((0.7, 0.7, 0.7))
    inner = [b.translate(b.rotate_y(b.cube((0, 0, 0), (0.6, 0.9, 0.6), m), 30.0), (0.4, 0.0, 0.2))]
    b.add(b.translate(b.rotate_y(b.bvh([b.sphere((-1.0 + 0.5 * k, 0.3, 0.0), 0.2, white) for k in range(4)] + inner),
                                 15.0), (-0.5, 0.0, 0.0)))
    b.add(b.medium(b.bvh([b.sphere((1.2, 0.4, 0.3 * k), 0.35, white) for k in range(3)]), 1.0,
                   b.isotropic((0.4, 0.7, 0.9))))
    b.add(_deep_chain(b, b.sphere((0.0, 1.4, -1.0), 0.4, b.metal((0.9, 0.9, 0.9), 0.2)), 6))
    b.add(b.sphere((0.0, -101.0, 0.0), 100.0, white))
    b.background_solid((0.5, 0.6, 0.8))
    sc = scenes.Scene("general_all", b.build(), _camera(64), fixed_spp(6))
    _check(sc, seed=9)
    one, oc = g.render(sc, seed=9)
    from grayshift_amd import _native as N
    N.check(N.lib.gs_debug_set_multi_same_device(1))
    try:
        mr = g.MultiRenderer(sc, devices=[0] * 8, tile=16, plan=False)
    finally:
        N.check(N.lib.gs_debug_set_multi_same_device(0))
    try:
        res = mr.render(seed=9, rgb=True)
        assert mr.scene_info()["feat"] & 512  # GS_FEAT_GENERAL
    finally:
        mr.close()
    assert np.array_equal(res["rgb"], one) and res["counters"] == oc
