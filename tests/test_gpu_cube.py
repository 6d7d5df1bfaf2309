"""Quad::cube lists as straight-line code (render.hip cube_test): every frame
and counter must equal the generic list loop's bit for bit (gs_debug_set_cube_lists(0)),
and the oracle within the north star's tolerance.  Cubes reached directly, under
Translate/RotateY chains, as ConstantMedium boundaries, inside BVHs; rays parallel to faces
(the Cornell camera's centre column and row), from inside a box, and the lists that must
keep the loop (a flat box, six quads out of cube order)."""
import os
import sys

import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import _native as N
from grayshift_amd import scenes
from grayshift_amd.scene import camera_spec
from grayshift_amd.scenes import fixed_spp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import oracle  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = 1e-3


def _both(sc, seed):
    try:
        N.check(N.lib.gs_debug_set_cube_lists(0))
        ref, rc = g.render(sc, seed=seed)
    finally:
        N.check(N.lib.gs_debug_set_cube_lists(1))
    out, oc = g.render(sc, seed=seed)
    assert np.array_equal(out, ref) and oc == rc
    return out, oc


@pytest.mark.parametrize("scene,kw", [("cornell_box", {}), ("cornell_smoke", {}),
                                      ("final_scene", {"boxes_per_side": 5, "n_balls": 40})])
def test_cube_lists_equal_loop_and_oracle(scene, kw):
    sc = scenes.SCENES[scene](width=48, **kw)
    out, oc = _both(sc, seed=4)
    ref, rc = oracle.render(sc, seed=4)
    assert float(np.abs(out.astype(np.float64) - ref).max()) < TOL
    assert oc == rc


def _box_scene(width, spp=6):
    b = g.SceneBuilder()
    red, white = b.lambertian((0.65, 0.05, 0.05)), b.lambertian((0.73, 0.73, 0.73))
    glass, light = b.dielectric(1.5), b.diffuse_light((7.0, 7.0, 7.0))
    members = [
        b.cube((-1, 0, -1), (1, 2, 1), red),                                # plain
        b.translate(b.rotate_y(b.cube((0, 0, 0), (1, 1, 1), white), 30.0), (2, 0, 0)),  # under a chain
        b.medium_isotropic(b.cube((-3, 0, -1), (-2, 1.5, 0.5), white), 0.6, (0.2, 0.4, 0.9)),  # boundary
        b.cube((-0.5, 2.5, -0.5), (0.5, 2.5, 0.5), glass),                 # flat: degenerate faces, loop
        b.hittable_list([b.quad((3, 0, 2), (1, 0, 0), (0, 1, 0), white),  # six quads out of cube order
                         b.quad((3, 0, 2), (0, 1, 0), (0, 0, 1), white),
                         b.quad((3, 1, 2), (1, 0, 0), (0, 0, 1), white),
                         b.quad((4, 0, 2), (0, 1, 0), (0, 0, 1), white),
                         b.quad((3, 0, 3), (1, 0, 0), (0, 1, 0), white),
                         b.quad((3, 0, 2), (1, 0, 0), (0, 0, 1), white)]),
        b.bvh([b.cube((x, 0, 3), (x + 0.4, 0.4 + 0.1 * x, 3.4), white) for x in np.arange(-3.0, 3.0, 0.5)]),
        b.quad((-1, 4, -1), (2, 0, 0), (0, 0, 2), light),
        b.sphere((0, -1000, 0), 1000.0, white),
    ]
    for m in members:
        b.add(m)
    b.background_solid((0.3, 0.4, 0.5))
    cam = camera_spec(1.0, width, 10, 50.0, (0.0, 1.0, 0.0), (0, 1, 5), (0, 1, 0), 0.0, 5.0)
    return scenes.Scene("boxes", b.build(), cam, fixed_spp(spp))


def test_cube_lists_everywhere_a_list_is_reached():
    """The camera sits inside the plain cube at (0, 1, 0) and looks along +z: the centre
    column and row of rays run parallel to four faces."""
    sc = _box_scene(41)
    out, oc = _both(sc, seed=11)
    ref, rc = oracle.render(sc, seed=11)
    assert float(np.abs(out.astype(np.float64) - ref).max()) < TOL
    assert oc == rc
    assert oc["quad_tests"] > 0 and oc["medium_tests"] > 0


def test_cube_lists_hook_rejects_bad_values():
    assert N.lib.gs_debug_set_cube_lists(2) == N.GS_ERR_ARG
    assert N.lib.gs_debug_set_cube_lists(-1) == N.GS_ERR_ARG
