"""GPU parity of participating media: ConstantMedium (hittable/volume.rs:10-68) with an
Isotropic or Lambertian phase function (material.rs:171-200), against the CPU oracle.

The medium draws its free-flight distance from the lane's RNG stream *during*
traversal (volume.rs:48), so these renders also pin the device's traversal order:
a medium test reached in another order than the reference's left-first walk would
consume the stream at a different point and diverge.  Tolerance as everywhere:
per-channel |delta| < 1e-3 (north star); counters as tests/test_gpu_parity.py.
"""
import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import scenes
from grayshift_amd.scene import camera_spec, fixed_spp
import oracle

from tests.test_gpu_parity import TOL, _render_partitioned, counters_match, maxdiff

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("width,settings", [(40, fixed_spp(16)), (32, None)])
def test_cornell_smoke_matches_oracle(width, settings):
    """main.rs:519-624: two media bounded by Translate(RotateY(cube)) lists."""
    sc = scenes.cornell_smoke(width=width, settings=settings)
    out, gc = g.render(sc, seed=3)
    ref, rc = oracle.render(sc, seed=3)
    assert maxdiff(out, ref) < TOL
    assert counters_match(gc, rc)
    assert gc["medium_tests"] > 0


def fog_scene(width=40, spp=16, phase="lambertian", instanced=False):
    """final_scene's media (main.rs:713-738): a foggy sphere with a Lambertian phase
    function inside a world fog, plus an isotropic cube medium under Translate/RotateY."""
    b = g.SceneBuilder()
    glass = b.dielectric(1.5)
    fog = b.lambertian((0.2, 0.4, 0.9)) if phase == "lambertian" else b.isotropic((0.2, 0.4, 0.9))
    med = b.medium(b.sphere((0.0, 0.0, 0.0), 1.2, glass), 0.9, fog)
    b.add(b.translate(med, (0.5, 0.2, 0.0)) if instanced else med)
    b.add(b.sphere((0.0, 0.0, 0.0), 1.2, glass))  # the visible glass shell, as final_scene
    b.add(b.medium(b.sphere((0.0, 0.0, 0.0), 50.0, glass), 0.02, b.lambertian((1.0, 1.0, 1.0))))
    cube = b.cube((0.0, 0.0, 0.0), (1.0, 1.0, 1.0), b.lambertian((0.73, 0.73, 0.73)))
    b.add(b.medium(b.translate(b.rotate_y(cube, 20.0), (1.5, -1.0, -1.0)), 1.5, b.isotropic((0.9, 0.9, 0.9))))
    b.add(b.sphere((0.0, -101.0, 0.0), 100.0, b.lambertian((0.5, 0.5, 0.5))))
    b.add(b.quad((-2.0, 3.0, -2.0), (4.0, 0.0, 0.0), (0.0, 0.0, 4.0), b.diffuse_light((4.0, 4.0, 4.0))))
    b.background_solid((0.3, 0.4, 0.5))
    cam = camera_spec(1.0, width, 20, 40.0, (0.0, 1.0, 8.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.0, 8.0)
    return scenes.Scene("fog", b.build(), cam, fixed_spp(spp))


@pytest.mark.parametrize("phase", ["lambertian", "isotropic"])
@pytest.mark.parametrize("instanced", [False, True])
def test_media_variants_match_oracle(phase, instanced):
    sc = fog_scene(phase=phase, instanced=instanced)
    out, gc = g.render(sc, seed=5)
    ref, rc = oracle.render(sc, seed=5)
    assert maxdiff(out, ref) < TOL
    assert counters_match(gc, rc)
    assert gc["medium_tests"] > 0


def test_media_partition_invariance():
    """RNG draws inside traversal stay per (pixel, sample): tiles and chunks do not move them."""
    sc = fog_scene(width=48, spp=8)
    full, fc = g.render(sc, seed=2)
    part, pc = _render_partitioned(sc, 3, 16, seed=2)
    assert np.array_equal(full, part) and fc == pc


@pytest.mark.parametrize("phase", ["isotropic", "lambertian"])
def test_media_inside_a_bvh_under_instances_match_oracle(phase):
    """ConstantMedium leaves inside a BVH under Translate(RotateY(...)) (volume.rs:10-68 in a
    BVHNode, hittable.rs:107-211 around it): accepted since round 5, when the device began
    walking such trees in its main node and leaf passes, where a medium leaf is tested as at
    the top level and its hit carries the tree's chain.  Frames and counters against the
    oracle; the media draw inside traversal, so this also pins the walk's visit order."""
    b = g.SceneBuilder()
    glass = b.dielectric(1.5)
    fog = b.lambertian((0.2, 0.4, 0.9)) if phase == "lambertian" else b.isotropic((0.2, 0.4, 0.9))
    white = b.lambertian((0.73, 0.73, 0.73))
    items = [b.sphere((0.3 * k - 1.2, 0.25 * (k % 3), 0.0), 0.12, white) for k in range(9)]
    items.append(b.medium(b.sphere((0.0, 0.2, 0.0), 0.8, glass), 1.2, fog))
    items.append(b.medium(b.cube((0.6, -0.4, -0.4), (1.2, 0.3, 0.4), white), 2.0, b.isotropic((0.9, 0.8, 0.7))))
    b.add(b.translate(b.rotate_y(b.bvh(items), 25.0), (0.2, 0.1, -0.3)))
    b.add(b.sphere((0.0, -101.0, 0.0), 100.0, b.lambertian((0.5, 0.5, 0.5))))
    b.add(b.quad((-2.0, 3.0, -2.0), (4.0, 0.0, 0.0), (0.0, 0.0, 4.0), b.diffuse_light((4.0, 4.0, 4.0))))
    b.background_solid((0.3, 0.4, 0.5))
    cam = camera_spec(1.0, 40, 20, 40.0, (0.0, 1.0, 6.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.0, 6.0)
    sc = scenes.Scene("nested_fog", b.build(), cam, fixed_spp(16))
    out, gc = g.render(sc, seed=9)
    ref, rc = oracle.render(sc, seed=9)
    assert maxdiff(out, ref) < TOL
    assert counters_match(gc, rc)
    assert gc["medium_tests"] > 0 and gc["instance_tests"] > 0
