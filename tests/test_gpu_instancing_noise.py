"""GPU parity of SURVEY.md §8f rank 4: BVHs under Translate/RotateY (final_scene's
rotated box of balls, main.rs:741-755) and NoiseTexture (texture.rs:97-131; noise 0.9
Perlin restated, parity with the crate unpinned — DESIGN.md §2), against the CPU oracle.

Tolerance as everywhere: per-channel |delta| < 1e-3 (north star); counters as
tests/test_gpu_parity.py (the nested walk counts node visits like the top level).
"""
import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import scenes
from grayshift_amd.scene import camera_spec, fixed_spp
import oracle

from tests.test_gpu_parity import TOL, _render_partitioned, counters_match, maxdiff

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,width,spp", [("perlin_spheres", 48, 8), ("simple_light", 48, 8),
                                            ("final_scene", 40, 8), ("final_scene", 16, None)])
def test_scene_matches_oracle(name, width, spp):
    sc = scenes.SCENES[name](width=width, settings=fixed_spp(spp) if spp else None)
    out, gc = g.render(sc, seed=21)
    ref, rc = oracle.render(sc, seed=21)
    assert maxdiff(out, ref) < TOL
    assert counters_match(gc, rc)
    assert gc["noise_evals"] > 0
    if name == "final_scene":
        assert gc["instance_tests"] > 0 and gc["medium_tests"] > 0


def nested_scene(width=40, spp=8, depth_chain=2, leaf="spheres", radii=1):
    """A BVH of spheres / cubes (lists) / triangles under a Translate/RotateY chain,
    next to top-level geometry.  `radii`: distinct sphere radii (round 4's inline nested-sphere
    records took at most 16; since round 5 a nested tree's leaves are ordinary leaf records of
    the main walk, spheres inline whatever their radii)."""
    b = g.SceneBuilder()
    rng = np.random.default_rng(7)
    white = b.lambertian((0.73, 0.73, 0.73))
    metal = b.metal((0.8, 0.8, 0.9), 0.2)
    glass = b.dielectric(1.5)
    members = []
    for k in range(120):
        c = tuple(float(v) for v in rng.uniform(-3, 3, 3))
        m = (white, metal, glass)[k % 3]
        if leaf == "spheres" or k % 3 == 0:
            members.append(b.sphere(c, 0.3 + 0.01 * (k % radii), m))
        elif leaf == "cubes":
            members.append(b.cube(c, (c[0] + 0.4, c[1] + 0.5, c[2] + 0.3), m))
        else:
            members.append(b.triangle(c, (c[0] + 0.5, c[1], c[2]), (c[0], c[1] + 0.5, c[2] + 0.2), m))
    obj = b.bvh(members)
    obj = b.rotate_y(obj, 30.0)
    if depth_chain >= 2:
        obj = b.translate(obj, (0.5, 1.0, -0.5))
    if depth_chain >= 3:
        obj = b.rotate_y(obj, -12.0)
    b.add(obj)
    b.add(b.sphere((0.0, -1004.0, 0.0), 1000.0, b.lambertian_texture(b.noise(1.5))))
    b.add(b.quad((-2.0, 6.0, -2.0), (4.0, 0.0, 0.0), (0.0, 0.0, 4.0), b.diffuse_light((5.0, 5.0, 5.0))))
    b.background_solid((0.4, 0.5, 0.7))
    cam = camera_spec(1.0, width, 20, 50.0, (0.0, 2.0, 12.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    return scenes.Scene("nested", b.build(), cam, fixed_spp(spp))


@pytest.mark.parametrize("leaf,radii", [("spheres", 1), ("spheres", 16), ("spheres", 17), ("cubes", 1),
                                        ("triangles", 1)])
@pytest.mark.parametrize("depth_chain", [1, 3])
def test_nested_bvh_variants_match_oracle(leaf, radii, depth_chain):
    sc = nested_scene(leaf=leaf, depth_chain=depth_chain, radii=radii)
    r = g.Renderer(sc)
    assert r.scene_info()["feat"] & 2  # GS_FEAT_NESTED: the trees are walked in the main loop
    r.close()
    out, gc = g.render(sc, seed=4)
    ref, rc = oracle.render(sc, seed=4)
    assert maxdiff(out, ref) < TOL
    assert counters_match(gc, rc)
    assert gc["instance_tests"] > 0


def test_final_scene_partition_invariance():
    sc = scenes.final_scene(width=48, settings=fixed_spp(4))
    full, fc = g.render(sc, seed=2)
    part, pc = _render_partitioned(sc, 3, 16, seed=2)
    assert np.array_equal(full, part) and fc == pc


def test_final_scene_ppm_matches_oracle():
    sc = scenes.final_scene(width=32, settings=fixed_spp(4))
    assert g.render_ppm(sc, seed=9)[0] == oracle.render_ppm(sc, seed=9)[0]


def test_final_scene_is_independent_of_leaf_batch_and_node_steps():
    """The scene's launch choices (leaf batch 48 and full node passes for BVHs under
    instances, kind-batched leaf passes) only regroup which lanes a pass serves: every lane
    tests its own records in its own order, so frames and counters equal any other
    choice's, and the oracle's."""
    from grayshift_amd import _native as N
    sc = scenes.final_scene(width=40, settings=fixed_spp(4))
    ref, rc = oracle.render(sc, seed=5)
    runs = []
    try:
        for lb, ns in [(0, 0), (1, 1), (12, 3), (64, 8)]:
            g.set_tuning(52, 0, lb, -1)
            N.check(N.lib.gs_set_node_steps(ns))
            runs.append(g.render(sc, seed=5))
    finally:
        g.set_tuning(0, 0, 0, -1)
        N.check(N.lib.gs_set_node_steps(0))
    for out, gc in runs:
        assert np.array_equal(out, runs[0][0]) and gc == runs[0][1]
    assert maxdiff(runs[0][0], ref) < TOL
    assert counters_match(runs[0][1], rc)
