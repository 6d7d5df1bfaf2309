"""Known-answer tests of the CPU oracle, hand-derived from the reference formulas.

The reference ships no tests, so these are the oracle's pins: each
expected value is worked out from the cited Rust lines, independently of both the
oracle and the product code.  No GPU needed.
"""
import math
import struct

import numpy as np
import pytest

import oracle

M64 = (1 << 64) - 1


def wyrand_ref(state, n):
    """fastrand 2.1.1 gen_u64 + f64, written out again with Python integers."""
    out_u, out_f = [], []
    for _ in range(n):
        state = (state + 0x2D358DCCAA6C78A5) & M64
        t = state * (state ^ 0x8BB84B93962EACC9)
        u = (t & M64) ^ (t >> 64)
        out_u.append(u)
        bits = 0x3FF0000000000000 | (u >> 12)
        out_f.append(struct.unpack("<d", struct.pack("<Q", bits))[0] - 1.0)
    return out_u, out_f


@pytest.mark.parametrize("seed", [0, 1, 42, 0x6772617973686966, M64])
def test_wyrand_stream(seed):
    f, u = oracle.wyrand(seed, 16)
    ru, rf = wyrand_ref(seed, 16)
    assert [int(x) for x in u] == ru
    assert list(f) == rf
    assert all(0.0 <= x < 1.0 for x in f)


def test_wyrand_f64_mapping_edges():
    # f64 = from_bits(0x3FF0... | u >> 12) - 1: u = 0 -> 0.0, u = 2^64-1 -> 1 - 2^-52
    lo = struct.unpack("<d", struct.pack("<Q", 0x3FF0000000000000))[0] - 1.0
    hi = struct.unpack("<d", struct.pack("<Q", 0x3FF0000000000000 | (M64 >> 12)))[0] - 1.0
    assert lo == 0.0 and hi == 1.0 - 2.0 ** -52


def splitmix(x):
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


@pytest.mark.parametrize("seed,pixel,sample", [(1, 0, 0), (1, 12345, 511), (7, 2073599, 4095), (M64, 1, 2)])
def test_stream_seed(seed, pixel, sample):
    assert oracle.stream_seed(seed, pixel, sample) == splitmix(seed ^ splitmix((sample << 32) | pixel))


# ------------------------------------------------------------------ AABB.rs:58-113
def test_aabb_straight_hit_and_miss():
    mn, mx = (-1, -1, -1), (1, 1, 1)
    assert oracle.aabb_hit(mn, mx, (-5, 0, 0), (1, 0, 0), 0.001, 1e300)
    assert not oracle.aabb_hit(mn, mx, (-5, 2, 0), (1, 0, 0), 0.001, 1e300)
    # box behind the ray
    assert not oracle.aabb_hit(mn, mx, (5, 0, 0), (1, 0, 0), 0.001, 1e300)
    # negative direction component: t0 > t1 branch
    assert oracle.aabb_hit(mn, mx, (5, 0, 0), (-1, 0, 0), 0.001, 1e300)
    # interval ends before the box (t enters at 4)
    assert not oracle.aabb_hit(mn, mx, (-5, 0, 0), (1, 0, 0), 0.001, 3.9)
    assert oracle.aabb_hit(mn, mx, (-5, 0, 0), (1, 0, 0), 0.001, 4.1)


def test_aabb_zero_direction_component():
    mn, mx = (-1, -1, -1), (1, 1, 1)
    # d.y = 0: 1/0 = +inf; inside the slab -> (-inf, +inf), outside -> (+inf, +inf) = miss
    assert oracle.aabb_hit(mn, mx, (-5, 0.5, 0), (1, 0, 0), 0.001, 1e300)
    assert not oracle.aabb_hit(mn, mx, (-5, 1.5, 0), (1, 0, 0), 0.001, 1e300)
    # origin exactly on the max plane: t0 = -2*inf = -inf, t1 = 0*inf = NaN; t0 < t1 is
    # false so the else branch runs: `t0 < max` sets max = -inf -> miss
    assert not oracle.aabb_hit(mn, mx, (-5, 1.0, 0), (1, 0, 0), 0.001, 1e300)
    # on the min plane: t0 = NaN, t1 = +inf; else branch: `t1 > min` sets min = +inf -> miss
    assert not oracle.aabb_hit(mn, mx, (-5, -1.0, 0), (1, 0, 0), 0.001, 1e300)


def test_aabb_zero_width_interval_misses():
    # entry 4, exit 6 clipped to [2, 2]: min becomes 4 > max 2 -> miss
    assert not oracle.aabb_hit((0, -1, -1), (2, 1, 1), (-4, 0, 0), (1, 0, 0), 2.0, 2.0)


# ------------------------------------------------------------- sphere.rs:55-106
def test_sphere_front_hit_and_uv():
    from grayshift_amd._native import GS_OBJ_SPHERE
    h = oracle.prim_hit(GS_OBJ_SPHERE, (0, 0, 0, 1), (0, 0, -5), (0, 0, 1), 0.001, 1e300)
    assert h["t"] == 4.0
    assert list(h["p"]) == [0.0, 0.0, -1.0]
    assert list(h["n"]) == [0.0, 0.0, -1.0] and h["front"]
    # p = (0,0,-1): theta = acos(-(-0)) wait: theta = acos(-p.y) = acos(-0) = pi/2 -> v = 0.5
    # phi = atan2(-p.z, p.x) + pi = atan2(1, 0) + pi = 3pi/2 -> u = 0.75
    assert h["u"] == pytest.approx(0.75, abs=1e-15) and h["v"] == pytest.approx(0.5, abs=1e-15)


def test_sphere_inside_far_root_and_flip():
    from grayshift_amd._native import GS_OBJ_SPHERE
    h = oracle.prim_hit(GS_OBJ_SPHERE, (0, 0, 0, 1), (0, 0, 0), (0, 0, 1), 0.001, 1e300)
    assert h["t"] == 1.0 and not h["front"]
    assert list(h["n"]) == [-0.0, -0.0, -1.0]  # outward (0,0,1) flipped


def test_sphere_unnormalised_direction_and_open_interval():
    from grayshift_amd._native import GS_OBJ_SPHERE
    h = oracle.prim_hit(GS_OBJ_SPHERE, (0, 0, 0, 1), (0, 0, -5), (0, 0, 2), 0.001, 1e300)
    assert h["t"] == 2.0  # a = |d|^2 = 4 (camera rays are not normalised, camera.rs:217)
    # surrounds is open: t == tmax is rejected, and the far root (t=6) is beyond it
    assert oracle.prim_hit(GS_OBJ_SPHERE, (0, 0, 0, 1), (0, 0, -5), (0, 0, 1), 0.001, 4.0) is None
    # near root before tmin: the far root is taken
    h = oracle.prim_hit(GS_OBJ_SPHERE, (0, 0, 0, 1), (0, 0, -5), (0, 0, 1), 4.5, 1e300)
    assert h["t"] == 6.0 and not h["front"]


def test_moving_sphere_center_at_time():
    from grayshift_amd._native import GS_OBJ_MOVING_SPHERE
    # center moves (0,0,0) -> (2,0,0); at time 0.5 it is (1,0,0)
    h = oracle.prim_hit(GS_OBJ_MOVING_SPHERE, (0, 0, 0, 2, 0, 0, 1), (1, 0, -5), (0, 0, 1), 0.001, 1e300, time=0.5)
    assert h["t"] == 4.0 and list(h["p"]) == [1.0, 0.0, -1.0]


# --------------------------------------------------------- quad.rs / plane.rs
def test_quad_hit_uv_and_closed_edges():
    from grayshift_amd._native import GS_OBJ_QUAD
    q = (0, 0, 0, 1, 0, 0, 0, 1, 0)
    h = oracle.prim_hit(GS_OBJ_QUAD, q, (0.25, 0.5, 1), (0, 0, -1), 0.001, 1e300)
    assert h["t"] == 1.0 and h["u"] == 0.25 and h["v"] == 0.5
    assert list(h["n"]) == [0.0, 0.0, 1.0] and h["front"]
    # alpha == 1 and beta == 0 are inside (Interval::UNIT.contains is closed)
    assert oracle.prim_hit(GS_OBJ_QUAD, q, (1.0, 0.0, 1), (0, 0, -1), 0.001, 1e300) is not None
    assert oracle.prim_hit(GS_OBJ_QUAD, q, (1.0 + 1e-12, 0.5, 1), (0, 0, -1), 0.001, 1e300) is None
    # t == tmax is accepted (contains is closed)
    assert oracle.prim_hit(GS_OBJ_QUAD, q, (0.5, 0.5, 1), (0, 0, -1), 0.001, 1.0) is not None
    # |n . d| < 1e-8: parallel -> miss
    assert oracle.prim_hit(GS_OBJ_QUAD, q, (0.5, 0.5, 1), (1, 0, 0), 0.001, 1e300) is None
    # back side: normal flipped
    h = oracle.prim_hit(GS_OBJ_QUAD, q, (0.5, 0.5, -1), (0, 0, 1), 0.001, 1e300)
    assert not h["front"] and list(h["n"]) == [-0.0, -0.0, -1.0]


# -------------------------------------------------------------- triangle.rs
def test_triangle_one_sided_unnormalised_and_ignores_interval():
    from grayshift_amd._native import GS_OBJ_TRIANGLE
    tri = (0, 0, 0, 2, 0, 0, 0, 2, 0)  # normal = (b-a)x(c-a) = (0,0,4), not unit
    # e1 = c-a = (0,2,0), e2 = b-a = (2,0,0).  Looking down -z: p = d x e2 = (0,-2,0),
    # det = e1.p = -4 < 1e-8 -> culled (the visible side is opposite the stored normal)
    assert oracle.prim_hit(GS_OBJ_TRIANGLE, tri, (0.5, 0.5, 1), (0, 0, -1), 0.001, 1e300) is None
    # Looking up +z from below: p = (0,2,0), det = 4; t_vec = (.5,.5,-1), u = 1;
    # q = t_vec x e1 = (2,0,1), v = 1; t = e2.q = 4 -> /det: t = 1, u = v = 0.25
    h = oracle.prim_hit(GS_OBJ_TRIANGLE, tri, (0.5, 0.5, -1), (0, 0, 1), 0.001, 1e300)
    assert (h["t"], h["u"], h["v"]) == (1.0, 0.25, 0.25)
    # d.n = 4 > 0 -> back face, normal flipped and left unnormalised
    assert not h["front"] and list(h["n"]) == [-0.0, -0.0, -4.0]
    # triangle.rs never checks ray_t: a hit behind the origin (t = -1) is returned
    h = oracle.prim_hit(GS_OBJ_TRIANGLE, tri, (0.5, 0.5, 1), (0, 0, 1), 0.001, 1e300)
    assert h is not None and h["t"] == -1.0


# ------------------------------------------------------------------- ONB.rs
def test_onb_axis_switch():
    b = oracle.onb((1.0, 0.0, 0.0))  # |w.x| > 0.9 -> a = (0,1,0)
    assert b[2].tolist() == [1.0, 0.0, 0.0]
    assert b[1].tolist() == [0.0, 0.0, 1.0]       # v = w x a
    assert b[0].tolist() == [0.0, -1.0, 0.0]      # u = w x v
    b = oracle.onb((0.0, 0.0, 3.0))  # w = unit(n) = (0,0,1); a = (1,0,0)
    assert b[2].tolist() == [0.0, 0.0, 1.0]
    assert b[1].tolist() == [0.0, 1.0, 0.0]
    assert b[0].tolist() == [-1.0, 0.0, 0.0]


# ------------------------------------------------------------------ util.rs:48-60
def test_random_cosine_direction_quirk():
    assert oracle.random_cosine_direction(0.0, 1.0).tolist() == [1.0, 0.0, 0.0]
    v = oracle.random_cosine_direction(0.0, 0.0625)
    # x = cos(0) * sqrt(sqrt(0.0625)) = 0.5 (r2^(1/4), not r2^(1/2)); z = sqrt(0.9375)
    assert v[0] == 0.5 and v[1] == 0.0 and v[2] == math.sqrt(0.9375)
    assert v[0] ** 2 + v[2] ** 2 == pytest.approx(1.1875)  # not a unit vector


# ------------------------------------------------------- material.rs / vec3.rs
def test_schlick_reflectance():
    assert oracle.reflectance(1.0, 1.5) == pytest.approx(0.04, abs=1e-17)
    assert oracle.reflectance(0.0, 1.5) == pytest.approx(1.0, abs=1e-16)
    x = 0.5
    r0 = ((1 - 1.5) / (1 + 1.5)) ** 2
    assert oracle.reflectance(0.5, 1.5) == r0 + (1 - r0) * (x * ((x * x) * (x * x)))


def test_refract_normal_incidence():
    r = oracle.refract((0, 0, -1), (0, 0, 1), 1 / 1.5)
    assert r.tolist() == [0.0, 0.0, -1.0]


def test_rotate_vector():
    assert oracle.rotate_vector((1, 2, 3), (0, 0, 0)).tolist() == [1.0, 2.0, 3.0]
    r = oracle.rotate_vector((1, 0, 0), (0, math.pi / 2, 0))
    assert r == pytest.approx([0.0, 0.0, 1.0], abs=1e-15)


# ------------------------------------------------------------------- color.rs
def test_luminance_blue_weight_quirk():
    assert oracle.luminance((1.0, 1.0, 1.0)) == 0.299 + 0.587 + 0.144  # 1.03, not 1.0
    assert oracle.luminance((0.0, 0.0, 1.0)) == 0.144


@pytest.mark.parametrize("c,byte", [(0.0, 0), (-1.0, 0), (1.0, 255), (4.0, 255), (0.25, 128), (float("nan"), 0),
                                    (0.0625, 64)])
def test_write_color_byte(c, byte):
    assert oracle.color_byte(c) == byte


# ------------------------------------------------------------------ texture.rs
def test_checkered_parity_truncating_mod():
    assert oracle.checker_even(1.0, (0.5, 0.5, 0.5))            # 0+0+0 even
    assert not oracle.checker_even(1.0, (-0.5, 0.5, 0.5))       # -1 % 2 = -1 -> odd
    assert oracle.checker_even(1.0, (-0.5, -0.5, 0.5))          # -2 even
    assert not oracle.checker_even(0.32, (0.33, 0.0, 0.0))      # floor(1.03) = 1 odd


# ---------------------------------------------------------------- BVH.rs:18-65
def _world(n, positions=None):
    from grayshift_amd.scene import SceneBuilder
    b = SceneBuilder()
    m = b.lambertian((0.5, 0.5, 0.5))
    for k in range(n):
        p = positions[k] if positions else (float(k) * 3.0, 0.0, 0.0)
        b.add(b.sphere(p, 1.0, m))
    return b.build()


def _pairs(t):
    return [tuple(t[i:i + 2]) for i in range(0, len(t), 2)]


def test_bvh_n1_wraps_with_no_right_child():
    assert _pairs(oracle.bvh_topology(_world(1)).tolist()) == [(1, 0), (-1, 1), (0, 1)]


def test_bvh_n2_holds_both_objects():
    assert _pairs(oracle.bvh_topology(_world(2)).tolist()) == [(1, 0), (-1, 1), (-1, 1)]


def test_bvh_n3_median_split():
    # 3 objects: split at len/2 = 1 -> left = 1 object (n==1 wrapper), right = 2 objects
    assert _pairs(oracle.bvh_topology(_world(3)).tolist()) == [
        (1, 0), (1, 1), (-1, 2), (0, 2), (1, 1), (-1, 2), (-1, 2)]


def test_bvh_depth_is_logarithmic():
    t = _pairs(oracle.bvh_topology(_world(1000)).tolist())
    assert max(d for k, d in t) <= 11  # ceil(log2(1000)) + 1


# ------------------------------------------------------ NoiseTexture (noise 0.9)
def test_noise_permutation_is_a_permutation_and_host_agrees():
    """PermutationTable::new(0) restated twice (oracle, product host): the same table, a
    permutation of 0..=255.  Parity with the real crate is unpinned."""
    import ctypes as C
    from grayshift_amd import _native as N
    for seed in (0, 1, 0xDEADBEEF):
        p = oracle.noise_perm(seed)
        assert sorted(p.tolist()) == list(range(256))
        h = np.zeros(256, dtype=np.uint8)
        N.lib.gs_host_noise_permutation(seed, h.ctypes.data)
        assert np.array_equal(h, p)
    assert not np.array_equal(oracle.noise_perm(0), oracle.noise_perm(1))


def test_perlin_known_properties():
    # zero on the integer lattice; continuous across cell faces; bounded
    for q in [(0, 0, 0), (3, -7, 12), (-1, -1, -1), (255, 256, 257)]:
        assert oracle.perlin3(np.array(q, float)) == 0.0
    rng = np.random.default_rng(3)
    for _ in range(200):
        c = np.floor(rng.uniform(-20, 20, 3))
        axis = rng.integers(0, 3)
        a, b = c.copy(), c.copy()
        a[axis] -= 1e-9
        b[axis] += 1e-9
        a += rng.uniform(0.1, 0.9, 3) * (np.arange(3) != axis)
        b = a.copy()
        b[axis] = c[axis] + 1e-9
        assert abs(oracle.perlin3(a) - oracle.perlin3(b)) < 1e-6
    v = [oracle.perlin3(rng.uniform(-100, 100, 3)) for _ in range(5000)]
    assert max(abs(x) for x in v) < 1.2 and np.std(v) > 0.1


def test_noise_texture_value_formula():
    # texture.rs:127-130 at a lattice point where every octave is 0: 0.5 * (1 + sin(scale*z))
    for scale, z in [(4.0, 3.0), (0.2, -8.0)]:
        p = np.array([5.0, -2.0, z])
        assert oracle.noise_value(scale, p) == 0.5 * (1.0 + math.sin(scale * z))
