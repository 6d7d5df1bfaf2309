"""Device known-answer tests: the megakernel's own device functions (geometry.hpp,
devmath.hpp), run through the test-only harness tests/hip/kat_device.hip, against the
CPU oracle bit-for-bit on random and adversarial cases."""
import ctypes as C
import math
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def kat(built):
    L = C.CDLL(os.path.join(HERE, "hip", "libkat_device.so"))
    P = C.c_void_p
    for f, args in {"kat_aabb": [C.c_int, P, P, P, P], "kat_aabb_cert": [C.c_int, P, P, P, P, P],
                    "kat_sphere": [C.c_int, P, P, P, P, P],
                    "kat_tri": [C.c_int, P, P, P, P], "kat_rng": [C.c_int, P, P, P, C.c_int, P],
                    "kat_math": [C.c_int, C.c_int, P, P, P],
                    "kat_noise": [C.c_int, C.c_int, P, C.c_double, P, P],
                    "kat_sky": [C.c_int, C.c_uint32, C.c_uint32, P, P],
                    "kat_rcp_cert": [C.c_int, P, P, P], "kat_div_by": [C.c_int, P, P, P, P]}.items():
        getattr(L, f).argtypes = args
        getattr(L, f).restype = C.c_int
    return L


def ptr(a):
    return a.ctypes.data


def _rays(rng, n, special=True):
    o = rng.uniform(-4, 4, (n, 3))
    d = rng.normal(size=(n, 3))
    if special:
        k = n // 4
        d[np.arange(k), rng.integers(0, 3, k)] = 0.0             # axis-parallel rays (1/0 = inf)
        d[k:2 * k, 0] = -0.0                                     # negative zero component
        o[2 * k:3 * k, 1] = np.round(o[2 * k:3 * k, 1])          # origins on integer planes
    return np.ascontiguousarray(np.hstack([o, d]))


def test_aabb_matches_oracle(kat):
    rng = np.random.default_rng(1)
    n = 20000
    ray = _rays(rng, n)
    lo = np.floor(rng.uniform(-3, 2, (n, 3)))
    ext = 1.0 + np.floor(rng.uniform(0, 3, (n, 3)))
    ext[rng.random(n) < 0.05, rng.integers(0, 3)] = 0.0                 # a few flat boxes
    box = np.ascontiguousarray(np.hstack([lo, lo + ext]))
    # aim 60% of the rays near their box (keeping the zero / negative-zero components) so
    # hits and misses are both common
    aim = rng.random(n) < 0.6
    to_box = 0.5 * (box[:, :3] + box[:, 3:]) - ray[:, :3] + rng.normal(scale=0.4, size=(n, 3))
    d = ray[:, 3:]
    ray[:, 3:] = np.where(aim[:, None] & (d != 0), to_box, d)
    iv = np.ascontiguousarray(np.stack([np.full(n, 0.001), np.where(rng.random(n) < 0.5, 1e300,
                                                                      rng.uniform(0, 6, n))], 1))
    out = np.zeros(n, np.int32)
    assert kat.kat_aabb(n, ptr(box), ptr(ray), ptr(iv), ptr(out)) == 0
    ref = np.array([oracle.aabb_hit(box[i, :3], box[i, 3:], ray[i, :3], ray[i, 3:], iv[i, 0], iv[i, 1])
                    for i in range(n)], np.int32)
    assert np.array_equal(out, ref)
    assert 0.05 < out.mean() < 0.95  # both outcomes exercised


def _grazing_cases(rng, n):
    """Rays aimed at box edges, faces and corners (tiny offsets, where f32 cannot decide),
    at unit and at C4 scales (boxes up to 2000 wide, origins up to 60 away)."""
    scale = np.where(rng.random(n) < 0.5, 1.0, rng.uniform(1, 60, n))[:, None]
    lo = rng.uniform(-3, 2, (n, 3)) * scale
    ext = rng.uniform(0.01, 3, (n, 3)) * np.where(rng.random((n, 1)) < 0.1, 700.0, 1.0) * scale
    box = np.hstack([lo, lo + ext])
    o = rng.uniform(-6, 6, (n, 3)) * scale
    # a target on the box surface: a corner, an edge or a face point, nudged by +-ulps
    t = lo + ext * rng.integers(0, 2, (n, 3))
    face = rng.integers(0, 3, n)
    frac = rng.random((n, 3))
    for k in range(3):
        m = (face == k) & (rng.random(n) < 0.5)
        t[m, k] = lo[m, k] + ext[m, k] * frac[m, k]
    t = t * (1.0 + rng.choice([-1, 1], (n, 3)) * rng.choice([0.0, 1e-16, 1e-12, 1e-9, 1e-7, 1e-5], (n, 3)))
    d = t - o
    d = d / np.where(rng.random((n, 1)) < 0.5, 1.0, np.linalg.norm(d, axis=1, keepdims=True))
    ray = np.hstack([o, d])
    tmax = np.where(rng.random(n) < 0.6, 1.7976931348623157e308, rng.uniform(0.2, 3.0, n))
    iv = np.stack([np.full(n, 0.001), tmax], 1)
    return np.ascontiguousarray(box), np.ascontiguousarray(ray), np.ascontiguousarray(iv)


def test_certified_f32_slab_matches_oracle(kat):
    """The node test the kernel runs for cert rays (box_cert in f32, the f64 test where it
    is undecided) decides exactly as the reference's f64 AABB::hit, on random boxes and
    on rays grazing box corners / edges / faces by 1e-16 .. 1e-5 relative; every
    decision f32 certifies is correct, and undecided ones are rare on random rays."""
    rng = np.random.default_rng(11)
    n = 40000
    box, ray, iv = _grazing_cases(rng, n)
    # plus the random cases of test_aabb_matches_oracle (non-cert rays report -1)
    rb = rng.uniform(-3, 2, (n, 3))
    box = np.ascontiguousarray(np.vstack([box, np.hstack([rb, rb + rng.uniform(0.1, 3, (n, 3))])]))
    ray = np.ascontiguousarray(np.vstack([ray, _rays(rng, n)]))
    iv = np.ascontiguousarray(np.vstack([iv, np.stack([np.full(n, 0.001), rng.uniform(0, 6, n)], 1)]))
    m = 2 * n
    out = np.zeros(m, np.int32)
    dec = np.zeros(m, np.int32)
    assert kat.kat_aabb_cert(m, ptr(box), ptr(ray), ptr(iv), ptr(out), ptr(dec)) == 0
    ref = np.array([oracle.aabb_hit(box[i, :3], box[i, 3:], ray[i, :3], ray[i, 3:], iv[i, 0], iv[i, 1])
                    for i in range(m)], np.int32)
    cert = dec >= 0
    assert cert[:n].all() and 0.4 < cert[n:].mean() < 1.0  # grazing cases are cert rays; the zero / -0 direction cases are not
    assert np.array_equal(out[cert], ref[cert])
    sure = (dec == 0) | (dec == 1)
    assert np.array_equal(dec[sure], ref[sure])  # what f32 certifies is right
    assert (dec[:n] == 2).sum() > 50  # the grazing cases do reach the f64 fallback
    assert (dec[n:][cert[n:]] == 2).mean() < 1e-3  # and random rays almost never need it


def test_sphere_matches_oracle_bitwise(kat):
    from grayshift_amd._native import GS_OBJ_SPHERE
    rng = np.random.default_rng(2)
    n = 20000
    ray = _rays(rng, n)
    sph = np.ascontiguousarray(np.hstack([rng.uniform(-2, 2, (n, 3)), rng.uniform(0.1, 3, (n, 1))]))
    iv = np.ascontiguousarray(np.stack([np.full(n, 0.001), np.where(rng.random(n) < 0.7, 1e300,
                                                                      rng.uniform(0, 5, n))], 1))
    t = np.zeros(n)
    hit = np.zeros(n, np.int32)
    assert kat.kat_sphere(n, ptr(sph), ptr(ray), ptr(iv), ptr(t), ptr(hit)) == 0
    for i in range(n):
        h = oracle.prim_hit(GS_OBJ_SPHERE, sph[i], ray[i, :3], ray[i, 3:], iv[i, 0], iv[i, 1])
        assert (h is not None) == bool(hit[i]), i
        if h is not None:
            assert h["t"] == t[i], i  # sqrt and / are correctly rounded on both sides


@pytest.mark.parametrize("W,H", [(1024, 512), (4096, 2048), (7, 3)])
def test_certified_sky_index_equals_f64(kat, W, H):
    """sky_index_f32 (f32 atan2f angles, accepted only away from texel boundaries) gives the
    f64 path's texel column and row whenever it decides, on uniform directions and on
    directions within 1e-10 .. 1e-4 rad of column and row boundaries, and decides almost
    all uniform directions."""
    rng = np.random.default_rng(13)
    n = 1_000_000
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    k = n // 2
    # near column boundaries: theta = 2 pi (i / W - 0.5) + delta; near row boundaries:
    # phi = pi (0.5 - j / H) + delta (the inverse of u, v in HDRI::sample)
    delta = np.where(rng.random(k) < 0.5, -1, 1) * 10.0 ** rng.uniform(-10, -4, k)
    th = 2 * np.pi * (rng.integers(0, W + 1, k) / W - 0.5) + delta
    ph = np.arcsin(np.clip(d[:k, 2], -1, 1))
    half = k // 2
    ph[:half] = np.pi * (0.5 - rng.integers(0, H + 1, half) / H) + delta[:half]
    th[:half] = rng.uniform(-np.pi, np.pi, half)
    d[:k] = np.stack([np.cos(ph) * np.cos(th), np.cos(ph) * np.sin(th), np.sin(ph)], 1)
    d = np.ascontiguousarray(d)
    out = np.zeros((n, 4), np.int32)
    assert kat.kat_sky(n, W, H, ptr(d), ptr(out)) == 0
    dec = out[:, 0] >= 0
    assert np.array_equal(out[dec, :2], out[dec, 2:])
    # undecided share of uniform directions ~ 2 (1e-6 W + 2e-6 H): 0.4% for the 1024x512 sky
    assert dec[k:].mean() > 1.0 - 6e-6 * (W + H)
    assert (~dec[:k]).sum() > 1000  # the boundary cases do reach the f64 path


def test_triangle_matches_oracle_bitwise(kat):
    from grayshift_amd._native import GS_OBJ_TRIANGLE
    rng = np.random.default_rng(3)
    n = 20000
    ray = _rays(rng, n, special=False)
    tri = np.ascontiguousarray(rng.uniform(-2, 2, (n, 9)))
    aim = rng.random(n) < 0.6  # towards the centroid, so hits are common
    cen = (tri[:, 0:3] + tri[:, 3:6] + tri[:, 6:9]) / 3.0
    ray[aim, 3:] = cen[aim] - ray[aim, :3] + rng.normal(scale=0.3, size=(int(aim.sum()), 3))
    tuv = np.zeros((n, 3))
    hit = np.zeros(n, np.int32)
    assert kat.kat_tri(n, ptr(tri), ptr(ray), ptr(tuv), ptr(hit)) == 0
    for i in range(n):
        h = oracle.prim_hit(GS_OBJ_TRIANGLE, tri[i], ray[i, :3], ray[i, 3:], 0.001, 1e300)
        assert (h is not None) == bool(hit[i]), i
        if h is not None:
            assert (h["t"], h["u"], h["v"]) == tuple(tuv[i]), i
    assert 0.02 < hit.mean() < 0.9


def test_rng_streams_match_oracle(kat):
    rng = np.random.default_rng(4)
    n, draws = 4096, 24
    seed = rng.integers(0, 2 ** 63, n, dtype=np.uint64)
    pix = rng.integers(0, 2 ** 31, n).astype(np.uint32)
    smp = rng.integers(0, 5000, n).astype(np.uint32)
    out = np.zeros((n, draws))
    assert kat.kat_rng(n, ptr(seed), ptr(pix), ptr(smp), draws, ptr(out)) == 0
    for i in range(0, n, 7):
        f, _ = oracle.wyrand(oracle.stream_seed(int(seed[i]), int(pix[i]), int(smp[i])), draws)
        assert np.array_equal(out[i], f)


@pytest.mark.parametrize("which,fn,lo,hi", [(0, math.sin, 0.0, 2 * math.pi), (1, math.cos, 0.0, 2 * math.pi),
                                            (2, math.acos, -1.0, 1.0), (3, math.asin, -1.0, 1.0)])
def test_transcendentals_within_one_ulp_of_libm(kat, which, fn, lo, hi):
    """OCML vs glibc (what the reference's Rust f64::sin etc. call): never more than
    1 ulp apart on the ranges the path uses; the mismatch rate is the source of the
    rare traversal-counter differences."""
    rng = np.random.default_rng(5 + which)
    n = 50000
    x = np.ascontiguousarray(rng.uniform(lo, hi, n))
    out = np.zeros(n)
    assert kat.kat_math(n, which, ptr(x), None, ptr(out)) == 0
    ref = np.array([fn(v) for v in x])
    ulps = np.abs(out - ref) / np.spacing(np.abs(ref))
    assert ulps.max() <= 1.0
    print("which=%d mismatch rate %.4f" % (which, float((out != ref).mean())))


def test_perlin_matches_oracle_bitwise(kat):
    """NoiseTexture's Perlin (noise 0.9 restated, perlin.hpp) against the oracle's
    independent restatement: bit-identical (pure f64 + - * and floor)."""
    rng = np.random.default_rng(11)
    n = 20000
    p = rng.uniform(-300, 300, (n, 3))
    p[: n // 10] = np.round(p[: n // 10])          # lattice points (exactly 0)
    p[n // 10: n // 5] *= 1e-3                      # near the origin, both signs
    p = np.ascontiguousarray(p)
    perm = np.ascontiguousarray(oracle.noise_perm(0))
    out = np.zeros(n)
    assert kat.kat_noise(n, 0, ptr(perm), 0.0, ptr(p), ptr(out)) == 0
    ref = np.array([oracle.perlin3(q) for q in p])
    assert np.array_equal(out, ref)
    assert (out[: n // 10] == 0.0).all()


def test_noise_texture_value_within_libm_ulps(kat):
    """value_at = 0.5 * (1 + sin(scale * z + 10 * turbulence)): turbulence is bit-exact,
    sin is OCML vs glibc (<= 1 ulp), so the channel differs by at most a few ulps."""
    rng = np.random.default_rng(12)
    n = 5000
    p = np.ascontiguousarray(rng.uniform(-400, 600, (n, 3)))
    perm = np.ascontiguousarray(oracle.noise_perm(0))
    for scale in (4.0, 0.2):
        out = np.zeros(n)
        assert kat.kat_noise(n, 1, ptr(perm), scale, ptr(p), ptr(out)) == 0
        ref = np.array([oracle.noise_value(scale, q) for q in p])
        assert np.abs(out - ref).max() <= 4 * np.spacing(1.0)


def test_rcp_cert_within_the_certificates_bound(kat):
    """rcp_cert (geometry.hpp, round 6): the certified test's 1/d from the hardware reciprocal
    and two Newton steps must be within 2^-50 of the exact quotient over the cert range (|1/d|
    in [1e-25, 1e15]); outside it -- zeros, infinities, denormals -- it must give a value
    cert_ray_ok rejects (NaN, an infinity, or a magnitude out of range), never a finite
    in-range wrong one."""
    rng = np.random.default_rng(7)
    n = 400000
    mant = rng.uniform(1.0, 2.0, n) * np.where(rng.random(n) < 0.5, -1.0, 1.0)
    d = mant * np.exp2(rng.integers(-83, 50, n)).astype(np.float64)
    d[:8] = [0.0, -0.0, np.inf, -np.inf, 5e-324, -1e-310, 1e-16, 1e26]
    d = np.ascontiguousarray(d)
    approx, exact = np.zeros(n), np.zeros(n)
    assert kat.kat_rcp_cert(n, ptr(d), ptr(approx), ptr(exact)) == 0
    with np.errstate(all="ignore"):
        inrange = (np.abs(exact) <= 1e15) & (np.abs(exact) >= 1e-25)
        rel = np.abs(approx[inrange] - exact[inrange]) / np.abs(exact[inrange])
        assert rel.max() <= 2.0 ** -50, rel.max()
        ok = lambda v: (np.abs(v) <= 1e15) & (np.abs(v) >= 1e-25)
        # a component clearly outside the range (zero, infinite, denormal, or 2x past a bound) is
        # rejected with the approximate value too; at a bound either choice is sound (the f64 test)
        out = ~((np.abs(exact) <= 2e15) & (np.abs(exact) >= 0.5e-25))
        assert out[:8].sum() >= 6 and not ok(approx[out]).any()


def test_root_division_through_the_reciprocal_is_exact(kat):
    """div_by (geometry.hpp, round 6: the sphere roots' (h -+ sqrt(disc)) / a through a refined
    reciprocal of a) equals the correctly rounded division bit for bit for every denominator in
    [2^-900, 2^900] and numerator >= 2^-968 in magnitude, incl. mantissas at the edges (all ones,
    powers of two), exact quotients and signed zeros' neighbours; a quotient under 2^-68 (below
    tmin) or an overflow may differ, and is rejected by the root's interval test either way."""
    rng = np.random.default_rng(11)
    n = 600000
    def draw(lo, hi, m):
        x = rng.uniform(1.0, 2.0, m) * np.exp2(rng.integers(lo, hi, m)).astype(np.float64)
        return np.where(rng.random(m) < 0.5, -x, x)
    den = np.abs(draw(-900, 900, n))
    num = draw(-968, 1000, n)
    k = n // 6  # edge mantissas: 1.111...1 and exact powers of two, exact small-integer quotients
    den[:k] = np.nextafter(np.exp2(rng.integers(-60, 60, k)).astype(np.float64), 0.0)
    num[k:2 * k] = np.exp2(rng.integers(-60, 60, k)).astype(np.float64)
    den[2 * k:3 * k] = rng.integers(1, 1 << 20, k).astype(np.float64)
    num[2 * k:3 * k] = den[2 * k:3 * k] * rng.integers(-1000, 1000, k)
    # the sphere's own shapes: a = |d|^2 of unit-ish directions, numerators h -+ sqrt(disc)
    den[3 * k:4 * k] = rng.uniform(0.01, 100.0, k)
    num[3 * k:4 * k] = rng.normal(scale=50.0, size=k)
    num, den = np.ascontiguousarray(num), np.ascontiguousarray(den)
    fast, exact = np.zeros(n), np.zeros(n)
    assert kat.kat_div_by(n, ptr(num), ptr(den), ptr(fast), ptr(exact)) == 0
    with np.errstate(all="ignore"):
        q = np.abs(num / den)
    inside = (q >= 2.0 ** -68) & np.isfinite(q) & (q < 1.7e308)
    assert inside.sum() > n // 2
    same = fast.view(np.uint64) == exact.view(np.uint64)
    assert same[inside].all(), (num[inside & ~same][:4], den[inside & ~same][:4])
