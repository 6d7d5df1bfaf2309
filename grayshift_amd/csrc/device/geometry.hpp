// geometry.hpp — device-side restatements of the reference's geometric tests
// (AABB.rs, sphere.rs, quad.rs/plane.rs, triangle.rs, hittable.rs Translate/RotateY)
// and the device records they read.  Shared by the megakernel (render.hip) and the
// device known-answer-test harness (tests/hip/kat_device.hip).
#pragma once
#include "../../../include/grayshift_gpu.h"
#include "devmath.hpp"

namespace gsd {

struct alignas(16) DNode {  // 64 B: box (f64, as AABB.rs) + children
    double mnx, mny, mnz, mxx, mxy, mxz;
    uint32_t left, right, pad0, pad1;
};
struct alignas(16) DSphere {  // 32 B: what Sphere::hit reads; material kept apart
    double cx, cy, cz, r;
};
struct Ray {
    d3 o, d;
    double time;
};

__device__ __forceinline__ DNode load_node(const DNode* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    DNode n;
    n.mnx = __hiloint2double((int)a.y, (int)a.x);
    n.mny = __hiloint2double((int)a.w, (int)a.z);
    n.mnz = __hiloint2double((int)b.y, (int)b.x);
    n.mxx = __hiloint2double((int)b.w, (int)b.z);
    n.mxy = __hiloint2double((int)c.y, (int)c.x);
    n.mxz = __hiloint2double((int)c.w, (int)c.z);
    n.left = d.x;
    n.right = d.y;
    n.pad0 = d.z;
    n.pad1 = d.w;
    return n;
}

// The box and the two links only (56 B: 3 x dwordx4 + dwordx2): the vector-memory pipe,
// not the bytes, limits the traversal loop, so the pad word is not fetched.
__device__ __forceinline__ DNode load_node56(const DNode* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const uint4 a = q[0], b = q[1], c = q[2];
    const uint2 d = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(p) + 48);
    DNode n;
    n.mnx = __hiloint2double((int)a.y, (int)a.x);
    n.mny = __hiloint2double((int)a.w, (int)a.z);
    n.mnz = __hiloint2double((int)b.y, (int)b.x);
    n.mxx = __hiloint2double((int)b.w, (int)b.z);
    n.mxy = __hiloint2double((int)c.y, (int)c.x);
    n.mxz = __hiloint2double((int)c.w, (int)c.z);
    n.left = d.x;
    n.right = d.y;
    n.pad0 = 0;
    n.pad1 = 0;
    return n;
}

// AABB::hit (AABB.rs:58-113) with the reference's 1.0/d hoisted per ray (same value).
// The early-outs of the reference do not change the boolean: once max <= min the
// later slabs only raise min / lower max, and NaN slabs never assign.
// `if a > lo { lo = a }` == fmax(lo, a) because lo is never NaN (tmin / tmax and only
// non-NaN values are ever assigned) and IEEE maxNum ignores a NaN operand, as the
// reference's failed comparison does (a == lo keeps an equal value).  Same for hi.
// The t0/t1 swap must stay a compare-select: min/max would treat a NaN t1 differently.
// (Round 1 issued bare v_max_f64 / v_min_f64 through inline asm, one with an SGPR-pair
// operand.  With the certified f32 test added, the media + nested-BVH kernel — which
// spills SGPRs and VGPRs — rendered final_scene wrongly and non-deterministically with
// the asm and correctly with these builtins (every node decision checked right, so the
// asm's operands were corrupted; a hazard the compiler does not guard inside inline asm
// is the likely cause).  The f64 test is now the rare path behind box_cert, so the
// builtins' canonicalisation costs nothing measurable.)
__device__ __forceinline__ double hw_max(double a, double b) { return __builtin_fmax(a, b); }
__device__ __forceinline__ double hw_min(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ double hw_max_u(double u, double b) { return __builtin_fmax(u, b); }

__device__ __forceinline__ void slab(double mn, double mx, double o, double inv, double& lo, double& hi) {
    const double t0 = (mn - o) * inv, t1 = (mx - o) * inv;
    const bool s = t0 < t1;
    const double a = s ? t0 : t1, b = s ? t1 : t0;
    lo = hw_max(lo, a);
    hi = hw_min(hi, b);
}
__device__ __forceinline__ bool box_hit(const DNode& n, const d3& o, const d3& inv, double tmin, double tmax) {
    double hi = tmax;
    double lo;
    {  // first slab: lo = max(tmin, a) with tmin uniform
        const double t0 = (n.mnx - o.x) * inv.x, t1 = (n.mxx - o.x) * inv.x;
        const bool s = t0 < t1;
        const double a = s ? t0 : t1, b = s ? t1 : t0;
        lo = hw_max_u(tmin, a);
        hi = hw_min(hi, b);
    }
    slab(n.mny, n.mxy, o.y, inv.y, lo, hi);
    slab(n.mnz, n.mxz, o.z, inv.z, lo, hi);
    return !(hi <= lo);
}

// box_hit with a per-lane tmin (no SGPR operand): for walks whose interval is not
// wave-uniform by construction (the nested BVH walk).
__device__ __forceinline__ bool box_hit_v(const DNode& n, const d3& o, const d3& inv, double tmin, double tmax) {
    double lo = tmin, hi = tmax;
    slab(n.mnx, n.mxx, o.x, inv.x, lo, hi);
    slab(n.mny, n.mxy, o.y, inv.y, lo, hi);
    slab(n.mnz, n.mxz, o.z, inv.z, lo, hi);
    return !(hi <= lo);
}

// Rays whose slab times can never be NaN — every 1/d finite and non-zero, |origin| and
// every box coordinate below 1e300 (so mn - o is finite; finite x finite non-zero is
// never NaN) — take the swap as (min, max): for non-NaN t0 != t1 that is exactly the
// compare-select; for t0 == t1 the two are the same value up to the sign of zero, and
// lo / hi only ever meet comparisons, where ±0 are equal.  3 x (cmp + 4 cndmask) -> 3 x 2.
__device__ __forceinline__ bool fast_slab_ray(const d3& o, const d3& inv) {
    auto ok = [](double v) { return __builtin_fabs(v) <= 1.7976931348623157e308 && v != 0.0; };
    auto small = [](double v) { return __builtin_fabs(v) < 1e300; };
    return ok(inv.x) && ok(inv.y) && ok(inv.z) && small(o.x) && small(o.y) && small(o.z);
}
__device__ __forceinline__ void slab_fast(double mn, double mx, double o, double inv, double& lo, double& hi) {
    const double t0 = (mn - o) * inv, t1 = (mx - o) * inv;
    lo = hw_max(lo, hw_min(t0, t1));
    hi = hw_min(hi, hw_max(t0, t1));
}
__device__ __forceinline__ bool box_hit_fast(const DNode& n, const d3& o, const d3& inv, double tmin, double tmax) {
    double hi = tmax;
    double lo;
    {
        const double t0 = (n.mnx - o.x) * inv.x, t1 = (n.mxx - o.x) * inv.x;
        lo = hw_max_u(tmin, hw_min(t0, t1));
        hi = hw_min(hi, hw_max(t0, t1));
    }
    slab_fast(n.mny, n.mxy, o.y, inv.y, lo, hi);
    slab_fast(n.mnz, n.mxz, o.z, inv.z, lo, hi);
    return !(hi <= lo);
}

// ------------------------------------------------------------------------------
// Certified f32 slab test.
//
// AABB::hit's decision (AABB.rs:58-113) is made in f64 by the reference, and the device
// must reproduce every decision (node visits and primitive tests equal the oracle's).
// But nearly every decision is far from its tie: the f32 form below decides it with a
// proven error bound and reports "undecided" otherwise, and only undecided lanes run the
// f64 test.  The f32 form takes fewer instructions — one FMA per slab plane (two per
// packed FMA) against a subtract and a multiply, 32-bit min/max against 64-bit ones — while
// MI355X issues f64 and f32 add/mul/FMA at about the same cost per wave-instruction
// (tools/ubench/valu_rate.hip: 4.9 / 5.7 cycles per SIMD at 4 waves); and its 32-B node
// record doubles what the LDS mirror holds (C4: 4673 -> 5263 Msamples/s).
//
// Per ray (rays with every |1/d| in [1e-25, 1e15] and |o| <= 1e15, scenes with every
// node coordinate |x| <= 1e15: "cert rays"): ix = f32(1/d), ox = f32(-(o * (1/d))) (the
// f64 product, rounded once), R = max over axes |o * (1/d)|.  Per plane: t' = fma(m32,
// ix, ox) with m32 = f32(m).  For the exact t = (m - o) / d and u = 2^-24:
//   |t' - t| <= u|t| (fma) + (2u + u^2)|m (1/d)| + u R  <=  3.01u (|t| + R)
// since |m (1/d)| <= |t| + R.  (Round 6: 1/d is the hardware reciprocal refined by two Newton
// steps, rcp_cert below, within 2^-50 |1/d| of the exact value for a normal d: that
// adds at most 2^-49 |m (1/d)| + 2^-50 R, under 2^-30 (|t| + R), to the terms above, and the
// 3.01u bound, like K below, has room for 0.01u = 2^-30.6.)  The f64 value the reference computes is within 2^-52 |t|
// of t.  lo = max(tmin, per-axis minima), hi = min(closest, per-axis maxima): x - k(|x|
// + R) and x + k(|x| + R) are increasing in x for k < 1, so a max / min of values each
// within k(|v'| + R) of its target is within k(|result'| + R) of the target's max / min;
// tmin' = f32(tmin) and closest' = f32(closest) are within u of theirs.  Hence with
//   thr = K (|hi'| + |lo'|) + 2 K R + 1e-30,   K = 2^-21 (= 8u: 2.6x the bound above,
//         covering the rounding of d and thr themselves),
// d = hi' - lo' > thr certifies the f64 hit (hi > lo) and d < -thr its miss (hi <= lo);
// the 1e-30 covers f32 underflow.  All values stay finite (|t'| < 2e30), so no NaN.
//
// The kernel drops both absolute values (round 3: two VOP3 source modifiers fewer per node
// step), thr' = K (hi' + lo') + 2 K R + 1e-30:  lo' >= tmin' = f32(0.001) > 0, so |lo'| =
// lo'; and hi' replaces |hi'|.  For hi' >= 0 nothing changes.  For hi' < 0, (a) d > thr'
// would need hi' (1 - K) > lo' (1 + K) + ... > 0, so no hit is certified, as with thr; (b)
// a miss is certified when d < -thr', i.e. lo' (1 - K) + |hi'| (1 + K) > 2 K R + 1e-30, so
// lo' + |hi'| > 16 u R / (1 + 8u), and the exact miss needs only lo' - hi' = lo' + |hi'| >
// 3.01u (|hi'| + lo' + 2R): (1 - 3.01u)(lo' + |hi'|) > 15.8 u R > 6.02 u R.  Undecided is
// then -thr' <= d <= thr'.
#define GS_CERT_K 4.76837158203125e-07f  // 2^-21

struct alignas(16) TNode {  // 32 B record of the threaded tree: f32 box (paired for box_cert) + hit / miss links
    float mnx, mny, mxx, mxy, mnz, mxz;
    uint32_t hit, miss;
};
struct alignas(16) TLeaf {  // 48 B leaf record: a stationary sphere inline, next link, ABI ref
    // rr = radius * radius, Sphere::hit's `self.radius * self.radius` (sphere.rs:70) taken
    // once on the host: the same IEEE product the test would take per ray (round 5)
    double cx, cy, cz, rr;
    uint32_t next, ref, pad0, pad1;
};
struct alignas(16) TBox {  // 48 B: the node's f64 box (AABB.rs), for undecided and non-cert rays
    double mnx, mny, mnz, mxx, mxy, mxz;
};
// 128 B traversal copy of a quad (the ABI gs_quad, material aside), ordered by use: the
// plane (normal, D: 32 B) decides most tests; Q, u, v, w (96 B) are read only for a plane
// hit inside the interval.
struct alignas(16) TQuad {
    double nx, ny, nz, d;
    double qx, qy, qz, ux, uy, uz, vx, vy, vz, wx, wy, wz;
};

typedef float gs_f2 __attribute__((ext_vector_type(2)));
// Per-ray constants of the certified test, paired so that one packed FMA (v_pk_fma_f32:
// the issue cost of one v_fma_f32, measured on MI355X) computes two planes: (min x, min
// y), (max x, max y) with the (x, y) pairs, (min z, max z) with the z pairs.
struct RayCert {
    gs_f2 ixy, oxy;  // f32(1/d), f32(-(o * (1/d))) of x and y
    gs_f2 izz, ozz;  // those of z, twice
    float r2;        // 2 K R + 1e-30
};

// 1/d for the certified test's constants only (make_cert, cert_ray_ok; round 6): the hardware
// reciprocal and two Newton steps, within ~2^-52 of 1/d for a normal, finite d -- the
// certificate's bound needs 2^-31 (above) -- in 5 instructions instead of a correctly
// rounded division's 11.  A zero, infinite or denormal component gives a NaN or infinity,
// which cert_ray_ok rejects (the ray then takes the f64 test, whose 1/d is render.hip's inv_of, an exact division).
__device__ __forceinline__ double rcp_cert(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(r, e, r);
}
__host__ __device__ __forceinline__ bool cert_ray_ok(const d3& o, const d3& inv) {
    auto ok_inv = [](double v) { return __builtin_fabs(v) <= 1e15 && __builtin_fabs(v) >= 1e-25; };
    auto ok_o = [](double v) { return __builtin_fabs(v) <= 1e15; };
    return ok_inv(inv.x) && ok_inv(inv.y) && ok_inv(inv.z) && ok_o(o.x) && ok_o(o.y) && ok_o(o.z);
}
__device__ __forceinline__ RayCert make_cert(const d3& o, const d3& inv) {
    RayCert c;
    const double px = o.x * inv.x, py = o.y * inv.y, pz = o.z * inv.z;
    const double R = __builtin_fmax(__builtin_fabs(px), __builtin_fmax(__builtin_fabs(py), __builtin_fabs(pz)));
    c.ixy = gs_f2{(float)inv.x, (float)inv.y};
    c.oxy = gs_f2{(float)(-px), (float)(-py)};
    c.izz = gs_f2{(float)inv.z, (float)inv.z};
    c.ozz = gs_f2{(float)(-pz), (float)(-pz)};
    c.r2 = (float)(2.0 * (double)GS_CERT_K * R * (1.0 + 0x1p-20)) + 1e-30f;
    return c;
}
// The certified test's difference and threshold: returns d > thr (a certified hit);
// d < -thr is a certified miss, anything between undecided (run the f64 test).
__device__ __forceinline__ bool box_cert_dt(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                            const RayCert& c, float tmin32, float closest32, float& d, float& thr) {
    // t = fma(coordinate, 1/d, -o/d) for both planes of an axis at once
    const gs_f2 t0 = __builtin_elementwise_fma(gs_f2{mnx, mny}, c.ixy, c.oxy);
    const gs_f2 t1 = __builtin_elementwise_fma(gs_f2{mxx, mxy}, c.ixy, c.oxy);
    const gs_f2 tz = __builtin_elementwise_fma(gs_f2{mnz, mxz}, c.izz, c.ozz);
    const float t0x = t0.x, t1x = t1.x, t0y = t0.y, t1y = t1.y, t0z = tz.x, t1z = tz.y;
    const float lo = __builtin_fmaxf(__builtin_fmaxf(tmin32, __builtin_fminf(t0x, t1x)),
                                     __builtin_fmaxf(__builtin_fminf(t0y, t1y), __builtin_fminf(t0z, t1z)));
    const float hi = __builtin_fminf(__builtin_fminf(closest32, __builtin_fmaxf(t0x, t1x)),
                                     __builtin_fminf(__builtin_fmaxf(t0y, t1y), __builtin_fmaxf(t0z, t1z)));
    d = hi - lo;
    thr = __builtin_fmaf(GS_CERT_K, hi + lo, c.r2);  // lo >= tmin32 > 0; hi for |hi| (above)
    return d > thr;
}
// Returns the certified decision (hit); `undecided` when f32 cannot decide (run the f64 test).
__device__ __forceinline__ bool box_cert(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                         const RayCert& c, float tmin32, float closest32, bool& undecided) {
    float d, thr;
    const bool h = box_cert_dt(mnx, mny, mnz, mxx, mxy, mxz, c, tmin32, closest32, d, thr);
    undecided = !h && d >= -thr;
    return h;
}
__device__ __forceinline__ DNode box64(const TBox& b) {
    DNode n;
    n.mnx = b.mnx;
    n.mny = b.mny;
    n.mnz = b.mnz;
    n.mxx = b.mxx;
    n.mxy = b.mxy;
    n.mxz = b.mxz;
    n.left = n.right = n.pad0 = n.pad1 = 0;
    return n;
}

// Sphere::hit acceptance (sphere.rs:64-88): whether a root lies in the open interval,
// and that root (t_out is written on every path, so callers carry no undefined value).
// (rr: the radius squared, r * r; leaf records carry it, TLeaf)
__device__ __forceinline__ bool sphere_accept_rr(d3 c, double rr, const Ray& ray, double a, double tmin, double tmax,
                                            double& t_out) {
    d3 oc = sub(c, ray.o);
    double h = dot(ray.d, oc);
    double cc = len2(oc) - rr;
    double disc = h * h - a * cc;
    t_out = tmax;
    if (disc < 0.0) return false;
    double sq = sqrt(disc);
    double t = (h - sq) / a;
    if (!(tmin < t && t < tmax)) {
        t = (h + sq) / a;
        if (!(tmin < t && t < tmax)) return false;
    }
    t_out = t;
    return true;
}
__device__ __forceinline__ bool sphere_accept(d3 c, double r, const Ray& ray, double a, double tmin, double tmax,
                                         double& t_out) {
    return sphere_accept_rr(c, r * r, ray, a, tmin, tmax, t_out);
}

// sphere_accept split at the discriminant: its first half (h, disc: no root, no
// interval), and its second half for a real disc -- the same operations in the same order.
// Lets a leaf pass run the square root and the divisions once for whichever of a lane's
// spheres needs them (GS_FEAT_SPHLEAF leaf runs, render.hip).
struct SphereDisc {
    double h, disc;
};
__device__ __forceinline__ SphereDisc sphere_disc_rr(d3 c, double rr, const Ray& ray, double a) {
    d3 oc = sub(c, ray.o);
    SphereDisc s;
    s.h = dot(ray.d, oc);
    double cc = len2(oc) - rr;
    s.disc = s.h * s.h - a * cc;
    return s;
}
__device__ __forceinline__ bool sphere_root_take(double h, double disc, double a, double tmin, double tmax, double& t_out) {
    double sq = sqrt(disc);
    double t = (h - sq) / a;
    if (!(tmin < t && t < tmax)) {
        t = (h + sq) / a;
        if (!(tmin < t && t < tmax)) return false;
    }
    t_out = t;
    return true;
}

// The same roots with the divisions by a taken from a refined reciprocal ra = rcp_cert(a)
// (round 6): q = num ra, r = fma(-a, q, num), fma(r, ra, q) is the f64 division's own sequence
// (v_div_scale, v_rcp, two Newton steps, v_div_fmas, v_div_fixup) with its scalings the
// identity -- which they are for a in [2^-900, 2^900] and every numerator |num| >= 2^-968 (the
// caller's condition on a; a smaller numerator gives |t| < 2^-68 < tmin, rejected either way,
// and an overflowing one a NaN or infinity, rejected either way).  So every root inside
// (tmin, tmax) is the correctly rounded quotient, bit for bit (test_gpu_device_kat.py).
__device__ __forceinline__ double div_by(double num, double den, double rden) {
    const double q = num * rden;
    const double r = __builtin_fma(-den, q, num);
    return __builtin_fma(r, rden, q);
}
__device__ __forceinline__ bool sphere_root_take_ra(double h, double disc, double a, double ra, double tmin, double tmax,
                                                    double& t_out) {
    double sq = sqrt(disc);
    double t = div_by(h - sq, a, ra);
    if (!(tmin < t && t < tmax)) {
        t = div_by(h + sq, a, ra);
        if (!(tmin < t && t < tmax)) return false;
    }
    t_out = t;
    return true;
}

// sphere_accept_rr with the roots' divisions through ra = rcp_cert(a) (the caller has checked a
// is in [2^-900, 2^900] for every active lane: sphere_root_take_ra's condition)
__device__ __forceinline__ bool sphere_accept_rr_ra(d3 c, double rr, const Ray& ray, double a, double ra, double tmin,
                                                    double tmax, double& t_out) {
    d3 oc = sub(c, ray.o);
    double h = dot(ray.d, oc);
    double cc = len2(oc) - rr;
    double disc = h * h - a * cc;
    t_out = tmax;
    if (disc < 0.0) return false;
    return sphere_root_take_ra(h, disc, a, ra, tmin, tmax, t_out);
}

// HDRI::sample's texel column and row (camera.rs:257-270) for the rotated, normalised
// direction `rot`: u = 0.5 + atan2(y, x) / 2pi, v = 0.5 - asin(z) / pi, then
// `(u * W) as usize % W`, `(v * H) as usize % H`.  sky_index_f64 is that, in f64.
__device__ __forceinline__ void sky_index_f64(d3 rot, uint32_t W, uint32_t H, uint32_t& x, uint32_t& y) {
    const double PI = 3.14159265358979323846;
    double theta = atan2(rot.y, rot.x);
    double phi = asin(rot.z);
    double u = 0.5 + theta / (2.0 * PI);
    double v = 0.5 - phi / PI;
    x = (uint32_t)(sat_u64(u * (double)W, 18446744073709551616.0, ~0ull) % (uint64_t)W);
    y = (uint32_t)(sat_u64(v * (double)H, 18446744073709551616.0, ~0ull) % (uint64_t)H);
}
// The same indices from f32 angles, certified: U = u*W and V = v*H are evaluated in f32
// (OCML atan2f; the elevation as atan2f(z, |(x, y)|), which equals asin(z) for a unit
// vector and is well conditioned at every elevation), and accepted only when both lie
// farther from a texel boundary (an integer, 0 and W included) than their error bound:
// |U32 - U| <= W (4 ulp(pi) atan2f + 2^-23 input rounding) / 2pi + the two f32 roundings
// ~= 2.4e-7 W, |V32 - V| ~= 2.6e-7 H; the margins are 1e-6 W and 2e-6 H (>= 4x), and
// |(x, y)| >= 1e-4 keeps the f64 asin's own sensitivity at the poles (tan(phi) 2^-53)
// negligible.  Returns false when undecided (about 0.4% of directions): the caller then
// runs sky_index_f64.  Decided indices equal sky_index_f64's
// (tests/test_gpu_device_kat.py: 4M random and near-boundary directions).
__device__ __forceinline__ bool sky_index_f32(d3 rot, uint32_t W, uint32_t H, uint32_t& x, uint32_t& y) {
    const float fx = (float)rot.x, fy = (float)rot.y, fz = (float)rot.z;
    const float r = __builtin_sqrtf(__builtin_fmaf(fx, fx, fy * fy));
    const float th = atan2f(fy, fx), ph = atan2f(fz, r);
    const float fW = (float)W, fH = (float)H;
    const float U = __builtin_fmaf(th, fW * 0.159154943f, fW * 0.5f);
    const float V = __builtin_fmaf(ph, fH * -0.318309886f, fH * 0.5f);
    const float iu = __builtin_floorf(U), iv = __builtin_floorf(V);
    const float du = U - iu, dv = V - iv;
    const float mu = fW * 1e-6f, mv = fH * 2e-6f;
    x = (uint32_t)(int32_t)iu;
    y = (uint32_t)(int32_t)iv;
    return r >= 1e-4f && du > mu && du < 1.0f - mu && dv > mv && dv < 1.0f - mv && iu >= 0.0f && iu < fW &&
           iv >= 0.0f && iv < fH;
}

// Quad::hit acceptance (quad.rs:84-95, plane.rs:20-32), given the plane (normal, D);
// `tail(Q, u, v, w)` fetches the rest only once the plane hit lies in [tmin, tmax].
template <class Tail>
__device__ __forceinline__ bool quad_accept_plane(d3 nrm, double qd, Tail tail, const Ray& ray, double tmin,
                                                  double tmax, double& t_out) {
    double den = dot(nrm, ray.d);
    if (fabs(den) < 1e-8) return false;
    double t = (qd - dot(nrm, ray.o)) / den;
    if (!(tmin <= t && t <= tmax)) return false;
    d3 Q, U, V, W;
    tail(Q, U, V, W);
    d3 inter = add(ray.o, muls(ray.d, t));
    d3 planar = sub(inter, Q);
    double alpha = dot(W, cross(planar, V));
    double beta = dot(W, cross(U, planar));
    if (!(0.0 <= alpha && alpha <= 1.0) || !(0.0 <= beta && beta <= 1.0)) return false;
    t_out = t;
    return true;
}
__device__ __forceinline__ bool quad_accept(const gs_quad& q, const Ray& ray, double tmin, double tmax, double& t_out) {
    return quad_accept_plane(
        ld3(q.normal), q.d,
        [&](d3& Q, d3& U, d3& V, d3& W) {
            Q = ld3(q.q);
            U = ld3(q.u);
            V = ld3(q.v);
            W = ld3(q.w);
        },
        ray, tmin, tmax, t_out);
}

// Triangle::hit (triangle.rs:34-68): one-sided, ray_t ignored (reference quirk).
__device__ __forceinline__ bool tri_hit(const gs_triangle& tr, const Ray& ray, double& t_out, double& u_out,
                                        double& v_out) {
    d3 a = ld3(tr.a);
    d3 e1 = sub(ld3(tr.c), a), e2 = sub(ld3(tr.b), a);
    d3 p_vec = cross(ray.d, e2);
    double det = dot(e1, p_vec);
    if (det < 1e-8) return false;
    d3 t_vec = sub(ray.o, a);
    double u = dot(t_vec, p_vec);
    if (u < 0.0 || u > det) return false;
    d3 q_vec = cross(t_vec, e1);
    double v = dot(ray.d, q_vec);
    if (v < 0.0 || u + v > det) return false;
    double t = dot(e2, q_vec);
    double inv_det = 1.0 / det;
    t_out = t * inv_det;
    u_out = u * inv_det;
    v_out = v * inv_det;
    return true;
}

// Translate/RotateY forward ray transforms (hittable.rs:107-113, :179-193).
__device__ __forceinline__ void inst_forward(const gs_instance& in, Ray& r) {
    if (in.kind == GS_INST_TRANSLATE) {
        r.o = sub(r.o, ld3(in.p));
    } else {
        double s = in.p[0], c = in.p[1];
        r.o = mk((c * r.o.x) - (s * r.o.z), r.o.y, (s * r.o.x) + (c * r.o.z));
        r.d = mk((c * r.d.x) - (s * r.d.z), r.d.y, (s * r.d.x) + (c * r.d.z));
    }
}
// Hit-record back transforms (hittable.rs:115-117, :195-207).
__device__ __forceinline__ void inst_backward(const gs_instance& in, d3& p, d3& n) {
    if (in.kind == GS_INST_TRANSLATE) {
        p = add(p, ld3(in.p));
    } else {
        double s = in.p[0], c = in.p[1];
        p = mk((c * p.x) + (s * p.z), p.y, (-s * p.x) + (c * p.z));
        n = mk((c * n.x) + (s * n.z), n.y, (-s * n.x) + (c * n.z));
    }
}

}  // namespace gsd
