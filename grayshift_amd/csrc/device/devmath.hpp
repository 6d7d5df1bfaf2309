// devmath.hpp — f64 vector helpers for the gfx950 megakernel.
//
// Every helper evaluates in exactly the order of the reference's util/vec3.rs
// (left-to-right sums, `a * s` componentwise, `unit` = divide by length).  The
// device code is compiled with -ffp-contract=off: Rust never fuses a*b+c, so an
// FMA here would move results by an ulp and flip rare geometric decisions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsd {

struct d3 {
    double x, y, z;
};

__device__ __forceinline__ d3 mk(double x, double y, double z) { return d3{x, y, z}; }
__device__ __forceinline__ d3 add(d3 a, d3 b) { return d3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ d3 sub(d3 a, d3 b) { return d3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ d3 neg(d3 a) { return d3{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ d3 muls(d3 a, double s) { return d3{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ d3 mulv(d3 a, d3 b) { return d3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ d3 divs(d3 a, double s) { return d3{a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double len2(d3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ d3 cross(d3 a, d3 b) {
    return d3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ d3 unit(d3 a) { return divs(a, sqrt(len2(a))); }
// vec3.rs:53-55: self - 2.0 * self.dot(n) * n
__device__ __forceinline__ d3 reflect(d3 v, d3 n) { return sub(v, muls(n, 2.0 * dot(v, n))); }
// vec3.rs:57-62
__device__ __forceinline__ d3 refract(d3 v, d3 n, double ratio) {
    double cos_theta = fmin(dot(n, neg(v)), 1.0);
    d3 perp = muls(add(v, muls(n, cos_theta)), ratio);
    d3 par = muls(n, -sqrt(fabs(1.0 - len2(perp))));
    return add(perp, par);
}
__device__ __forceinline__ d3 ld3(const double* p) { return d3{p[0], p[1], p[2]}; }

// fastrand 2.1.1 wyrand (the crate's Rng::gen_u64 / Rng::f64), see oracle.cpp for the
// restatement it is checked against.
__device__ __forceinline__ uint64_t wy_next(uint64_t& state) {
    const uint64_t C0 = 0x2d358dccaa6c78a5ULL, C1 = 0x8bb84b93962eacc9ULL;
    uint64_t s = state + C0;
    state = s;
    uint64_t b = s ^ C1;
    // The 128-bit product s * b from four 32x32->64 partial products, each a
    // v_mad_u64_u32 with its carry-in folded into the addend: the low half reuses the
    // partial products the high half needs (`s * b` and __umul64hi compiled separately
    // recomputed two of them: 22 -> 19 VALU per draw on gfx950).
    const uint32_t s0 = (uint32_t)s, s1 = (uint32_t)(s >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p00 = (uint64_t)s0 * b0;
    const uint64_t t = (uint64_t)s0 * b1 + (p00 >> 32);
    const uint64_t u = (uint64_t)s1 * b0 + (uint32_t)t;
    const uint64_t hi = (uint64_t)s1 * b1 + ((t >> 32) + (u >> 32));
    const uint64_t lo = (u << 32) | (uint32_t)p00;
    return lo ^ hi;
}
__device__ __forceinline__ double wy_f64(uint64_t& state) {
    uint64_t bits = 0x3FF0000000000000ULL | (wy_next(state) >> 12);
    return __longlong_as_double((long long)bits) - 1.0;
}
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
// Per-(pixel, sample) stream.
__device__ __forceinline__ uint64_t stream_seed(uint64_t seed, uint32_t pixel, uint32_t sample) {
    return splitmix64(seed ^ splitmix64(((uint64_t)sample << 32) | (uint64_t)pixel));
}

// Unsigned 32-bit division by a divisor fixed for a launch (image width, tiles per row,
// chunks per pixel, ...): the round-up multiply-shift method (Granlund & Montgomery
// 1994; Hacker's Delight 10-8), exact for every n < 2^32 and every d >= 1 -- 5 VALU
// instead of the ~18 of a division by a runtime value.  The host fills the magic.
struct UDiv {
    uint32_t d, m, s1, s2;
};
__host__ __device__ inline UDiv udiv_make(uint32_t d) {
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) l++;  // ceil(log2 d)
    UDiv u;
    u.d = d;
    u.m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
    u.s1 = l < 1 ? l : 1;
    u.s2 = l < 1 ? 0 : l - 1;
    return u;
}
__device__ __forceinline__ uint32_t udiv(uint32_t n, const UDiv& u) {
    const uint32_t t = __umulhi(n, u.m);
    return (t + ((n - t) >> u.s1)) >> u.s2;
}

// Rust `f64 as i32` (saturating, NaN -> 0).
__device__ __forceinline__ int32_t sat_i32(double f) {
    if (f != f) return 0;
    if (f >= 2147483647.0) return 2147483647;
    if (f <= -2147483648.0) return (int32_t)0x80000000u;
    return (int32_t)f;
}
// Rust `f64 as u32`/`as usize` clamped to [0, maxv] (NaN, negatives -> 0).
__device__ __forceinline__ uint64_t sat_u64(double f, double maxv_as_double, uint64_t maxv) {
    if (!(f > 0.0)) return 0;
    if (f >= maxv_as_double) return maxv;
    return (uint64_t)f;
}

// write_color's byte (color.rs:8-28): linear_to_gamma (sqrt of a positive value, else 0;
// NaN -> 0), INTENSITY.clamp to [0, 0.999], then `(256.0 * c) as i32`.
__device__ __forceinline__ uint8_t color_byte(double c) {
    double g = c > 0.0 ? sqrt(c) : 0.0;
    if (g < 0.000) g = 0.000;
    if (g > 0.999) g = 0.999;
    return (uint8_t)sat_i32(256.0 * g);
}

}  // namespace gsd
