// perlin.hpp — NoiseTexture (texture.rs:97-131) on the device: 3-D Perlin noise of the
// `noise` crate 0.9.0 (Perlin::default(), NoiseFn<f64, 3>::get), restated from the crate's
// published algorithm — the crate source is not in this image, so parity with it is
// unpinned; parity with the oracle's independent restatement is exact.
//
//   hash(x, y, z)  = P[P[P[x & 255] ^ (y & 255)] ^ (z & 255)]      (PermutationTable)
//   gradient(h, v) = the 16-entry edge-gradient table (12 cube edges + 4 repeats) · v
//   noise(p)       = trilinear blend of the 8 corner gradients with quintic s-curves,
//                    written as the crate's k0..k7 polynomial, times 2/sqrt(3)
// Expression order follows the crate's so the f64 results match bit for bit.
#pragma once
#include "devmath.hpp"

namespace gsd {

__device__ __forceinline__ double perlin_grad(uint32_t h, double x, double y, double z) {
    switch (h & 15u) {
        case 0: return x + y;
        case 1: return -x + y;
        case 2: return x - y;
        case 3: return -x - y;
        case 4: return x + z;
        case 5: return -x + z;
        case 6: return x - z;
        case 7: return -x - z;
        case 8: return y + z;
        case 9: return -y + z;
        case 10: return y - z;
        case 11: return -y - z;
        case 12: return x + y;
        case 13: return -x + y;
        case 14: return -y + z;
        default: return -y - z;
    }
}

__device__ __forceinline__ double s_curve5(double t) { return t * t * t * (t * (t * 6.0 - 15.0) + 10.0); }

// `floored.numcast::<isize>()`: saturating, NaN -> 0 (the crate would panic on those).
__device__ __forceinline__ int64_t perlin_corner(double f) {
    if (f != f) return 0;
    if (f >= 9.2233720368547758e18) return INT64_MAX;
    if (f <= -9.2233720368547758e18) return INT64_MIN;
    return (int64_t)f;
}

__device__ __forceinline__ double perlin3(const uint8_t* __restrict__ P, double px, double py, double pz) {
    const double SCALE_FACTOR = 1.1547005383792515;  // 2 / sqrt(3)
    const double fx = floor(px), fy = floor(py), fz = floor(pz);
    const int64_t cx = perlin_corner(fx), cy = perlin_corner(fy), cz = perlin_corner(fz);
    const double dx = px - fx, dy = py - fy, dz = pz - fz;
    auto hash = [&](int64_t x, int64_t y, int64_t z) -> uint32_t {
        uint32_t i = P[(uint32_t)(x & 255)];
        i = P[i ^ (uint32_t)(y & 255)];
        return P[i ^ (uint32_t)(z & 255)];
    };
    const double g000 = perlin_grad(hash(cx, cy, cz), dx, dy, dz);
    const double g100 = perlin_grad(hash(cx + 1, cy, cz), dx - 1.0, dy, dz);
    const double g010 = perlin_grad(hash(cx, cy + 1, cz), dx, dy - 1.0, dz);
    const double g110 = perlin_grad(hash(cx + 1, cy + 1, cz), dx - 1.0, dy - 1.0, dz);
    const double g001 = perlin_grad(hash(cx, cy, cz + 1), dx, dy, dz - 1.0);
    const double g101 = perlin_grad(hash(cx + 1, cy, cz + 1), dx - 1.0, dy, dz - 1.0);
    const double g011 = perlin_grad(hash(cx, cy + 1, cz + 1), dx, dy - 1.0, dz - 1.0);
    const double g111 = perlin_grad(hash(cx + 1, cy + 1, cz + 1), dx - 1.0, dy - 1.0, dz - 1.0);
    const double a = s_curve5(dx), b = s_curve5(dy), c = s_curve5(dz);
    const double k0 = g000;
    const double k1 = g100 - g000;
    const double k2 = g010 - g000;
    const double k3 = g001 - g000;
    const double k4 = g000 + g110 - g100 - g010;
    const double k5 = g000 + g101 - g100 - g001;
    const double k6 = g000 + g011 - g010 - g001;
    const double k7 = g100 + g010 + g001 + g111 - g000 - g110 - g101 - g011;
    const double result = k0 + k1 * a + k2 * b + k3 * c + k4 * a * b + k5 * a * c + k6 * b * c + k7 * a * b * c;
    return result * SCALE_FACTOR;
}

// NoiseTexture::turbulence(p, depth) (texture.rs:107-124).
__device__ __forceinline__ double turbulence(const uint8_t* __restrict__ P, double x, double y, double z, int depth) {
    double accum = 0.0, weight = 1.0;
#pragma unroll 1
    for (int i = 0; i < depth; i++) {
        accum += weight * perlin3(P, x, y, z);
        weight /= 2.0;
        x *= 2.0;
        y *= 2.0;
        z *= 2.0;
    }
    return fabs(accum);
}

// NoiseTexture::value_at (texture.rs:127-130): every channel 0.5 * (1 + sin(...)).
__device__ __forceinline__ double noise_value(const uint8_t* __restrict__ P, double scale, double x, double y,
                                              double z) {
    return 0.5 * (1.0 + sin(scale * z + 10.0 * turbulence(P, x, y, z, 7)));
}

}  // namespace gsd
