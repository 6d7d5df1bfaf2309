// kat_device.hip — TEST INFRASTRUCTURE: runs the megakernel's own device functions
// (grayshift_amd/csrc/device/geometry.hpp, devmath.hpp) over arrays of test cases so
// tests/test_gpu_device_kat.py can compare them bit-for-bit with the CPU oracle on
// adversarial inputs (zero / negative-zero direction components, origins on slab
// planes, tangent rays, closed/open interval ends).  Not part of the product.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../grayshift_amd/csrc/device/devmath.hpp"
#include "../../grayshift_amd/csrc/device/geometry.hpp"
#include "../../grayshift_amd/csrc/device/perlin.hpp"

using namespace gsd;

__global__ void k_aabb(int n, const double* box, const double* ray, const double* iv, int* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    DNode nd{box[6 * i], box[6 * i + 1], box[6 * i + 2], box[6 * i + 3], box[6 * i + 4], box[6 * i + 5], 0, 0, 0, 0};
    d3 o = mk(ray[6 * i], ray[6 * i + 1], ray[6 * i + 2]);
    d3 d = mk(ray[6 * i + 3], ray[6 * i + 4], ray[6 * i + 5]);
    d3 inv = mk(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
    out[i] = box_hit(nd, o, inv, iv[2 * i], iv[2 * i + 1]) ? 1 : 0;
}

// The megakernel's node decision for cert rays: box_cert (f32, certified), and the f64
// box_hit_fast where box_cert is undecided.  out: 0/1 the decision, dec: 0 miss / 1 hit
// certified by f32, 2 undecided; -1 for rays that are not cert rays (not decided here).
__global__ void k_aabb_cert(int n, const double* box, const double* ray, const double* iv, int* out, int* dec) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* b = box + 6 * i;
    DNode nd{b[0], b[1], b[2], b[3], b[4], b[5], 0, 0, 0, 0};
    d3 o = mk(ray[6 * i], ray[6 * i + 1], ray[6 * i + 2]);
    d3 d = mk(ray[6 * i + 3], ray[6 * i + 4], ray[6 * i + 5]);
    d3 inv = mk(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
    bool boxes_ok = true;
    for (int k = 0; k < 6; k++) boxes_ok = boxes_ok && __builtin_fabs(b[k]) <= 1e15;
    // (the product's constants: the refined hardware reciprocal, rcp_cert; the f64 test below
    // keeps the exact 1/d, as the megakernel's inv_of)
    const d3 invc = mk(rcp_cert(d.x), rcp_cert(d.y), rcp_cert(d.z));
    if (!boxes_ok || !cert_ray_ok(o, invc)) {
        out[i] = -1;
        dec[i] = -1;
        return;
    }
    const RayCert rc = make_cert(o, invc);
    bool und;
    bool h = box_cert((float)b[0], (float)b[1], (float)b[2], (float)b[3], (float)b[4], (float)b[5], rc,
                      (float)iv[2 * i], (float)iv[2 * i + 1], und);
    dec[i] = und ? 2 : (h ? 1 : 0);
    if (und) h = box_hit_fast(nd, o, inv, iv[2 * i], iv[2 * i + 1]);
    out[i] = h ? 1 : 0;
}

// rcp_cert (the certified test's 1/d) next to the exact division, per case.
__global__ void k_rcp_cert(int n, const double* d, double* approx, double* exact) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    approx[i] = rcp_cert(d[i]);
    exact[i] = 1.0 / d[i];
}

// div_by (the sphere roots' division through a refined reciprocal) next to the exact quotient.
__global__ void k_div_by(int n, const double* num, const double* den, double* fast, double* exact) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fast[i] = div_by(num[i], den[i], rcp_cert(den[i]));
    exact[i] = num[i] / den[i];
}

__global__ void k_sphere(int n, const double* sph, const double* ray, const double* iv, double* t, int* hit) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r;
    r.o = mk(ray[6 * i], ray[6 * i + 1], ray[6 * i + 2]);
    r.d = mk(ray[6 * i + 3], ray[6 * i + 4], ray[6 * i + 5]);
    r.time = 0.0;
    double tt = 0.0;
    bool h = sphere_accept(mk(sph[4 * i], sph[4 * i + 1], sph[4 * i + 2]), sph[4 * i + 3], r, len2(r.d), iv[2 * i],
                           iv[2 * i + 1], tt);
    hit[i] = h ? 1 : 0;
    t[i] = tt;
}

__global__ void k_tri(int n, const double* tri, const double* ray, double* tuv, int* hit) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    gs_triangle g;
    for (int k = 0; k < 3; k++) {
        g.a[k] = tri[9 * i + k];
        g.b[k] = tri[9 * i + 3 + k];
        g.c[k] = tri[9 * i + 6 + k];
    }
    Ray r;
    r.o = mk(ray[6 * i], ray[6 * i + 1], ray[6 * i + 2]);
    r.d = mk(ray[6 * i + 3], ray[6 * i + 4], ray[6 * i + 5]);
    r.time = 0.0;
    double t = 0, u = 0, v = 0;
    hit[i] = tri_hit(g, r, t, u, v) ? 1 : 0;
    tuv[3 * i] = t;
    tuv[3 * i + 1] = u;
    tuv[3 * i + 2] = v;
}

__global__ void k_rng(int n, const uint64_t* seed, const uint32_t* pix, const uint32_t* smp, int draws, double* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t st = stream_seed(seed[i], pix[i], smp[i]);
    for (int k = 0; k < draws; k++) out[(size_t)i * draws + k] = wy_f64(st);
}

// which: 0 sin, 1 cos, 2 acos, 3 asin, 4 atan2(x, y)
__global__ void k_math(int n, int which, const double* x, const double* y, double* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double r;
    if (which == 0) {
        double s, c;
        sincos(x[i], &s, &c);
        r = s;
    } else if (which == 1) {
        double s, c;
        sincos(x[i], &s, &c);
        r = c;
    } else if (which == 2) {
        r = acos(x[i]);
    } else if (which == 3) {
        r = asin(x[i]);
    } else {
        r = atan2(x[i], y[i]);
    }
    out[i] = r;
}

// The sky texel index: f32 certified (-1, -1 when undecided) and the f64 reference path.
__global__ void k_sky(int n, uint32_t W, uint32_t H, const double* dir, int* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const d3 r = mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
    uint32_t x = 0, y = 0, x64 = 0, y64 = 0;
    const bool ok = sky_index_f32(r, W, H, x, y);
    sky_index_f64(r, W, H, x64, y64);
    out[4 * i] = ok ? (int)x : -1;
    out[4 * i + 1] = ok ? (int)y : -1;
    out[4 * i + 2] = (int)x64;
    out[4 * i + 3] = (int)y64;
}

template <class T>
static T* dcopy(const T* h, size_t n) {
    T* d = nullptr;
    if (hipMalloc(&d, n * sizeof(T) + 8) != hipSuccess) return nullptr;
    if (h) (void)hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice);
    return d;
}
template <class T>
static void back(T* h, T* d, size_t n) {
    (void)hipMemcpy(h, d, n * sizeof(T), hipMemcpyDeviceToHost);
    (void)hipFree(d);
}
static dim3 grid(int n) { return dim3((unsigned)((n + 255) / 256)); }

// perlin3 (which 0) or NoiseTexture's channel value at scale s (which 1) per point.
__global__ void k_noise(int n, int which, const uint8_t* perm, double scale, const double* p, double* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* q = p + 3 * i;
    out[i] = which == 0 ? perlin3(perm, q[0], q[1], q[2]) : noise_value(perm, scale, q[0], q[1], q[2]);
}

extern "C" {

int kat_aabb(int n, const double* box, const double* ray, const double* iv, int* out) {
    double *db = dcopy(box, 6 * (size_t)n), *dr = dcopy(ray, 6 * (size_t)n), *di = dcopy(iv, 2 * (size_t)n);
    int* dout = dcopy<int>(nullptr, n);
    hipLaunchKernelGGL(k_aabb, grid(n), dim3(256), 0, 0, n, db, dr, di, dout);
    back(out, dout, n);
    (void)hipFree(db); (void)hipFree(dr); (void)hipFree(di);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int kat_aabb_cert(int n, const double* box, const double* ray, const double* iv, int* out, int* dec) {
    double *db = dcopy(box, 6 * (size_t)n), *dr = dcopy(ray, 6 * (size_t)n), *di = dcopy(iv, 2 * (size_t)n);
    int* dout = dcopy<int>(nullptr, n);
    int* ddec = dcopy<int>(nullptr, n);
    hipLaunchKernelGGL(k_aabb_cert, grid(n), dim3(256), 0, 0, n, db, dr, di, dout, ddec);
    back(out, dout, n);
    back(dec, ddec, n);
    (void)hipFree(db); (void)hipFree(dr); (void)hipFree(di);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int kat_rcp_cert(int n, const double* d, double* approx, double* exact) {
    double* dd = dcopy(d, n);
    double *da = dcopy<double>(nullptr, n), *de = dcopy<double>(nullptr, n);
    hipLaunchKernelGGL(k_rcp_cert, grid(n), dim3(256), 0, 0, n, dd, da, de);
    back(approx, da, n);
    back(exact, de, n);
    (void)hipFree(dd);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int kat_div_by(int n, const double* num, const double* den, double* fast, double* exact) {
    double *dn = dcopy(num, n), *dd = dcopy(den, n);
    double *df = dcopy<double>(nullptr, n), *de = dcopy<double>(nullptr, n);
    hipLaunchKernelGGL(k_div_by, grid(n), dim3(256), 0, 0, n, dn, dd, df, de);
    back(fast, df, n);
    back(exact, de, n);
    (void)hipFree(dn); (void)hipFree(dd);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int kat_sphere(int n, const double* sph, const double* ray, const double* iv, double* t, int* hit) {
    double *ds = dcopy(sph, 4 * (size_t)n), *dr = dcopy(ray, 6 * (size_t)n), *di = dcopy(iv, 2 * (size_t)n);
    double* dt = dcopy<double>(nullptr, n);
    int* dh = dcopy<int>(nullptr, n);
    hipLaunchKernelGGL(k_sphere, grid(n), dim3(256), 0, 0, n, ds, dr, di, dt, dh);
    back(t, dt, n);
    back(hit, dh, n);
    (void)hipFree(ds); (void)hipFree(dr); (void)hipFree(di);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int kat_tri(int n, const double* tri, const double* ray, double* tuv, int* hit) {
    double *dt = dcopy(tri, 9 * (size_t)n), *dr = dcopy(ray, 6 * (size_t)n);
    double* dtuv = dcopy<double>(nullptr, 3 * (size_t)n);
    int* dh = dcopy<int>(nullptr, n);
    hipLaunchKernelGGL(k_tri, grid(n), dim3(256), 0, 0, n, dt, dr, dtuv, dh);
    back(tuv, dtuv, 3 * (size_t)n);
    back(hit, dh, n);
    (void)hipFree(dt); (void)hipFree(dr);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int kat_rng(int n, const uint64_t* seed, const uint32_t* pix, const uint32_t* smp, int draws, double* out) {
    uint64_t* ds = dcopy(seed, n);
    uint32_t *dp = dcopy(pix, n), *dm = dcopy(smp, n);
    double* dout = dcopy<double>(nullptr, (size_t)n * draws);
    hipLaunchKernelGGL(k_rng, grid(n), dim3(256), 0, 0, n, ds, dp, dm, draws, dout);
    back(out, dout, (size_t)n * draws);
    (void)hipFree(ds); (void)hipFree(dp); (void)hipFree(dm);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int kat_math(int n, int which, const double* x, const double* y, double* out) {
    double *dx = dcopy(x, n), *dy = dcopy(y ? y : x, n);
    double* dout = dcopy<double>(nullptr, n);
    hipLaunchKernelGGL(k_math, grid(n), dim3(256), 0, 0, n, which, dx, dy, dout);
    back(out, dout, n);
    (void)hipFree(dx); (void)hipFree(dy);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int kat_sky(int n, uint32_t W, uint32_t H, const double* dir, int* out) {
    double* dd = dcopy(dir, 3 * (size_t)n);
    int* dout = dcopy<int>(nullptr, 4 * (size_t)n);
    hipLaunchKernelGGL(k_sky, grid(n), dim3(256), 0, 0, n, W, H, dd, dout);
    back(out, dout, 4 * (size_t)n);
    (void)hipFree(dd);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int kat_noise(int n, int which, const uint8_t* perm256, double scale, const double* p, double* out) {
    uint8_t* dperm = dcopy(perm256, 256);
    double* dp = dcopy(p, 3 * (size_t)n);
    double* dout = dcopy<double>(nullptr, n);
    hipLaunchKernelGGL(k_noise, grid(n), dim3(256), 0, 0, n, which, dperm, scale, dp, dout);
    back(out, dout, n);
    (void)hipFree(dperm); (void)hipFree(dp);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

}  // extern "C"
