/*
 * oracle.cpp — CPU restatement of the grayshift reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker or the CPU
 * baseline.  The product (grayshift_amd/) never links, loads or calls it.
 *
 * PARITY UNPINNED: the reference (Rust, /root/reference) has no tests, no golden
 * vectors and no fixtures, and cannot be built here (no rustc/cargo, no crate
 * registry).  This file is therefore pinned only by hand-derived known-answer
 * tests (tests/test_oracle_kat.py) and by its line-by-line correspondence with the
 * reference sources cited below.  Third-party arithmetic the reference delegates
 * to crates absent from the container is restated from their published
 * algorithms: fastrand 2.1.1 (wyrand + f64 mapping), radiant 0.3.0 (RGBE -> f32,
 * done by the asset loader, not here), image 0.25.2 (JPEG decode, replaced by a
 * committed decoded fixture).
 *
 * The one intended semantic change from the reference: fastrand's unseeded
 * thread-local generator is replaced by a per-(pixel, sample) wyrand stream
 * (DESIGN.md §3), seeded at the top of each sample — equivalent to the Rust
 * reference with `fastrand::seed(stream(seed, pixel, sample))` inserted at the
 * top of the batch-loop body (camera.rs:138).
 *
 * Build: oracle/Makefile (g++ -O2 -ffp-contract=off, no -march, no fast-math).
 */
#include <cmath>
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <cfloat>
#include <climits>
#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <vector>
#include <algorithm>
#include <stdexcept>
#include <string>

#include "../include/grayshift_scene.h"

namespace oracle {

static const double PI = 3.14159265358979323846; /* std::f64::consts::PI */

/* ---------------------------------------------------------------- RNG ---- */
/* fastrand 2.1.1 Rng::gen_u64 (wyrand, v4.2 constants) and Rng::f64.
 * Restated from the crate's published source; the crate is not in the container. */
struct Wyrand {
    uint64_t state;
    uint64_t next_u64() {
        const uint64_t C0 = 0x2d358dccaa6c78a5ULL, C1 = 0x8bb84b93962eacc9ULL;
        uint64_t s = state + C0;
        state = s;
        unsigned __int128 t = (unsigned __int128)s * (unsigned __int128)(s ^ C1);
        return (uint64_t)t ^ (uint64_t)(t >> 64);
    }
    double next_f64() {
        uint64_t bits = 0x3FF0000000000000ULL | (next_u64() >> 12);
        double d;
        std::memcpy(&d, &bits, 8);
        return d - 1.0;
    }
};

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* Per-(pixel, sample) stream seed — DESIGN.md §3. */
static uint64_t stream_seed(uint64_t seed, uint32_t pixel, uint32_t sample) {
    return splitmix64(seed ^ splitmix64(((uint64_t)sample << 32) | (uint64_t)pixel));
}

/* The reference's thread-local fastrand generator (util.rs:5-7 fastrand::f64()). */
static thread_local Wyrand tl_rng = {0};
static double rand_f64() { return tl_rng.next_f64(); }

/* Work counters, thread-local like the RNG, summed at the end of a render. */
static thread_local gs_counters tl_cnt;

/* --------------------------------------------------------------- Vec3 ---- */
/* util/vec3.rs */
struct Vec3 {
    double x, y, z;
    Vec3() : x(0), y(0), z(0) {}
    Vec3(double a, double b, double c) : x(a), y(b), z(c) {}
    double length_squared() const { return x * x + y * y + z * z; }   /* :19-21 */
    double length() const { return std::sqrt(length_squared()); }    /* :23-25 */
    Vec3 unit() const;                                                 /* :27-29 */
    double dot(const Vec3& o) const { return x * o.x + y * o.y + z * o.z; } /* :31-35 */
    Vec3 cross(const Vec3& o) const {                                 /* :37-43 */
        return Vec3(y * o.z - z * o.y, z * o.x - x * o.z, x * o.y - y * o.x);
    }
    Vec3 operator-() const { return Vec3(-x, -y, -z); }
    Vec3 operator+(const Vec3& o) const { return Vec3(x + o.x, y + o.y, z + o.z); }
    Vec3 operator-(const Vec3& o) const { return Vec3(x - o.x, y - o.y, z - o.z); }
    Vec3 operator*(double s) const { return Vec3(x * s, y * s, z * s); }
    Vec3 operator*(const Vec3& o) const { return Vec3(x * o.x, y * o.y, z * o.z); }
    Vec3 operator/(double s) const { return Vec3(x / s, y / s, z / s); }
    Vec3& operator+=(const Vec3& o) { x += o.x; y += o.y; z += o.z; return *this; }
    Vec3& operator/=(double s) { x /= s; y /= s; z /= s; return *this; }
    Vec3 reflect(const Vec3& n) const { return *this - n * (2.0 * dot(n)); } /* :53-55 */
    Vec3 refract(const Vec3& n, double ratio) const {                        /* :57-62 */
        double cos_theta = std::fmin(n.dot(-(*this)), 1.0);
        Vec3 r_out_perp = (*this + n * cos_theta) * ratio;
        Vec3 r_out_parallel = n * (-std::sqrt(std::fabs(1.0 - r_out_perp.length_squared())));
        return r_out_perp + r_out_parallel;
    }
};
/* `f64 * Vec3` is `rhs * self` (vec3.rs:144-149): componentwise v.c * s. */
static inline Vec3 operator*(double s, const Vec3& v) { return v * s; }
Vec3 Vec3::unit() const { return *this / length(); }

/* ----------------------------------------------------------- Interval ---- */
/* util/interval.rs */
struct Interval {
    double min, max;
    Interval(double a, double b) : min(a), max(b) {}
    static Interval EMPTY() { return Interval(DBL_MAX, -DBL_MAX); }    /* :10 */
    static Interval UNIVERSE() { return Interval(-DBL_MAX, DBL_MAX); } /* :11 */
    static Interval pair(const Interval& a, const Interval& b) {       /* :18-23 */
        return Interval(a.min <= b.min ? a.min : b.min, a.max >= b.max ? a.max : b.max);
    }
    double size() const { return max - min; }
    bool contains(double t) const { return min <= t && t <= max; }  /* :29-31 */
    bool surrounds(double t) const { return min < t && t < max; }   /* :33-35 */
    double clamp(double t) const {                                    /* :37-39, Rust f64::clamp */
        double r = t;
        if (r < min) r = min;
        if (r > max) r = max;
        return r;
    }
    Interval expand(double delta) const {                              /* :41-44 */
        double padding = delta / 2.0;
        return Interval(min - padding, max + padding);
    }
};

/* ---------------------------------------------------------------- Ray ---- */
struct Ray { /* ray.rs */
    Vec3 origin, direction;
    double time;
    Ray(const Vec3& o, const Vec3& d, double t) : origin(o), direction(d), time(t) {}
    Vec3 at(double t) const { return origin + direction * t; }
};

/* --------------------------------------------------------------- AABB ---- */
/* AABB.rs */
struct AABB {
    Interval x, y, z;
    AABB() : x(Interval::EMPTY()), y(Interval::EMPTY()), z(Interval::EMPTY()) {}
    AABB(Interval a, Interval b, Interval c) : x(a), y(b), z(c) {}
    static AABB from_corners(const Vec3& a, const Vec3& b) { /* :24-47 */
        AABB r(a.x <= b.x ? Interval(a.x, b.x) : Interval(b.x, a.x),
               a.y <= b.y ? Interval(a.y, b.y) : Interval(b.y, a.y),
               a.z <= b.z ? Interval(a.z, b.z) : Interval(b.z, a.z));
        r.pad_to_minimums();
        return r;
    }
    static AABB pair(const AABB& a, const AABB& b) { /* :49-56 */
        return AABB(Interval::pair(a.x, b.x), Interval::pair(a.y, b.y), Interval::pair(a.z, b.z));
    }
    const Interval& axis(int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    static bool slab(const Interval& s, double o, double d, Interval& iv) {
        double ad_inv = 1.0 / d;
        double t0 = (s.min - o) * ad_inv;
        double t1 = (s.max - o) * ad_inv;
        if (t0 < t1) {
            if (t0 > iv.min) iv.min = t0;
            if (t1 < iv.max) iv.max = t1;
        } else {
            if (t1 > iv.min) iv.min = t1;
            if (t0 < iv.max) iv.max = t0;
        }
        return !(iv.max <= iv.min);
    }
    bool hit(const Ray& r, Interval ray_t) const { /* :58-113 */
        Interval iv = ray_t;
        if (!slab(x, r.origin.x, r.direction.x, iv)) return false;
        if (!slab(y, r.origin.y, r.direction.y, iv)) return false;
        if (!slab(z, r.origin.z, r.direction.z, iv)) return false;
        return true;
    }
    int longest_axis() const { /* :115-121 */
        if (x.size() > y.size()) return x.size() > z.size() ? 0 : 2;
        return y.size() > z.size() ? 1 : 2;
    }
    void pad_to_minimums() { /* :123-128 */
        double delta = 0.0001;
        if (x.size() < delta) x = x.expand(delta);
        if (y.size() < delta) y = y.expand(delta);
        if (z.size() < delta) z = z.expand(delta);
    }
    AABB operator+(const Vec3& o) const { /* :144-153, Interval + f64 interval.rs:47-55 */
        return AABB(Interval(x.min + o.x, x.max + o.x), Interval(y.min + o.y, y.max + o.y),
                    Interval(z.min + o.z, z.max + o.z));
    }
};

/* ------------------------------------------------------------ Texture ---- */
/* texture.rs */
struct Texture {
    virtual ~Texture() {}
    virtual Vec3 value_at(double u, double v, const Vec3& p) const = 0;
};
struct SolidColorTexture : Texture { /* :13-31 */
    Vec3 albedo;
    explicit SolidColorTexture(Vec3 a) : albedo(a) {}
    Vec3 value_at(double, double, const Vec3&) const override { return albedo; }
};
/* Rust `f64 as i32`: saturating, NaN -> 0. */
static int32_t sat_i32(double f) {
    if (std::isnan(f)) return 0;
    if (f >= 2147483647.0) return INT32_MAX;
    if (f <= -2147483648.0) return INT32_MIN;
    return (int32_t)f;
}
/* Rust `f64 as u32` / `as usize`: saturating, NaN and negatives -> 0. */
static uint64_t sat_u64(double f, uint64_t maxv) {
    if (!(f > 0.0)) return 0;
    if (f >= (double)maxv) return maxv; /* (double)maxv rounds up for 2^64-1: still saturates */
    return (uint64_t)f;
}
struct CheckeredTexture : Texture { /* :33-71 */
    double scale_inv;
    const Texture* even;
    const Texture* odd;
    CheckeredTexture(double scale, const Texture* e, const Texture* o) : scale_inv(1.0 / scale), even(e), odd(o) {}
    Vec3 value_at(double u, double v, const Vec3& p) const override {
        int32_t xi = sat_i32(std::floor(scale_inv * p.x));
        int32_t yi = sat_i32(std::floor(scale_inv * p.y));
        int32_t zi = sat_i32(std::floor(scale_inv * p.z));
        /* i32 addition wraps in a release build; `%` truncates like C. */
        int32_t s = (int32_t)((uint32_t)xi + (uint32_t)yi + (uint32_t)zi);
        bool is_even = (s % 2) == 0;
        return is_even ? even->value_at(u, v, p) : odd->value_at(u, v, p);
    }
};
/* NoiseTexture (texture.rs:97-131) over `noise` 0.9.0's Perlin::default().  The crate
 * (and rand 0.8 / rand_xorshift 0.3 under it) is not in this image: this restates the
 * published algorithms — PARITY UNPINNED against the real crate. */
namespace noise09 {
struct XorShiftRng { /* rand_xorshift 0.3 */
    uint32_t x, y, z, w;
    explicit XorShiftRng(const uint8_t seed[16]) {
        uint32_t v[4];
        for (int i = 0; i < 4; i++) std::memcpy(&v[i], seed + 4 * i, 4); /* read_u32_into (LE) */
        x = v[0]; y = v[1]; z = v[2]; w = v[3];
    }
    uint32_t next_u32() {
        uint32_t t = x ^ (x << 11);
        x = y; y = z; z = w;
        w = w ^ (w >> 19) ^ (t ^ (t >> 8));
        return w;
    }
    /* rand 0.8 UniformInt<u32>::sample_single(0, n): Lemire widening multiply, rejection zone */
    uint32_t gen_range(uint32_t n) {
        uint32_t range = n;
        uint32_t zone = (range << __builtin_clz(range)) - 1u;
        for (;;) {
            uint64_t m = (uint64_t)next_u32() * (uint64_t)range;
            uint32_t hi = (uint32_t)(m >> 32), lo = (uint32_t)m;
            if (lo <= zone) return hi;
        }
    }
};
struct PermutationTable { /* noise 0.9 permutationtable.rs */
    uint8_t values[256];
    explicit PermutationTable(uint32_t seed) {
        uint8_t real[16] = {0};
        real[0] = 1;
        for (int i = 1; i < 4; i++) {
            real[i * 4] = (uint8_t)seed;
            real[i * 4 + 1] = (uint8_t)(seed >> 8);
            real[i * 4 + 2] = (uint8_t)(seed >> 16);
            real[i * 4 + 3] = (uint8_t)(seed >> 24);
        }
        XorShiftRng rng(real);
        for (int i = 0; i < 256; i++) values[i] = (uint8_t)i;
        for (int i = 255; i >= 1; i--) std::swap(values[i], values[rng.gen_range((uint32_t)i + 1)]); /* shuffle */
    }
    size_t hash(const int64_t* v, int n) const { /* fold: values[a] ^ b, then values[.] */
        size_t idx = (size_t)(v[0] & 0xff);
        for (int k = 1; k < n; k++) idx = (size_t)values[idx] ^ (size_t)(v[k] & 0xff);
        return values[idx];
    }
};
static int64_t numcast_isize(double f) { /* panics in the crate for NaN / out of range; saturate here */
    if (std::isnan(f)) return 0;
    if (f >= 9223372036854775808.0) return INT64_MAX;
    if (f <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)f;
}
static double gradient_dot_v(size_t perm, double x, double y, double z) {
    switch (perm & 0xF) {
        case 0: return x + y;   case 1: return -x + y;  case 2: return x - y;   case 3: return -x - y;
        case 4: return x + z;   case 5: return -x + z;  case 6: return x - z;   case 7: return -x - z;
        case 8: return y + z;   case 9: return -y + z;  case 10: return y - z;  case 11: return -y - z;
        case 12: return x + y;  case 13: return -x + y; case 14: return -y + z; default: return -y - z;
    }
}
static double s_curve5(double t) { return t * t * t * (t * (t * 6.0 - 15.0) + 10.0); }
/* core/perlin.rs perlin_3d */
static double perlin_3d(const double point[3], const PermutationTable& hasher) {
    const double SCALE_FACTOR = 1.1547005383792515;
    double floored[3] = {std::floor(point[0]), std::floor(point[1]), std::floor(point[2])};
    int64_t corner[3] = {numcast_isize(floored[0]), numcast_isize(floored[1]), numcast_isize(floored[2])};
    double distance[3] = {point[0] - floored[0], point[1] - floored[1], point[2] - floored[2]};
    auto g = [&](int ox, int oy, int oz) {
        int64_t c[3] = {corner[0] + ox, corner[1] + oy, corner[2] + oz};
        return gradient_dot_v(hasher.hash(c, 3), distance[0] - (double)ox, distance[1] - (double)oy,
                              distance[2] - (double)oz);
    };
    double g000 = g(0, 0, 0), g100 = g(1, 0, 0), g010 = g(0, 1, 0), g110 = g(1, 1, 0);
    double g001 = g(0, 0, 1), g101 = g(1, 0, 1), g011 = g(0, 1, 1), g111 = g(1, 1, 1);
    double a = s_curve5(distance[0]), b = s_curve5(distance[1]), c = s_curve5(distance[2]);
    double k0 = g000;
    double k1 = g100 - g000;
    double k2 = g010 - g000;
    double k3 = g001 - g000;
    double k4 = g000 + g110 - g100 - g010;
    double k5 = g000 + g101 - g100 - g001;
    double k6 = g000 + g011 - g010 - g001;
    double k7 = g100 + g010 + g001 + g111 - g000 - g110 - g101 - g011;
    double result = k0 + k1 * a + k2 * b + k3 * c + k4 * a * b + k5 * a * c + k6 * b * c + k7 * a * b * c;
    return result * SCALE_FACTOR;
}
} /* namespace noise09 */

struct NoiseTexture : Texture { /* :97-131 */
    double scale;
    noise09::PermutationTable noise; /* Perlin::default(): seed 0 */
    explicit NoiseTexture(double s) : scale(s), noise(0) {}
    double turbulence(Vec3 p, uint32_t depth) const { /* :107-124 */
        double accum = 0.0;
        Vec3 sample_point = p;
        double weight = 1.0;
        for (uint32_t i = 0; i < depth; i++) {
            double pt[3] = {sample_point.x, sample_point.y, sample_point.z};
            accum += weight * noise09::perlin_3d(pt, noise);
            weight /= 2.0;
            sample_point = sample_point * 2.0;
        }
        return std::fabs(accum);
    }
    Vec3 value_at(double, double, const Vec3& p) const override { /* :127-130 */
        tl_cnt.noise_evals++;
        return Vec3(0.5, 0.5, 0.5) * (1.0 + std::sin(scale * p.z + 10.0 * turbulence(p, 7)));
    }
};

struct ImageTexture : Texture { /* :73-95 */
    int32_t w, h;
    const uint8_t* rgb;
    ImageTexture(int32_t w_, int32_t h_, const uint8_t* p) : w(w_), h(h_), rgb(p) {}
    Vec3 value_at(double u, double v, const Vec3&) const override {
        double u_clamp = Interval(0.0, 1.0).clamp(u);
        double v_clamp = 1.0 - Interval(0.0, 1.0).clamp(v);
        uint64_t i = sat_u64(u_clamp * (double)w, UINT32_MAX);
        uint64_t j = sat_u64(v_clamp * (double)h, UINT32_MAX);
        /* Reference panics in get_pixel when i == w (u == 1) or j == h (v == 0);
         * documented deviation: clamp to the last texel. */
        if (i > (uint64_t)(w - 1)) i = (uint64_t)(w - 1);
        if (j > (uint64_t)(h - 1)) j = (uint64_t)(h - 1);
        const uint8_t* px = rgb + ((size_t)j * (size_t)w + (size_t)i) * 3;
        tl_cnt.image_texels++;
        return Vec3((double)px[0], (double)px[1], (double)px[2]) * (1.0 / 255.0);
    }
};

/* ------------------------------------------------------------- Hittable ---- */
struct Material;

struct HitRecord { /* hittable.rs:15-43 */
    double t;
    Vec3 position, normal;
    bool is_front_face;
    const Material* material;
    double u, v;
    HitRecord() : t(0), is_front_face(false), material(nullptr), u(0), v(0) {}
    static HitRecord make(const Ray& ray, double t, const Vec3& position, const Vec3& normal,
                          const Material* m, double u, double v) {
        HitRecord r;
        r.is_front_face = ray.direction.dot(normal) < 0.0;
        r.normal = r.is_front_face ? normal : -normal;
        r.t = t; r.position = position; r.material = m; r.u = u; r.v = v;
        return r;
    }
};

struct Hittable { /* hittable.rs:10-13 */
    virtual ~Hittable() {}
    virtual bool hit(const Ray& ray, Interval ray_t, HitRecord& rec) const = 0;
    virtual AABB bounding_box() const = 0;
};
using HittablePtr = std::unique_ptr<Hittable>;

struct HittableList : Hittable { /* hittable.rs:45-91 */
    std::vector<HittablePtr> objects;
    AABB bbox;
    void add(HittablePtr o) { bbox = AABB::pair(bbox, o->bounding_box()); objects.push_back(std::move(o)); }
    bool hit(const Ray& ray, Interval ray_t, HitRecord& rec) const override {
        tl_cnt.list_tests++;
        double closest = ray_t.max;
        bool any = false;
        HitRecord tmp;
        for (const auto& o : objects) {
            if (o->hit(ray, Interval(ray_t.min, closest), tmp)) {
                closest = tmp.t;
                rec = tmp;
                any = true;
            }
        }
        return any;
    }
    AABB bounding_box() const override { return bbox; }
};

static double deg_to_rad(double d) { return d / 180.0 * PI; } /* util.rs:62-64 */

struct Translate : Hittable { /* hittable.rs:93-125 */
    HittablePtr object;
    Vec3 offset;
    AABB bbox;
    Translate(HittablePtr o, Vec3 off) : object(std::move(o)), offset(off) { bbox = object->bounding_box() + offset; }
    bool hit(const Ray& ray, Interval ray_t, HitRecord& rec) const override {
        tl_cnt.instance_tests++;
        Ray offset_ray(ray.origin - offset, ray.direction, ray.time);
        if (object->hit(offset_ray, ray_t, rec)) {
            rec.position += offset;
            return true;
        }
        return false;
    }
    AABB bounding_box() const override { return bbox; }
};

struct RotateY : Hittable { /* hittable.rs:127-215 */
    HittablePtr object;
    double sin_theta, cos_theta;
    AABB bbox;
    RotateY(HittablePtr o, double angle) : object(std::move(o)) {
        double radians = deg_to_rad(angle);
        sin_theta = std::sin(radians);
        cos_theta = std::cos(radians);
        AABB b = object->bounding_box();
        Vec3 mn(DBL_MAX, DBL_MAX, DBL_MAX), mx(-DBL_MAX, -DBL_MAX, -DBL_MAX);
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++)
                for (int k = 0; k < 2; k++) {
                    double x = (double)i * b.x.max + (double)(1 - i) * b.x.min;
                    double y = (double)j * b.y.max + (double)(1 - j) * b.y.min;
                    double z = (double)k * b.z.max + (double)(1 - k) * b.z.min;
                    double nx = cos_theta * x + sin_theta * z;
                    double nz = -sin_theta * x + cos_theta * z;
                    mn.x = std::fmin(mn.x, nx); mx.x = std::fmax(mx.x, nx);
                    mn.y = std::fmin(mn.y, y);  mx.y = std::fmax(mx.y, y);
                    mn.z = std::fmin(mn.z, nz); mx.z = std::fmax(mx.z, nz);
                }
        bbox = AABB::from_corners(mn, mx);
    }
    bool hit(const Ray& ray, Interval ray_t, HitRecord& rec) const override {
        tl_cnt.instance_tests++;
        Vec3 o((cos_theta * ray.origin.x) - (sin_theta * ray.origin.z), ray.origin.y,
               (sin_theta * ray.origin.x) + (cos_theta * ray.origin.z));
        Vec3 d((cos_theta * ray.direction.x) - (sin_theta * ray.direction.z), ray.direction.y,
               (sin_theta * ray.direction.x) + (cos_theta * ray.direction.z));
        Ray rotated(o, d, ray.time);
        if (object->hit(rotated, ray_t, rec)) {
            Vec3 p = rec.position, n = rec.normal;
            rec.position = Vec3((cos_theta * p.x) + (sin_theta * p.z), p.y, (-sin_theta * p.x) + (cos_theta * p.z));
            rec.normal = Vec3((cos_theta * n.x) + (sin_theta * n.z), n.y, (-sin_theta * n.x) + (cos_theta * n.z));
            return true;
        }
        return false;
    }
    AABB bounding_box() const override { return bbox; }
};

struct Sphere : Hittable { /* hittable/sphere.rs */
    Vec3 center_start, center_path;
    bool is_moving;
    double radius;
    const Material* material;
    AABB bbox;
    static std::unique_ptr<Sphere> stationary(Vec3 c, double r, const Material* m) { /* :21-33 */
        auto s = std::make_unique<Sphere>();
        Vec3 rv(r, r, r);
        s->bbox = AABB::from_corners(c - rv, c + rv);
        s->center_start = c; s->center_path = Vec3(0, 0, 0); s->is_moving = false; s->radius = r; s->material = m;
        return s;
    }
    static std::unique_ptr<Sphere> moving(Vec3 c1, Vec3 c2, double r, const Material* m) { /* :35-49 */
        auto s = std::make_unique<Sphere>();
        Vec3 rv(r, r, r);
        AABB b1 = AABB::from_corners(c1 - rv, c1 + rv);
        AABB b2 = AABB::from_corners(c2 - rv, c2 + rv);
        s->bbox = AABB::pair(b1, b2);
        s->center_start = c1; s->center_path = c2 - c1; s->is_moving = true; s->radius = r; s->material = m;
        return s;
    }
    static void sphere_uv(const Vec3& p, double& u, double& v) { /* :55-60 */
        double theta = std::acos(-p.y);
        double phi = std::atan2(-p.z, p.x) + PI;
        u = phi / (2.0 * PI);
        v = theta / PI;
    }
    bool hit(const Ray& ray, Interval ray_t, HitRecord& rec) const override { /* :64-106 */
        if (is_moving) tl_cnt.msphere_tests++; else tl_cnt.sphere_tests++;
        Vec3 center = is_moving ? center_start + ray.time * center_path : center_start;
        Vec3 oc = center - ray.origin;
        double a = ray.direction.length_squared();
        double h = ray.direction.dot(oc);
        double c = oc.length_squared() - radius * radius;
        double discriminant = h * h - a * c;
        if (discriminant < 0.0) return false;
        double sqrt_d = std::sqrt(discriminant);
        double t = (h - sqrt_d) / a;
        if (!ray_t.surrounds(t)) {
            t = (h + sqrt_d) / a;
            if (!ray_t.surrounds(t)) return false;
        }
        Vec3 hit_pos = ray.at(t);
        Vec3 outward = (hit_pos - center) / radius;
        double u, v;
        sphere_uv(outward, u, v);
        rec = HitRecord::make(ray, t, hit_pos, outward, material, u, v);
        return true;
    }
    AABB bounding_box() const override { return bbox; }
};

struct Plane { /* hittable/plane.rs */
    Vec3 normal;
    double d;
    Plane() : d(0) {}
    Plane(Vec3 n, Vec3 origin) : normal(n), d(n.dot(origin)) {}
    bool hit(const Ray& ray, const Interval& ray_t, double& t, Vec3& inter) const { /* :20-32 */
        double denominator = normal.dot(ray.direction);
        if (std::fabs(denominator) < 1e-8) return false;
        t = (d - normal.dot(ray.origin)) / denominator;
        if (!ray_t.contains(t)) return false;
        inter = ray.at(t);
        return true;
    }
};

struct Quad : Hittable { /* hittable/quad.rs */
    Plane plane;
    Vec3 q, u, v, w;
    const Material* material;
    AABB bbox;
    Quad(Vec3 q_, Vec3 u_, Vec3 v_, const Material* m) : q(q_), u(u_), v(v_), material(m) { /* :25-38 */
        AABB d1 = AABB::from_corners(q, q + u + v);
        AABB d2 = AABB::from_corners(q + u, q + v);
        bbox = AABB::pair(d1, d2);
        Vec3 n = u.cross(v);
        Vec3 normal = n.unit();
        w = n / n.dot(n);
        plane = Plane(normal, q);
    }
    bool hit(const Ray& ray, Interval ray_t, HitRecord& rec) const override { /* :84-109 */
        tl_cnt.quad_tests++;
        double t;
        Vec3 inter;
        if (!plane.hit(ray, ray_t, t, inter)) return false;
        Vec3 planar = inter - q;
        double alpha = w.dot(planar.cross(v));
        double beta = w.dot(u.cross(planar));
        Interval unit(0.0, 1.0);
        if (!unit.contains(alpha) || !unit.contains(beta)) return false;
        rec = HitRecord::make(ray, t, inter, plane.normal, material, alpha, beta);
        return true;
    }
    AABB bounding_box() const override { return bbox; }
    static std::unique_ptr<HittableList> cube(Vec3 a, Vec3 b, const Material* m) { /* :54-80 */
        auto sides = std::make_unique<HittableList>();
        Vec3 mn(std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z));
        Vec3 mx(std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z));
        Vec3 dx(mx.x - mn.x, 0.0, 0.0), dy(0.0, mx.y - mn.y, 0.0), dz(0.0, 0.0, mx.z - mn.z);
        sides->add(std::make_unique<Quad>(Vec3(mn.x, mn.y, mx.z), dx, dy, m));
        sides->add(std::make_unique<Quad>(Vec3(mx.x, mn.y, mx.z), -dz, dy, m));
        sides->add(std::make_unique<Quad>(Vec3(mx.x, mn.y, mn.z), -dx, dy, m));
        sides->add(std::make_unique<Quad>(Vec3(mn.x, mn.y, mn.z), dz, dy, m));
        sides->add(std::make_unique<Quad>(Vec3(mn.x, mx.y, mx.z), dx, -dz, m));
        sides->add(std::make_unique<Quad>(Vec3(mn.x, mn.y, mn.z), dx, dz, m));
        return sides;
    }
};

struct Triangle : Hittable { /* hittable/triangle.rs */
    Vec3 normal, a, b, c;
    const Material* material;
    AABB bbox;
    Triangle(Vec3 a_, Vec3 b_, Vec3 c_, const Material* m) : a(a_), b(b_), c(c_), material(m) { /* :20-28 */
        normal = (b - a).cross(c - a);
        bbox = AABB::pair(AABB::from_corners(a, b), AABB::from_corners(a, c));
    }
    bool hit(const Ray& ray, Interval, HitRecord& rec) const override { /* :34-68; ray_t unused (quirk) */
        tl_cnt.tri_tests++;
        const double EPS = 1e-8;
        Vec3 e1 = c - a, e2 = b - a;
        Vec3 p_vec = ray.direction.cross(e2);
        double det = e1.dot(p_vec);
        if (det < EPS) return false;
        Vec3 t_vec = ray.origin - a;
        double u = t_vec.dot(p_vec);
        if (u < 0.0 || u > det) return false;
        Vec3 q_vec = t_vec.cross(e1);
        double v = ray.direction.dot(q_vec);
        if (v < 0.0 || u + v > det) return false;
        double t = e2.dot(q_vec);
        double inv_det = 1.0 / det;
        t *= inv_det; u *= inv_det; v *= inv_det;
        Vec3 pos = ray.at(t);
        rec = HitRecord::make(ray, t, pos, normal, material, u, v);
        return true;
    }
    AABB bounding_box() const override { return bbox; }
};

struct BVHNode : Hittable { /* hittable/BVH.rs */
    HittablePtr left, right;
    AABB bbox;
    static HittablePtr construct_tree(std::vector<HittablePtr> objects) { /* :18-65 */
        auto node = std::make_unique<BVHNode>();
        if (objects.size() == 1) {
            node->bbox = objects[0]->bounding_box();
            node->left = std::move(objects[0]);
            return node;
        }
        if (objects.size() == 2) {
            node->bbox = AABB::pair(objects[0]->bounding_box(), objects[1]->bounding_box());
            node->left = std::move(objects[0]);
            node->right = std::move(objects[1]);
            return node;
        }
        AABB bbox;
        for (auto& o : objects) bbox = AABB::pair(bbox, o->bounding_box());
        int axis = bbox.longest_axis();
        /* sort_by is a stable sort; partial_cmp().unwrap() panics on NaN (BVH.rs:54). */
        std::stable_sort(objects.begin(), objects.end(), [axis](const HittablePtr& a, const HittablePtr& b) {
            double am = a->bounding_box().axis(axis).min, bm = b->bounding_box().axis(axis).min;
            if (std::isnan(am) || std::isnan(bm)) throw std::runtime_error("BVH sort: NaN bbox (reference panics)");
            return am < bm;
        });
        size_t middle = objects.size() / 2;
        std::vector<HittablePtr> right_objs, left_objs;
        for (size_t i = 0; i < objects.size(); i++)
            (i < middle ? left_objs : right_objs).push_back(std::move(objects[i]));
        node->left = construct_tree(std::move(left_objs));
        node->right = construct_tree(std::move(right_objs));
        node->bbox = bbox;
        return node;
    }
    bool hit(const Ray& ray, Interval ray_t, HitRecord& rec) const override { /* :69-90 */
        tl_cnt.node_visits++;
        if (!bbox.hit(ray, ray_t)) return false;
        HitRecord hl;
        if (left->hit(ray, ray_t, hl)) {
            if (right) {
                HitRecord hr;
                if (right->hit(ray, Interval(ray_t.min, hl.t), hr)) { rec = hr; return true; }
            }
            rec = hl;
            return true;
        }
        if (right) return right->hit(ray, ray_t, rec);
        return false;
    }
    AABB bounding_box() const override { return bbox; }
};

struct ConstantMedium : Hittable { /* hittable/volume.rs:10-68 */
    HittablePtr boundary;
    double density_neg_inv;
    const Material* phase_function;
    ConstantMedium(HittablePtr b, double density, const Material* m) /* :17-21 */
        : boundary(std::move(b)), density_neg_inv(-1.0 / density), phase_function(m) {}
    bool hit(const Ray& ray, Interval ray_t, HitRecord& rec) const override { /* :32-63 */
        tl_cnt.medium_tests++;
        HitRecord r1, r2;
        if (!boundary->hit(ray, Interval::UNIVERSE(), r1)) return false;
        if (!boundary->hit(ray, Interval(r1.t + 0.0001, DBL_MAX), r2)) return false;
        double t1 = r1.t, t2 = r2.t;
        if (t1 < ray_t.min) t1 = ray_t.min;
        if (t2 > ray_t.max) t2 = ray_t.max;
        if (t1 >= t2) return false;
        if (t1 < 0.0) t1 = 0.0;
        double ray_len = ray.direction.length();
        double dist_inside_boundary = (t2 - t1) * ray_len;
        double hit_dist = density_neg_inv * std::log(rand_f64()); /* the RNG draw inside traversal (:48) */
        if (hit_dist > dist_inside_boundary) return false;
        double t = t1 + hit_dist / ray_len;
        rec = HitRecord::make(ray, t, ray.at(t), Vec3(1.0, 0.0, 0.0), phase_function, 0.0, 0.0);
        return true;
    }
    AABB bounding_box() const override { return boundary->bounding_box(); } /* :65-67 */
};

/* ------------------------------------------------------------ Material ---- */
/* material.rs */
struct ScatterRecord {
    Ray scattered_ray;
    Vec3 attenuation;
    double pdf;
    ScatterRecord() : scattered_ray(Vec3(), Vec3(), 0.0), pdf(0) {}
};

static Vec3 random_vector(double mn, double mx) { /* util.rs:9-16; fields evaluated x, y, z */
    double x = rand_f64() * (mx - mn) + mn;
    double y = rand_f64() * (mx - mn) + mn;
    double z = rand_f64() * (mx - mn) + mn;
    return Vec3(x, y, z);
}
static Vec3 random_vector_in_unit_sphere() { /* util.rs:18-25 */
    for (;;) {
        Vec3 v = random_vector(-1.0, 1.0);
        if (v.length_squared() < 1.0) return v;
    }
}
static Vec3 random_unit_vector() { return random_vector_in_unit_sphere().unit(); } /* :27-29 */
static Vec3 random_vector_in_unit_disk() { /* :36-46 */
    for (;;) {
        double x = rand_f64() * (1.0 - -1.0) + -1.0;
        double y = rand_f64() * (1.0 - -1.0) + -1.0;
        Vec3 v(x, y, 0.0);
        if (v.length_squared() < 1.0) return v;
    }
}
static Vec3 random_cosine_direction_from(double r_1, double r_2) { /* :48-60 */
    double phi = 2.0 * PI * r_1;
    double r_2_sqrt = std::sqrt(r_2);
    double x = std::cos(phi) * std::sqrt(r_2_sqrt);
    double y = std::sin(phi) * std::sqrt(r_2_sqrt);
    double z = std::sqrt(1.0 - r_2);
    return Vec3(x, y, z);
}
static Vec3 random_cosine_direction() {
    double r_1 = rand_f64();
    double r_2 = rand_f64();
    return random_cosine_direction_from(r_1, r_2);
}

struct ONB { /* ONB.rs */
    Vec3 u, v, w;
    explicit ONB(const Vec3& normal) { /* :10-23 */
        w = normal.unit();
        Vec3 a = std::fabs(w.x) > 0.9 ? Vec3(0.0, 1.0, 0.0) : Vec3(1.0, 0.0, 0.0);
        v = w.cross(a).unit();
        u = w.cross(v);
    }
    Vec3 transform(const Vec3& vec) const { return u * vec.x + v * vec.y + w * vec.z; } /* :25-27 */
};

struct Material { /* material.rs:11-21 */
    virtual ~Material() {}
    virtual bool scatter(const Ray&, const HitRecord&, ScatterRecord&) const { return false; }
    virtual Vec3 emitted(double, double, const Vec3&) const { return Vec3(0, 0, 0); }
};
struct Lambertian : Material { /* :29-73 */
    const Texture* texture;
    explicit Lambertian(const Texture* t) : texture(t) {}
    bool scatter(const Ray& ray_in, const HitRecord& rec, ScatterRecord& s) const override {
        s.attenuation = texture->value_at(rec.u, rec.v, rec.position);
        ONB basis(rec.normal);
        Vec3 dir = basis.transform(random_cosine_direction()).unit();
        s.scattered_ray = Ray(rec.position, dir, ray_in.time);
        s.pdf = basis.w.dot(dir) / PI;
        return true;
    }
};
struct Metal : Material { /* :75-103 */
    Vec3 albedo;
    double fuzz;
    Metal(Vec3 a, double f) : albedo(a), fuzz(f) {}
    bool scatter(const Ray& ray_in, const HitRecord& rec, ScatterRecord& s) const override {
        Vec3 reflected = ray_in.direction.reflect(rec.normal);
        reflected = reflected.unit() + fuzz * random_unit_vector();
        Ray scattered(rec.position, reflected, ray_in.time);
        if (scattered.direction.dot(rec.normal) > 0.0) {
            s.attenuation = albedo; s.scattered_ray = scattered; s.pdf = 0.0;
            return true;
        }
        return false;
    }
};
struct Dielectric : Material { /* :105-149 */
    double refraction_index;
    explicit Dielectric(double ri) : refraction_index(ri) {}
    static double reflectance(double cosine, double ri) { /* :114-119 */
        double r0 = (1.0 - ri) / (1.0 + ri);
        r0 = r0 * r0;
        double x = 1.0 - cosine;
        /* f64::powi(x, 5): LLVM expands a constant powi by repeated squaring: x * (x^2)^2 */
        double x2 = x * x;
        double x4 = x2 * x2;
        double p5 = x * x4;
        return r0 + (1.0 - r0) * p5;
    }
    bool scatter(const Ray& ray_in, const HitRecord& rec, ScatterRecord& s) const override {
        double ri = rec.is_front_face ? 1.0 / refraction_index : refraction_index;
        Vec3 unit_direction = ray_in.direction.unit();
        double cos_theta = std::fmin((-unit_direction).dot(rec.normal), 1.0);
        double sin_theta = std::sqrt(1.0 - cos_theta * cos_theta);
        bool cannot_refract = ri * sin_theta > 1.0;
        bool fresnel = reflectance(cos_theta, ri) > rand_f64(); /* draw is unconditional (:135) */
        Vec3 direction = (cannot_refract || fresnel) ? unit_direction.reflect(rec.normal)
                                                     : unit_direction.refract(rec.normal, ri);
        s.attenuation = Vec3(1.0, 1.0, 1.0);
        s.scattered_ray = Ray(rec.position, direction, ray_in.time);
        s.pdf = 0.0;
        return true;
    }
};
struct DiffuseLight : Material { /* :151-169 */
    const Texture* texture;
    explicit DiffuseLight(const Texture* t) : texture(t) {}
    Vec3 emitted(double u, double v, const Vec3& p) const override { return texture->value_at(u, v, p); }
};
struct Isotropic : Material { /* :171-200 */
    const Texture* texture;
    explicit Isotropic(const Texture* t) : texture(t) {}
    bool scatter(const Ray& ray_in, const HitRecord& rec, ScatterRecord& s) const override {
        s.attenuation = texture->value_at(rec.u, rec.v, rec.position);
        s.scattered_ray = Ray(rec.position, random_unit_vector(), ray_in.time);
        s.pdf = 1.0 / (4.0 * PI);
        return true;
    }
};

/* ------------------------------------------------------------- Camera ---- */
/* util.rs:67-86 */
static Vec3 rotate_vector(const Vec3& vector, const Vec3& rotation) {
    double sin_x = std::sin(rotation.x), cos_x = std::cos(rotation.x);
    double sin_y = std::sin(rotation.y), cos_y = std::cos(rotation.y);
    double sin_z = std::sin(rotation.z), cos_z = std::cos(rotation.z);
    double x = vector.x * (cos_y * cos_z) +
               vector.y * (cos_x * sin_z + sin_x * sin_y * cos_z) +
               vector.z * (sin_x * sin_z - cos_x * sin_y * cos_z);
    double y = vector.x * (-cos_y * sin_z) +
               vector.y * (cos_x * cos_z - sin_x * sin_y * sin_z) +
               vector.z * (sin_x * cos_z + cos_x * sin_y * sin_z);
    double z = vector.x * sin_y +
               vector.y * (-sin_x * cos_y) +
               vector.z * (cos_x * cos_y);
    return Vec3(x, y, z);
}

struct HDRI { /* camera.rs:251-270 */
    int32_t width, height;
    const float* rgb;
    Vec3 rotation;
    Vec3 sample(const Vec3& direction) const {
        Vec3 rotated = rotate_vector(direction, rotation).unit();
        double theta = std::atan2(rotated.y, rotated.x);
        double phi = std::asin(rotated.z);
        double u = 0.5 + theta / (2.0 * PI);
        double v = 0.5 - phi / PI;
        uint64_t x = sat_u64(u * (double)width, UINT64_MAX) % (uint64_t)width;
        uint64_t y = sat_u64(v * (double)height, UINT64_MAX) % (uint64_t)height;
        const float* px = rgb + ((size_t)y * (size_t)width + (size_t)x) * 3;
        tl_cnt.hdri_texels++;
        return Vec3((double)px[0], (double)px[1], (double)px[2]);
    }
};

static double luminance(const Vec3& v) { return 0.299 * v.x + 0.587 * v.y + 0.144 * v.z; } /* color.rs:31-33 */

struct Camera { /* camera.rs:17-98 */
    int32_t image_width, image_height;
    gs_sample_settings ss;
    uint32_t max_depth;
    Vec3 center, starting_pixel_pos, pixel_delta_u, pixel_delta_v;
    bool bg_hdri;
    Vec3 bg_color;
    HDRI hdri;
    double defocus_angle;
    Vec3 defocus_disk_u, defocus_disk_v;
    uint64_t seed;

    Camera(const gs_camera_spec& c, const gs_sample_settings& s, const gs_background_spec& bg, uint64_t seed_) {
        image_width = c.image_width;
        image_height = (int32_t)((double)c.image_width / c.aspect_ratio); /* `as i32` */
        ss = s;
        max_depth = c.max_depth;
        Vec3 look_from(c.look_from[0], c.look_from[1], c.look_from[2]);
        Vec3 look_at(c.look_at[0], c.look_at[1], c.look_at[2]);
        Vec3 vup(c.vup[0], c.vup[1], c.vup[2]);
        double theta = c.v_fov / 180.0 * PI;
        double h = std::tan(theta / 2.0);
        double viewport_height = 2.0 * h * c.focus_distance;
        double viewport_width = viewport_height * ((double)image_width / (double)image_height);
        Vec3 w = (look_from - look_at).unit();
        Vec3 u = vup.cross(w).unit();
        Vec3 v = w.cross(u);
        Vec3 viewport_u = viewport_width * u;
        Vec3 viewport_v = viewport_height * -v;
        pixel_delta_u = viewport_u / (double)image_width;
        pixel_delta_v = viewport_v / (double)image_height;
        Vec3 viewport_upper_left = look_from - c.focus_distance * w - viewport_u / 2.0 - viewport_v / 2.0;
        starting_pixel_pos = viewport_upper_left + 0.5 * (pixel_delta_u + pixel_delta_v);
        double defocus_radius = c.focus_distance * std::tan(deg_to_rad(c.defocus_angle / 2.0));
        defocus_disk_u = u * defocus_radius;
        defocus_disk_v = v * defocus_radius;
        center = look_from;
        defocus_angle = c.defocus_angle;
        bg_hdri = bg.kind == GS_BG_HDRI;
        bg_color = Vec3(bg.color[0], bg.color[1], bg.color[2]);
        hdri.width = bg.width; hdri.height = bg.height; hdri.rgb = bg.rgb;
        hdri.rotation = Vec3(bg.rotation[0], bg.rotation[1], bg.rotation[2]);
        seed = seed_;
    }

    Vec3 defocus_disk_sample() const { /* :223-226 */
        Vec3 v = random_vector_in_unit_disk();
        return center + v.x * defocus_disk_u + v.y * defocus_disk_v;
    }
    Ray get_ray(int32_t i, int32_t j) const { /* :204-221 */
        double offset_x = rand_f64() - 0.5;
        double offset_y = rand_f64() - 0.5;
        Vec3 pixel_sample = starting_pixel_pos + ((double)i + offset_x) * pixel_delta_u +
                            ((double)j + offset_y) * pixel_delta_v;
        Vec3 origin = defocus_angle <= 0.0 ? center : defocus_disk_sample();
        Vec3 direction = pixel_sample - origin;
        double t = rand_f64();
        return Ray(origin, direction, t);
    }
    Vec3 sample_background(const Ray& ray) const { /* :228-233 */
        return bg_hdri ? hdri.sample(ray.direction) : bg_color;
    }
    Vec3 ray_color(const Ray& ray, uint32_t depth, const Hittable& world) const { /* :174-202 */
        if (depth <= 0) return Vec3(0, 0, 0);
        tl_cnt.rays++;
        HitRecord rec;
        if (world.hit(ray, Interval(0.001, DBL_MAX), rec)) {
            tl_cnt.hits++;
            Vec3 emission = rec.material->emitted(rec.u, rec.v, rec.position);
            ScatterRecord s;
            if (rec.material->scatter(ray, rec, s)) {
                Vec3 scatter_color = ray_color(s.scattered_ray, depth - 1, world);
                Vec3 color_from_scatter = scatter_color * s.attenuation;
                return emission + color_from_scatter;
            }
            return emission;
        }
        return sample_background(ray);
    }
    Vec3 sample(int32_t i, int32_t j, const Hittable& world) const { /* :125-171 */
        Vec3 pixel_color(0, 0, 0);
        double tolerance_sq = ss.tolerance * ss.tolerance;
        double confidence_sq = ss.confidence * ss.confidence;
        double sum = 0.0, sq_sum = 0.0, sample_count = 0.0;
        uint32_t pixel = (uint32_t)j * (uint32_t)image_width + (uint32_t)i;
        uint32_t sample_index = 0;
        for (;;) {
            sample_count += (double)ss.batch_size;
            for (uint32_t b = 0; b < ss.batch_size; b++) {
                tl_rng.state = stream_seed(seed, pixel, sample_index++); /* the seeded stream */
                tl_cnt.paths++;
                Ray ray = get_ray(i, j);
                Vec3 sample_color = ray_color(ray, max_depth, world);
                pixel_color += sample_color;
                double lum = luminance(sample_color);
                sum += lum;
                sq_sum += lum * lum;
            }
            double mean = sum / sample_count;
            double variance_sq = 1.0 / (sample_count - 1.0) * (sq_sum - sum * sum / sample_count);
            double convergence_sq = confidence_sq * variance_sq / sample_count;
            if (convergence_sq < (mean * mean * tolerance_sq)) break;
            /* `sample_count as u32` saturates */
            if ((uint32_t)sat_u64(sample_count, UINT32_MAX) > ss.max_samples) break;
        }
        pixel_color /= sample_count;
        tl_cnt.pixels++;
        return pixel_color;
    }
};

/* ---------------------------------------------------------- Scene build ---- */
struct World {
    std::vector<std::unique_ptr<Texture>> textures;
    std::vector<std::unique_ptr<Material>> materials;
    HittablePtr root;
};

static const Texture* build_texture(const gs_scene_spec& s, int idx, World& w, std::vector<const Texture*>& memo) {
    if (idx < 0 || idx >= s.n_textures) throw std::runtime_error("texture index out of range");
    if (memo[idx]) return memo[idx];
    const gs_texture_spec& t = s.textures[idx];
    std::unique_ptr<Texture> tex;
    switch (t.kind) {
        case GS_TEX_SOLID: tex = std::make_unique<SolidColorTexture>(Vec3(t.p[0], t.p[1], t.p[2])); break;
        case GS_TEX_CHECKERED: {
            const Texture* e = build_texture(s, t.a, w, memo);
            const Texture* o = build_texture(s, t.b, w, memo);
            tex = std::make_unique<CheckeredTexture>(t.p[0], e, o);
            break;
        }
        case GS_TEX_IMAGE: {
            if (t.a < 0 || t.a >= s.n_images) throw std::runtime_error("image index out of range");
            const gs_image_spec& im = s.images[t.a];
            tex = std::make_unique<ImageTexture>(im.width, im.height, im.rgb8);
            break;
        }
        case GS_TEX_NOISE: tex = std::make_unique<NoiseTexture>(t.p[0]); break;
        default: throw std::runtime_error("unknown texture kind");
    }
    memo[idx] = tex.get();
    w.textures.push_back(std::move(tex));
    return memo[idx];
}

static HittablePtr build_object(const gs_scene_spec& s, int idx, const std::vector<const Material*>& mats) {
    if (idx < 0 || idx >= s.n_objects) throw std::runtime_error("object index out of range");
    const gs_object& o = s.objects[idx];
    const double* p = o.p;
    auto mat = [&]() -> const Material* {
        if (o.material < 0 || o.material >= (int)mats.size()) throw std::runtime_error("material index out of range");
        return mats[o.material];
    };
    switch (o.kind) {
        case GS_OBJ_SPHERE: return Sphere::stationary(Vec3(p[0], p[1], p[2]), p[3], mat());
        case GS_OBJ_MOVING_SPHERE: return Sphere::moving(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), p[6], mat());
        case GS_OBJ_QUAD: return std::make_unique<Quad>(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), Vec3(p[6], p[7], p[8]), mat());
        case GS_OBJ_TRIANGLE: return std::make_unique<Triangle>(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), Vec3(p[6], p[7], p[8]), mat());
        case GS_OBJ_CUBE: return Quad::cube(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), mat());
        case GS_OBJ_LIST: {
            auto l = std::make_unique<HittableList>();
            for (int k = 0; k < o.count; k++) l->add(build_object(s, s.children[o.first + k], mats));
            return l;
        }
        case GS_OBJ_BVH: {
            std::vector<HittablePtr> v;
            for (int k = 0; k < o.count; k++) v.push_back(build_object(s, s.children[o.first + k], mats));
            if (v.empty()) throw std::runtime_error("BVH of empty list (reference panics)");
            return BVHNode::construct_tree(std::move(v));
        }
        case GS_OBJ_TRANSLATE: return std::make_unique<Translate>(build_object(s, o.first, mats), Vec3(p[0], p[1], p[2]));
        case GS_OBJ_ROTATE_Y: return std::make_unique<RotateY>(build_object(s, o.first, mats), p[0]);
        case GS_OBJ_MEDIUM: return std::make_unique<ConstantMedium>(build_object(s, o.first, mats), p[0], mat());
        default: throw std::runtime_error("unknown object kind");
    }
}

static void build_world(const gs_scene_spec& s, World& w) {
    std::vector<const Texture*> tmemo(s.n_textures > 0 ? s.n_textures : 0, nullptr);
    std::vector<const Material*> mats;
    for (int i = 0; i < s.n_materials; i++) {
        const gs_material_spec& m = s.materials[i];
        std::unique_ptr<Material> mm;
        switch (m.kind) {
            case GS_MAT_LAMBERTIAN: mm = std::make_unique<Lambertian>(build_texture(s, m.texture, w, tmemo)); break;
            case GS_MAT_METAL: mm = std::make_unique<Metal>(Vec3(m.p[0], m.p[1], m.p[2]), m.p[3]); break;
            case GS_MAT_DIELECTRIC: mm = std::make_unique<Dielectric>(m.p[0]); break;
            case GS_MAT_DIFFUSE_LIGHT: mm = std::make_unique<DiffuseLight>(build_texture(s, m.texture, w, tmemo)); break;
            case GS_MAT_ISOTROPIC: mm = std::make_unique<Isotropic>(build_texture(s, m.texture, w, tmemo)); break;
            default: throw std::runtime_error("unknown material kind");
        }
        mats.push_back(mm.get());
        w.materials.push_back(std::move(mm));
    }
    /* The world HittableList, then BVHNode::from_list(world) as every scene does. */
    std::vector<HittablePtr> objs;
    for (int i = 0; i < s.n_world; i++) objs.push_back(build_object(s, s.world[i], mats));
    if (objs.empty()) throw std::runtime_error("empty world (reference panics)");
    w.root = BVHNode::construct_tree(std::move(objs));
}

static void add_counters(gs_counters& a, const gs_counters& b) {
    const uint64_t* pb = (const uint64_t*)&b;
    uint64_t* pa = (uint64_t*)&a;
    for (size_t k = 0; k < sizeof(gs_counters) / 8; k++) pa[k] += pb[k];
}

static thread_local std::string tl_err;

} // namespace oracle

using namespace oracle;

extern "C" {

const char* oracle_last_error(void) { return tl_err.c_str(); }

int32_t oracle_color_byte(double c);

/* Render pixels of the frame (all, or the listed subset) into out_rgb
 * (n_pixels*3 f32, in subset order, or the full W*H*3 frame), and, when out_rgb8 is
 * not NULL, write_color's bytes of the f64 colour in the same order.
 * Returns 0 on success, -1 on error (message in oracle_last_error). */
int oracle_render_timed(const gs_scene_spec* spec, const gs_camera_spec* cam, const gs_sample_settings* ss,
                        uint64_t seed, int32_t n_threads, const int32_t* subset, int64_t n_subset,
                        float* out_rgb, gs_counters* counters, uint8_t* out_rgb8, double* render_seconds) {
    try {
        World w;
        build_world(*spec, w);
        Camera camera(*cam, *ss, spec->background, seed);
        /* render time only: the pixel loop (camera.rs:105-114), not the world / BVH build */
        const auto t0 = std::chrono::steady_clock::now();
        int64_t n = subset ? n_subset : (int64_t)camera.image_width * camera.image_height;
        if (n_threads <= 0) n_threads = (int32_t)std::max(1u, std::thread::hardware_concurrency());
        std::atomic<int64_t> next(0);
        std::vector<gs_counters> per(n_threads);
        std::vector<std::thread> th;
        std::vector<std::string> errs(n_threads);
        const int64_t CHUNK = 64; /* rayon-like dynamic chunks */
        for (int t = 0; t < n_threads; t++) {
            th.emplace_back([&, t]() {
                try {
                    std::memset(&tl_cnt, 0, sizeof(tl_cnt));
                    for (;;) {
                        int64_t b = next.fetch_add(CHUNK);
                        if (b >= n) break;
                        int64_t e = std::min(n, b + CHUNK);
                        for (int64_t k = b; k < e; k++) {
                            int64_t pix = subset ? subset[k] : k;
                            int32_t i = (int32_t)(pix % camera.image_width), j = (int32_t)(pix / camera.image_width);
                            Vec3 c = camera.sample(i, j, *w.root);
                            out_rgb[k * 3 + 0] = (float)c.x;
                            out_rgb[k * 3 + 1] = (float)c.y;
                            out_rgb[k * 3 + 2] = (float)c.z;
                            if (out_rgb8) { /* write_color (color.rs:8-18) of the f64 colour */
                                out_rgb8[k * 3 + 0] = (uint8_t)oracle_color_byte(c.x);
                                out_rgb8[k * 3 + 1] = (uint8_t)oracle_color_byte(c.y);
                                out_rgb8[k * 3 + 2] = (uint8_t)oracle_color_byte(c.z);
                            }
                        }
                    }
                    per[t] = tl_cnt;
                } catch (const std::exception& ex) { errs[t] = ex.what(); }
            });
        }
        for (auto& x : th) x.join();
        if (render_seconds)
            *render_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (auto& e : errs) if (!e.empty()) throw std::runtime_error(e);
        if (counters) {
            std::memset(counters, 0, sizeof(*counters));
            for (auto& c : per) add_counters(*counters, c);
        }
        return 0;
    } catch (const std::exception& ex) {
        tl_err = ex.what();
        return -1;
    }
}

int oracle_render(const gs_scene_spec* spec, const gs_camera_spec* cam, const gs_sample_settings* ss,
                  uint64_t seed, int32_t n_threads, const int32_t* subset, int64_t n_subset,
                  float* out_rgb, gs_counters* counters, uint8_t* out_rgb8) {
    return oracle_render_timed(spec, cam, ss, seed, n_threads, subset, n_subset, out_rgb, counters, out_rgb8,
                               nullptr);
}

/* Camera::new derived fields, for KATs: image_height, center, starting_pixel_pos,
 * pixel_delta_u, pixel_delta_v, defocus_disk_u, defocus_disk_v (19 doubles). */
int oracle_camera_fields(const gs_camera_spec* cam, double* out19) {
    gs_sample_settings ss = {0.95, 0.0, 1, 0};
    gs_background_spec bg;
    std::memset(&bg, 0, sizeof(bg));
    bg.kind = GS_BG_SOLID;
    Camera c(*cam, ss, bg, 0);
    out19[0] = c.image_height;
    const Vec3* v[6] = {&c.center, &c.starting_pixel_pos, &c.pixel_delta_u, &c.pixel_delta_v, &c.defocus_disk_u, &c.defocus_disk_v};
    for (int k = 0; k < 6; k++) { out19[1 + 3 * k] = v[k]->x; out19[2 + 3 * k] = v[k]->y; out19[3 + 3 * k] = v[k]->z; }
    return 0;
}

/* ---- known-answer-test hooks (tests/test_oracle_kat.py) ---- */
uint64_t oracle_stream_seed(uint64_t seed, uint32_t pixel, uint32_t sample) { return stream_seed(seed, pixel, sample); }
void oracle_wyrand_f64(uint64_t state, int32_t n, double* out, uint64_t* out_u64) {
    Wyrand r{state};
    for (int k = 0; k < n; k++) {
        Wyrand c = r;
        if (out_u64) out_u64[k] = c.next_u64();
        out[k] = r.next_f64();
    }
}
int oracle_aabb_hit(const double* mn, const double* mx, const double* o, const double* d, double tmin, double tmax) {
    AABB b(Interval(mn[0], mx[0]), Interval(mn[1], mx[1]), Interval(mn[2], mx[2]));
    return b.hit(Ray(Vec3(o[0], o[1], o[2]), Vec3(d[0], d[1], d[2]), 0.0), Interval(tmin, tmax)) ? 1 : 0;
}
/* Single-primitive hit: kind = GS_OBJ_SPHERE/QUAD/TRIANGLE, p as in gs_object.
 * out: t, position[3], normal[3], front, u, v (10 doubles). */
int oracle_prim_hit(int32_t kind, const double* p, const double* o, const double* d, double time,
                    double tmin, double tmax, double* out) {
    Lambertian dummy(nullptr);
    HittablePtr h;
    if (kind == GS_OBJ_SPHERE) h = Sphere::stationary(Vec3(p[0], p[1], p[2]), p[3], &dummy);
    else if (kind == GS_OBJ_MOVING_SPHERE) h = Sphere::moving(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), p[6], &dummy);
    else if (kind == GS_OBJ_QUAD) h = std::make_unique<Quad>(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), Vec3(p[6], p[7], p[8]), &dummy);
    else if (kind == GS_OBJ_TRIANGLE) h = std::make_unique<Triangle>(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), Vec3(p[6], p[7], p[8]), &dummy);
    else return -1;
    HitRecord rec;
    bool ok = h->hit(Ray(Vec3(o[0], o[1], o[2]), Vec3(d[0], d[1], d[2]), time), Interval(tmin, tmax), rec);
    if (!ok) return 0;
    out[0] = rec.t;
    out[1] = rec.position.x; out[2] = rec.position.y; out[3] = rec.position.z;
    out[4] = rec.normal.x; out[5] = rec.normal.y; out[6] = rec.normal.z;
    out[7] = rec.is_front_face ? 1.0 : 0.0; out[8] = rec.u; out[9] = rec.v;
    return 1;
}
void oracle_random_cosine_direction(double r1, double r2, double* out3) {
    Vec3 v = random_cosine_direction_from(r1, r2);
    out3[0] = v.x; out3[1] = v.y; out3[2] = v.z;
}
void oracle_onb(const double* n, double* out9) {
    ONB b(Vec3(n[0], n[1], n[2]));
    const Vec3* v[3] = {&b.u, &b.v, &b.w};
    for (int k = 0; k < 3; k++) { out9[3 * k] = v[k]->x; out9[3 * k + 1] = v[k]->y; out9[3 * k + 2] = v[k]->z; }
}
double oracle_reflectance(double cosine, double ri) { return Dielectric::reflectance(cosine, ri); }
void oracle_refract(const double* v, const double* n, double ratio, double* out3) {
    Vec3 r = Vec3(v[0], v[1], v[2]).refract(Vec3(n[0], n[1], n[2]), ratio);
    out3[0] = r.x; out3[1] = r.y; out3[2] = r.z;
}
void oracle_rotate_vector(const double* v, const double* rot, double* out3) {
    Vec3 r = rotate_vector(Vec3(v[0], v[1], v[2]), Vec3(rot[0], rot[1], rot[2]));
    out3[0] = r.x; out3[1] = r.y; out3[2] = r.z;
}
double oracle_luminance(const double* c) { return luminance(Vec3(c[0], c[1], c[2])); }
/* write_color (color.rs:8-18): linear f64 -> byte */
int32_t oracle_color_byte(double c) {
    double g = c > 0.0 ? std::sqrt(c) : 0.0;
    double cl = Interval(0.0, 0.999).clamp(g);
    return sat_i32(256.0 * cl);
}
/* Camera::render's text (camera.rs:101-103,116-118; color.rs:17 `writeln!` of
 * "{r} {g} {b}") from a W*H*3 byte frame.  Returns the length, or the length needed
 * when out is NULL / too small. */
int64_t oracle_ppm_text(const uint8_t* rgb8, int32_t w, int32_t h, char* out, int64_t cap) {
    std::string t = "P3\n" + std::to_string(w) + " " + std::to_string(h) + "\n255\n";
    const int64_t n = (int64_t)w * h;
    for (int64_t k = 0; k < n; k++)
        t += std::to_string(rgb8[3 * k]) + " " + std::to_string(rgb8[3 * k + 1]) + " " + std::to_string(rgb8[3 * k + 2]) + "\n";
    if (out && cap >= (int64_t)t.size()) std::memcpy(out, t.data(), t.size());
    return (int64_t)t.size();
}
/* noise 0.9 Perlin::default() pieces, for KATs: the seed-0 permutation table, one
 * perlin_3d value, and NoiseTexture::value_at's channel value. */
void oracle_noise_perm(uint32_t seed, uint8_t* out256) {
    noise09::PermutationTable t(seed);
    std::memcpy(out256, t.values, 256);
}
double oracle_perlin3(const double* p) {
    static const noise09::PermutationTable t(0);
    return noise09::perlin_3d(p, t);
}
double oracle_noise_value(double scale, const double* p) {
    NoiseTexture n(scale);
    return n.value_at(0.0, 0.0, Vec3(p[0], p[1], p[2])).x;
}
/* Checkered texture parity (texture.rs:58-70): returns 1 for even. */
int oracle_checker_even(double scale, const double* p) {
    SolidColorTexture e(Vec3(1, 1, 1)), o(Vec3(0, 0, 0));
    CheckeredTexture c(scale, &e, &o);
    return c.value_at(0, 0, Vec3(p[0], p[1], p[2])).x == 1.0 ? 1 : 0;
}
/* BVH topology of the world list: writes a pre-order description:
 * for each node visited: (depth, n_leaf_children) ... returns node count. */
static void bvh_walk(const Hittable* h, int depth, std::vector<int32_t>& out) {
    const BVHNode* n = dynamic_cast<const BVHNode*>(h);
    if (!n) { out.push_back(-1); out.push_back(depth); return; }
    out.push_back(1); out.push_back(depth);
    bvh_walk(n->left.get(), depth + 1, out);
    if (n->right) bvh_walk(n->right.get(), depth + 1, out);
    else { out.push_back(0); out.push_back(depth + 1); }
}
int64_t oracle_bvh_topology(const gs_scene_spec* spec, int32_t* out, int64_t cap) {
    try {
        World w;
        build_world(*spec, w);
        std::vector<int32_t> v;
        bvh_walk(w.root.get(), 0, v);
        if (out) for (int64_t k = 0; k < (int64_t)v.size() && k < cap; k++) out[k] = v[k];
        return (int64_t)v.size();
    } catch (const std::exception& ex) {
        tl_err = ex.what();
        return -1;
    }
}

} /* extern "C" */
