// world.hpp — C++ host mirror of the reference's scene surface.
//
// The reference's host-side types (Rust trait objects) restated as C++ classes with
// the same names and constructor arguments, so a Rust `Camera::render` caller maps
// one-for-one:  Hittable (hittable/hittable.rs:10-13), HittableList, Translate,
// RotateY, BVHNode::from_list (BVH.rs:15), Sphere::new_stationary/new_moving,
// Quad::new / Quad::cube, Triangle::new, Material (Lambertian::from_color,
// from_texture, Metal::new, Dielectric::new, DiffuseLight::new/from_color),
// Texture (SolidColorTexture, CheckeredTexture::from_colors, ImageTexture),
// Camera::new / Camera::render, SampleSettings, Background::{SOLID, HDRI}.
//
// The one addition to the reference surface is `flatten(Flattener&)` on every
// concrete type: the world is turned into the plain arrays of
// include/grayshift_gpu.h and rendered by the HIP megakernel.  There is no CPU
// `hit()` here — the only place the scene is intersected is the device.
#pragma once

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <map>
#include <memory>
#include <ostream>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../../../include/grayshift_gpu.h"

namespace grayshift {

static const double PI = 3.14159265358979323846;

struct Vec3 {  // util/vec3.rs
    double x = 0, y = 0, z = 0;
    Vec3() = default;
    Vec3(double a, double b, double c) : x(a), y(b), z(c) {}
    static Vec3 ZERO() { return Vec3(); }
    double length_squared() const { return x * x + y * y + z * z; }
    double length() const { return std::sqrt(length_squared()); }
    Vec3 unit() const { return Vec3(x / length(), y / length(), z / length()); }
    double dot(const Vec3& o) const { return x * o.x + y * o.y + z * o.z; }
    Vec3 cross(const Vec3& o) const { return Vec3(y * o.z - z * o.y, z * o.x - x * o.z, x * o.y - y * o.x); }
    Vec3 operator-() const { return Vec3(-x, -y, -z); }
    Vec3 operator+(const Vec3& o) const { return Vec3(x + o.x, y + o.y, z + o.z); }
    Vec3 operator-(const Vec3& o) const { return Vec3(x - o.x, y - o.y, z - o.z); }
    Vec3 operator*(double s) const { return Vec3(x * s, y * s, z * s); }
    Vec3 operator/(double s) const { return Vec3(x / s, y / s, z / s); }
    void store(double* p) const { p[0] = x; p[1] = y; p[2] = z; }
};
inline Vec3 operator*(double s, const Vec3& v) { return v * s; }  // vec3.rs:144-149

struct Interval {  // util/interval.rs
    double min, max;
    Interval(double a, double b) : min(a), max(b) {}
    static Interval EMPTY() { return Interval(DBL_MAX, -DBL_MAX); }
    static Interval from_interval_pair(const Interval& a, const Interval& b) {
        return Interval(a.min <= b.min ? a.min : b.min, a.max >= b.max ? a.max : b.max);
    }
    double size() const { return max - min; }
    Interval expand(double delta) const {
        double padding = delta / 2.0;
        return Interval(min - padding, max + padding);
    }
};

struct AABB {  // AABB.rs
    Interval x = Interval::EMPTY(), y = Interval::EMPTY(), z = Interval::EMPTY();
    AABB() = default;
    AABB(Interval a, Interval b, Interval c) : x(a), y(b), z(c) {}
    static AABB from_corners(const Vec3& a, const Vec3& b);
    static AABB from_AABB_pair(const AABB& a, const AABB& b) {
        return AABB(Interval::from_interval_pair(a.x, b.x), Interval::from_interval_pair(a.y, b.y),
                    Interval::from_interval_pair(a.z, b.z));
    }
    const Interval& operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    int longest_axis() const {
        if (x.size() > y.size()) return x.size() > z.size() ? 0 : 2;
        return y.size() > z.size() ? 1 : 2;
    }
    AABB operator+(const Vec3& o) const {
        return AABB(Interval(x.min + o.x, x.max + o.x), Interval(y.min + o.y, y.max + o.y),
                    Interval(z.min + o.z, z.max + o.z));
    }
};

class Flattener;

// ---------------------------------------------------------------- textures
class Texture {
public:
    virtual ~Texture() = default;
    virtual uint32_t flatten(Flattener& f) const = 0;
};
using TexturePtr = std::shared_ptr<Texture>;  // Arc<dyn Texture>

class SolidColorTexture : public Texture {
public:
    explicit SolidColorTexture(Vec3 albedo) : albedo(albedo) {}
    uint32_t flatten(Flattener& f) const override;
    Vec3 albedo;
};

class CheckeredTexture : public Texture {
public:
    CheckeredTexture(double scale, TexturePtr even, TexturePtr odd)
        : scale_inv(1.0 / scale), even(std::move(even)), odd(std::move(odd)) {}
    static std::shared_ptr<CheckeredTexture> from_colors(double scale, Vec3 even, Vec3 odd) {
        return std::make_shared<CheckeredTexture>(scale, std::make_shared<SolidColorTexture>(even),
                                                  std::make_shared<SolidColorTexture>(odd));
    }
    uint32_t flatten(Flattener& f) const override;
    double scale_inv;
    TexturePtr even, odd;
};

// ImageTexture over caller-owned RGB8 texels (the decoded earthmap.jpg).
class ImageTexture : public Texture {
public:
    ImageTexture(int32_t width, int32_t height, const uint8_t* rgb8) : width(width), height(height), rgb8(rgb8) {}
    uint32_t flatten(Flattener& f) const override;
    int32_t width, height;
    const uint8_t* rgb8;
};

// NoiseTexture (texture.rs:97-131): Perlin::default() of the `noise` crate; the device
// evaluates it from the crate's seed-0 permutation table, which flatten() generates.
class NoiseTexture : public Texture {
public:
    explicit NoiseTexture(double scale) : scale(scale) {}
    uint32_t flatten(Flattener& f) const override;
    double scale;
};

// noise 0.9 PermutationTable::new(seed): XorShiftRng seeded from `seed`, then a rand 0.8
// Fisher-Yates shuffle of 0..=255.  Restated from the crates' published algorithms
// (their source is not in this image: parity unpinned).
void noise_permutation(uint32_t seed, uint8_t out[256]);

// --------------------------------------------------------------- materials
class Material {
public:
    virtual ~Material() = default;
    virtual uint32_t flatten(Flattener& f) const = 0;
};
using MaterialPtr = std::shared_ptr<Material>;  // Arc<dyn Material>

class Lambertian : public Material {
public:
    explicit Lambertian(TexturePtr t) : texture(std::move(t)) {}
    static std::shared_ptr<Lambertian> from_color(Vec3 albedo) {
        return std::make_shared<Lambertian>(std::make_shared<SolidColorTexture>(albedo));
    }
    static std::shared_ptr<Lambertian> from_texture(TexturePtr t) { return std::make_shared<Lambertian>(std::move(t)); }
    uint32_t flatten(Flattener& f) const override;
    TexturePtr texture;
};
class Metal : public Material {
public:
    Metal(Vec3 albedo, double fuzz) : albedo(albedo), fuzz(fuzz) {}
    uint32_t flatten(Flattener& f) const override;
    Vec3 albedo;
    double fuzz;
};
class Dielectric : public Material {
public:
    explicit Dielectric(double refraction_index) : refraction_index(refraction_index) {}
    uint32_t flatten(Flattener& f) const override;
    double refraction_index;
};
class DiffuseLight : public Material {
public:
    explicit DiffuseLight(TexturePtr t) : texture(std::move(t)) {}
    static std::shared_ptr<DiffuseLight> from_color(Vec3 c) {
        return std::make_shared<DiffuseLight>(std::make_shared<SolidColorTexture>(c));
    }
    uint32_t flatten(Flattener& f) const override;
    TexturePtr texture;
};

class Isotropic : public Material {  // material.rs:171-200 (phase function of a ConstantMedium)
public:
    explicit Isotropic(TexturePtr t) : texture(std::move(t)) {}
    static std::shared_ptr<Isotropic> from_color(Vec3 c) {
        return std::make_shared<Isotropic>(std::make_shared<SolidColorTexture>(c));
    }
    uint32_t flatten(Flattener& f) const override;
    TexturePtr texture;
};

// --------------------------------------------------------------- hittables
class Hittable {
public:
    virtual ~Hittable() = default;
    virtual AABB bounding_box() const = 0;
    // Append this object to the flat arrays; returns its tagged reference.
    virtual uint32_t flatten(Flattener& f) const = 0;
};
using HittablePtr = std::unique_ptr<Hittable>;  // Box<dyn Hittable>

class Sphere : public Hittable {
public:
    static std::unique_ptr<Sphere> new_stationary(Vec3 center, double radius, MaterialPtr m);
    static std::unique_ptr<Sphere> new_moving(Vec3 c1, Vec3 c2, double radius, MaterialPtr m);
    AABB bounding_box() const override { return bbox; }
    uint32_t flatten(Flattener& f) const override;
    Vec3 center_start, center_path;
    bool is_moving = false;
    double radius = 0;
    MaterialPtr material;
    AABB bbox;
};

class Quad : public Hittable {
public:
    Quad(Vec3 q, Vec3 u, Vec3 v, MaterialPtr m);
    static std::unique_ptr<class HittableList> cube(Vec3 a, Vec3 b, MaterialPtr m);
    AABB bounding_box() const override { return bbox; }
    uint32_t flatten(Flattener& f) const override;
    Vec3 q, u, v, w, normal;
    double d;
    MaterialPtr material;
    AABB bbox;
};

class Triangle : public Hittable {
public:
    Triangle(Vec3 a, Vec3 b, Vec3 c, MaterialPtr m);
    AABB bounding_box() const override { return bbox; }
    uint32_t flatten(Flattener& f) const override;
    Vec3 normal, a, b, c;
    MaterialPtr material;
    AABB bbox;
};

class HittableList : public Hittable {
public:
    void add(HittablePtr o) {
        bbox = AABB::from_AABB_pair(bbox, o->bounding_box());
        objects.push_back(std::move(o));
    }
    AABB bounding_box() const override { return bbox; }
    uint32_t flatten(Flattener& f) const override;
    std::vector<HittablePtr> objects;
    AABB bbox;
};

class Translate : public Hittable {
public:
    Translate(HittablePtr o, Vec3 offset) : object(std::move(o)), offset(offset) { bbox = object->bounding_box() + offset; }
    AABB bounding_box() const override { return bbox; }
    uint32_t flatten(Flattener& f) const override;
    HittablePtr object;
    Vec3 offset;
    AABB bbox;
};

class RotateY : public Hittable {
public:
    RotateY(HittablePtr o, double angle);
    AABB bounding_box() const override { return bbox; }
    uint32_t flatten(Flattener& f) const override;
    HittablePtr object;
    double sin_theta, cos_theta;
    AABB bbox;
};

class BVHNode : public Hittable {
public:
    static std::unique_ptr<BVHNode> from_list(HittableList list) { return construct_tree(std::move(list.objects)); }
    static std::unique_ptr<BVHNode> construct_tree(std::vector<HittablePtr> objects);
    AABB bounding_box() const override { return bbox; }
    uint32_t flatten(Flattener& f) const override;
    HittablePtr left, right;  // right may be null (n == 1)
    AABB bbox;
};

// hittable/volume.rs:10-68.  The boundary is a primitive, a list, a BVH of those, or (one
// level) another medium on the device path (round 6; the device's validation and flatten say
// so otherwise); the medium itself may sit in a BVH under Translate/RotateY (round 5).
class ConstantMedium : public Hittable {
public:
    ConstantMedium(HittablePtr boundary, double density, MaterialPtr phase_function)
        : boundary(std::move(boundary)), density_neg_inv(-1.0 / density), phase_function(std::move(phase_function)) {}
    static std::unique_ptr<ConstantMedium> from_isotropic_color(HittablePtr boundary, double density, Vec3 color) {
        return std::make_unique<ConstantMedium>(std::move(boundary), density, Isotropic::from_color(color));
    }
    AABB bounding_box() const override { return boundary->bounding_box(); }
    uint32_t flatten(Flattener& f) const override;
    HittablePtr boundary;
    double density_neg_inv;
    MaterialPtr phase_function;
};

// ------------------------------------------------------------------ camera
struct SampleSettings {  // camera.rs:239-244
    double confidence, tolerance;
    uint32_t batch_size, max_samples;
};

struct HDRI {  // camera.rs:251-254 (image = f32 RGB texels, caller-owned)
    int32_t width = 0, height = 0;
    const float* rgb = nullptr;
    Vec3 rotation;
};

struct Background {  // camera.rs:246-249
    enum Kind { SOLID, HDRI_ } kind = SOLID;
    Vec3 color;
    HDRI hdri;
    static Background solid(Vec3 c) { Background b; b.kind = SOLID; b.color = c; return b; }
    static Background hdr(HDRI h) { Background b; b.kind = HDRI_; b.hdri = h; return b; }
};

// Collects the flat arrays of include/grayshift_gpu.h.
class Flattener {
public:
    uint32_t material_index(const Material* m);
    uint32_t texture_index(const Texture* t);
    uint32_t image_index(const ImageTexture* t);
    std::vector<gs_node> nodes;
    std::vector<gs_sphere> spheres;
    std::vector<gs_msphere> mspheres;
    std::vector<gs_quad> quads;
    std::vector<gs_triangle> triangles;
    std::vector<gs_list> lists;
    std::vector<uint32_t> list_refs;
    std::vector<gs_instance> instances;
    std::vector<gs_medium> media;
    std::vector<uint8_t> noise_perm;  // 256 B once any NoiseTexture is flattened
    std::vector<gs_material> materials;
    std::vector<gs_texture> textures;
    std::vector<gs_image> images;
    std::vector<uint8_t> texels8;
    // Identity -> slot (hash maps: a linear scan per lookup was O(n^2) in unique
    // materials, minutes for a million-sphere world).
    std::unordered_map<const Material*, uint32_t> mat_slot;
    std::unordered_map<const Texture*, uint32_t> tex_slot;
    std::map<std::tuple<const uint8_t*, int32_t, int32_t>, uint32_t> img_slot;  // same texels = one image
    uint32_t depth = 0, max_depth = 0;  // BVH node nesting while flattening
    bool inside_instance = false;
    bool inside_medium = false;  // flattening a ConstantMedium boundary
    int medium_depth = 0;        // ConstantMedium boundaries being flattened (round 6: up to 2)
    bool inside_nested_bvh = false;  // flattening a BVH under Translate/RotateY
    bool instance_in_nested = false;  // flattening a Translate/RotateY inside such a BVH (round 6)
};

// A flattened world + background, ready for gs_render / gs_device_scene_create.
struct FlatScene {
    Flattener f;
    std::vector<float> hdri_rgb;
    gs_flat_scene view{};
    void finalize(uint32_t root, const Background& bg);
};

class Camera {
public:
    Camera(double aspect_ratio, int32_t image_width, SampleSettings sample_settings, uint32_t max_depth,
           double v_fov, Vec3 look_from, Vec3 look_at, Vec3 vup, double defocus_angle, double focus_distance,
           Background background);
    // camera.rs:100 — same contract: PPM "P3" text, one `r g b` line per pixel.
    void render(const Hittable& world, std::ostream& image_file, uint64_t seed = 1) const;
    // The linear framebuffer (pixel_color / sample_count, camera.rs:167) instead of PPM.
    void render_linear(const Hittable& world, float* out_rgb, gs_stats* stats, uint64_t seed = 1) const;
    // The PPM text Camera::render writes (device-formatted).
    std::string render_ppm(const Hittable& world, gs_stats* stats, uint64_t seed = 1) const;
    const gs_camera& fields() const { return cam; }
    const gs_sample_settings& settings() const { return ss; }
    const Background& background() const { return bg; }
    int32_t image_width() const { return cam.image_width; }
    int32_t image_height() const { return cam.image_height; }

private:
    gs_camera cam{};
    gs_sample_settings ss{};
    Background bg;
};

// Flatten a world (the BVH root) for the device.
std::unique_ptr<FlatScene> flatten_world(const Hittable& world, const Background& bg);
// color.rs:8-18 — linear f64 -> PPM byte.
int32_t color_byte(double c);
void write_ppm(std::ostream& os, int32_t w, int32_t h, const float* rgb);

}  // namespace grayshift
