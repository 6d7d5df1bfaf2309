// world.cpp — constructors, BVH build and flattening of the host mirror.
// Every constructor follows the cited reference lines exactly (same f64 expression
// order), because bounding boxes decide BVH topology and node-box tests.
#include "world.hpp"

#include <algorithm>
#include <cstring>

namespace grayshift {

AABB AABB::from_corners(const Vec3& a, const Vec3& b) {  // AABB.rs:24-47, pad :123-128
    AABB r(a.x <= b.x ? Interval(a.x, b.x) : Interval(b.x, a.x), a.y <= b.y ? Interval(a.y, b.y) : Interval(b.y, a.y),
           a.z <= b.z ? Interval(a.z, b.z) : Interval(b.z, a.z));
    const double delta = 0.0001;
    if (r.x.size() < delta) r.x = r.x.expand(delta);
    if (r.y.size() < delta) r.y = r.y.expand(delta);
    if (r.z.size() < delta) r.z = r.z.expand(delta);
    return r;
}

std::unique_ptr<Sphere> Sphere::new_stationary(Vec3 center, double radius, MaterialPtr m) {  // sphere.rs:21-33
    auto s = std::make_unique<Sphere>();
    Vec3 r(radius, radius, radius);
    s->bbox = AABB::from_corners(center - r, center + r);
    s->center_start = center;
    s->is_moving = false;
    s->radius = radius;
    s->material = std::move(m);
    return s;
}

std::unique_ptr<Sphere> Sphere::new_moving(Vec3 c1, Vec3 c2, double radius, MaterialPtr m) {  // sphere.rs:35-49
    auto s = std::make_unique<Sphere>();
    Vec3 r(radius, radius, radius);
    s->bbox = AABB::from_AABB_pair(AABB::from_corners(c1 - r, c1 + r), AABB::from_corners(c2 - r, c2 + r));
    s->center_start = c1;
    s->center_path = c2 - c1;
    s->is_moving = true;
    s->radius = radius;
    s->material = std::move(m);
    return s;
}

Quad::Quad(Vec3 q_, Vec3 u_, Vec3 v_, MaterialPtr m) : q(q_), u(u_), v(v_), material(std::move(m)) {  // quad.rs:25-38
    bbox = AABB::from_AABB_pair(AABB::from_corners(q, q + u + v), AABB::from_corners(q + u, q + v));
    Vec3 n = u.cross(v);
    normal = n.unit();
    w = n / n.dot(n);
    d = normal.dot(q);  // Plane::new plane.rs:15-18
}

std::unique_ptr<HittableList> Quad::cube(Vec3 a, Vec3 b, MaterialPtr m) {  // quad.rs:54-80
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

Triangle::Triangle(Vec3 a_, Vec3 b_, Vec3 c_, MaterialPtr m) : a(a_), b(b_), c(c_), material(std::move(m)) {  // triangle.rs:20-28
    normal = (b - a).cross(c - a);
    bbox = AABB::from_AABB_pair(AABB::from_corners(a, b), AABB::from_corners(a, c));
}

RotateY::RotateY(HittablePtr o, double angle) : object(std::move(o)) {  // hittable.rs:135-175
    double radians = angle / 180.0 * PI;  // deg_to_rad util.rs:62-64
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

std::unique_ptr<BVHNode> BVHNode::construct_tree(std::vector<HittablePtr> objects) {  // BVH.rs:18-65
    if (objects.empty()) throw std::invalid_argument("BVHNode::from_list of an empty list");
    auto node = std::make_unique<BVHNode>();
    if (objects.size() == 1) {
        node->bbox = objects[0]->bounding_box();
        node->left = std::move(objects[0]);
        return node;
    }
    if (objects.size() == 2) {
        node->bbox = AABB::from_AABB_pair(objects[0]->bounding_box(), objects[1]->bounding_box());
        node->left = std::move(objects[0]);
        node->right = std::move(objects[1]);
        return node;
    }
    AABB bbox;
    for (auto& o : objects) bbox = AABB::from_AABB_pair(bbox, o->bounding_box());
    const int axis = bbox.longest_axis();
    // Stable sort on bbox[axis].min, as Rust's sort_by; NaN keys panic there (unwrap).
    std::vector<std::pair<double, size_t>> keys(objects.size());
    for (size_t i = 0; i < objects.size(); i++) {
        double k = objects[i]->bounding_box()[axis].min;
        if (std::isnan(k)) throw std::invalid_argument("BVH sort: NaN bounding box");
        keys[i] = {k, i};
    }
    std::stable_sort(keys.begin(), keys.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    const size_t middle = objects.size() / 2;
    std::vector<HittablePtr> left_objs, right_objs;
    for (size_t r = 0; r < keys.size(); r++)
        (r < middle ? left_objs : right_objs).push_back(std::move(objects[keys[r].second]));
    node->left = construct_tree(std::move(left_objs));
    node->right = construct_tree(std::move(right_objs));
    node->bbox = bbox;
    return node;
}

// ---------------------------------------------------------------- flatten
static void check_index(size_t n, const char* what) {
    if (n >= GS_REF_MASK) throw std::length_error(std::string("too many ") + what + " for a 28-bit reference");
}

uint32_t Flattener::material_index(const Material* m) {
    auto it = mat_slot.find(m);
    if (it != mat_slot.end()) return it->second;
    // Reserve the slot first so recursive texture flattening cannot reorder it.
    const uint32_t idx = (uint32_t)materials.size();
    mat_slot.emplace(m, idx);
    materials.push_back(gs_material{});
    m->flatten(*this);  // fills materials[idx]
    return idx;
}
uint32_t Flattener::texture_index(const Texture* t) {
    auto it = tex_slot.find(t);
    if (it != tex_slot.end()) return it->second;
    const uint32_t idx = (uint32_t)textures.size();
    tex_slot.emplace(t, idx);
    textures.push_back(gs_texture{});
    t->flatten(*this);
    return idx;
}
uint32_t Flattener::image_index(const ImageTexture* t) {
    const auto key = std::make_tuple(t->rgb8, t->width, t->height);
    auto it = img_slot.find(key);
    if (it != img_slot.end()) return it->second;
    gs_image im{(uint32_t)t->width, (uint32_t)t->height, (uint64_t)texels8.size()};
    size_t n = (size_t)t->width * (size_t)t->height * 3;
    texels8.insert(texels8.end(), t->rgb8, t->rgb8 + n);
    images.push_back(im);
    const uint32_t idx = (uint32_t)(images.size() - 1);
    img_slot.emplace(key, idx);
    return idx;
}

// A texture/material writes itself into the slot its *_index call reserved.
static size_t slot_of(const std::unordered_map<const Texture*, uint32_t>& slots, const Texture* t) {
    auto it = slots.find(t);
    if (it == slots.end()) throw std::logic_error("texture slot");
    return it->second;
}
static size_t slot_of(const std::unordered_map<const Material*, uint32_t>& slots, const Material* m) {
    auto it = slots.find(m);
    if (it == slots.end()) throw std::logic_error("material slot");
    return it->second;
}

uint32_t SolidColorTexture::flatten(Flattener& f) const {
    size_t s = slot_of(f.tex_slot, this);
    gs_texture& t = f.textures[s];
    t.kind = GS_TEX_SOLID;
    albedo.store(t.color);
    return (uint32_t)s;
}
uint32_t CheckeredTexture::flatten(Flattener& f) const {
    size_t s = slot_of(f.tex_slot, this);
    uint32_t e = f.texture_index(even.get());
    uint32_t o = f.texture_index(odd.get());
    gs_texture& t = f.textures[s];
    t.kind = GS_TEX_CHECKERED;
    t.even = e;
    t.odd = o;
    t.scale_inv = scale_inv;
    return (uint32_t)s;
}
uint32_t ImageTexture::flatten(Flattener& f) const {
    size_t s = slot_of(f.tex_slot, this);
    if (width <= 0 || height <= 0 || !rgb8) throw std::invalid_argument("ImageTexture without texels");
    uint32_t im = f.image_index(this);
    gs_texture& t = f.textures[s];
    t.kind = GS_TEX_IMAGE;
    t.image = im;
    return (uint32_t)s;
}

void noise_permutation(uint32_t seed, uint8_t out[256]) {
    // PermutationTable::new: a 16-byte XorShift seed, byte 0 = 1, then the seed's
    // little-endian bytes repeated in words 1..3.
    uint8_t real[16] = {0};
    real[0] = 1;
    for (int i = 1; i < 4; i++)
        for (int k = 0; k < 4; k++) real[i * 4 + k] = (uint8_t)(seed >> (8 * k));
    uint32_t x[4];
    for (int i = 0; i < 4; i++)
        x[i] = (uint32_t)real[4 * i] | ((uint32_t)real[4 * i + 1] << 8) | ((uint32_t)real[4 * i + 2] << 16) |
               ((uint32_t)real[4 * i + 3] << 24);
    auto next_u32 = [&]() {  // rand_xorshift 0.3 XorShiftRng::next_u32
        const uint32_t t = x[0] ^ (x[0] << 11);
        x[0] = x[1];
        x[1] = x[2];
        x[2] = x[3];
        x[3] = x[3] ^ (x[3] >> 19) ^ (t ^ (t >> 8));
        return x[3];
    };
    auto gen_index = [&](uint32_t range) {  // rand 0.8 gen_range(0..range) for u32: widening multiply + zone
        const uint32_t zone = (range << __builtin_clz(range)) - 1u;
        for (;;) {
            const uint64_t m = (uint64_t)next_u32() * range;
            if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
        }
    };
    for (int i = 0; i < 256; i++) out[i] = (uint8_t)i;
    for (uint32_t i = 255; i >= 1; i--) {  // SliceRandom::shuffle
        const uint32_t j = gen_index(i + 1);
        const uint8_t t = out[i];
        out[i] = out[j];
        out[j] = t;
    }
}

uint32_t NoiseTexture::flatten(Flattener& f) const {
    size_t s = slot_of(f.tex_slot, this);
    if (f.noise_perm.empty()) {
        f.noise_perm.resize(256);
        noise_permutation(0, f.noise_perm.data());  // Perlin::DEFAULT_SEED
    }
    gs_texture& t = f.textures[s];
    t.kind = GS_TEX_NOISE;
    t.color[0] = scale;
    return (uint32_t)s;
}

uint32_t Lambertian::flatten(Flattener& f) const {
    size_t s = slot_of(f.mat_slot, this);
    uint32_t tex = f.texture_index(texture.get());
    f.materials[s].kind = GS_MAT_LAMBERTIAN;
    f.materials[s].texture = tex;
    return (uint32_t)s;
}
uint32_t Metal::flatten(Flattener& f) const {
    size_t s = slot_of(f.mat_slot, this);
    f.materials[s].kind = GS_MAT_METAL;
    albedo.store(f.materials[s].albedo);
    f.materials[s].param = fuzz;
    return (uint32_t)s;
}
uint32_t Dielectric::flatten(Flattener& f) const {
    size_t s = slot_of(f.mat_slot, this);
    f.materials[s].kind = GS_MAT_DIELECTRIC;
    f.materials[s].param = refraction_index;
    return (uint32_t)s;
}
uint32_t DiffuseLight::flatten(Flattener& f) const {
    size_t s = slot_of(f.mat_slot, this);
    uint32_t tex = f.texture_index(texture.get());
    f.materials[s].kind = GS_MAT_DIFFUSE_LIGHT;
    f.materials[s].texture = tex;
    return (uint32_t)s;
}

uint32_t Isotropic::flatten(Flattener& f) const {
    size_t s = slot_of(f.mat_slot, this);
    uint32_t tex = f.texture_index(texture.get());
    f.materials[s].kind = GS_MAT_ISOTROPIC;
    f.materials[s].texture = tex;
    return (uint32_t)s;
}

uint32_t Sphere::flatten(Flattener& f) const {
    uint32_t m = f.material_index(material.get());
    if (!is_moving) {
        gs_sphere s{};
        center_start.store(s.center);
        s.radius = radius;
        s.material = m;
        check_index(f.spheres.size(), "spheres");
        f.spheres.push_back(s);
        return GS_MAKE_REF(GS_REF_SPHERE, f.spheres.size() - 1);
    }
    gs_msphere s{};
    center_start.store(s.center_start);
    center_path.store(s.center_path);
    s.radius = radius;
    s.material = m;
    check_index(f.mspheres.size(), "moving spheres");
    f.mspheres.push_back(s);
    return GS_MAKE_REF(GS_REF_MSPHERE, f.mspheres.size() - 1);
}
uint32_t Quad::flatten(Flattener& f) const {
    gs_quad g{};
    q.store(g.q); u.store(g.u); v.store(g.v); w.store(g.w); normal.store(g.normal);
    g.d = d;
    g.material = f.material_index(material.get());
    check_index(f.quads.size(), "quads");
    f.quads.push_back(g);
    return GS_MAKE_REF(GS_REF_QUAD, f.quads.size() - 1);
}
uint32_t Triangle::flatten(Flattener& f) const {
    gs_triangle g{};
    a.store(g.a); b.store(g.b); c.store(g.c); normal.store(g.normal);
    g.material = f.material_index(material.get());
    check_index(f.triangles.size(), "triangles");
    f.triangles.push_back(g);
    return GS_MAKE_REF(GS_REF_TRIANGLE, f.triangles.size() - 1);
}
static bool is_primitive(uint32_t ref) {
    uint32_t k = ref >> GS_REF_SHIFT;
    return k == GS_REF_SPHERE || k == GS_REF_MSPHERE || k == GS_REF_QUAD || k == GS_REF_TRIANGLE;
}
uint32_t HittableList::flatten(Flattener& f) const {
    // A list is scanned linearly on the device; its members must be primitives.
    std::vector<uint32_t> refs;
    for (auto& o : objects) {
        uint32_t r = o->flatten(f);
        if (!is_primitive(r))
            throw std::domain_error("HittableList member that is not a primitive (nested list/instance/BVH) "
                                    "is not supported on the device path");
        refs.push_back(r);
    }
    gs_list l{(uint32_t)f.list_refs.size(), (uint32_t)refs.size()};
    f.list_refs.insert(f.list_refs.end(), refs.begin(), refs.end());
    check_index(f.lists.size(), "lists");
    f.lists.push_back(l);
    return GS_MAKE_REF(GS_REF_LIST, f.lists.size() - 1);
}
static uint32_t flatten_instance_child(Flattener& f, const Hittable& o) {
    // (round 6: a chain inside a BVH that is itself under a chain is accepted -- the device keeps
    // both chains of such a hit -- but not a further BVH under it, BVHNode::flatten)
    bool was = f.inside_instance, was_in = f.instance_in_nested;
    f.inside_instance = true;
    if (f.inside_nested_bvh) f.instance_in_nested = true;
    uint32_t r = o.flatten(f);
    f.inside_instance = was;
    f.instance_in_nested = was_in;
    return r;
}
uint32_t Translate::flatten(Flattener& f) const {
    // Reserve first: instance order = outer before inner.
    size_t idx = f.instances.size();
    check_index(idx, "instances");
    f.instances.push_back(gs_instance{});
    uint32_t child = flatten_instance_child(f, *object);
    gs_instance& in = f.instances[idx];
    in.kind = GS_INST_TRANSLATE;
    in.child = child;
    offset.store(in.p);
    return GS_MAKE_REF(GS_REF_INSTANCE, idx);
}
uint32_t RotateY::flatten(Flattener& f) const {
    size_t idx = f.instances.size();
    check_index(idx, "instances");
    f.instances.push_back(gs_instance{});
    uint32_t child = flatten_instance_child(f, *object);
    gs_instance& in = f.instances[idx];
    in.kind = GS_INST_ROTATE_Y;
    in.child = child;
    in.p[0] = sin_theta;
    in.p[1] = cos_theta;
    in.p[2] = 0.0;
    return GS_MAKE_REF(GS_REF_INSTANCE, idx);
}
uint32_t BVHNode::flatten(Flattener& f) const {
    // (round 6: a BVH as a ConstantMedium boundary is walked by the device's catch-all kernel;
    // its leaves must be lists or primitives -- the device's validation says so otherwise)
    if (f.instance_in_nested)
        throw std::domain_error("a BVH under Translate/RotateY inside a BVH that is itself under Translate/RotateY "
                                "(two levels of nested BVHs) is not supported on the device path");
    // A BVH under Translate/RotateY (final_scene's balls, main.rs:741-755) is walked by the
    // device as a second-level tree on its own stack: its depth does not count towards
    // the top-level (LDS) stack.
    const bool top = !f.inside_instance && f.medium_depth == 0;
    const bool was_nested = f.inside_nested_bvh;
    if (!top) f.inside_nested_bvh = true;
    // Pre-order: the left subtree follows its parent in memory (cache locality).
    size_t idx = f.nodes.size();
    check_index(idx, "nodes");
    f.nodes.push_back(gs_node{});
    if (top) {
        f.depth++;
        if (f.depth > f.max_depth) f.max_depth = f.depth;
    }
    uint32_t l = left->flatten(f);
    uint32_t r = right ? right->flatten(f) : (uint32_t)GS_REF_NONE;
    if (top) f.depth--;
    f.inside_nested_bvh = was_nested;
    gs_node& n = f.nodes[idx];
    n.min[0] = bbox.x.min; n.min[1] = bbox.y.min; n.min[2] = bbox.z.min;
    n.max[0] = bbox.x.max; n.max[1] = bbox.y.max; n.max[2] = bbox.z.max;
    n.left = l;
    n.right = r;
    return GS_MAKE_REF(GS_REF_NODE, idx);
}

uint32_t ConstantMedium::flatten(Flattener& f) const {  // volume.rs:10-29
    // (round 6: one medium as another's boundary is walked by the device's catch-all kernel)
    if (f.medium_depth >= 2)
        throw std::domain_error("ConstantMedium two deep inside ConstantMedium boundaries is not supported on the "
                                "device path");
    // (inside a BVH under Translate/RotateY: supported since round 5, the device walks such
    // trees in its main passes and tests their media like the top level's)
    size_t idx = f.media.size();
    check_index(idx, "media");
    f.media.push_back(gs_medium{});
    const bool was = f.inside_medium;
    f.inside_medium = true;
    f.medium_depth++;
    uint32_t b = boundary->flatten(f);
    f.medium_depth--;
    f.inside_medium = was;
    uint32_t m = f.material_index(phase_function.get());
    gs_medium& md = f.media[idx];
    md.boundary = b;
    md.material = m;
    md.density_neg_inv = density_neg_inv;
    return GS_MAKE_REF(GS_REF_MEDIUM, idx);
}

void FlatScene::finalize(uint32_t root, const Background& bg) {
    gs_flat_scene& v = view;
    std::memset(&v, 0, sizeof(v));
    v.root = root;
    v.max_bvh_depth = f.max_depth;
    v.nodes = f.nodes.data();           v.n_nodes = (uint32_t)f.nodes.size();
    v.spheres = f.spheres.data();       v.n_spheres = (uint32_t)f.spheres.size();
    v.mspheres = f.mspheres.data();     v.n_mspheres = (uint32_t)f.mspheres.size();
    v.quads = f.quads.data();           v.n_quads = (uint32_t)f.quads.size();
    v.triangles = f.triangles.data();   v.n_triangles = (uint32_t)f.triangles.size();
    v.lists = f.lists.data();           v.n_lists = (uint32_t)f.lists.size();
    v.list_refs = f.list_refs.data();   v.n_list_refs = (uint32_t)f.list_refs.size();
    v.instances = f.instances.data();   v.n_instances = (uint32_t)f.instances.size();
    v.media = f.media.data();           v.n_media = (uint32_t)f.media.size();
    v.noise_perm = f.noise_perm.empty() ? nullptr : f.noise_perm.data();
    v.n_noise_perm = (uint32_t)f.noise_perm.size();
    v.materials = f.materials.data();   v.n_materials = (uint32_t)f.materials.size();
    v.textures = f.textures.data();     v.n_textures = (uint32_t)f.textures.size();
    v.images = f.images.data();         v.n_images = (uint32_t)f.images.size();
    v.texels8 = f.texels8.data();       v.n_texels8 = f.texels8.size();
    gs_background& b = v.background;
    if (bg.kind == Background::SOLID) {
        b.kind = GS_BG_SOLID;
        bg.color.store(b.color);
    } else {
        b.kind = GS_BG_HDRI;
        b.width = (uint32_t)bg.hdri.width;
        b.height = (uint32_t)bg.hdri.height;
        // rotate_vector's coefficients (util.rs:67-86), same expressions, computed once.
        const Vec3& r = bg.hdri.rotation;
        double sin_x = std::sin(r.x), cos_x = std::cos(r.x);
        double sin_y = std::sin(r.y), cos_y = std::cos(r.y);
        double sin_z = std::sin(r.z), cos_z = std::cos(r.z);
        b.rot[0] = cos_y * cos_z;
        b.rot[1] = cos_x * sin_z + sin_x * sin_y * cos_z;
        b.rot[2] = sin_x * sin_z - cos_x * sin_y * cos_z;
        b.rot[3] = -cos_y * sin_z;
        b.rot[4] = cos_x * cos_z - sin_x * sin_y * sin_z;
        b.rot[5] = sin_x * cos_z + cos_x * sin_y * sin_z;
        b.rot[6] = sin_y;
        b.rot[7] = -sin_x * cos_y;
        b.rot[8] = cos_x * cos_y;
        size_t n = (size_t)bg.hdri.width * (size_t)bg.hdri.height * 3;
        if (!bg.hdri.rgb || n == 0) throw std::invalid_argument("HDRI background without texels");
        hdri_rgb.assign(bg.hdri.rgb, bg.hdri.rgb + n);
        v.hdri_rgb = hdri_rgb.data();
        v.n_hdri_floats = n;
    }
}

std::unique_ptr<FlatScene> flatten_world(const Hittable& world, const Background& bg) {
    auto fs = std::make_unique<FlatScene>();
    uint32_t root = world.flatten(fs->f);
    fs->finalize(root, bg);
    return fs;
}

}  // namespace grayshift
