// host_capi.cpp — gs_scene_spec -> world objects, and the C-ABI of grayshift_host.h.
#include <cstring>
#include <fstream>
#include <string>

#include "../../../include/grayshift_host.h"
#include "world.hpp"

namespace grayshift {

struct SpecBuilder {
    const gs_scene_spec& s;
    std::vector<TexturePtr> tex;
    std::vector<MaterialPtr> mat;
    explicit SpecBuilder(const gs_scene_spec& spec) : s(spec) {}

    TexturePtr texture(int idx, int depth = 0) {
        if (idx < 0 || idx >= s.n_textures) throw std::invalid_argument("texture index out of range");
        if (depth > 16) throw std::invalid_argument("texture nesting too deep");
        if (tex[idx]) return tex[idx];
        const gs_texture_spec& t = s.textures[idx];
        TexturePtr r;
        switch (t.kind) {
            case GS_TEX_SOLID: r = std::make_shared<SolidColorTexture>(Vec3(t.p[0], t.p[1], t.p[2])); break;
            case GS_TEX_CHECKERED:
                r = std::make_shared<CheckeredTexture>(t.p[0], texture(t.a, depth + 1), texture(t.b, depth + 1));
                break;
            case GS_TEX_IMAGE: {
                if (t.a < 0 || t.a >= s.n_images) throw std::invalid_argument("image index out of range");
                const gs_image_spec& im = s.images[t.a];
                r = std::make_shared<ImageTexture>(im.width, im.height, im.rgb8);
                break;
            }
            case GS_TEX_NOISE: r = std::make_shared<NoiseTexture>(t.p[0]); break;
            default: throw std::invalid_argument("unknown texture kind");
        }
        tex[idx] = r;
        return r;
    }
    MaterialPtr material(int idx) {
        if (idx < 0 || idx >= (int)mat.size()) throw std::invalid_argument("material index out of range");
        return mat[idx];
    }
    HittablePtr object(int idx, int depth = 0) {
        if (idx < 0 || idx >= s.n_objects) throw std::invalid_argument("object index out of range");
        if (depth > 64) throw std::invalid_argument("object nesting too deep");
        const gs_object& o = s.objects[idx];
        const double* p = o.p;
        auto children = [&]() {
            if (o.first < 0 || o.count < 0 || o.first + o.count > s.n_children)
                throw std::invalid_argument("children range out of bounds");
            std::vector<HittablePtr> v;
            for (int k = 0; k < o.count; k++) v.push_back(object(s.children[o.first + k], depth + 1));
            return v;
        };
        switch (o.kind) {
            case GS_OBJ_SPHERE: return Sphere::new_stationary(Vec3(p[0], p[1], p[2]), p[3], material(o.material));
            case GS_OBJ_MOVING_SPHERE:
                return Sphere::new_moving(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), p[6], material(o.material));
            case GS_OBJ_QUAD:
                return std::make_unique<Quad>(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), Vec3(p[6], p[7], p[8]),
                                              material(o.material));
            case GS_OBJ_TRIANGLE:
                return std::make_unique<Triangle>(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]),
                                                  Vec3(p[6], p[7], p[8]), material(o.material));
            case GS_OBJ_CUBE: return Quad::cube(Vec3(p[0], p[1], p[2]), Vec3(p[3], p[4], p[5]), material(o.material));
            case GS_OBJ_LIST: {
                auto l = std::make_unique<HittableList>();
                for (auto& c : children()) l->add(std::move(c));
                return l;
            }
            case GS_OBJ_BVH: return BVHNode::construct_tree(children());
            case GS_OBJ_TRANSLATE: return std::make_unique<Translate>(object(o.first, depth + 1), Vec3(p[0], p[1], p[2]));
            case GS_OBJ_ROTATE_Y: return std::make_unique<RotateY>(object(o.first, depth + 1), p[0]);
            case GS_OBJ_MEDIUM:
                return std::make_unique<ConstantMedium>(object(o.first, depth + 1), p[0], material(o.material));
            default: throw std::invalid_argument("unknown object kind");
        }
    }
    std::unique_ptr<BVHNode> world() {
        tex.assign(s.n_textures > 0 ? s.n_textures : 0, nullptr);
        for (int i = 0; i < s.n_materials; i++) {
            const gs_material_spec& m = s.materials[i];
            switch (m.kind) {
                case GS_MAT_LAMBERTIAN: mat.push_back(Lambertian::from_texture(texture(m.texture))); break;
                case GS_MAT_METAL: mat.push_back(std::make_shared<Metal>(Vec3(m.p[0], m.p[1], m.p[2]), m.p[3])); break;
                case GS_MAT_DIELECTRIC: mat.push_back(std::make_shared<Dielectric>(m.p[0])); break;
                case GS_MAT_DIFFUSE_LIGHT: mat.push_back(std::make_shared<DiffuseLight>(texture(m.texture))); break;
                case GS_MAT_ISOTROPIC: mat.push_back(std::make_shared<Isotropic>(texture(m.texture))); break;
                default: throw std::invalid_argument("unknown material kind");
            }
        }
        HittableList world;
        for (int i = 0; i < s.n_world; i++) world.add(object(s.world[i]));
        return BVHNode::from_list(std::move(world));
    }
    Background background() {
        const gs_background_spec& b = s.background;
        if (b.kind == GS_BG_SOLID) return Background::solid(Vec3(b.color[0], b.color[1], b.color[2]));
        if (b.kind == GS_BG_HDRI) {
            HDRI h;
            h.width = b.width;
            h.height = b.height;
            h.rgb = b.rgb;
            h.rotation = Vec3(b.rotation[0], b.rotation[1], b.rotation[2]);
            if (h.width <= 0 || h.height <= 0 || !h.rgb) throw std::invalid_argument("HDRI without texels");
            return Background::hdr(h);
        }
        throw std::invalid_argument("unknown background kind");
    }
};

static void topo(const gs_flat_scene& v, uint32_t ref, int depth, std::vector<int32_t>& out) {
    uint32_t k = ref >> GS_REF_SHIFT, i = ref & GS_REF_MASK;
    if (k != GS_REF_NODE) {
        out.push_back(-1);
        out.push_back(depth);
        return;
    }
    out.push_back(1);
    out.push_back(depth);
    topo(v, v.nodes[i].left, depth + 1, out);
    if ((v.nodes[i].right >> GS_REF_SHIFT) != GS_REF_NONE) topo(v, v.nodes[i].right, depth + 1, out);
    else {
        out.push_back(0);
        out.push_back(depth + 1);
    }
}

}  // namespace grayshift

using namespace grayshift;

struct gs_host_scene {
    std::unique_ptr<FlatScene> flat;
};

// The device library owns gs_last_error(); the host reports through it.
extern "C" void gs_set_last_error(const char* msg);

static gs_status fail(gs_status code, const char* what) {
    gs_set_last_error(what);
    return code;
}

template <class F>
static gs_status guarded(F&& f) {
    try {
        return f();
    } catch (const std::domain_error& e) {
        return fail(GS_ERR_UNSUPPORTED, e.what());
    } catch (const std::bad_alloc&) {
        return fail(GS_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(GS_ERR_ARG, e.what());
    }
}

extern "C" {

gs_status gs_host_scene_from_spec(const gs_scene_spec* spec, gs_host_scene** out) {
    if (!spec || !out) return fail(GS_ERR_ARG, "null argument");
    return guarded([&]() {
        SpecBuilder b(*spec);
        auto world = b.world();
        auto bg = b.background();
        auto hs = std::make_unique<gs_host_scene>();
        hs->flat = flatten_world(*world, bg);
        *out = hs.release();
        return GS_OK;
    });
}

gs_status gs_host_scene_destroy(gs_host_scene* scene) {
    delete scene;
    return GS_OK;
}

const gs_flat_scene* gs_host_scene_flat(const gs_host_scene* scene) { return scene ? &scene->flat->view : nullptr; }

gs_status gs_host_camera(const gs_camera_spec* c, gs_camera* out) {
    if (!c || !out) return fail(GS_ERR_ARG, "null argument");
    if (c->image_width <= 0 || !(c->aspect_ratio > 0.0)) return fail(GS_ERR_ARG, "bad image size");
    return guarded([&]() {
        SampleSettings ss{0.95, 0.0, 1, 0};
        Camera cam(c->aspect_ratio, c->image_width, ss, c->max_depth, c->v_fov,
                   Vec3(c->look_from[0], c->look_from[1], c->look_from[2]),
                   Vec3(c->look_at[0], c->look_at[1], c->look_at[2]), Vec3(c->vup[0], c->vup[1], c->vup[2]),
                   c->defocus_angle, c->focus_distance, Background::solid(Vec3()));
        if (cam.image_height() <= 0) throw std::invalid_argument("image height is zero");
        *out = cam.fields();
        return GS_OK;
    });
}

gs_status gs_host_render_spec(const gs_scene_spec* spec, const gs_camera_spec* c, const gs_sample_settings* ss,
                              uint64_t seed, float* out_rgb, gs_stats* stats) {
    if (!spec || !c || !ss || !out_rgb) return fail(GS_ERR_ARG, "null argument");
    return guarded([&]() {
        SpecBuilder b(*spec);
        auto world = b.world();
        Camera cam(c->aspect_ratio, c->image_width, SampleSettings{ss->confidence, ss->tolerance, ss->batch_size, ss->max_samples},
                   c->max_depth, c->v_fov, Vec3(c->look_from[0], c->look_from[1], c->look_from[2]),
                   Vec3(c->look_at[0], c->look_at[1], c->look_at[2]), Vec3(c->vup[0], c->vup[1], c->vup[2]),
                   c->defocus_angle, c->focus_distance, b.background());
        auto fs = flatten_world(*world, cam.background());
        return gs_render(&fs->view, &cam.fields(), &cam.settings(), seed, out_rgb, stats);
    });
}

gs_status gs_host_render_ppm_spec(const gs_scene_spec* spec, const gs_camera_spec* c, const gs_sample_settings* ss,
                                  uint64_t seed, char* out_text, int64_t text_capacity, int64_t* out_len,
                                  gs_stats* stats) {
    if (!spec || !c || !ss || !out_text || !out_len) return fail(GS_ERR_ARG, "null argument");
    return guarded([&]() {
        SpecBuilder b(*spec);
        auto world = b.world();
        Camera cam(c->aspect_ratio, c->image_width, SampleSettings{ss->confidence, ss->tolerance, ss->batch_size, ss->max_samples},
                   c->max_depth, c->v_fov, Vec3(c->look_from[0], c->look_from[1], c->look_from[2]),
                   Vec3(c->look_at[0], c->look_at[1], c->look_at[2]), Vec3(c->vup[0], c->vup[1], c->vup[2]),
                   c->defocus_angle, c->focus_distance, b.background());
        auto fs = flatten_world(*world, cam.background());
        return gs_render_ppm(&fs->view, &cam.fields(), &cam.settings(), seed, out_text, text_capacity, out_len,
                             stats);
    });
}

gs_status gs_host_write_ppm(const char* path, int32_t width, int32_t height, const float* rgb) {
    if (!path || !rgb || width <= 0 || height <= 0) return fail(GS_ERR_ARG, "bad argument");
    return guarded([&]() {
        std::ofstream f(path);
        if (!f) throw std::runtime_error(std::string("cannot open ") + path);
        write_ppm(f, width, height, rgb);
        return GS_OK;
    });
}

int32_t gs_host_color_byte(double linear) { return color_byte(linear); }

void gs_host_noise_permutation(uint32_t seed, uint8_t* out256) {
    if (out256) noise_permutation(seed, out256);
}

int64_t gs_host_bvh_topology(const gs_scene_spec* spec, int32_t* out, int64_t cap) {
    if (!spec) return -1;
    try {
        SpecBuilder b(*spec);
        auto world = b.world();
        Background bg = Background::solid(Vec3());
        auto fs = flatten_world(*world, bg);
        std::vector<int32_t> v;
        topo(fs->view, fs->view.root, 0, v);
        if (out)
            for (int64_t k = 0; k < (int64_t)v.size() && k < cap; k++) out[k] = v[k];
        return (int64_t)v.size();
    } catch (const std::exception& e) {
        gs_set_last_error(e.what());
        return -1;
    }
}

int64_t gs_host_struct_size(const char* name) {
    if (!name) return -1;
    const std::string n(name);
#define GS_SZ(T) if (n == #T) return (int64_t)sizeof(T);
    GS_SZ(gs_object) GS_SZ(gs_material_spec) GS_SZ(gs_texture_spec) GS_SZ(gs_image_spec)
    GS_SZ(gs_background_spec) GS_SZ(gs_scene_spec) GS_SZ(gs_camera_spec) GS_SZ(gs_sample_settings)
    GS_SZ(gs_counters) GS_SZ(gs_node) GS_SZ(gs_sphere) GS_SZ(gs_msphere) GS_SZ(gs_quad) GS_SZ(gs_triangle)
    GS_SZ(gs_list) GS_SZ(gs_instance) GS_SZ(gs_medium) GS_SZ(gs_material) GS_SZ(gs_texture) GS_SZ(gs_image)
    GS_SZ(gs_background) GS_SZ(gs_flat_scene) GS_SZ(gs_camera) GS_SZ(gs_partition)
    GS_SZ(gs_render_outputs) GS_SZ(gs_launch) GS_SZ(gs_multi_outputs) GS_SZ(gs_stats) GS_SZ(gs_scene_info)
#undef GS_SZ
    return -1;
}

}  // extern "C"
