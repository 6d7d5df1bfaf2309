/*
 * grayshift_scene.h — the scene *description* both sides of the parity check consume.
 *
 * A gs_scene_spec is the neutral, plain-C statement of what the reference's scene
 * builders (src/main.rs:61-888) construct: the objects added to the world
 * `HittableList` (hittable/hittable.rs:63-66), their materials (material.rs),
 * textures (texture.rs), the background (camera.rs:246-255) and the camera
 * arguments (camera.rs:39-51).  It carries no BVH and no derived data: the
 * product host (grayshift_amd/csrc/host) and the CPU oracle (oracle/) each build
 * their own world, BVH and camera from it, independently.
 *
 * All arrays are caller-owned and only read during a call.
 */
#ifndef GRAYSHIFT_SCENE_H
#define GRAYSHIFT_SCENE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Object kinds.  p[] layout per kind is given beside each. */
enum gs_obj_kind {
    GS_OBJ_SPHERE        = 1, /* Sphere::new_stationary  sphere.rs:21   p: center[3], radius                 */
    GS_OBJ_MOVING_SPHERE = 2, /* Sphere::new_moving      sphere.rs:35   p: center1[3], center2[3], radius     */
    GS_OBJ_QUAD          = 3, /* Quad::new               quad.rs:25     p: q[3], u[3], v[3]                  */
    GS_OBJ_TRIANGLE      = 4, /* Triangle::new           triangle.rs:20 p: a[3], b[3], c[3]                  */
    GS_OBJ_LIST          = 5, /* HittableList            hittable.rs:45 children[first .. first+count)       */
    GS_OBJ_BVH           = 6, /* BVHNode::from_list      BVH.rs:15      children[first .. first+count)       */
    GS_OBJ_TRANSLATE     = 7, /* Translate::new          hittable.rs:99 child = first; p: offset[3]          */
    GS_OBJ_ROTATE_Y      = 8, /* RotateY::new            hittable.rs:135 child = first; p: angle (degrees)   */
    GS_OBJ_CUBE          = 9, /* Quad::cube              quad.rs:54     p: point_a[3], point_b[3] (a list)   */
    GS_OBJ_MEDIUM        = 10 /* ConstantMedium::new     volume.rs:17   boundary = first, phase function =
                                 material; p: density                                                      */
};

typedef struct gs_object {
    int32_t kind;      /* gs_obj_kind */
    int32_t material;  /* index into materials (primitives and cubes); -1 otherwise */
    int32_t first;     /* LIST/BVH: first index into children[]; TRANSLATE/ROTATE_Y: child object */
    int32_t count;     /* LIST/BVH: number of children */
    double  p[9];
} gs_object;

enum gs_mat_kind {
    GS_MAT_LAMBERTIAN    = 1, /* material.rs:29  texture                        */
    GS_MAT_METAL         = 2, /* material.rs:75  p: albedo[3], fuzz             */
    GS_MAT_DIELECTRIC    = 3, /* material.rs:105 p: refraction_index            */
    GS_MAT_DIFFUSE_LIGHT = 4, /* material.rs:151 texture                        */
    GS_MAT_ISOTROPIC     = 5  /* material.rs:171 texture (phase function of a ConstantMedium) */
};

typedef struct gs_material_spec {
    int32_t kind;     /* gs_mat_kind */
    int32_t texture;  /* index into textures; -1 for METAL / DIELECTRIC */
    double  p[4];
} gs_material_spec;

enum gs_tex_kind {
    GS_TEX_SOLID     = 1, /* texture.rs:13  p: albedo[3]                               */
    GS_TEX_CHECKERED = 2, /* texture.rs:33  a = even texture, b = odd texture, p[0] = scale */
    GS_TEX_IMAGE     = 3, /* texture.rs:73  a = image index                            */
    GS_TEX_NOISE     = 4  /* texture.rs:97  p[0] = scale; Perlin::default() (noise 0.9) */
};

typedef struct gs_texture_spec {
    int32_t kind;  /* gs_tex_kind */
    int32_t a, b;
    int32_t pad;
    double  p[3];
} gs_texture_spec;

/* 8-bit RGB image, row-major, top row first (what image::open yields for earthmap.jpg). */
typedef struct gs_image_spec {
    int32_t width, height;
    const uint8_t* rgb8; /* width*height*3 bytes */
} gs_image_spec;

enum gs_bg_kind {
    GS_BG_SOLID = 1, /* Background::SOLID(color)      camera.rs:247 */
    GS_BG_HDRI  = 2  /* Background::HDRI(HDRI)        camera.rs:248 */
};

typedef struct gs_background_spec {
    int32_t kind;          /* gs_bg_kind */
    int32_t width, height; /* HDRI size */
    int32_t pad;
    double  color[3];      /* SOLID */
    double  rotation[3];   /* HDRI::rotation, radians as the reference passes them (camera.rs:252) */
    const float* rgb;      /* HDRI texels, f32 RGB, row-major top-down (radiant::Image) */
} gs_background_spec;

typedef struct gs_scene_spec {
    const gs_object* objects;           int32_t n_objects;
    const int32_t* children;            int32_t n_children; /* object indices for LIST/BVH */
    const int32_t* world;               int32_t n_world;    /* top-level HittableList, add() order */
    const gs_material_spec* materials;  int32_t n_materials;
    const gs_texture_spec* textures;    int32_t n_textures;
    const gs_image_spec* images;        int32_t n_images;
    gs_background_spec background;
} gs_scene_spec;

/* Camera::new arguments (camera.rs:39-51), minus SampleSettings and Background. */
typedef struct gs_camera_spec {
    double   aspect_ratio;
    int32_t  image_width;
    uint32_t max_depth;
    double   v_fov;
    double   look_from[3];
    double   look_at[3];
    double   vup[3];
    double   defocus_angle;
    double   focus_distance;
} gs_camera_spec;

/* SampleSettings (camera.rs:239-244). Fixed spp = {tol 0, batch spp, max spp-1}. */
typedef struct gs_sample_settings {
    double   confidence;
    double   tolerance;
    uint32_t batch_size;
    uint32_t max_samples;
} gs_sample_settings;

/* Work counters.  Identical definitions on the oracle and on the device; they
 * define the algorithmic bytes of DESIGN.md §4. */
typedef struct gs_counters {
    uint64_t rays;            /* world.hit calls               camera.rs:177 */
    uint64_t node_visits;     /* AABB::hit calls on BVH nodes  BVH.rs:70     */
    uint64_t sphere_tests;    /* Sphere::hit (stationary)      sphere.rs:64  */
    uint64_t msphere_tests;   /* Sphere::hit (moving)                        */
    uint64_t quad_tests;      /* Quad::hit                     quad.rs:84    */
    uint64_t tri_tests;       /* Triangle::hit                 triangle.rs:34*/
    uint64_t instance_tests;  /* Translate::hit + RotateY::hit               */
    uint64_t list_tests;      /* HittableList::hit                           */
    uint64_t hits;            /* rays that hit (material record read)        */
    uint64_t image_texels;    /* ImageTexture::value_at        texture.rs:84 */
    uint64_t hdri_texels;     /* HDRI::sample                  camera.rs:257 */
    uint64_t paths;           /* camera samples (get_ray calls)              */
    uint64_t pixels;          /* pixels finished                             */
    uint64_t medium_tests;    /* ConstantMedium::hit           volume.rs:32  */
    uint64_t noise_evals;     /* NoiseTexture::value_at        texture.rs:127 */
    uint64_t reserved[1];
} gs_counters;

#ifdef __cplusplus
}
#endif
#endif /* GRAYSHIFT_SCENE_H */
