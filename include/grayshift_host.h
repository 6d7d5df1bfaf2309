/*
 * grayshift_host.h — C-ABI of the C++ host mirror (grayshift_amd/csrc/host).
 *
 * The reference's host is Rust (src/main.rs scene builders + Camera).  No Rust
 * toolchain exists in this image, so the host side above the device boundary
 * (grayshift_gpu.h) is C++ mirroring the reference's types; this header exposes it
 * to Python (ctypes) and to any C caller.  A scene is given as a gs_scene_spec
 * (grayshift_scene.h) — the objects main.rs adds to the world — and the host builds
 * the world objects, `BVHNode::from_list(world)`, and the flat arrays, exactly as the
 * Rust host would before calling gs_render.
 */
#ifndef GRAYSHIFT_HOST_H
#define GRAYSHIFT_HOST_H

#include "grayshift_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gs_host_scene gs_host_scene; /* world + BVH + flat arrays (host memory) */

/* Build the world from a spec: objects, BVHNode::from_list(world), flatten. */
gs_status gs_host_scene_from_spec(const gs_scene_spec* spec, gs_host_scene** out);
gs_status gs_host_scene_destroy(gs_host_scene* scene);
/* View of the flattened arrays (valid while the scene lives). */
const gs_flat_scene* gs_host_scene_flat(const gs_host_scene* scene);

/* Camera::new (camera.rs:39-98): the derived fields the device needs. */
gs_status gs_host_camera(const gs_camera_spec* spec, gs_camera* out);

/* Camera::render minus the PPM stage: spec -> world -> BVH -> flat -> gs_render.
 * out_rgb: host W*H*3 f32 linear.  stats: host, nullable (ABI 6: was gs_counters*). */
gs_status gs_host_render_spec(const gs_scene_spec* spec, const gs_camera_spec* cam, const gs_sample_settings* ss,
                              uint64_t seed, float* out_rgb, gs_stats* stats);

/* The whole of Camera::render (camera.rs:100-121): spec -> world -> BVH -> flat ->
 * gs_render_ppm.  out_text: host, >= gs_ppm_max_bytes(W, H); *out_len = text length. */
gs_status gs_host_render_ppm_spec(const gs_scene_spec* spec, const gs_camera_spec* cam, const gs_sample_settings* ss,
                                  uint64_t seed, char* out_text, int64_t text_capacity, int64_t* out_len,
                                  gs_stats* stats);

/* Camera::render output stage on the host, from an f32 frame (camera.rs:101-103,116-118; color.rs:8-18). */
gs_status gs_host_write_ppm(const char* path, int32_t width, int32_t height, const float* rgb);
int32_t gs_host_color_byte(double linear);

/* BVH topology of the built world, pre-order: per BVH node (1, depth) then its left
 * subtree then its right subtree (or (0, depth+1) when absent); per non-node (-1, depth).
 * Returns the number of int32 written (or needed when out is NULL), -1 on error. */
int64_t gs_host_bvh_topology(const gs_scene_spec* spec, int32_t* out, int64_t cap);

/* noise 0.9 PermutationTable::new(seed) as the host generates it for NoiseTexture. */
void gs_host_noise_permutation(uint32_t seed, uint8_t* out256);

/* sizeof() of a public struct by name ("gs_object", "gs_camera", ...), for FFI
 * mirrors to check their layout; -1 if unknown. */
int64_t gs_host_struct_size(const char* name);

#ifdef __cplusplus
}
#endif
#endif /* GRAYSHIFT_HOST_H */
