//! Rust FFI binding of include/grayshift_gpu.h — what the reference crate
//! (benjisu03/grayshift) would add to call the MI355X path from `Camera::render`
//! (src/camera.rs:100).  Documentation of the drop-in: not compiled in this image
//! (no Rust toolchain); the layouts mirror the C header field for field and are
//! checked against it from Python (tests/test_host.py::test_struct_layouts_match).
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_void};

pub type gs_status = i32;
pub const GS_OK: gs_status = 0;
pub const GS_ERR_ARG: gs_status = -1;
pub const GS_ERR_HIP: gs_status = -2;
pub const GS_ERR_OOM: gs_status = -3;
pub const GS_ERR_UNSUPPORTED: gs_status = -4;
pub const GS_ERR_NO_DEVICE: gs_status = -5;

pub const GS_REF_SHIFT: u32 = 28;
pub const GS_REF_NONE: u32 = 0;
pub const GS_REF_NODE: u32 = 1;
pub const GS_REF_SPHERE: u32 = 2;
pub const GS_REF_MSPHERE: u32 = 3;
pub const GS_REF_QUAD: u32 = 4;
pub const GS_REF_TRIANGLE: u32 = 5;
pub const GS_REF_LIST: u32 = 6;
pub const GS_REF_INSTANCE: u32 = 7;
pub const GS_REF_MEDIUM: u32 = 8;
pub const GS_ABI_VERSION: i32 = 3;
pub const fn gs_make_ref(kind: u32, idx: u32) -> u32 { (kind << GS_REF_SHIFT) | (idx & 0x0FFF_FFFF) }

#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_node { pub min: [f64; 3], pub max: [f64; 3], pub left: u32, pub right: u32, pub pad: [u32; 2] }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_sphere { pub center: [f64; 3], pub radius: f64, pub material: u32, pub pad: u32 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_msphere { pub center_start: [f64; 3], pub center_path: [f64; 3], pub radius: f64, pub material: u32, pub pad: u32 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_quad { pub q: [f64; 3], pub u: [f64; 3], pub v: [f64; 3], pub w: [f64; 3], pub normal: [f64; 3], pub d: f64, pub material: u32, pub pad: u32 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_triangle { pub a: [f64; 3], pub b: [f64; 3], pub c: [f64; 3], pub normal: [f64; 3], pub material: u32, pub pad: u32 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_list { pub first: u32, pub count: u32 }
pub const GS_INST_TRANSLATE: u32 = 1;
pub const GS_INST_ROTATE_Y: u32 = 2;
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_instance { pub kind: u32, pub child: u32, pub p: [f64; 3] }
/// ConstantMedium (hittable/volume.rs:10-29) (ABI 2).
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_medium { pub boundary: u32, pub material: u32, pub density_neg_inv: f64 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_material { pub kind: u32, pub texture: u32, pub albedo: [f64; 3], pub param: f64 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_texture { pub kind: u32, pub even: u32, pub odd: u32, pub image: u32, pub color: [f64; 3], pub scale_inv: f64 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_image { pub width: u32, pub height: u32, pub offset: u64 }
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_background { pub kind: u32, pub width: u32, pub height: u32, pub pad: u32, pub color: [f64; 3], pub rot: [f64; 9] }

#[repr(C)]
pub struct gs_flat_scene {
    pub root: u32, pub max_bvh_depth: u32,
    pub nodes: *const gs_node, pub n_nodes: u32,
    pub spheres: *const gs_sphere, pub n_spheres: u32,
    pub mspheres: *const gs_msphere, pub n_mspheres: u32,
    pub quads: *const gs_quad, pub n_quads: u32,
    pub triangles: *const gs_triangle, pub n_triangles: u32,
    pub lists: *const gs_list, pub n_lists: u32,
    pub list_refs: *const u32, pub n_list_refs: u32,
    pub instances: *const gs_instance, pub n_instances: u32,
    pub materials: *const gs_material, pub n_materials: u32,
    pub textures: *const gs_texture, pub n_textures: u32,
    pub images: *const gs_image, pub n_images: u32,
    pub texels8: *const u8, pub n_texels8: u64,
    pub background: gs_background,
    pub hdri_rgb: *const f32, pub n_hdri_floats: u64,
    pub media: *const gs_medium, pub n_media: u32,
    pub noise_perm: *const u8, pub n_noise_perm: u32,
}

/// The fields `Camera::new` derives (camera.rs:17-98).
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_camera {
    pub image_width: i32, pub image_height: i32, pub max_depth: u32, pub pad: u32,
    pub center: [f64; 3], pub starting_pixel_pos: [f64; 3],
    pub pixel_delta_u: [f64; 3], pub pixel_delta_v: [f64; 3],
    pub defocus_angle: f64, pub defocus_disk_u: [f64; 3], pub defocus_disk_v: [f64; 3],
}

/// SampleSettings (camera.rs:239-244).
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_sample_settings { pub confidence: f64, pub tolerance: f64, pub batch_size: u32, pub max_samples: u32 }

#[repr(C)] #[derive(Clone, Copy)]
pub struct gs_partition {
    pub rank: i32, pub world_size: i32, pub tile_w: i32, pub tile_h: i32,
    pub d_tile_order: *const i32, pub slots_per_rank: i32, pub pad: i32,
}

#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_counters {
    pub rays: u64, pub node_visits: u64, pub sphere_tests: u64, pub msphere_tests: u64,
    pub quad_tests: u64, pub tri_tests: u64, pub instance_tests: u64, pub list_tests: u64,
    pub hits: u64, pub image_texels: u64, pub hdri_texels: u64, pub paths: u64, pub pixels: u64,
    pub medium_tests: u64, pub noise_evals: u64, pub reserved: [u64; 1],
}

/// Outputs of one launch (ABI 3): either or both of the linear f32 colour and
/// write_color's bytes of the f64 colour, per packed pixel.
#[repr(C)]
pub struct gs_render_outputs { pub rgb: *mut f32, pub rgb8: *mut u8, pub item_visits: *mut u32 }

#[repr(C)] pub struct gs_device_scene { _private: [u8; 0] }

#[link(name = "grayshift")]
extern "C" {
    pub fn gs_last_error() -> *const c_char;
    pub fn gs_version() -> i32;
    pub fn gs_set_tuning(shade_batch: i32, blocks_per_cu: i32, leaf_batch: i32, sample_chunk: i32) -> gs_status;
    pub fn gs_device_scene_create(scene: *const gs_flat_scene, out: *mut *mut gs_device_scene) -> gs_status;
    pub fn gs_device_scene_destroy(scene: *mut gs_device_scene) -> gs_status;
    pub fn gs_partition_capacity(cam: *const gs_camera, part: *const gs_partition) -> i64;
    pub fn gs_render_tiles_async(scene: *const gs_device_scene, cam: *const gs_camera, ss: *const gs_sample_settings,
                                 seed: u64, part: *const gs_partition, d_packed_rgb: *mut f32,
                                 d_counters: *mut gs_counters, stream: *mut c_void) -> gs_status;
    pub fn gs_render_tiles_debug_async(scene: *const gs_device_scene, cam: *const gs_camera,
                                       ss: *const gs_sample_settings, seed: u64, part: *const gs_partition,
                                       d_packed_rgb: *mut f32, d_counters: *mut gs_counters,
                                       d_item_visits: *mut u32, stream: *mut c_void) -> gs_status;
    pub fn gs_unpack_tiles_async(cam: *const gs_camera, world_size: i32, tile_w: i32, tile_h: i32, capacity: i64,
                                 d_gathered: *const f32, d_frame: *mut f32, stream: *mut c_void) -> gs_status;
    pub fn gs_render_tiles_ex_async(scene: *const gs_device_scene, cam: *const gs_camera,
                                    ss: *const gs_sample_settings, seed: u64, part: *const gs_partition,
                                    out: *const gs_render_outputs, d_counters: *mut gs_counters,
                                    stream: *mut c_void) -> gs_status;
    pub fn gs_unpack_tiles_u8_async(cam: *const gs_camera, world_size: i32, tile_w: i32, tile_h: i32, capacity: i64,
                                    d_gathered: *const u8, d_frame: *mut u8, stream: *mut c_void) -> gs_status;
    pub fn gs_plan_tiles(scene: *const gs_device_scene, cam: *const gs_camera, seed: u64, world_size: i32,
                         tile_w: i32, tile_h: i32, order_out: *mut i32, order_cap: i64,
                         slots_per_rank: *mut i32) -> gs_status;
    pub fn gs_unpack_tiles_part_async(cam: *const gs_camera, part: *const gs_partition, capacity: i64,
                                      d_gathered: *const c_void, d_frame: *mut c_void, elem_bytes: i32,
                                      stream: *mut c_void) -> gs_status;
    pub fn gs_device_alloc(bytes: i64, d_out: *mut *mut c_void) -> gs_status;
    pub fn gs_device_free(d_ptr: *mut c_void) -> gs_status;
    pub fn gs_device_upload(d_dst: *mut c_void, host_src: *const c_void, bytes: i64) -> gs_status;
    pub fn gs_ppm_max_bytes(width: i32, height: i32) -> i64;
    pub fn gs_ppm_scratch_bytes(width: i32, height: i32) -> i64;
    pub fn gs_ppm_encode_async(d_rgb8: *const u8, width: i32, height: i32, d_text: *mut c_char, text_capacity: i64,
                               d_len: *mut i64, d_scratch: *mut c_void, scratch_bytes: i64,
                               stream: *mut c_void) -> gs_status;
    /// The whole of camera.rs:100-121 past the world build: PPM text into `out_text`.
    pub fn gs_render_ppm(scene: *const gs_flat_scene, cam: *const gs_camera, ss: *const gs_sample_settings, seed: u64,
                         out_text: *mut c_char, text_capacity: i64, out_len: *mut i64,
                         counters: *mut gs_counters) -> gs_status;
    /// The one-call replacement of camera.rs:105-114.
    pub fn gs_render(scene: *const gs_flat_scene, cam: *const gs_camera, ss: *const gs_sample_settings, seed: u64,
                     out_rgb: *mut f32, counters: *mut gs_counters) -> gs_status;
}

pub fn last_error() -> String {
    unsafe { std::ffi::CStr::from_ptr(gs_last_error()).to_string_lossy().into_owned() }
}

/// `Camera::render` (camera.rs:100-121) on the device: flatten, render, write the
/// device-formatted PPM text with one call.  `flat`, `cam` and `ss` come from the
/// crate's `flatten` trait method and `Camera::new`.
pub fn render_ppm(flat: &gs_flat_scene, cam: &gs_camera, ss: &gs_sample_settings, seed: u64,
                  out: &mut impl std::io::Write) -> std::io::Result<()> {
    let cap = unsafe { gs_ppm_max_bytes(cam.image_width, cam.image_height) };
    if cap < 0 { return Err(std::io::Error::new(std::io::ErrorKind::InvalidInput, "bad image size")); }
    let mut text = vec![0u8; cap as usize];
    let mut len: i64 = 0;
    let st = unsafe {
        gs_render_ppm(flat, cam, ss, seed, text.as_mut_ptr() as *mut c_char, cap, &mut len, std::ptr::null_mut())
    };
    if st != GS_OK { return Err(std::io::Error::new(std::io::ErrorKind::Other, last_error())); }
    out.write_all(&text[..len as usize])
}
