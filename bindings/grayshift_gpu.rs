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
pub const GS_ABI_VERSION: i32 = 11;
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

/// The N-GPU render behind one call (ABI 4): devices, tiles, plan.
#[repr(C)] #[derive(Clone, Copy)]
pub struct gs_launch { pub num_gpus: i32, pub tile_w: i32, pub tile_h: i32, pub plan: i32, pub devices: *const i32 }

/// Host outputs of gs_render_multi (ABI 4): any subset of the linear frame, the
/// write_color bytes and the PPM text.
#[repr(C)]
pub struct gs_multi_outputs {
    pub rgb: *mut f32, pub rgb8: *mut u8, pub ppm_text: *mut c_char, pub ppm_capacity: i64, pub ppm_len: *mut i64,
}

/// What one frame did (SURVEY.md §5 metrics): every synchronous render call fills it (ABI 6).
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_stats {
    pub counters: gs_counters, pub setup_ms: f64, pub total_ms: f64, pub render_ms_max: f64, pub render_ms_min: f64,
    pub gather_ms: f64, pub algorithmic_bytes: u64, pub gathered_bytes: u64, pub num_gpus: i32, pub pad: i32,
    pub kernel_ms_max: f64, pub kernel_ms_min: f64,
}

/// The persistent N-GPU frame context (ABI 6, opaque).
#[repr(C)] pub struct gs_multi { _private: [u8; 0] }

/// What gs_device_scene_create built (ABI 5).
#[repr(C)] #[derive(Clone, Copy, Default)]
pub struct gs_scene_info {
    pub node_records: u32, pub leaf_records: u32, pub lds_nodes: u32, pub lds_leaves: u32, pub lds_quads: u32,
    pub feat: i32, pub node_steps: i32, pub cert_boxes: i32, pub nodes_per_leaf: f64, pub other_leaf_frac: f64,
    pub placement: i32, pub long_samples: i32, pub pilot_ms: f64,
}

#[link(name = "grayshift")]
extern "C" {
    pub fn gs_last_error() -> *const c_char;
    pub fn gs_version() -> i32;
    pub fn gs_set_tuning(shade_batch: i32, blocks_per_cu: i32, leaf_batch: i32, sample_chunk: i32) -> gs_status;
    pub fn gs_debug_set_partial_budget(bytes: u64) -> gs_status;
    pub fn gs_debug_set_guided_tail(fine_chunk: i32, tail_pct: i32) -> gs_status;
    pub fn gs_set_node_steps(node_steps: i32) -> gs_status;
    pub fn gs_set_camera_batch(cam_batch: i32) -> gs_status;
    pub fn gs_set_placement(mode: i32) -> gs_status;
    pub fn gs_set_adaptive_mode(mode: i32) -> gs_status;
    pub fn gs_debug_set_round_items(mode: i32) -> gs_status;
    pub fn gs_debug_set_cube_lists(on: i32) -> gs_status;
    pub fn gs_debug_record_visits(scene: *const gs_device_scene, cam: *const gs_camera, ss: *const gs_sample_settings,
                                  seed: u64, part: *const gs_partition, d_packed_rgb: *mut f32, d_visits: *mut u32,
                                  stream: *mut c_void) -> gs_status;
    pub fn gs_device_scene_create(scene: *const gs_flat_scene, out: *mut *mut gs_device_scene) -> gs_status;
    pub fn gs_device_scene_destroy(scene: *mut gs_device_scene) -> gs_status;
    pub fn gs_device_scene_info(scene: *const gs_device_scene, out: *mut gs_scene_info) -> gs_status;
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
    pub fn gs_device_download(host_dst: *mut c_void, d_src: *const c_void, bytes: i64) -> gs_status;
    pub fn gs_ppm_max_bytes(width: i32, height: i32) -> i64;
    pub fn gs_ppm_scratch_bytes(width: i32, height: i32) -> i64;
    pub fn gs_ppm_encode_async(d_rgb8: *const u8, width: i32, height: i32, d_text: *mut c_char, text_capacity: i64,
                               d_len: *mut i64, d_scratch: *mut c_void, scratch_bytes: i64,
                               stream: *mut c_void) -> gs_status;
    /// The whole of camera.rs:100-121 past the world build: PPM text into `out_text`.
    pub fn gs_render_ppm(scene: *const gs_flat_scene, cam: *const gs_camera, ss: *const gs_sample_settings, seed: u64,
                         out_text: *mut c_char, text_capacity: i64, out_len: *mut i64,
                         stats: *mut gs_stats) -> gs_status;
    /// The one-call replacement of camera.rs:105-114.
    pub fn gs_render(scene: *const gs_flat_scene, cam: *const gs_camera, ss: *const gs_sample_settings, seed: u64,
                     out_rgb: *mut f32, stats: *mut gs_stats) -> gs_status;
    /// camera.rs:105-114 (and, with ppm_text, :100-121) on the GPUs of one node, one RCCL gather.
    pub fn gs_render_multi(scene: *const gs_flat_scene, cam: *const gs_camera, ss: *const gs_sample_settings,
                           seed: u64, launch: *const gs_launch, out: *const gs_multi_outputs,
                           stats: *mut gs_stats) -> gs_status;
    pub fn gs_rccl_library() -> *const c_char;
    /// The persistent N-GPU context (ABI 6): upload + communicator once, then frames.
    pub fn gs_multi_create(scene: *const gs_flat_scene, launch: *const gs_launch, out: *mut *mut gs_multi) -> gs_status;
    pub fn gs_multi_render(m: *mut gs_multi, cam: *const gs_camera, ss: *const gs_sample_settings, seed: u64,
                           out: *const gs_multi_outputs, stats: *mut gs_stats) -> gs_status;
    pub fn gs_multi_frame(m: *const gs_multi, d_rgb: *mut *const f32, d_rgb8: *mut *const u8,
                          device: *mut i32) -> gs_status;
    pub fn gs_multi_devices(m: *const gs_multi, num_gpus: *mut i32, devices: *mut i32, capacity: i32) -> gs_status;
    pub fn gs_multi_scene(m: *const gs_multi, rank: i32, scene: *mut *const gs_device_scene) -> gs_status;
    pub fn gs_multi_destroy(m: *mut gs_multi) -> gs_status;
    pub fn gs_debug_set_multi_collective(always: i32) -> gs_status;
    pub fn gs_debug_set_multi_same_device(on: i32) -> gs_status;
}

pub fn last_error() -> String {
    unsafe { std::ffi::CStr::from_ptr(gs_last_error()).to_string_lossy().into_owned() }
}

/// `Camera::render` (camera.rs:100-121) on the device: flatten, render, write the
/// device-formatted PPM text with one call.  `flat`, `cam` and `ss` come from the
/// crate's `flatten` trait method and `Camera::new`.
pub fn render_ppm(flat: &gs_flat_scene, cam: &gs_camera, ss: &gs_sample_settings, seed: u64,
                  out: &mut impl std::io::Write) -> std::io::Result<gs_stats> {
    let cap = unsafe { gs_ppm_max_bytes(cam.image_width, cam.image_height) };
    if cap < 0 { return Err(std::io::Error::new(std::io::ErrorKind::InvalidInput, "bad image size")); }
    let mut text = vec![0u8; cap as usize];
    let mut len: i64 = 0;
    let mut stats = gs_stats::default();
    let st = unsafe { gs_render_ppm(flat, cam, ss, seed, text.as_mut_ptr() as *mut c_char, cap, &mut len, &mut stats) };
    if st != GS_OK { return Err(std::io::Error::new(std::io::ErrorKind::Other, last_error())); }
    out.write_all(&text[..len as usize])?;
    Ok(stats)
}

/// Many frames of one world on `num_gpus` GPUs (an animation, a benchmark): the scene
/// upload and the RCCL communicator happen once in `new`, each `frame` is one call.
pub struct Frames { ctx: *mut gs_multi }

impl Frames {
    pub fn new(flat: &gs_flat_scene, num_gpus: i32) -> std::io::Result<Frames> {
        let launch = gs_launch { num_gpus, tile_w: 64, tile_h: 64, plan: 1, devices: std::ptr::null() };
        let mut ctx: *mut gs_multi = std::ptr::null_mut();
        let st = unsafe { gs_multi_create(flat, &launch, &mut ctx) };
        if st != GS_OK { return Err(std::io::Error::new(std::io::ErrorKind::Other, last_error())); }
        Ok(Frames { ctx })
    }
    /// One frame's linear colour (W*H*3 f32) into `rgb`.
    pub fn frame(&mut self, cam: &gs_camera, ss: &gs_sample_settings, seed: u64, rgb: &mut [f32]) -> std::io::Result<gs_stats> {
        if rgb.len() < (cam.image_width as usize) * (cam.image_height as usize) * 3 {
            return Err(std::io::Error::new(std::io::ErrorKind::InvalidInput, "rgb buffer too small"));
        }
        let outs = gs_multi_outputs { rgb: rgb.as_mut_ptr(), rgb8: std::ptr::null_mut(), ppm_text: std::ptr::null_mut(),
                                      ppm_capacity: 0, ppm_len: std::ptr::null_mut() };
        let mut stats = gs_stats::default();
        let st = unsafe { gs_multi_render(self.ctx, cam, ss, seed, &outs, &mut stats) };
        if st != GS_OK { return Err(std::io::Error::new(std::io::ErrorKind::Other, last_error())); }
        Ok(stats)
    }
}

impl Drop for Frames {
    fn drop(&mut self) { unsafe { gs_multi_destroy(self.ctx); } }
}

/// `Camera::render` (camera.rs:100-121) on `num_gpus` GPUs of this node (0 = all): the
/// tiles are rendered concurrently and gathered over RCCL, the PPM text is formatted on
/// the first device and written with one call.  Same bytes as `render_ppm`.
pub fn render_ppm_multi(flat: &gs_flat_scene, cam: &gs_camera, ss: &gs_sample_settings, seed: u64, num_gpus: i32,
                        out: &mut impl std::io::Write) -> std::io::Result<gs_stats> {
    let cap = unsafe { gs_ppm_max_bytes(cam.image_width, cam.image_height) };
    if cap < 0 { return Err(std::io::Error::new(std::io::ErrorKind::InvalidInput, "bad image size")); }
    let mut text = vec![0u8; cap as usize];
    let mut len: i64 = 0;
    let launch = gs_launch { num_gpus, tile_w: 64, tile_h: 64, plan: 1, devices: std::ptr::null() };
    let outs = gs_multi_outputs { rgb: std::ptr::null_mut(), rgb8: std::ptr::null_mut(),
                                  ppm_text: text.as_mut_ptr() as *mut c_char, ppm_capacity: cap, ppm_len: &mut len };
    let mut stats = gs_stats::default();
    let st = unsafe { gs_render_multi(flat, cam, ss, seed, &launch, &outs, &mut stats) };
    if st != GS_OK { return Err(std::io::Error::new(std::io::ErrorKind::Other, last_error())); }
    out.write_all(&text[..len as usize])?;
    Ok(stats)
}

// ---------------------------------------------------------------------------------
// Flattening: the one method the reference's traits gain.
//
// `SceneBuilder` collects the flat arrays of gs_flat_scene the way the C++ host's
// `Flattener` does (grayshift_amd/csrc/host/world.cpp): every `Hittable::flatten` appends
// its record(s) and returns a tagged ref; a `BVHNode` reserves its slot first, so nodes
// land in pre-order; materials / textures / images are deduplicated by identity (hash
// maps keyed by the `Arc` pointer: O(1) per lookup, so a million-sphere world flattens in
// linear time) and reserve their slot before flattening their children.

pub const GS_MAT_LAMBERTIAN: u32 = 1;
pub const GS_MAT_METAL: u32 = 2;
pub const GS_MAT_DIELECTRIC: u32 = 3;
pub const GS_MAT_DIFFUSE_LIGHT: u32 = 4;
pub const GS_MAT_ISOTROPIC: u32 = 5;
pub const GS_TEX_SOLID: u32 = 1;
pub const GS_TEX_CHECKERED: u32 = 2;
pub const GS_TEX_IMAGE: u32 = 3;
pub const GS_TEX_NOISE: u32 = 4;
pub const GS_BG_SOLID: u32 = 1;
pub const GS_BG_HDRI: u32 = 2;

use std::collections::HashMap;

#[derive(Default)]
pub struct SceneBuilder {
    pub nodes: Vec<gs_node>,
    pub spheres: Vec<gs_sphere>,
    pub mspheres: Vec<gs_msphere>,
    pub quads: Vec<gs_quad>,
    pub triangles: Vec<gs_triangle>,
    pub lists: Vec<gs_list>,
    pub list_refs: Vec<u32>,
    pub instances: Vec<gs_instance>,
    pub media: Vec<gs_medium>,
    pub materials: Vec<gs_material>,
    pub textures: Vec<gs_texture>,
    pub images: Vec<gs_image>,
    pub texels8: Vec<u8>,
    pub noise_perm: Vec<u8>,
    mat_slot: HashMap<usize, u32>,
    tex_slot: HashMap<usize, u32>,
    img_slot: HashMap<(usize, u32, u32), u32>,
    depth: u32,
    pub max_depth: u32,
}

/// A flattened world plus the storage its view points into (keep it alive while the
/// view is used).
pub struct FlatScene {
    pub builder: SceneBuilder,
    pub hdri_rgb: Vec<f32>,
    pub view: gs_flat_scene,
}

impl SceneBuilder {
    /// `BVHNode::flatten`: reserve the node (pre-order), flatten the children, fill the box.
    /// `left` / `right` flatten the children (right: `None` for the n == 1 wrapper, BVH.rs:20-28).
    pub fn node(&mut self, bbox_min: [f64; 3], bbox_max: [f64; 3],
                left: impl FnOnce(&mut SceneBuilder) -> u32,
                right: Option<&dyn Fn(&mut SceneBuilder) -> u32>) -> u32 {
        let idx = self.nodes.len() as u32;
        self.nodes.push(gs_node::default());
        self.depth += 1;
        self.max_depth = self.max_depth.max(self.depth);
        let l = left(self);
        let r = match right { Some(f) => f(self), None => GS_REF_NONE };
        self.depth -= 1;
        let n = &mut self.nodes[idx as usize];
        n.min = bbox_min;
        n.max = bbox_max;
        n.left = l;
        n.right = r;
        gs_make_ref(GS_REF_NODE, idx)
    }
    pub fn sphere(&mut self, center: [f64; 3], radius: f64, material: u32) -> u32 {
        self.spheres.push(gs_sphere { center, radius, material, pad: 0 });
        gs_make_ref(GS_REF_SPHERE, self.spheres.len() as u32 - 1)
    }
    pub fn moving_sphere(&mut self, center_start: [f64; 3], center_path: [f64; 3], radius: f64, material: u32) -> u32 {
        self.mspheres.push(gs_msphere { center_start, center_path, radius, material, pad: 0 });
        gs_make_ref(GS_REF_MSPHERE, self.mspheres.len() as u32 - 1)
    }
    /// `Quad::flatten` (quad.rs:12-38): q, u, v plus the derived w, normal and plane d.
    pub fn quad(&mut self, q: [f64; 3], u: [f64; 3], v: [f64; 3], w: [f64; 3], normal: [f64; 3], d: f64,
                material: u32) -> u32 {
        self.quads.push(gs_quad { q, u, v, w, normal, d, material, pad: 0 });
        gs_make_ref(GS_REF_QUAD, self.quads.len() as u32 - 1)
    }
    pub fn triangle(&mut self, a: [f64; 3], b: [f64; 3], c: [f64; 3], normal: [f64; 3], material: u32) -> u32 {
        self.triangles.push(gs_triangle { a, b, c, normal, material, pad: 0 });
        gs_make_ref(GS_REF_TRIANGLE, self.triangles.len() as u32 - 1)
    }
    /// `HittableList::flatten`: its members' refs (primitives only on the device path).
    pub fn list(&mut self, member_refs: &[u32]) -> u32 {
        let first = self.list_refs.len() as u32;
        self.list_refs.extend_from_slice(member_refs);
        self.lists.push(gs_list { first, count: member_refs.len() as u32 });
        gs_make_ref(GS_REF_LIST, self.lists.len() as u32 - 1)
    }
    /// `Translate::flatten` / `RotateY::flatten`: reserve (outer before inner), then the child.
    pub fn instance(&mut self, kind: u32, p: [f64; 3], child: impl FnOnce(&mut SceneBuilder) -> u32) -> u32 {
        let idx = self.instances.len();
        self.instances.push(gs_instance::default());
        let c = child(self);
        self.instances[idx] = gs_instance { kind, child: c, p };
        gs_make_ref(GS_REF_INSTANCE, idx as u32)
    }
    /// `ConstantMedium::flatten` (volume.rs:10-29).
    pub fn medium(&mut self, density: f64, boundary: impl FnOnce(&mut SceneBuilder) -> u32, phase: u32) -> u32 {
        let idx = self.media.len();
        self.media.push(gs_medium::default());
        let b = boundary(self);
        self.media[idx] = gs_medium { boundary: b, material: phase, density_neg_inv: -1.0 / density };
        gs_make_ref(GS_REF_MEDIUM, idx as u32)
    }
    /// The material slot of `key` (the `Arc<dyn Material>` pointer): found, or reserved
    /// and filled by `fill` (which may flatten textures first).
    pub fn material_index(&mut self, key: *const (), fill: impl FnOnce(&mut SceneBuilder) -> gs_material) -> u32 {
        if let Some(&i) = self.mat_slot.get(&(key as usize)) { return i; }
        let i = self.materials.len() as u32;
        self.mat_slot.insert(key as usize, i);
        self.materials.push(gs_material::default());
        let m = fill(self);
        self.materials[i as usize] = m;
        i
    }
    pub fn texture_index(&mut self, key: *const (), fill: impl FnOnce(&mut SceneBuilder) -> gs_texture) -> u32 {
        if let Some(&i) = self.tex_slot.get(&(key as usize)) { return i; }
        let i = self.textures.len() as u32;
        self.tex_slot.insert(key as usize, i);
        self.textures.push(gs_texture::default());
        let t = fill(self);
        self.textures[i as usize] = t;
        i
    }
    /// One image per distinct texel buffer (RGB8, row-major, top row first).
    pub fn image_index(&mut self, rgb8: &[u8], width: u32, height: u32) -> u32 {
        let key = (rgb8.as_ptr() as usize, width, height);
        if let Some(&i) = self.img_slot.get(&key) { return i; }
        let offset = self.texels8.len() as u64;
        self.texels8.extend_from_slice(rgb8);
        self.images.push(gs_image { width, height, offset });
        let i = self.images.len() as u32 - 1;
        self.img_slot.insert(key, i);
        i
    }
    /// Close the world: `root` from `world.flatten`, the background (camera.rs:246-249;
    /// for HDRI, `rot` = rotate_vector's coefficients and `hdri_rgb` the f32 texels).
    pub fn finish(self, root: u32, background: gs_background, hdri_rgb: Vec<f32>) -> FlatScene {
        let mut fs = FlatScene { builder: self, hdri_rgb, view: unsafe { std::mem::zeroed() } };
        let b = &fs.builder;
        fs.view = gs_flat_scene {
            root, max_bvh_depth: b.max_depth,
            nodes: b.nodes.as_ptr(), n_nodes: b.nodes.len() as u32,
            spheres: b.spheres.as_ptr(), n_spheres: b.spheres.len() as u32,
            mspheres: b.mspheres.as_ptr(), n_mspheres: b.mspheres.len() as u32,
            quads: b.quads.as_ptr(), n_quads: b.quads.len() as u32,
            triangles: b.triangles.as_ptr(), n_triangles: b.triangles.len() as u32,
            lists: b.lists.as_ptr(), n_lists: b.lists.len() as u32,
            list_refs: b.list_refs.as_ptr(), n_list_refs: b.list_refs.len() as u32,
            instances: b.instances.as_ptr(), n_instances: b.instances.len() as u32,
            materials: b.materials.as_ptr(), n_materials: b.materials.len() as u32,
            textures: b.textures.as_ptr(), n_textures: b.textures.len() as u32,
            images: b.images.as_ptr(), n_images: b.images.len() as u32,
            texels8: b.texels8.as_ptr(), n_texels8: b.texels8.len() as u64,
            background,
            hdri_rgb: fs.hdri_rgb.as_ptr(), n_hdri_floats: fs.hdri_rgb.len() as u64,
            media: b.media.as_ptr(), n_media: b.media.len() as u32,
            noise_perm: if b.noise_perm.is_empty() { std::ptr::null() } else { b.noise_perm.as_ptr() },
            n_noise_perm: b.noise_perm.len() as u32,
        };
        fs
    }
}
