"""ctypes mirror of include/grayshift_scene.h, grayshift_gpu.h and grayshift_host.h.

Loads the in-tree ``libgrayshift.so``.  There is no fallback: if the library is
missing or fails to load, importing this module raises — the product path is the
HIP extension or nothing.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GS_LIB") or os.path.join(HERE, "libgrayshift.so")  # GS_LIB: A/B variant builds

# ------------------------------------------------------------------ enums
GS_OBJ_SPHERE, GS_OBJ_MOVING_SPHERE, GS_OBJ_QUAD, GS_OBJ_TRIANGLE = 1, 2, 3, 4
GS_OBJ_LIST, GS_OBJ_BVH, GS_OBJ_TRANSLATE, GS_OBJ_ROTATE_Y, GS_OBJ_CUBE, GS_OBJ_MEDIUM = 5, 6, 7, 8, 9, 10
GS_MAT_LAMBERTIAN, GS_MAT_METAL, GS_MAT_DIELECTRIC, GS_MAT_DIFFUSE_LIGHT, GS_MAT_ISOTROPIC = 1, 2, 3, 4, 5
GS_TEX_SOLID, GS_TEX_CHECKERED, GS_TEX_IMAGE, GS_TEX_NOISE = 1, 2, 3, 4
GS_BG_SOLID, GS_BG_HDRI = 1, 2
GS_ABI_VERSION = 11
GS_OK, GS_ERR_ARG, GS_ERR_HIP, GS_ERR_OOM, GS_ERR_UNSUPPORTED, GS_ERR_NO_DEVICE = 0, -1, -2, -3, -4, -5

D3 = C.c_double * 3


class gs_object(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material", C.c_int32), ("first", C.c_int32), ("count", C.c_int32),
                ("p", C.c_double * 9)]


class gs_material_spec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("texture", C.c_int32), ("p", C.c_double * 4)]


class gs_texture_spec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("a", C.c_int32), ("b", C.c_int32), ("pad", C.c_int32),
                ("p", C.c_double * 3)]


class gs_image_spec(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("rgb8", C.c_void_p)]


class gs_background_spec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("width", C.c_int32), ("height", C.c_int32), ("pad", C.c_int32),
                ("color", D3), ("rotation", D3), ("rgb", C.c_void_p)]


class gs_scene_spec(C.Structure):
    _fields_ = [("objects", C.POINTER(gs_object)), ("n_objects", C.c_int32),
                ("children", C.POINTER(C.c_int32)), ("n_children", C.c_int32),
                ("world", C.POINTER(C.c_int32)), ("n_world", C.c_int32),
                ("materials", C.POINTER(gs_material_spec)), ("n_materials", C.c_int32),
                ("textures", C.POINTER(gs_texture_spec)), ("n_textures", C.c_int32),
                ("images", C.POINTER(gs_image_spec)), ("n_images", C.c_int32),
                ("background", gs_background_spec)]


class gs_camera_spec(C.Structure):
    _fields_ = [("aspect_ratio", C.c_double), ("image_width", C.c_int32), ("max_depth", C.c_uint32),
                ("v_fov", C.c_double), ("look_from", D3), ("look_at", D3), ("vup", D3),
                ("defocus_angle", C.c_double), ("focus_distance", C.c_double)]


class gs_sample_settings(C.Structure):
    _fields_ = [("confidence", C.c_double), ("tolerance", C.c_double), ("batch_size", C.c_uint32),
                ("max_samples", C.c_uint32)]


COUNTER_NAMES = ["rays", "node_visits", "sphere_tests", "msphere_tests", "quad_tests", "tri_tests",
                 "instance_tests", "list_tests", "hits", "image_texels", "hdri_texels", "paths", "pixels",
                 "medium_tests", "noise_evals"]


class gs_counters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in COUNTER_NAMES] + [("reserved", C.c_uint64 * 1)]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n in COUNTER_NAMES}


class gs_camera(C.Structure):
    _fields_ = [("image_width", C.c_int32), ("image_height", C.c_int32), ("max_depth", C.c_uint32),
                ("pad", C.c_uint32), ("center", D3), ("starting_pixel_pos", D3), ("pixel_delta_u", D3),
                ("pixel_delta_v", D3), ("defocus_angle", C.c_double), ("defocus_disk_u", D3),
                ("defocus_disk_v", D3)]


class gs_medium_rec(C.Structure):  # gs_medium (a flat-scene record)
    _fields_ = [("boundary", C.c_uint32), ("material", C.c_uint32), ("density_neg_inv", C.c_double)]


class gs_partition(C.Structure):
    _fields_ = [("rank", C.c_int32), ("world_size", C.c_int32), ("tile_w", C.c_int32), ("tile_h", C.c_int32),
                ("d_tile_order", C.c_void_p), ("slots_per_rank", C.c_int32), ("pad", C.c_int32)]


class gs_background(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32), ("pad", C.c_uint32),
                ("color", D3), ("rot", C.c_double * 9)]


class gs_flat_scene(C.Structure):
    _fields_ = [("root", C.c_uint32), ("max_bvh_depth", C.c_uint32),
                ("nodes", C.c_void_p), ("n_nodes", C.c_uint32),
                ("spheres", C.c_void_p), ("n_spheres", C.c_uint32),
                ("mspheres", C.c_void_p), ("n_mspheres", C.c_uint32),
                ("quads", C.c_void_p), ("n_quads", C.c_uint32),
                ("triangles", C.c_void_p), ("n_triangles", C.c_uint32),
                ("lists", C.c_void_p), ("n_lists", C.c_uint32),
                ("list_refs", C.c_void_p), ("n_list_refs", C.c_uint32),
                ("instances", C.c_void_p), ("n_instances", C.c_uint32),
                ("materials", C.c_void_p), ("n_materials", C.c_uint32),
                ("textures", C.c_void_p), ("n_textures", C.c_uint32),
                ("images", C.c_void_p), ("n_images", C.c_uint32),
                ("texels8", C.c_void_p), ("n_texels8", C.c_uint64),
                ("background", gs_background),
                ("hdri_rgb", C.c_void_p), ("n_hdri_floats", C.c_uint64),
                ("media", C.c_void_p), ("n_media", C.c_uint32),
                ("noise_perm", C.c_void_p), ("n_noise_perm", C.c_uint32)]


class gs_render_outputs(C.Structure):
    _fields_ = [("rgb", C.c_void_p), ("rgb8", C.c_void_p), ("item_visits", C.c_void_p)]


class gs_launch(C.Structure):
    _fields_ = [("num_gpus", C.c_int32), ("tile_w", C.c_int32), ("tile_h", C.c_int32), ("plan", C.c_int32),
                ("devices", C.c_void_p)]


class gs_multi_outputs(C.Structure):
    _fields_ = [("rgb", C.c_void_p), ("rgb8", C.c_void_p), ("ppm_text", C.c_void_p), ("ppm_capacity", C.c_int64),
                ("ppm_len", C.POINTER(C.c_int64))]


class gs_stats(C.Structure):
    _fields_ = [("counters", gs_counters), ("setup_ms", C.c_double), ("total_ms", C.c_double),
                ("render_ms_max", C.c_double), ("render_ms_min", C.c_double), ("gather_ms", C.c_double),
                ("algorithmic_bytes", C.c_uint64), ("gathered_bytes", C.c_uint64), ("num_gpus", C.c_int32),
                ("pad", C.c_int32), ("kernel_ms_max", C.c_double), ("kernel_ms_min", C.c_double)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("counters", "pad")}
        d["counters"] = self.counters.as_dict()
        return d


class gs_scene_info(C.Structure):
    _fields_ = [("node_records", C.c_uint32), ("leaf_records", C.c_uint32), ("lds_nodes", C.c_uint32),
                ("lds_leaves", C.c_uint32), ("lds_quads", C.c_uint32), ("feat", C.c_int32), ("node_steps", C.c_int32),
                ("cert_boxes", C.c_int32), ("nodes_per_leaf", C.c_double), ("other_leaf_frac", C.c_double),
                ("placement", C.c_int32), ("long_samples", C.c_int32), ("pilot_ms", C.c_double)]


# Every symbol include/*.h declares, with its ctypes signature.
_P = C.c_void_p
SIGNATURES = {
    # grayshift_gpu.h
    "gs_last_error": (C.c_char_p, []),
    "gs_version": (C.c_int32, []),
    "gs_set_tuning": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "gs_debug_set_partial_budget": (C.c_int32, [C.c_uint64]),
    "gs_debug_set_guided_tail": (C.c_int32, [C.c_int32, C.c_int32]),
    "gs_set_node_steps": (C.c_int32, [C.c_int32]),
    "gs_set_camera_batch": (C.c_int32, [C.c_int32]),
    "gs_set_placement": (C.c_int32, [C.c_int32]),
    "gs_set_adaptive_mode": (C.c_int32, [C.c_int32]),
    "gs_debug_set_round_items": (C.c_int32, [C.c_int32]),
    "gs_debug_set_cube_lists": (C.c_int32, [C.c_int32]),
    "gs_debug_record_visits": (C.c_int32, [_P, C.POINTER(gs_camera), C.POINTER(gs_sample_settings), C.c_uint64,
                                           C.POINTER(gs_partition), _P, _P, _P]),
    "gs_device_scene_create": (C.c_int32, [_P, C.POINTER(_P)]),
    "gs_device_scene_destroy": (C.c_int32, [_P]),
    "gs_device_scene_info": (C.c_int32, [_P, C.POINTER(gs_scene_info)]),
    "gs_partition_capacity": (C.c_int64, [C.POINTER(gs_camera), C.POINTER(gs_partition)]),
    "gs_render_tiles_async": (C.c_int32, [_P, C.POINTER(gs_camera), C.POINTER(gs_sample_settings), C.c_uint64,
                                          C.POINTER(gs_partition), _P, _P, _P]),
    "gs_render_tiles_debug_async": (C.c_int32, [_P, C.POINTER(gs_camera), C.POINTER(gs_sample_settings), C.c_uint64,
                                                C.POINTER(gs_partition), _P, _P, _P, _P]),
    "gs_unpack_tiles_async": (C.c_int32, [C.POINTER(gs_camera), C.c_int32, C.c_int32, C.c_int32, C.c_int64, _P, _P,
                                          _P]),
    "gs_render_tiles_ex_async": (C.c_int32, [_P, C.POINTER(gs_camera), C.POINTER(gs_sample_settings), C.c_uint64,
                                             C.POINTER(gs_partition), C.POINTER(gs_render_outputs), _P, _P]),
    "gs_unpack_tiles_u8_async": (C.c_int32, [C.POINTER(gs_camera), C.c_int32, C.c_int32, C.c_int32, C.c_int64, _P,
                                             _P, _P]),
    "gs_ppm_max_bytes": (C.c_int64, [C.c_int32, C.c_int32]),
    "gs_ppm_scratch_bytes": (C.c_int64, [C.c_int32, C.c_int32]),
    "gs_ppm_encode_async": (C.c_int32, [_P, C.c_int32, C.c_int32, _P, C.c_int64, _P, _P, C.c_int64, _P]),
    "gs_render_ppm": (C.c_int32, [_P, C.POINTER(gs_camera), C.POINTER(gs_sample_settings), C.c_uint64, _P,
                                  C.c_int64, C.POINTER(C.c_int64), C.POINTER(gs_stats)]),
    "gs_plan_tiles": (C.c_int32, [_P, C.POINTER(gs_camera), C.c_uint64, C.c_int32, C.c_int32, C.c_int32, _P,
                                  C.c_int64, C.POINTER(C.c_int32)]),
    "gs_unpack_tiles_part_async": (C.c_int32, [C.POINTER(gs_camera), C.POINTER(gs_partition), C.c_int64, _P, _P,
                                               C.c_int32, _P]),
    "gs_device_alloc": (C.c_int32, [C.c_int64, C.POINTER(_P)]),
    "gs_device_free": (C.c_int32, [_P]),
    "gs_device_upload": (C.c_int32, [_P, _P, C.c_int64]),
    "gs_device_download": (C.c_int32, [_P, _P, C.c_int64]),
    "gs_render": (C.c_int32, [_P, C.POINTER(gs_camera), C.POINTER(gs_sample_settings), C.c_uint64, _P,
                              C.POINTER(gs_stats)]),
    "gs_render_multi": (C.c_int32, [_P, C.POINTER(gs_camera), C.POINTER(gs_sample_settings), C.c_uint64,
                                    C.POINTER(gs_launch), C.POINTER(gs_multi_outputs), C.POINTER(gs_stats)]),
    "gs_rccl_library": (C.c_char_p, []),
    "gs_multi_create": (C.c_int32, [_P, C.POINTER(gs_launch), C.POINTER(_P)]),
    "gs_multi_render": (C.c_int32, [_P, C.POINTER(gs_camera), C.POINTER(gs_sample_settings), C.c_uint64,
                                    C.POINTER(gs_multi_outputs), C.POINTER(gs_stats)]),
    "gs_multi_frame": (C.c_int32, [_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_int32)]),
    "gs_multi_devices": (C.c_int32, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_int32]),
    "gs_multi_scene": (C.c_int32, [_P, C.c_int32, C.POINTER(_P)]),
    "gs_multi_destroy": (C.c_int32, [_P]),
    "gs_debug_set_multi_collective": (C.c_int32, [C.c_int32]),
    "gs_debug_set_multi_same_device": (C.c_int32, [C.c_int32]),
    # grayshift_host.h
    "gs_host_scene_from_spec": (C.c_int32, [C.POINTER(gs_scene_spec), C.POINTER(_P)]),
    "gs_host_scene_destroy": (C.c_int32, [_P]),
    "gs_host_scene_flat": (_P, [_P]),
    "gs_host_camera": (C.c_int32, [C.POINTER(gs_camera_spec), C.POINTER(gs_camera)]),
    "gs_host_render_spec": (C.c_int32, [C.POINTER(gs_scene_spec), C.POINTER(gs_camera_spec),
                                        C.POINTER(gs_sample_settings), C.c_uint64, _P, C.POINTER(gs_stats)]),
    "gs_host_render_ppm_spec": (C.c_int32, [C.POINTER(gs_scene_spec), C.POINTER(gs_camera_spec),
                                            C.POINTER(gs_sample_settings), C.c_uint64, _P, C.c_int64,
                                            C.POINTER(C.c_int64), C.POINTER(gs_stats)]),
    "gs_host_write_ppm": (C.c_int32, [C.c_char_p, C.c_int32, C.c_int32, _P]),
    "gs_host_color_byte": (C.c_int32, [C.c_double]),
    "gs_host_noise_permutation": (None, [C.c_uint32, _P]),
    "gs_host_bvh_topology": (C.c_int64, [C.POINTER(gs_scene_spec), C.POINTER(C.c_int32), C.c_int64]),
    "gs_host_struct_size": (C.c_int64, [C.c_char_p]),
}


class GrayshiftError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("grayshift error %d: %s" % (code, msg))
        self.code = code


def _preload_hip_runtime():
    """One HIP runtime per process.  torch wheels bundle their own libamdhip64.so.7 /
    libhsa-runtime64 (the same sonames as /opt/rocm's).  Loaded first, they also serve
    this library; if /opt/rocm's were loaded first, a later `import torch` would find no
    GPU ("No HIP GPUs are available").  So when torch is installed, load torch's HIP
    runtime library (by path: no `import torch`, so importing this package stays cheap)
    before this library; without torch, /opt/rocm's is used."""
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.submodule_search_locations:
        return None
    hip = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if not os.path.exists(hip):
        return None
    return C.CDLL(hip, mode=C.RTLD_GLOBAL)


def load(path=LIB_PATH):
    if not os.path.exists(path):
        raise ImportError("libgrayshift.so not built (%s): run `python -m grayshift_amd.build`" % path)
    _preload_hip_runtime()
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = load()


def check(status):
    if status != GS_OK:
        raise GrayshiftError(status, lib.gs_last_error().decode("utf-8", "replace"))
    return status
