"""CPU tests of the product library: it loads, exports every declared symbol, its
ctypes mirror matches the C layouts, and the C++ host mirror builds the same world,
BVH and camera as the oracle.  No compute on a device."""
import ctypes as C
import hashlib
import json
import os
import re

import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import _native as N
from grayshift_amd import partition, scenes
from grayshift_amd.scene import SceneBuilder, fixed_spp
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = []
    for h in ("grayshift_gpu.h", "grayshift_host.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(gs_[a-z0-9_]+)\s*\(", src, re.M):
            names.append(m.group(1))
    return names


def test_every_declared_symbol_is_exported(built):
    names = declared_functions()
    assert len(names) >= 15
    lib = C.CDLL(N.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
        assert n in N.SIGNATURES, "ctypes mirror lacks " + n


def test_version_and_error_channel():
    assert N.lib.gs_version() == N.GS_ABI_VERSION == 11
    assert N.lib.gs_set_tuning(-1, 0, 0, -1) == N.GS_ERR_ARG
    assert b"tuning" in N.lib.gs_last_error()
    assert N.lib.gs_set_tuning(65, 0, 0, -1) == N.GS_ERR_ARG
    assert N.lib.gs_set_tuning(60, 0, 0, -1) == N.GS_OK
    assert N.lib.gs_set_tuning(60, 0, 8, -2) == N.GS_ERR_ARG
    assert N.lib.gs_set_tuning(60, 0, 8, -1) == N.GS_OK
    assert N.lib.gs_set_tuning(0, 0, 0, -1) == N.GS_OK  # (0: the scene's own shade batch, ABI 8)
    # the guided tail's test hook (ABI 10): 0 = the defaults, negative values rejected; ABI 11:
    # tail items are single samples (other sizes would tie the bits to the tail's tiles)
    assert N.lib.gs_debug_set_guided_tail(-1, 0) == N.GS_ERR_ARG
    assert N.lib.gs_debug_set_guided_tail(0, -5) == N.GS_ERR_ARG
    assert b"fine_chunk" in N.lib.gs_last_error()
    assert N.lib.gs_debug_set_guided_tail(4, 300) == N.GS_ERR_ARG
    assert N.lib.gs_debug_set_guided_tail(1, 300) == N.GS_OK
    assert N.lib.gs_debug_set_guided_tail(0, 0) == N.GS_OK
    # the same-device frame-context hook (ABI 11)
    assert N.lib.gs_debug_set_multi_same_device(2) == N.GS_ERR_ARG
    assert N.lib.gs_debug_set_multi_same_device(0) == N.GS_OK


@pytest.mark.parametrize("name", ["gs_object", "gs_material_spec", "gs_texture_spec", "gs_image_spec",
                                  "gs_background_spec", "gs_scene_spec", "gs_camera_spec", "gs_sample_settings",
                                  "gs_counters", "gs_camera", "gs_partition", "gs_background", "gs_flat_scene",
                                  "gs_render_outputs", "gs_launch", "gs_multi_outputs", "gs_stats",
                                  "gs_scene_info"])
def test_struct_layouts_match(name):
    assert N.lib.gs_host_struct_size(name.encode()) == C.sizeof(getattr(N, name))


def test_device_record_sizes():
    # the per-unit record sizes DESIGN.md §5 prices
    for name, size in [("gs_node", 64), ("gs_sphere", 40), ("gs_msphere", 64), ("gs_quad", 136),
                       ("gs_triangle", 104), ("gs_instance", 32), ("gs_medium", 16), ("gs_material", 40)]:
        assert N.lib.gs_host_struct_size(name.encode()) == size, name


ALL_SCENES = ["C1", "C3", "C4", "C5", "earth", "quads", "triangles", "checkered_spheres", "hdri", "cornell_box",
              "cornell_smoke"]


def _scene(name):
    if name.startswith("C"):
        return scenes.config(name, width=64, spp=4)
    return scenes.SCENES[name](width=64)


@pytest.mark.parametrize("name", ALL_SCENES)
def test_bvh_topology_matches_oracle(name):
    sc = _scene(name)
    n = N.lib.gs_host_bvh_topology(sc.spec.ptr(), None, 0)
    mine = np.zeros(n, np.int32)
    N.lib.gs_host_bvh_topology(sc.spec.ptr(), mine.ctypes.data_as(C.POINTER(C.c_int32)), n)
    assert np.array_equal(mine, oracle.bvh_topology(sc.spec))


@pytest.mark.parametrize("name", ALL_SCENES + ["C2"])
def test_camera_fields_bit_exact(name):
    sc = scenes.config(name) if name.startswith("C") else scenes.SCENES[name]()
    cam = g.camera(sc.camera)
    mine = [cam.image_height] + [x for f in ("center", "starting_pixel_pos", "pixel_delta_u", "pixel_delta_v",
                                            "defocus_disk_u", "defocus_disk_v") for x in getattr(cam, f)]
    assert np.array_equal(np.array(mine, np.float64), oracle.camera_fields(sc.camera))


def test_config_sizes():
    for name, (w, h) in {"C1": (400, 225), "C2": (1920, 1080), "C3": (1024, 1024), "C4": (1920, 1080),
                         "C5": (3840, 2160)}.items():
        cam = g.camera(scenes.config(name).camera)
        assert (cam.image_width, cam.image_height) == (w, h)


def test_c4_world_is_the_10k_sphere_bvh():
    hs = g.HostScene(scenes.config("C4").spec)
    st = hs.stats()
    assert st["spheres"] == 10002 and st["nodes"] == 11811 and st["max_bvh_depth"] == 14


def test_scene_generator_is_deterministic():
    a = scenes.config("C4").spec
    b = scenes.config("C4").spec
    ba = bytes(C.string_at(C.addressof(a.objects), a.spec.n_objects * C.sizeof(N.gs_object)))
    bb = bytes(C.string_at(C.addressof(b.objects), b.spec.n_objects * C.sizeof(N.gs_object)))
    assert ba == bb


def test_assets_match_manifest():
    from grayshift_amd import assets
    man = json.load(open(os.path.join(ROOT, "grayshift_amd", "assets", "manifest.json")))
    e = assets.earthmap_rgb8()
    assert e.shape == (512, 1024, 3)
    assert hashlib.sha256(e.tobytes()).hexdigest() == man["earthmap.jpg"]["decoded_sha256"]
    h = assets.airport_hdr_f32()
    assert h.shape == (512, 1024, 3) and h.dtype == np.float32 and float(h.max()) == 3808.0


def test_rgbe_conversion():
    from grayshift_amd.assets import rgbe_to_f32
    px = np.array([[[128, 64, 0, 129], [255, 255, 255, 0], [1, 2, 3, 136]]], np.uint8)
    out = rgbe_to_f32(px)
    assert out[0, 0].tolist() == [1.0, 0.5, 0.0]     # m * 2^(129-136)
    assert out[0, 1].tolist() == [0.0, 0.0, 0.0]     # e == 0 -> black
    assert out[0, 2].tolist() == [1.0, 2.0, 3.0]


@pytest.mark.parametrize("w,h,world,tile", [(1920, 1080, 1, 64), (1920, 1080, 8, 64), (400, 225, 3, 64),
                                            (37, 23, 2, 16), (1, 1, 4, 8)])
def test_partition_covers_every_pixel_once(w, h, world, tile):
    seen = np.zeros(w * h, np.int32)
    cam = N.gs_camera(image_width=w, image_height=h)
    for r in range(world):
        cap = N.lib.gs_partition_capacity(C.byref(cam), C.byref(N.gs_partition(r, world, tile, tile)))
        assert cap == partition.capacity(w, h, r, world, tile, tile)
        ids = partition.packed_pixel_ids(w, h, r, world, tile, tile)
        np.add.at(seen, ids[ids >= 0], 1)
    assert (seen == 1).all()


def test_color_byte_matches_oracle():
    for c in [0.0, 1e-9, 0.0625, 0.25, 0.5, 0.998, 0.999, 1.0, 7.0, -3.0, float("nan"), float("inf")]:
        assert N.lib.gs_host_color_byte(c) == oracle.color_byte(c)


def test_write_ppm(tmp_path):
    rgb = np.array([[[0.0, 0.25, 1.0], [4.0, -1.0, 0.0625]]], np.float32)
    p = str(tmp_path / "x.ppm")
    g.write_ppm(p, rgb)
    assert open(p).read() == "P3\n2 1\n255\n0 128 255\n255 0 64\n"


# ---------------------------------------------------------------- errors
def _flat_copy(name="C3"):
    hs = g.HostScene(_scene(name).spec)
    f = N.gs_flat_scene.from_buffer_copy(hs.flat)
    return hs, f


def test_malformed_scene_is_rejected_before_the_device():
    hs, f = _flat_copy()
    f.root = (1 << 28) | 9999  # node index out of range
    out = C.c_void_p()
    assert N.lib.gs_device_scene_create(C.byref(f), C.byref(out)) == N.GS_ERR_ARG
    assert b"node index" in N.lib.gs_last_error()
    hs, f = _flat_copy()
    f.n_materials = 0
    assert N.lib.gs_device_scene_create(C.byref(f), C.byref(out)) == N.GS_ERR_ARG


def test_media_flatten_to_medium_records():
    """cornell_smoke (main.rs:519-624): two ConstantMedium over Translate(RotateY(cube))."""
    hs = g.HostScene(scenes.cornell_smoke(width=32).spec)
    f = hs.flat
    assert f.n_media == 2
    recs = (N.gs_medium_rec * 2).from_address(f.media)
    for r in recs:
        assert r.boundary >> 28 == 7  # an instance chain (Translate)
        assert r.density_neg_inv == -1.0 / 0.01
    hs.close()


@pytest.mark.parametrize("case", ["bvh_boundary", "nested_medium", "nested_medium_3", "medium_in_list"])
def test_medium_boundaries_accepted_and_rejected(case):
    """Round 6: a BVH as a medium boundary and one medium as another's boundary are accepted (the
    device's catch-all kernel walks them; GPU parity: test_gpu_composition.py); media two deep
    inside media and a medium as a list member stay unsupported."""
    b = SceneBuilder()
    m = b.lambertian((1, 1, 1))
    iso = b.isotropic((1, 1, 1))
    s1, s2, s3 = (b.sphere((3.0 * k, 0, 0), 1, m) for k in range(3))
    if case == "bvh_boundary":
        b.add(b.medium(b.bvh([s1, s2, s3]), 0.5, iso))
    elif case == "nested_medium":
        b.add(b.medium(b.medium(s1, 0.5, iso), 0.5, iso))
    elif case == "nested_medium_3":
        b.add(b.medium(b.medium(b.medium(s1, 0.5, iso), 0.5, iso), 0.5, iso))
    else:
        b.add(b.hittable_list([b.medium(s1, 0.5, iso), s2]))
    h = C.c_void_p()
    rc = N.lib.gs_host_scene_from_spec(b.build().ptr(), C.byref(h))
    if case in ("bvh_boundary", "nested_medium"):
        assert rc == N.GS_OK
        N.lib.gs_host_scene_destroy(h)
    else:
        assert rc == N.GS_ERR_UNSUPPORTED


def test_bvh_under_instance_flattens_as_a_second_level_tree():
    """final_scene's Translate(RotateY(BVHNode::from_list(balls))) (main.rs:741-755): the
    inner tree's nodes are flattened but do not count towards the top-level depth."""
    b = SceneBuilder()
    m = b.lambertian((1, 1, 1))
    inner = b.bvh([b.sphere((float(i), 0, 0), 0.4, m) for i in range(40)])
    b.add(b.translate(b.rotate_y(inner, 15.0), (1, 0, 0)))
    b.add(b.sphere((0, -100, 0), 99, m))
    hs = g.HostScene(b.build())
    st = hs.stats()
    assert st["instances"] == 2 and st["spheres"] == 41
    assert st["nodes"] > 1 + 19  # top-level root + the inner tree (>= n/2 nodes for n leaves)
    assert st["max_bvh_depth"] == 1
    hs.close()


@pytest.mark.parametrize("case", ["instance_in_nested", "medium_in_nested", "bvh_in_instance_in_nested"])
def test_nested_bvh_leaves(case):
    """A ConstantMedium inside a BVH that is itself under Translate/RotateY is accepted since
    round 5, a Translate/RotateY chain there since round 6 (the device keeps both chains of
    such a hit; GPU parity: test_gpu_composition.py); a further BVH under that chain (two
    levels of nested BVHs) stays unsupported."""
    b = SceneBuilder()
    m = b.lambertian((1, 1, 1))
    s1 = b.sphere((0, 0, 0), 1, m)
    if case == "instance_in_nested":
        odd = b.translate(b.sphere((3, 0, 0), 1, m), (0, 1, 0))
    elif case == "medium_in_nested":
        odd = b.medium(b.sphere((3, 0, 0), 1, m), 0.5, b.isotropic((1, 1, 1)))
    else:
        odd = b.translate(b.bvh([b.sphere((3, 0, 0), 1, m), b.sphere((3, 3, 0), 1, m)]), (0, 1, 0))
    b.add(b.translate(b.bvh([s1, odd, b.sphere((6, 0, 0), 1, m)]), (1, 0, 0)))
    h = C.c_void_p()
    rc = N.lib.gs_host_scene_from_spec(b.build().ptr(), C.byref(h))
    if case == "bvh_in_instance_in_nested":
        assert rc == N.GS_ERR_UNSUPPORTED
    else:
        assert rc == N.GS_OK
        N.lib.gs_host_scene_destroy(h)


def test_empty_world_is_an_error():
    h = C.c_void_p()
    assert N.lib.gs_host_scene_from_spec(SceneBuilder().build().ptr(), C.byref(h)) == N.GS_ERR_ARG


def test_no_cpu_fallback_without_device():
    # Without a GPU the product must fail loudly, never compute on the CPU.
    import subprocess
    import sys
    code = ("import grayshift_amd as g; from grayshift_amd import scenes\n"
            "try:\n g.render(scenes.config('C1', width=8, spp=1))\n"
            "except g._native.GrayshiftError as e: print('ERR', e.code)\n"
            "else: print('RENDERED')\n")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert "ERR" in r.stdout, r.stdout + r.stderr


# ------------------------------------------------- output stage (PPM text)
def _ppm_reference_text(b8):
    """camera.rs:101-103 header, then color.rs:17 `writeln!("{r} {g} {b}")` per pixel."""
    h, w = b8.shape[0], b8.shape[1]
    lines = ["P3", "%d %d" % (w, h), "255"] + ["%d %d %d" % tuple(p) for p in b8.reshape(-1, 3)]
    return ("\n".join(lines) + "\n").encode()


@pytest.mark.parametrize("w,h", [(1, 1), (2, 1), (7, 3), (64, 32)])
def test_oracle_ppm_text_format(w, h):
    rng = np.random.default_rng(w * 100 + h)
    b8 = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    b8.flat[:4] = [0, 9, 10, 255][:min(4, b8.size)]
    assert oracle.ppm_text(b8) == _ppm_reference_text(b8)


def test_oracle_bytes_are_write_color_of_the_f64_colour():
    sc = _scene("C3")
    sc = type(sc)(sc.name, sc.spec, g.camera_spec(1.0, 12, 20, 40.0, (278.0, 278.0, -800.0), (278.0, 278.0, 0.0),
                                                  (0.0, 1.0, 0.0), 0.0, 10.0), g.fixed_spp(2))
    rgb, _, b8 = oracle.render(sc, seed=4, bytes_out=True)
    # bytes come from the f64 colour: equal to the f32 frame's bytes except where the
    # f32 rounding crosses a quantisation step (rare); every byte is write_color's range
    f32_bytes = np.vectorize(oracle.color_byte)(rgb.astype(np.float64))
    assert (np.abs(f32_bytes - b8.astype(np.int64)) <= 1).all()
    assert (f32_bytes == b8).mean() > 0.99


def test_ppm_sizes():
    hdr = len(b"P3\n3840 2160\n255\n")
    assert N.lib.gs_ppm_max_bytes(3840, 2160) == hdr + 3840 * 2160 * 12
    assert N.lib.gs_ppm_max_bytes(0, 5) == -1 and N.lib.gs_ppm_scratch_bytes(5, -1) == -1
    assert N.lib.gs_ppm_scratch_bytes(1, 1) == 8
    assert N.lib.gs_ppm_scratch_bytes(2048, 1) == 8 and N.lib.gs_ppm_scratch_bytes(2049, 1) == 16


def test_ppm_encode_rejects_bad_arguments_before_the_device():
    P = C.c_void_p
    ok = P(0x1000)
    assert N.lib.gs_ppm_encode_async(None, 4, 4, ok, 1 << 20, ok, ok, 1 << 20, None) == N.GS_ERR_ARG
    assert N.lib.gs_ppm_encode_async(ok, 0, 4, ok, 1 << 20, ok, ok, 1 << 20, None) == N.GS_ERR_ARG
    assert N.lib.gs_ppm_encode_async(ok, 4, 4, ok, 10, ok, ok, 1 << 20, None) == N.GS_ERR_ARG
    assert b"capacity" in N.lib.gs_last_error()
    assert N.lib.gs_ppm_encode_async(ok, 4, 4, ok, 1 << 20, ok, ok, 4, None) == N.GS_ERR_ARG
    assert N.lib.gs_ppm_encode_async(P(0x1001), 4, 4, ok, 1 << 20, ok, ok, 1 << 20, None) == N.GS_ERR_ARG
    assert b"aligned" in N.lib.gs_last_error()


# ------------------------------------------------- Rust binding
def _rust():
    return open(os.path.join(ROOT, "bindings", "grayshift_gpu.rs")).read()


def test_rust_binding_declares_every_gpu_entry_point():
    src = open(os.path.join(ROOT, "include", "grayshift_gpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    c_fns = set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(gs_[a-z0-9_]+)\s*\(", src, re.M))
    rs_fns = set(re.findall(r"pub fn (gs_[a-z0-9_]+)\s*\(", _rust()))
    assert c_fns == rs_fns
    assert "pub const GS_ABI_VERSION: i32 = %d;" % N.GS_ABI_VERSION in _rust()


@pytest.mark.parametrize("name", ["gs_counters", "gs_flat_scene", "gs_camera", "gs_render_outputs", "gs_medium",
                                  "gs_launch", "gs_multi_outputs", "gs_stats", "gs_scene_info"])
def test_rust_struct_fields_follow_the_header(name):
    """Field names in declaration order (arrays flattened by name) match the C struct."""
    hdrs = "".join(open(os.path.join(ROOT, "include", h)).read() for h in ("grayshift_gpu.h", "grayshift_scene.h"))
    hdrs = re.sub(r"/\*.*?\*/", "", hdrs, flags=re.S)
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), hdrs, re.S).group(1)
    c_names = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        for part in decl.split(","):
            m = re.search(r"([A-Za-z_][A-Za-z0-9_]*)\s*(\[[^\]]*\])?\s*$", part.strip())
            c_names.append(m.group(1))
    rs = re.search(r"pub struct %s \{(.*?)\}" % name, _rust(), re.S).group(1)
    rs_names = re.findall(r"pub ([a-z_0-9]+)\s*:", rs)
    norm = {"min": "mn", "max": "mx"}
    assert [norm.get(n, n) for n in rs_names] == [norm.get(n, n) for n in c_names]


# ------------------------------------------------------- tile plans (N > 1)
def test_planned_partition_capacity_and_validation():
    cam = g.camera(scenes.config("C4", width=200, spp=1).camera)
    # with an order table every rank holds slots_per_rank tiles (padded)
    p = N.gs_partition(1, 4, 64, 64, 0x1000, 3, 0)
    assert N.lib.gs_partition_capacity(C.byref(cam), C.byref(p)) == 3 * 64 * 64
    p_bad = N.gs_partition(1, 4, 64, 64, 0x1000, 0, 0)  # an order table needs slots_per_rank > 0
    assert N.lib.gs_partition_capacity(C.byref(cam), C.byref(p_bad)) == -1
    rr = N.gs_partition(1, 4, 64, 64, None, 0, 0)       # round-robin: ceil((tiles - rank) / world)
    tiles = ((200 + 63) // 64) * ((112 + 63) // 64)
    assert N.lib.gs_partition_capacity(C.byref(cam), C.byref(rr)) == ((tiles - 1 + 3) // 4) * 4096


def test_plan_and_device_helpers_reject_bad_arguments_before_the_device():
    cam = g.camera(scenes.config("C4", width=64, spp=1).camera)
    slots = C.c_int32()
    assert N.lib.gs_plan_tiles(None, C.byref(cam), 1, 2, 64, 64, None, 0, C.byref(slots)) == N.GS_ERR_ARG
    d = C.c_void_p()
    assert N.lib.gs_device_alloc(-1, C.byref(d)) == N.GS_ERR_ARG
    assert N.lib.gs_device_upload(None, None, 4) == N.GS_ERR_ARG
    p = N.gs_partition(0, 2, 64, 64, None, 0, 0)
    assert N.lib.gs_unpack_tiles_part_async(C.byref(cam), C.byref(p), 4096, C.c_void_p(0x1000),
                                            C.c_void_p(0x2000), 7, None) == N.GS_ERR_ARG
    p2 = N.gs_partition(0, 2, 64, 64, 0x1000, 2, 0)  # capacity must match the plan
    assert N.lib.gs_unpack_tiles_part_async(C.byref(cam), C.byref(p2), 4096, C.c_void_p(0x1000),
                                            C.c_void_p(0x2000), 12, None) == N.GS_ERR_ARG


def test_library_shares_torchs_hip_runtime():
    """_native loads torch's bundled libamdhip64.so.7 (by path, without importing torch)
    before libgrayshift.so, so one HIP runtime serves both (torch's and /opt/rocm's share
    a soname; whichever loads first wins)."""
    pytest.importorskip("torch")
    import grayshift_amd  # noqa: F401  (the library is loaded at import)
    maps = open("/proc/self/maps").read()
    hips = {line.split()[-1] for line in maps.splitlines() if "libamdhip64" in line}
    assert len(hips) == 1, hips
    assert "/torch/lib/" in next(iter(hips)), hips


# ------------------------------------------------------- flattener scalability
def _million_sphere_spec(n_side=1000):
    """A bouncing_spheres-like world of n_side^2 small spheres, every one with its own
    Lambertian over its own solid texture (unique materials, as main.rs:85-110 makes),
    plus the checkered ground; built directly as spec arrays (numpy), not by the Python
    scene builder."""
    n = n_side * n_side
    rng = np.random.default_rng(7)
    objs = np.zeros(n + 1, dtype=np.dtype(N.gs_object))
    objs["kind"] = N.GS_OBJ_SPHERE
    a, b = np.meshgrid(np.arange(n_side) - n_side // 2, np.arange(n_side) - n_side // 2, indexing="ij")
    objs["p"][:n, 0] = a.ravel() + 0.9 * rng.random(n)
    objs["p"][:n, 1] = 0.2
    objs["p"][:n, 2] = b.ravel() + 0.9 * rng.random(n)
    objs["p"][:n, 3] = 0.2
    objs["material"][:n] = np.arange(n)
    objs["p"][n, :4] = (0.0, -1000.0, 0.0, 1000.0)  # ground
    objs["material"][n] = n
    mats = np.zeros(n + 1, dtype=np.dtype(N.gs_material_spec))
    mats["kind"] = N.GS_MAT_LAMBERTIAN
    mats["texture"] = np.arange(n + 1)
    mats["texture"][n] = n + 2  # ground: the checker over two solids
    texs = np.zeros(n + 3, dtype=np.dtype(N.gs_texture_spec))
    texs["kind"] = N.GS_TEX_SOLID
    texs["p"][:n] = rng.random((n, 3))
    texs["kind"][n + 2], texs["a"][n + 2], texs["b"][n + 2] = N.GS_TEX_CHECKERED, n, n + 1
    texs["p"][n + 2, 0] = 0.32
    world = np.arange(n + 1, dtype=np.int32)
    s = N.gs_scene_spec()
    s.objects, s.n_objects = C.cast(objs.ctypes.data, C.POINTER(N.gs_object)), n + 1
    s.world, s.n_world = C.cast(world.ctypes.data, C.POINTER(C.c_int32)), n + 1
    s.materials, s.n_materials = C.cast(mats.ctypes.data, C.POINTER(N.gs_material_spec)), n + 1
    s.textures, s.n_textures = C.cast(texs.ctypes.data, C.POINTER(N.gs_texture_spec)), n + 3
    s.background = N.gs_background_spec(kind=N.GS_BG_SOLID)
    return s, (objs, mats, texs, world)


def test_million_sphere_world_flattens_in_seconds():
    """World + BVHNode::from_list + flatten of ~1M spheres with ~1M unique materials: the
    flattener's identity lookups are hash maps (a linear scan per lookup took hours)."""
    import time
    spec, keep = _million_sphere_spec()
    t0 = time.perf_counter()
    h = C.c_void_p()
    N.check(N.lib.gs_host_scene_from_spec(C.byref(spec), C.byref(h)))
    dt = time.perf_counter() - t0
    try:
        f = N.gs_flat_scene.from_address(N.lib.gs_host_scene_flat(h))
        assert f.n_spheres == 1000 * 1000 + 1
        assert f.n_materials == 1000 * 1000 + 1 and f.n_textures == 1000 * 1000 + 3
        assert f.n_nodes >= f.n_spheres // 2
    finally:
        N.lib.gs_host_scene_destroy(h)
    assert dt < 15.0, "flatten took %.1f s" % dt


# ------------------------------------------- Rust flattener
def test_rust_scene_builder_mirrors_the_cpp_flattener():
    rs = _rust()
    assert "pub struct SceneBuilder" in rs and "pub struct FlatScene" in rs
    impl = rs[rs.index("impl SceneBuilder"):]
    methods = set(re.findall(r"pub fn ([a-z_]+)\s*\(", impl))
    # one builder method per flattened record kind, the identity lookups, and finish
    assert {"node", "sphere", "moving_sphere", "quad", "triangle", "list", "instance", "medium", "material_index",
            "texture_index", "image_index", "finish"} <= methods
    # identity lookups are hash maps (O(1)), as the C++ Flattener's
    assert "HashMap" in rs and "mat_slot" in rs and "tex_slot" in rs
    # SceneBuilder fills every array of gs_flat_scene
    fin = impl[impl.index("pub fn finish"):]
    body = re.search(r"typedef struct gs_flat_scene \{(.*?)\} gs_flat_scene;",
                     re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "grayshift_gpu.h")).read(), flags=re.S),
                     re.S).group(1)
    for field in re.findall(r"([a-z_0-9]+)\s*;", body):
        assert field + ":" in fin or field + "," in fin, field


def test_integration_example_uses_the_binding():
    """The Rust example in INTEGRATION.md calls only what bindings/grayshift_gpu.rs defines."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    rs = _rust()
    for name in re.findall(r"gs::([A-Za-z_]+)", doc):
        assert re.search(r"pub (?:fn|struct|const) %s\b" % name, rs), name
    assert "b.finish(" in doc and "pub fn finish" in rs
