"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the checker / CPU baseline.  Parity unpinned (see oracle.cpp header).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        from grayshift_amd import _native as N  # struct definitions only
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.oracle_last_error.restype = C.c_char_p
        L.oracle_render.restype = C.c_int
        L.oracle_render.argtypes = [C.POINTER(N.gs_scene_spec), C.POINTER(N.gs_camera_spec),
                                    C.POINTER(N.gs_sample_settings), C.c_uint64, C.c_int32, P, C.c_int64, P,
                                    C.POINTER(N.gs_counters), P]
        L.oracle_render_timed.restype = C.c_int
        L.oracle_render_timed.argtypes = L.oracle_render.argtypes + [C.POINTER(C.c_double)]
        L.oracle_noise_perm.argtypes = [C.c_uint32, P]
        L.oracle_perlin3.restype = C.c_double
        L.oracle_perlin3.argtypes = [P]
        L.oracle_noise_value.restype = C.c_double
        L.oracle_noise_value.argtypes = [C.c_double, P]
        L.oracle_ppm_text.restype = C.c_int64
        L.oracle_ppm_text.argtypes = [P, C.c_int32, C.c_int32, P, C.c_int64]
        L.oracle_camera_fields.argtypes = [C.POINTER(N.gs_camera_spec), P]
        L.oracle_stream_seed.restype = C.c_uint64
        L.oracle_stream_seed.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32]
        L.oracle_wyrand_f64.argtypes = [C.c_uint64, C.c_int32, P, P]
        L.oracle_aabb_hit.argtypes = [P, P, P, P, C.c_double, C.c_double]
        L.oracle_prim_hit.argtypes = [C.c_int32, P, P, P, C.c_double, C.c_double, C.c_double, P]
        L.oracle_random_cosine_direction.argtypes = [C.c_double, C.c_double, P]
        L.oracle_onb.argtypes = [P, P]
        L.oracle_reflectance.restype = C.c_double
        L.oracle_reflectance.argtypes = [C.c_double, C.c_double]
        L.oracle_refract.argtypes = [P, P, C.c_double, P]
        L.oracle_rotate_vector.argtypes = [P, P, P]
        L.oracle_luminance.restype = C.c_double
        L.oracle_luminance.argtypes = [P]
        L.oracle_color_byte.restype = C.c_int32
        L.oracle_color_byte.argtypes = [C.c_double]
        L.oracle_checker_even.argtypes = [C.c_double, P]
        L.oracle_bvh_topology.restype = C.c_int64
        L.oracle_bvh_topology.argtypes = [C.POINTER(N.gs_scene_spec), P, C.c_int64]
        _lib = L
    return _lib


def _d(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data


def render(scene, seed=1, threads=0, subset=None, bytes_out=False, timing=None):
    """Render `scene` (scenes.Scene) on the CPU.  Returns (rgb f32 [n,3] or [H,W,3], counters dict),
    plus write_color's bytes of the f64 colour (u8, same shape) when bytes_out.
    timing: a dict that receives "render_s", the pixel loop's wall time (world/BVH build excluded)."""
    from grayshift_amd import _native as N
    L = lib()
    if not threads:  # the GPU box's CPU share is 16 cores; nproc reports the whole machine
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    cnt = N.gs_counters()
    if subset is not None:
        sub = np.ascontiguousarray(subset, dtype=np.int32)
        out = np.zeros((len(sub), 3), dtype=np.float32)
        sub_ptr, n_sub = sub.ctypes.data, len(sub)
    else:
        out = np.zeros((scene.height, scene.width, 3), dtype=np.float32)
        sub_ptr, n_sub = None, 0
    b8 = np.zeros(out.shape, dtype=np.uint8) if bytes_out else None
    secs = C.c_double(0.0)
    r = L.oracle_render_timed(scene.spec.ptr(), C.byref(scene.camera), C.byref(scene.settings), seed, threads,
                              sub_ptr, n_sub, out.ctypes.data, C.byref(cnt), b8.ctypes.data if bytes_out else None,
                              C.byref(secs))
    if timing is not None:
        timing["render_s"] = secs.value
    if r != 0:
        raise RuntimeError("oracle: " + L.oracle_last_error().decode())
    if bytes_out:
        return out, cnt.as_dict(), b8
    return out, cnt.as_dict()


def ppm_text(rgb8):
    """Camera::render's PPM text (camera.rs:101-103,116-118) for an [H,W,3] byte frame."""
    a = np.ascontiguousarray(rgb8, dtype=np.uint8)
    h, w = a.shape[0], a.shape[1]
    L = lib()
    n = L.oracle_ppm_text(a.ctypes.data, w, h, None, 0)
    buf = C.create_string_buffer(int(n))
    L.oracle_ppm_text(a.ctypes.data, w, h, buf, n)
    return buf.raw[:n]


def render_ppm(scene, seed=1, threads=0):
    """The oracle's Camera::render output: (PPM bytes, counters)."""
    _, cnt, b8 = render(scene, seed=seed, threads=threads, bytes_out=True)
    return ppm_text(b8), cnt


def bvh_topology(spec):
    L = lib()
    n = L.oracle_bvh_topology(spec.ptr(), None, 0)
    if n < 0:
        raise RuntimeError("oracle: " + L.oracle_last_error().decode())
    out = np.zeros(n, dtype=np.int32)
    L.oracle_bvh_topology(spec.ptr(), out.ctypes.data, n)
    return out


def camera_fields(cam):
    out = np.zeros(19, dtype=np.float64)
    lib().oracle_camera_fields(C.byref(cam), out.ctypes.data)
    return out


def stream_seed(seed, pixel, sample):
    return lib().oracle_stream_seed(seed, pixel, sample)


def wyrand(state, n):
    f = np.zeros(n, dtype=np.float64)
    u = np.zeros(n, dtype=np.uint64)
    lib().oracle_wyrand_f64(state, n, f.ctypes.data, u.ctypes.data)
    return f, u


def aabb_hit(mn, mx, o, d, tmin, tmax):
    a, pa = _d(mn); b, pb = _d(mx); c, pc = _d(o); e, pe = _d(d)
    return bool(lib().oracle_aabb_hit(pa, pb, pc, pe, tmin, tmax))


def prim_hit(kind, p, o, d, tmin, tmax, time=0.0):
    pp, ppp = _d(list(p) + [0.0] * (9 - len(p)))
    oo, po = _d(o); dd, pd = _d(d)
    out = np.zeros(10, dtype=np.float64)
    r = lib().oracle_prim_hit(kind, ppp, po, pd, time, tmin, tmax, out.ctypes.data)
    if r < 0:
        raise ValueError("bad kind")
    if r == 0:
        return None
    return {"t": out[0], "p": out[1:4].copy(), "n": out[4:7].copy(), "front": bool(out[7]), "u": out[8], "v": out[9]}


def random_cosine_direction(r1, r2):
    out = np.zeros(3)
    lib().oracle_random_cosine_direction(r1, r2, out.ctypes.data)
    return out


def onb(n):
    nn, pn = _d(n)
    out = np.zeros(9)
    lib().oracle_onb(pn, out.ctypes.data)
    return out.reshape(3, 3)


def reflectance(c, ri):
    return lib().oracle_reflectance(c, ri)


def refract(v, n, ratio):
    vv, pv = _d(v); nn, pn = _d(n)
    out = np.zeros(3)
    lib().oracle_refract(pv, pn, ratio, out.ctypes.data)
    return out


def rotate_vector(v, rot):
    vv, pv = _d(v); rr, pr = _d(rot)
    out = np.zeros(3)
    lib().oracle_rotate_vector(pv, pr, out.ctypes.data)
    return out


def luminance(c):
    cc, pc = _d(c)
    return lib().oracle_luminance(pc)


def color_byte(c):
    return lib().oracle_color_byte(c)


def checker_even(scale, p):
    pp, ptr = _d(p)
    return bool(lib().oracle_checker_even(scale, ptr))


def noise_perm(seed=0):
    out = np.zeros(256, dtype=np.uint8)
    lib().oracle_noise_perm(seed, out.ctypes.data)
    return out


def perlin3(p):
    a, ptr = _d(p)
    return lib().oracle_perlin3(ptr)


def noise_value(scale, p):
    a, ptr = _d(p)
    return lib().oracle_noise_value(scale, ptr)
