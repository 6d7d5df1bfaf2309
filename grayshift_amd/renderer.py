"""Python entry points to the device path (libgrayshift.so, HIP for gfx950).

* ``render(scene)`` — the one-call ``Camera::render`` replacement (linear f32 frame).
* ``Renderer`` — device-resident scene for repeated / multi-GPU rendering: upload once,
  render this rank's tiles into a caller-provided device buffer on a given stream.
  Used by bench.py with torch tensors as the device buffers (torch is plumbing only).
"""
import ctypes as C

import numpy as np

from . import _native as N


def camera(cam_spec):
    """Camera::new (camera.rs:39-98) -> gs_camera (the fields the device reads)."""
    out = N.gs_camera()
    N.check(N.lib.gs_host_camera(C.byref(cam_spec), C.byref(out)))
    return out


def render(scene, seed=1, stats=None):
    """Render a scenes.Scene on the current HIP device.  Returns (rgb [H,W,3] f32, counters);
    `stats` (a dict, optional) receives the call's gs_stats (kernel / render ms, bytes)."""
    cam = camera(scene.camera)
    out = np.zeros((cam.image_height, cam.image_width, 3), dtype=np.float32)
    st = N.gs_stats()
    N.check(N.lib.gs_host_render_spec(scene.spec.ptr(), C.byref(scene.camera), C.byref(scene.settings), seed,
                                      out.ctypes.data, C.byref(st)))
    if stats is not None:
        stats.update(st.as_dict())
    return out, st.counters.as_dict()


def render_ppm(scene, seed=1):
    """The whole of Camera::render (camera.rs:100-121): returns (PPM text as bytes, counters).
    Pixel bytes (write_color of the f64 colour) and the text are produced on the device."""
    cam = camera(scene.camera)
    cap = N.lib.gs_ppm_max_bytes(cam.image_width, cam.image_height)
    if cap < 0:
        raise ValueError("bad image size")
    buf = C.create_string_buffer(int(cap))
    n = C.c_int64()
    st = N.gs_stats()
    N.check(N.lib.gs_host_render_ppm_spec(scene.spec.ptr(), C.byref(scene.camera), C.byref(scene.settings), seed,
                                          buf, cap, C.byref(n), C.byref(st)))
    return buf.raw[:n.value], st.counters.as_dict()


def _launch(num_gpus, tile, plan, devices):
    dev = None
    if devices is not None:
        dev = (C.c_int32 * len(devices))(*devices)
        num_gpus = len(devices)
    launch = N.gs_launch(num_gpus=num_gpus, tile_w=tile, tile_h=tile, plan=1 if plan else 0,
                         devices=C.cast(dev, C.c_void_p) if dev is not None else None)
    return launch, dev


def _outputs(W, H, rgb, rgb8, ppm):
    """gs_multi_outputs for the requested host outputs (None: the frame stays on the device)."""
    if not (rgb or rgb8 or ppm):
        return None, {}, None
    res = {}
    out = N.gs_multi_outputs()
    if rgb:
        res["rgb"] = np.zeros((H, W, 3), dtype=np.float32)
        out.rgb = res["rgb"].ctypes.data
    if rgb8:
        res["rgb8"] = np.zeros((H, W, 3), dtype=np.uint8)
        out.rgb8 = res["rgb8"].ctypes.data
    ppm_buf = None
    if ppm:
        cap = N.lib.gs_ppm_max_bytes(W, H)
        ppm_buf = (C.create_string_buffer(int(cap)), C.c_int64(0))
        out.ppm_text = C.addressof(ppm_buf[0])
        out.ppm_capacity = cap
        out.ppm_len = C.pointer(ppm_buf[1])
    return out, res, ppm_buf


def render_multi(scene, num_gpus=0, seed=1, tile=64, plan=True, rgb=True, rgb8=False, ppm=False, devices=None):
    """camera.rs:105-114 (and with ppm=True the whole of :100-121) on `num_gpus` GPUs of
    this node (0 = every visible one) through gs_render_multi: one scene per device,
    tiles rendered concurrently, one RCCL gather to the first device.  Returns a dict
    with the requested outputs ("rgb" [H,W,3] f32, "rgb8" [H,W,3] u8, "ppm" bytes), the
    summed "counters" and the call's "stats"."""
    host = HostScene(scene.spec)
    try:
        cam = camera(scene.camera)
        out, res, ppm_buf = _outputs(cam.image_width, cam.image_height, rgb, rgb8, ppm)
        if out is None:
            out = N.gs_multi_outputs()  # none requested: the library reports GS_ERR_ARG
        launch, _dev = _launch(num_gpus, tile, plan, devices)
        st = N.gs_stats()
        N.check(N.lib.gs_render_multi(host.flat_ptr, C.byref(cam), C.byref(scene.settings), seed, C.byref(launch),
                                      C.byref(out), C.byref(st)))
        if ppm:
            res["ppm"] = ppm_buf[0].raw[:ppm_buf[1].value]
        res["counters"] = st.counters.as_dict()
        res["stats"] = {k: v for k, v in st.as_dict().items() if k != "counters"}
        return res
    finally:
        host.close()


class MultiRenderer:
    """The persistent N-GPU frame context (gs_multi_*): the world uploaded to every device
    and the RCCL communicator built once, then any number of frames, each one synchronous
    call (plan, render on every device, one gather, unpack).  num_gpus=0: every visible
    device; num_gpus=1: no collective."""

    def __init__(self, scene, num_gpus=1, tile=64, plan=True, devices=None):
        self.scene = scene
        self.host = HostScene(scene.spec)
        self.cam = camera(scene.camera)
        self.settings = scene.settings
        launch, _dev = _launch(num_gpus, tile, plan, devices)
        h = C.c_void_p()
        N.check(N.lib.gs_multi_create(self.host.flat_ptr, C.byref(launch), C.byref(h)))
        self.handle = h
        n = C.c_int32()
        ids = (C.c_int32 * 64)()
        N.check(N.lib.gs_multi_devices(h, C.byref(n), ids, 64))
        self.devices = list(ids[:n.value])

    @property
    def width(self):
        return self.cam.image_width

    @property
    def height(self):
        return self.cam.image_height

    def render(self, seed=1, rgb=False, rgb8=False, ppm=False):
        """One frame.  With no host output requested the linear f32 frame stays on the first
        device (frame_ptr()).  Returns a dict: requested outputs, "counters", "stats"."""
        out, res, ppm_buf = _outputs(self.width, self.height, rgb, rgb8, ppm)
        st = N.gs_stats()
        N.check(N.lib.gs_multi_render(self.handle, C.byref(self.cam), C.byref(self.settings), seed,
                                      C.byref(out) if out is not None else None, C.byref(st)))
        if ppm:
            res["ppm"] = ppm_buf[0].raw[:ppm_buf[1].value]
        res["counters"] = st.counters.as_dict()
        res["stats"] = {k: v for k, v in st.as_dict().items() if k != "counters"}
        return res

    def render_stats(self, seed, st):
        """One frame, the frame left on the first device, its gs_stats written into `st` (a
        caller-owned N.gs_stats) -- render() without the per-call Python conversions, for
        timed loops (bench.py)."""
        N.check(N.lib.gs_multi_render(self.handle, C.byref(self.cam), C.byref(self.settings), seed, None,
                                      C.byref(st)))

    def scene_info(self, rank=0):
        """gs_device_scene_info of the scene on rank `rank`'s device."""
        d = C.c_void_p()
        N.check(N.lib.gs_multi_scene(self.handle, rank, C.byref(d)))
        i = N.gs_scene_info()
        N.check(N.lib.gs_device_scene_info(d, C.byref(i)))
        return {k: getattr(i, k) for k, _ in N.gs_scene_info._fields_}

    def frame_ptr(self):
        """(device pointer of the last W*H*3 f32 frame or None, its device id)."""
        p, p8, d = C.c_void_p(), C.c_void_p(), C.c_int32()
        N.check(N.lib.gs_multi_frame(self.handle, C.byref(p), C.byref(p8), C.byref(d)))
        return p.value, d.value

    def close(self):
        if getattr(self, "handle", None):
            N.lib.gs_multi_destroy(self.handle)
            self.handle = None
        if getattr(self, "host", None):
            self.host.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter shutdown: the binding may be gone)
            pass


def ppm_encode_async(d_rgb8, width, height, d_text, text_capacity, d_len, d_scratch, scratch_bytes, stream=0):
    """Format a device W*H*3 byte frame as the reference's PPM text on the device."""
    N.check(N.lib.gs_ppm_encode_async(C.c_void_p(d_rgb8), width, height, C.c_void_p(d_text), text_capacity,
                                      C.c_void_p(d_len), C.c_void_p(d_scratch), scratch_bytes, C.c_void_p(stream)))


def set_tuning(shade_batch=0, blocks_per_cu=0, leaf_batch=0, sample_chunk=-1):
    """Process-wide launch tuning (see gs_set_tuning in include/grayshift_gpu.h)."""
    N.check(N.lib.gs_set_tuning(shade_batch, blocks_per_cu, leaf_batch, sample_chunk))


def write_ppm(path, rgb):
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    N.check(N.lib.gs_host_write_ppm(path.encode(), rgb.shape[1], rgb.shape[0], rgb.ctypes.data))


class HostScene:
    """World + BVHNode::from_list + flat arrays, built by the C++ host mirror."""

    def __init__(self, spec):
        self._spec = spec
        h = C.c_void_p()
        N.check(N.lib.gs_host_scene_from_spec(spec.ptr(), C.byref(h)))
        self.handle = h
        self.flat_ptr = N.lib.gs_host_scene_flat(h)
        self.flat = N.gs_flat_scene.from_address(self.flat_ptr)

    def close(self):
        if self.handle:
            N.lib.gs_host_scene_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter shutdown: the binding may be gone)
            pass

    def stats(self):
        f = self.flat
        return {"nodes": f.n_nodes, "spheres": f.n_spheres, "mspheres": f.n_mspheres, "quads": f.n_quads,
                "triangles": f.n_triangles, "lists": f.n_lists, "instances": f.n_instances,
                "materials": f.n_materials, "textures": f.n_textures, "max_bvh_depth": f.max_bvh_depth}


class Renderer:
    """A scene resident in HBM of the current device, rendered tile-partitioned."""

    def __init__(self, scene, rank=0, world_size=1, tile=64, tile_h=None, plan=False, plan_seed=1, order=None):
        """plan: cost-balanced tile assignment (gs_plan_tiles: a 1-spp pilot of the whole
        frame on this device) instead of round-robin.  order: a plan computed elsewhere
        (e.g. on rank 0 and broadcast: int32, slots_per_rank * world_size entries, see
        gs_partition.d_tile_order), used as given."""
        self.scene = scene
        self.host = HostScene(scene.spec)
        self.cam = camera(scene.camera)
        self.settings = scene.settings
        self.part = N.gs_partition(rank=rank, world_size=world_size, tile_w=tile, tile_h=tile_h or tile)
        self.order = None
        self.d_order = None
        d = C.c_void_p()
        N.check(N.lib.gs_device_scene_create(self.host.flat_ptr, C.byref(d)))
        self.dev = d
        if order is not None:
            self._use_order(np.ascontiguousarray(order, dtype=np.int32))
        elif plan:
            self._plan(plan_seed)
        self.capacity = N.lib.gs_partition_capacity(C.byref(self.cam), C.byref(self.part))
        if self.capacity < 0:
            raise ValueError("bad partition")

    def _plan(self, seed):
        p = self.part
        slots = C.c_int32()
        N.check(N.lib.gs_plan_tiles(self.dev, C.byref(self.cam), seed, p.world_size, p.tile_w, p.tile_h, None, 0,
                                    C.byref(slots)))
        order = np.zeros(slots.value * p.world_size, dtype=np.int32)
        N.check(N.lib.gs_plan_tiles(self.dev, C.byref(self.cam), seed, p.world_size, p.tile_w, p.tile_h,
                                    order.ctypes.data, order.size, C.byref(slots)))
        self._use_order(order)

    def _use_order(self, order):
        p = self.part
        if order.size % p.world_size:
            raise ValueError("tile order of %d entries for %d ranks" % (order.size, p.world_size))
        slots = order.size // p.world_size
        ids = np.sort(order[order >= 0])
        tx = (self.cam.image_width + p.tile_w - 1) // p.tile_w
        ty = (self.cam.image_height + p.tile_h - 1) // p.tile_h
        if not np.array_equal(ids, np.arange(tx * ty)):
            raise ValueError("tile order must hold every tile exactly once")
        d = C.c_void_p()
        N.check(N.lib.gs_device_alloc(order.nbytes, C.byref(d)))
        self.d_order = d
        N.check(N.lib.gs_device_upload(d, order.ctypes.data, order.nbytes))
        self.order = order
        p.d_tile_order = d.value
        p.slots_per_rank = slots

    @property
    def width(self):
        return self.cam.image_width

    @property
    def height(self):
        return self.cam.image_height

    def scene_info(self):
        """gs_device_scene_info as a dict (tree records, LDS mirror prefixes, kernel choices)."""
        i = N.gs_scene_info()
        N.check(N.lib.gs_device_scene_info(self.dev, C.byref(i)))
        return {k: getattr(i, k) for k, _ in N.gs_scene_info._fields_}

    def render_async(self, d_packed, d_counters=0, stream=0, seed=1):
        """d_packed: device pointer to capacity*3 f32; d_counters: device gs_counters or 0."""
        N.check(N.lib.gs_render_tiles_async(self.dev, C.byref(self.cam), C.byref(self.settings), seed,
                                            C.byref(self.part), C.c_void_p(d_packed), C.c_void_p(d_counters),
                                            C.c_void_p(stream)))

    def render_ex_async(self, d_rgb=0, d_rgb8=0, d_counters=0, stream=0, seed=1, d_item_visits=0):
        """Either or both outputs: d_rgb capacity*3 f32, d_rgb8 capacity*3 u8 (write_color bytes)."""
        o = N.gs_render_outputs(d_rgb or None, d_rgb8 or None, d_item_visits or None)
        N.check(N.lib.gs_render_tiles_ex_async(self.dev, C.byref(self.cam), C.byref(self.settings), seed,
                                               C.byref(self.part), C.byref(o), C.c_void_p(d_counters),
                                               C.c_void_p(stream)))

    def unpack_u8_async(self, d_gathered, d_frame, world_size, stream=0):
        part = N.gs_partition(0, world_size, self.part.tile_w, self.part.tile_h, self.part.d_tile_order,
                              self.part.slots_per_rank, 0)
        N.check(N.lib.gs_unpack_tiles_part_async(C.byref(self.cam), C.byref(part), self.capacity,
                                                 C.c_void_p(d_gathered), C.c_void_p(d_frame), 3, C.c_void_p(stream)))

    def unpack_async(self, d_gathered, d_frame, world_size, stream=0):
        part = N.gs_partition(0, world_size, self.part.tile_w, self.part.tile_h, self.part.d_tile_order,
                              self.part.slots_per_rank, 0)
        N.check(N.lib.gs_unpack_tiles_part_async(C.byref(self.cam), C.byref(part), self.capacity,
                                                 C.c_void_p(d_gathered), C.c_void_p(d_frame), 12, C.c_void_p(stream)))

    def close(self):
        if getattr(self, "d_order", None):
            N.lib.gs_device_free(self.d_order)
            self.d_order = None
        if getattr(self, "dev", None):
            N.lib.gs_device_scene_destroy(self.dev)
            self.dev = None
        if getattr(self, "host", None):
            self.host.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter shutdown: the binding may be gone)
            pass
