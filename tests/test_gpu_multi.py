"""The frame context gs_multi_* (one process, one scene per device uploaded once, one
grouped RCCL gather over xGMI to the first device per frame, unpack there), the one-shot
gs_render_multi / gs_render / gs_render_ppm built on it, and bench.py's two launch modes
(the context in one process; torch.distributed's gather over an RCCL process group).

The box has one MI355X, so these run the RCCL code with a 1-rank communicator
(gs_debug_set_multi_collective forces ncclCommInitAll + ncclGather for one device; a
1-rank nccl process group for bench.py): the frame must equal the single-GPU gs_render
frame bit for bit, and the PPM text gs_render_ppm's byte for byte.  Multi-device
partitions themselves are covered by test_gpu_parity.py (partition invariance and planned
partitions, G in {1,2,3,4,8} on one GPU: the context's non-RCCL steps) and
test_gpu_multiprocess.py.  The context's N > 1 path has not run on more than one device."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import _native as N
from grayshift_amd import scenes

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _collective:
    """Force the RCCL communicator and gather for one-device contexts (test hook)."""
    def __enter__(self):
        N.check(N.lib.gs_debug_set_multi_collective(1))

    def __exit__(self, *a):
        N.check(N.lib.gs_debug_set_multi_collective(0))


@pytest.mark.parametrize("plan", [False, True])
@pytest.mark.parametrize("tile", [64, 24])
@pytest.mark.parametrize("rccl", [False, True])
def test_render_multi_one_gpu_equals_render(plan, tile, rccl):
    sc = scenes.config("C4", width=160, spp=8)
    ref, rc = g.render(sc, seed=5)
    if rccl:
        with _collective():
            res = g.render_multi(sc, num_gpus=1, seed=5, tile=tile, plan=plan, rgb=True, rgb8=True)
    else:
        res = g.render_multi(sc, num_gpus=1, seed=5, tile=tile, plan=plan, rgb=True, rgb8=True)
    assert np.array_equal(res["rgb"], ref)
    assert res["counters"] == rc
    st = res["stats"]
    # (one device without a collective renders into the frame itself: no gather, no unpack)
    assert st["num_gpus"] == 1 and st["render_ms_max"] > 0 and (st["gather_ms"] > 0) == rccl
    assert 0 < st["kernel_ms_max"] <= st["render_ms_max"]
    assert st["algorithmic_bytes"] > 0
    assert (st["gathered_bytes"] > 0) == rccl  # one device: no gather unless forced
    if rccl:
        assert N.lib.gs_rccl_library()  # RCCL was loaded and used


def test_render_stats_on_the_single_gpu_calls():
    """gs_render / gs_render_ppm fill gs_stats: counters equal the CPU
    oracle's, kernel and render times from HIP events, algorithmic bytes (camera.rs:100-121)."""
    import ctypes as C
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    sc = scenes.config("C4", width=96, spp=8)
    host = g.HostScene(sc.spec)
    cam = g.camera(sc.camera)
    rgb = np.zeros((cam.image_height, cam.image_width, 3), np.float32)
    st = N.gs_stats()
    N.check(N.lib.gs_render(host.flat_ptr, C.byref(cam), C.byref(sc.settings), 4, rgb.ctypes.data, C.byref(st)))
    ref, oc = oracle.render(sc, seed=4)
    assert float(np.abs(rgb.astype(np.float64) - ref).max()) < 1e-3
    assert st.counters.as_dict() == oc
    assert st.num_gpus == 1 and 0 < st.kernel_ms_max <= st.render_ms_max and st.total_ms > 0
    assert st.algorithmic_bytes > 0 and st.gathered_bytes == 0
    cap = N.lib.gs_ppm_max_bytes(cam.image_width, cam.image_height)
    buf = C.create_string_buffer(int(cap))
    n = C.c_int64()
    st2 = N.gs_stats()
    N.check(N.lib.gs_render_ppm(host.flat_ptr, C.byref(cam), C.byref(sc.settings), 4, buf, cap, C.byref(n),
                                C.byref(st2)))
    assert st2.counters.as_dict() == oc and st2.kernel_ms_max > 0
    host.close()


@pytest.mark.parametrize("rccl", [False, True])
def test_frame_context_many_frames(rccl):
    """gs_multi_*: the scene is uploaded once; every frame of the context equals the
    one-shot render of its seed, the device-resident frame equals the host copy, and the
    stats report the megakernel alone inside the render."""
    import ctypes as C
    sc = scenes.config("C5", width=96, spp=4)
    if rccl:
        with _collective():
            m = g.MultiRenderer(sc, num_gpus=1, tile=32, plan=True)
    else:
        m = g.MultiRenderer(sc, num_gpus=1, tile=32, plan=True)
    assert m.devices == [0]
    for seed in (1, 2, 1):
        ref, rc = g.render(sc, seed=seed)
        res = m.render(seed=seed, rgb=True)
        assert np.array_equal(res["rgb"], ref) and res["counters"] == rc
        dev = m.render(seed=seed)  # no host output: the frame stays on the device
        p, d = m.frame_ptr()
        assert p and d == 0 and dev["counters"] == rc
        host = np.zeros_like(ref)
        N.check(N.lib.gs_device_download(host.ctypes.data, C.c_void_p(p), host.nbytes))
        assert np.array_equal(host, ref)
        st = dev["stats"]
        assert 0 < st["kernel_ms_max"] <= st["render_ms_max"] and st["setup_ms"] == 0.0  # plan kept
    assert m.scene_info()["node_records"] > 0
    m.close()


def test_frame_context_rejects_bad_arguments():
    import ctypes as C
    sc = scenes.config("C4", width=32, spp=1)
    host = g.HostScene(sc.spec)
    h = C.c_void_p()
    ids = (C.c_int32 * 1)(0)
    bad = N.gs_launch(num_gpus=0, tile_w=64, tile_h=64, plan=0, devices=C.cast(ids, C.c_void_p))
    assert N.lib.gs_multi_create(host.flat_ptr, C.byref(bad), C.byref(h)) == N.GS_ERR_ARG  # devices need num_gpus
    assert b"device list" in N.lib.gs_last_error()
    bad = N.gs_launch(num_gpus=2, tile_w=64, tile_h=64, plan=0, devices=None)
    assert N.lib.gs_multi_create(host.flat_ptr, C.byref(bad), C.byref(h)) == N.GS_ERR_ARG  # one GPU visible
    ok = N.gs_launch(num_gpus=1, tile_w=64, tile_h=64, plan=0, devices=None)
    N.check(N.lib.gs_multi_create(host.flat_ptr, C.byref(ok), C.byref(h)))
    cam = g.camera(sc.camera)
    cam.image_width = 0
    assert N.lib.gs_multi_render(h, C.byref(cam), C.byref(sc.settings), 1, None, None) == N.GS_ERR_ARG
    s = C.c_void_p()
    assert N.lib.gs_multi_scene(h, 1, C.byref(s)) == N.GS_ERR_ARG
    N.check(N.lib.gs_multi_destroy(h))
    host.close()


def test_render_multi_ppm_equals_render_ppm():
    sc = scenes.config("C5", width=96, spp=8)
    text, c = g.render_ppm(sc, seed=2)
    res = g.render_multi(sc, num_gpus=0, seed=2, rgb=False, ppm=True)  # 0 = every visible device
    assert res["ppm"] == text and res["counters"] == c


def test_render_multi_rejects_bad_launches():
    sc = scenes.config("C4", width=32, spp=1)
    with pytest.raises(N.GrayshiftError) as e:
        g.render_multi(sc, num_gpus=64)
    assert e.value.code == N.GS_ERR_ARG
    with pytest.raises(N.GrayshiftError) as e:
        g.render_multi(sc, devices=[0, 0])
    assert e.value.code == N.GS_ERR_ARG
    with pytest.raises(N.GrayshiftError):
        g.render_multi(sc, rgb=False)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_gather_over_rccl_one_rank(tmp_path):
    """bench.py's gather branch on an RCCL (backend "nccl") process group of one rank:
    the gathered and unpacked frame equals the plain N=1 frame bit for bit."""
    common = ["--steps", "1", "--warmup", "1", "--no-cpu", "--width", "160", "--spp", "8"]
    one, two = tmp_path / "plain.npy", tmp_path / "rccl.npy"
    r1 = subprocess.run([sys.executable, "bench.py"] + common + ["--dump", str(one)], cwd=ROOT,
                        capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr[-2000:]
    r2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                         "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
                         "--gpus", "1", "--gather", "--backend", "nccl", "--dump", str(two)] + common,
                        cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r2.returncode == 0, r2.stderr[-3000:]
    line = [l for l in r2.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["config"]["collective"] == "rccl"
    assert np.array_equal(np.load(one), np.load(two))


def test_bench_context_path_and_too_many_gpus(tmp_path):
    """bench.py without a launcher drives the devices through the frame context: its frame
    equals the one-shot render; --gpus above the visible devices fails with a message."""
    out = tmp_path / "ctx.npy"
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--no-cpu", "--width", "160",
                        "--spp", "8", "--seed", "3", "--dump", str(out)], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 1 and d["config"]["collective"] == "none" and "gs_multi" in d["config"]["launch"]
    assert d["roofline"]["kernel_ms"] > 0 and d["config"]["scene"]["node_records"] > 0
    ref, _ = g.render(scenes.config("C4", width=160, spp=8), seed=3)
    assert np.array_equal(np.load(out), ref)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "64", "--steps", "1", "--no-cpu"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "visible" in r.stderr


def test_concurrent_launches_of_one_scene():
    """Launches of one device scene on two streams and from two host threads at once
    (more in flight than the scene's 4 launch slots): each launch has its own parameter
    block, queue counter and chunk sums, so every frame is the serial one."""
    import threading
    import torch
    sc = scenes.config("C4", width=128, spp=16)
    seeds = [3, 4, 5, 6, 7, 8]
    refs = {s: g.render(sc, seed=s)[0] for s in seeds}
    r = g.Renderer(sc)
    dev = torch.device("cuda", 0)
    bufs = {s: torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev) for s in seeds}
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    errors = []

    def worker(k):
        try:
            for s in seeds[k::2]:
                r.render_async(bufs[s].data_ptr(), 0, streams[k].cuda_stream, seed=s)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    torch.cuda.synchronize()
    assert not errors, errors
    for s in seeds:
        frame = torch.zeros(r.height * r.width * 3, dtype=torch.float32, device=dev)
        r.unpack_async(bufs[s].data_ptr(), frame.data_ptr(), 1, torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(frame.view(r.height, r.width, 3).cpu().numpy(), refs[s]), s
    r.close()


def test_frame_context_from_two_threads():
    """One frame context rendered from two host threads at once (gs_multi_render holds the
    context's mutex, taken before anything reads its state): every frame equals the
    one-shot render of its seed, the first frame's placement pilots run exactly once
    (spp 32: a launch of >= 16x the pilot's samples, so the pilot does run)."""
    import threading
    sc = scenes.config("C4", width=96, spp=32)
    seeds = [1, 2, 3, 4, 5, 6]
    refs = {s: g.render(sc, seed=s) for s in seeds}
    m = g.MultiRenderer(sc, num_gpus=1, tile=32, plan=False)
    got, errors = {}, []

    def worker(k):
        try:
            for s in seeds[k::2]:
                got[s] = m.render(seed=s, rgb=True)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    for s in seeds:
        assert np.array_equal(got[s]["rgb"], refs[s][0]) and got[s]["counters"] == refs[s][1], s
    assert sum(1 for s in seeds if got[s]["stats"]["setup_ms"] > 0.0) == 1
    assert m.scene_info()["placement"] == 2
    m.close()


def test_async_launch_returns_while_the_kernel_runs():
    """the N-device issue loop (multi_gpu.cpp) launches every device's
    frame before waiting for any, so a launch call must return while its kernel still runs,
    or the devices would serialise.  After a warm-up frame (the placement pilot and the
    slot's chunk-sum buffer are in place), the host call of a >= 100 ms C4 launch returns
    in a small fraction of the kernel's time, long before the stream drains."""
    import time
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    sc = scenes.config("C4", width=1920, spp=160)
    r = g.Renderer(sc, 0, 1, 64)
    st = torch.cuda.Stream(dev)
    buf = torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev)
    r.render_async(buf.data_ptr(), 0, st.cuda_stream, seed=1)  # warm-up: pilot, buffers
    torch.cuda.synchronize()
    calls = []
    for seed in (2, 3):
        t0 = time.perf_counter()
        r.render_async(buf.data_ptr(), 0, st.cuda_stream, seed=seed)
        calls.append(time.perf_counter() - t0)
        t1 = time.perf_counter()
        st.synchronize()
        calls.append(-(time.perf_counter() - t1))  # (negative: the wait, kept apart below)
    launches = [c for c in calls if c >= 0]
    waits = [-c for c in calls if c < 0]
    r.close()
    assert min(waits) > 0.05, waits  # the frames did run long (>= ~100 ms of kernel)
    # (relative, not an absolute bound: a loaded host may take a few ms for the call itself)
    assert max(launches) < 0.1 * min(waits), (launches, waits)
