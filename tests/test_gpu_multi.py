"""gs_render_multi — the N-GPU render behind one C-ABI call (one process, one scene per
device, one grouped RCCL gather over xGMI to the first device, unpack there) — and
bench.py's torch.distributed gather over an RCCL process group.

The box has one MI355X, so these run the RCCL code with a 1-rank communicator
(ncclCommInitAll over one device / a 1-rank nccl process group): the frame must equal
the single-GPU gs_render frame bit for bit, and the PPM text gs_render_ppm's byte for
byte.  Multi-device partitions themselves are covered by test_gpu_parity.py
(partition invariance, G in {1,2,3,4,8} on one GPU) and test_gpu_multiprocess.py."""
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


@pytest.mark.parametrize("plan", [False, True])
@pytest.mark.parametrize("tile", [64, 24])
def test_render_multi_one_gpu_equals_render(plan, tile):
    sc = scenes.config("C4", width=160, spp=8)
    ref, rc = g.render(sc, seed=5)
    res = g.render_multi(sc, num_gpus=1, seed=5, tile=tile, plan=plan, rgb=True, rgb8=True)
    assert np.array_equal(res["rgb"], ref)
    assert res["counters"] == rc
    st = res["stats"]
    assert st["num_gpus"] == 1 and st["render_ms_max"] > 0 and st["gather_ms"] > 0
    assert st["algorithmic_bytes"] > 0 and st["gathered_bytes"] > 0
    assert N.lib.gs_rccl_library()  # RCCL was loaded and used


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
