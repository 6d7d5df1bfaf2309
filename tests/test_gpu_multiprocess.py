"""The N>1 data path with real processes on the GPU: two ranks share the box's one
MI355X, each renders the tiles gs_partition assigns it through the C-ABI (sample
chunks on), the packed buffers are gathered to rank 0 (gloo over host memory here;
bench.py uses RCCL over xGMI, one GPU per rank) and unpacked by gs_unpack_tiles_async.
The frame and the summed counters must equal the single-rank render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tile, plan, q):
    import sys
    import ctypes as C
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import grayshift_amd as g
        from grayshift_amd import _native as N, scenes
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        sc = scenes.config("C4", width=200, spp=64)
        r = g.Renderer(sc, rank=rank, world_size=world, tile=tile, plan=plan)
        # planned partitions give every rank the same capacity; round-robin: rank 0's
        cap0 = r.capacity if plan else N.lib.gs_partition_capacity(C.byref(r.cam),
                                                                    C.byref(N.gs_partition(0, world, tile, tile)))
        packed = torch.zeros(cap0 * 3, dtype=torch.float32, device=dev)
        cnt = torch.zeros(16, dtype=torch.int64, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        r.render_async(packed.data_ptr(), cnt.data_ptr(), stream, seed=3)
        torch.cuda.synchronize()
        host = packed.cpu()
        cnt_h = cnt.cpu()
        dist.all_reduce(cnt_h)
        if rank == 0:
            bufs = [torch.empty_like(host) for _ in range(world)]
            dist.gather(host, gather_list=bufs, dst=0)
            gathered = torch.cat(bufs).to(dev)
            frame = torch.zeros(r.height * r.width * 3, dtype=torch.float32, device=dev)
            r.unpack_async(gathered.data_ptr(), frame.data_ptr(), world, stream)
            torch.cuda.synchronize()
            full, fc = g.render(sc, seed=3)
            mine = frame.view(r.height, r.width, 3).cpu().numpy()
            counters = {n: int(cnt_h[i]) for i, n in enumerate(N.COUNTER_NAMES)}
            q.put((bool(np.array_equal(mine, full)), counters == fc))
        else:
            dist.gather(host, dst=0)
        r.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,tile,plan", [(2, 64, False), (3, 16, False), (2, 64, True), (3, 32, True)])
def test_ranks_on_gpu_gather_equals_single_rank(world, tile, plan):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, tile, plan, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    frame_ok, counters_ok = q.get(timeout=5)
    assert frame_ok and counters_ok


def test_bench_two_ranks_shared_gpu(tmp_path):
    """bench.py's N>1 path end to end (cost-balanced plan, gather, unpack, max-over-ranks
    timing, one JSON line) rehearsed with 2 ranks on the box's one GPU over gloo: the
    gathered frame equals the 1-rank frame bit for bit."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["--steps", "1", "--warmup", "1", "--no-cpu", "--width", "160", "--spp", "8"]
    one = tmp_path / "one.npy"
    two = tmp_path / "two.npy"
    r1 = subprocess.run([sys.executable, "bench.py"] + common + ["--dump", str(one)], cwd=root,
                        capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr[-2000:]
    r2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                         "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
                         "--gpus", "2", "--share-gpu", "--backend", "gloo", "--dump", str(two)] + common,
                        cwd=root, capture_output=True, text=True, timeout=300)
    assert r2.returncode == 0, r2.stderr[-2000:]
    line = [l for l in r2.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["config"]["tile_plan"] == "cost-balanced"
    assert np.array_equal(np.load(one), np.load(two))
