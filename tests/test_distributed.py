"""The N>1 data path on CPU: world_size-2 (and 3) gloo process groups.

Each rank takes the tiles gs_partition assigns it (round-robin 64x64 tiles), fills
its packed buffer (here with the CPU oracle standing in for the device kernel —
there is no GPU in this container), pads to rank 0's capacity, and rank 0 gathers
every buffer in ONE gather and unpacks it.  The result must equal the single-rank
frame bit for bit: per-(pixel, sample) RNG streams make the output independent of
the partition.  bench.py uses the same protocol over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tile, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import ctypes as C
    from grayshift_amd import _native as N
    from grayshift_amd import partition
    from tests.golden import make_golden
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = make_golden.build("C5")
        W, H = sc.width, sc.height
        cam = N.gs_camera(image_width=W, image_height=H)
        cap0 = N.lib.gs_partition_capacity(C.byref(cam), C.byref(N.gs_partition(0, world, tile, tile)))
        ids = partition.packed_pixel_ids(W, H, rank, world, tile, tile)
        assert len(ids) == N.lib.gs_partition_capacity(C.byref(cam), C.byref(N.gs_partition(rank, world, tile, tile)))
        packed = np.zeros((cap0, 3), np.float32)
        valid = ids >= 0
        rgb, _ = oracle.render(sc, seed=5, threads=2, subset=ids[valid].astype(np.int32))
        packed[:len(ids)][valid] = rgb
        t = torch.from_numpy(packed.reshape(-1))
        if rank == 0:
            bufs = [torch.empty_like(t) for _ in range(world)]
            dist.gather(t, gather_list=bufs, dst=0)
            frame = partition.unpack(torch.cat(bufs).numpy(), W, H, world, tile, tile, cap0)
            full, _ = oracle.render(sc, seed=5, threads=2)
            q.put(bool(np.array_equal(frame, full)))
        else:
            dist.gather(t, dst=0)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,tile", [(2, 8), (3, 16)])
def test_tile_partitioned_gather_equals_single_rank(world, tile):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, tile, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True
