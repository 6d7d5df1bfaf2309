#!/usr/bin/env python3
"""Find pixels where the GPU and the oracle traverse differently.

python tools/diverge.py --config C5 --width 32 --spp 8
Prints per-pixel node-visit mismatches and the image difference statistics.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--width", type=int, default=32)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--per-pixel", action="store_true", help="oracle visits per pixel (slow for big frames)")
    a = ap.parse_args()
    import torch
    import grayshift_amd as g
    from grayshift_amd import _native as N, scenes, partition
    import oracle

    sc = scenes.config(a.config, width=a.width, spp=a.spp)
    r = g.Renderer(sc, 0, 1, 64)
    dev = torch.device("cuda", 0)
    packed = torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev)
    visits = torch.zeros(r.capacity, dtype=torch.int32, device=dev)
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)
    N.check(N.lib.gs_render_tiles_debug_async(r.dev, C.byref(r.cam), C.byref(r.settings), a.seed, C.byref(r.part),
                                              C.c_void_p(packed.data_ptr()), C.c_void_p(cnt.data_ptr()),
                                              C.c_void_p(visits.data_ptr()), None))
    torch.cuda.synchronize()
    ids = partition.packed_pixel_ids(r.width, r.height, 0, 1, 64, 64)
    ok = ids >= 0
    gv = np.zeros(r.width * r.height, np.int64)
    gv[ids[ok]] = visits.cpu().numpy()[ok]
    grgb = np.zeros((r.width * r.height, 3), np.float32)
    grgb[ids[ok]] = packed.cpu().numpy().reshape(-1, 3)[ok]
    ref, rc = oracle.render(sc, seed=a.seed)
    d = np.abs(grgb.astype(np.float64) - ref.reshape(-1, 3).astype(np.float64)).max(axis=1)
    gc = {n: int(x) for n, x in zip(N.COUNTER_NAMES, cnt.cpu().numpy())}
    print("frame %dx%d spp %d: max|d| %.3g, px>1e-3: %d, px!=: %d" % (r.width, r.height, a.spp, d.max(),
                                                                     (d > 1e-3).sum(), (d > 0).sum()))
    for k in rc:
        if rc[k] != gc[k]:
            print("  counter %s: oracle %d gpu %d (%+.3g%%)" % (k, rc[k], gc[k], 100.0 * (gc[k] - rc[k]) / max(1, rc[k])))
    if a.per_pixel:
        bad = []
        for pid in range(r.width * r.height):
            _, c = oracle.render(sc, seed=a.seed, subset=np.array([pid], np.int32), threads=1)
            if c["node_visits"] != gv[pid]:
                bad.append((pid, c["node_visits"], int(gv[pid])))
        print("pixels with different visit counts:", len(bad))
        for pid, o, gg in bad[:20]:
            print("  pixel %d (i=%d j=%d): oracle %d gpu %d  |d|=%.3g" % (pid, pid % r.width, pid // r.width, o, gg,
                                                                          d[pid]))


if __name__ == "__main__":
    main()
