#!/usr/bin/env python3
"""Which threaded records the rays of a frame test, and how much of that the per-block LDS
mirror serves under each placement: the static estimate (gs_set_placement(0)) and the
pilot-measured one (the default), both counted by gs_debug_record_visits over the same
frame; plus the best any budget could do (records ranked by measured visits per byte).

python tools/visitmap.py [--config C4] [--spp 16]"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--budgets", type=int, nargs="+", default=[56, 84, 111, 130, 159],
                    help="mirror budgets in KiB for the best-order column")
    a = ap.parse_args()
    import numpy as np
    import torch
    import grayshift_amd as g
    from grayshift_amd import _native as N, scenes
    sc = scenes.config(a.config, width=a.width, spp=a.spp)
    dev = torch.device("cuda", 0)
    for mode in (0, 1):
        N.check(N.lib.gs_set_placement(mode))
        r = g.Renderer(sc, 0, 1, 64)
        packed = torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev)
        i0 = r.scene_info()
        nn, nl = i0["node_records"], i0["leaf_records"]
        vm = torch.zeros(nn + nl, dtype=torch.int32, device=dev)
        N.check(N.lib.gs_debug_record_visits(r.dev, C.byref(r.cam), C.byref(r.settings), 1, C.byref(r.part),
                                             C.c_void_p(packed.data_ptr()), C.c_void_p(vm.data_ptr()), None))
        torch.cuda.synchronize()
        info = r.scene_info()
        v = vm.cpu().numpy().astype(np.int64)
        nodes, leaves = v[:nn], v[nn:]
        ln, ll = info["lds_nodes"], info["lds_leaves"]
        print("%s %s spp, placement %s (pilot %.1f ms): %d node records (%d mirrored), %d leaf records (%d mirrored); "
              "node visits %d, %.2f%% from the mirror; leaf tests %d, %.2f%% from the mirror" % (
                  a.config, a.spp, {0: "pending", 1: "static", 2: "measured"}[info["placement"]], info["pilot_ms"],
                  nn, ln, nl, ll, nodes.sum(), 100.0 * nodes[:ln].sum() / max(1, nodes.sum()), leaves.sum(),
                  100.0 * leaves[:ll].sum() / max(1, leaves.sum())), flush=True)
        r.close()
    N.check(N.lib.gs_set_placement(1))
    # the best order for other budgets (the last run's counts: records by visits per byte)
    val = np.concatenate([nodes / 32.0, leaves / 48.0])
    size = np.concatenate([np.full(nn, 32), np.full(nl, 48)])
    isleaf = np.concatenate([np.zeros(nn, bool), np.ones(nl, bool)])
    o = np.argsort(-val, kind="stable")
    cum = np.cumsum(size[o])
    for kib in a.budgets:
        k = np.searchsorted(cum, kib * 1024, side="right")
        sel = o[:k]
        sn, sl = sel[~isleaf[sel]], sel[isleaf[sel]] - nn
        print("budget %4d KiB, by visits per byte: %5d nodes + %5d leaves; node visits %.2f%%, leaf tests %.2f%%"
              % (kib, len(sn), len(sl), 100.0 * nodes[sn].sum() / max(1, nodes.sum()),
                 100.0 * leaves[sl].sum() / max(1, leaves.sum())))


if __name__ == "__main__":
    main()
