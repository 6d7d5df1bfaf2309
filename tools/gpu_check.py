#!/usr/bin/env python3
"""Quick GPU-vs-oracle parity sweep over small versions of the configs.

python tools/gpu_check.py [--configs C1,C3,C4,C5] [--width 64] [--spp 8]
Prints per config: max |delta|, pixels over 1e-3, counters equality.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import grayshift_amd as g  # noqa: E402
from grayshift_amd import scenes  # noqa: E402
import oracle  # noqa: E402


def counters_close(gpu, ref, rel=1e-4):
    """Same rule as tests/test_gpu_parity.py::counters_match."""
    if gpu["paths"] != ref["paths"] or gpu["pixels"] != ref["pixels"]:
        return False
    return all(abs(gpu[k] - v) <= rel * max(v, 1) + 2 for k, v in ref.items())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C3,C4,C5")
    ap.add_argument("--extra", default="quads,triangles,hdri,checkered_spheres,earth")
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--spp", type=int, default=8)
    a = ap.parse_args()
    todo = []
    for c in filter(None, a.configs.split(",")):
        todo.append((c, scenes.config(c, width=a.width, spp=a.spp)))
    for s in filter(None, a.extra.split(",")):
        todo.append((s, scenes.SCENES[s](width=a.width, settings=g.fixed_spp(a.spp))))
    ok = True
    for name, sc in todo:
        t0 = time.time()
        ref, rc = oracle.render(sc, seed=1)
        t1 = time.time()
        out, gc = g.render(sc, seed=1)
        t2 = time.time()
        d = np.abs(out.astype(np.float64) - ref.astype(np.float64))
        bad = int((d > 1e-3).any(axis=2).sum())
        same = counters_close(gc, rc)
        ok = ok and bad == 0 and same
        print("%-18s %4dx%-4d spp=%-4d max|d|=%.3g bad_px=%d counters_ok=%s oracle=%.2fs gpu=%.2fs"
              % (name, sc.width, sc.height, a.spp, d.max(), bad, same, t1 - t0, t2 - t1), flush=True)
        if not same:
            for k in rc:
                if rc[k] != gc[k]:
                    print("    %s: oracle=%d gpu=%d" % (k, rc[k], gc[k]))
    print("ALL OK" if ok else "MISMATCH")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
