#!/usr/bin/env python3
"""Measure the output stage on one GPU: the PPM text encoder
(gs_ppm_encode_async) and the byte-tile unpack, at 1080p and 4K, on random byte frames
resident in HBM.  Prints one JSON line per kernel.

Algorithmic bytes per launch: encoder = 3 B read per pixel + the text written
(header + Σ line lengths); unpack = 3 B read + 3 B written per packed pixel.
Both are HBM-bound byte work; roofline peak = 8 TB/s (MI355X_MICROARCH.md).

Usage: python tools/bench_output.py [--iters 50]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import numpy as np
    import torch
    import grayshift_amd as g
    from grayshift_amd import _native as N

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    for (w, h) in [(1920, 1080), (3840, 2160)]:
        rng = np.random.default_rng(1)
        # a rendered frame's byte distribution is mostly 2-3 digits; uniform bytes give
        # ~90% 3-digit values (≈11.6 B per line)
        b8 = torch.from_numpy(rng.integers(0, 256, size=w * h * 3, dtype=np.uint8)).to(dev)
        cap = N.lib.gs_ppm_max_bytes(w, h)
        scr = N.lib.gs_ppm_scratch_bytes(w, h)
        text = torch.empty(cap, dtype=torch.uint8, device=dev)
        n = torch.zeros(1, dtype=torch.int64, device=dev)
        scratch = torch.empty((scr + 7) // 8, dtype=torch.int64, device=dev)

        def enc():
            g.ppm_encode_async(b8.data_ptr(), w, h, text.data_ptr(), cap, n.data_ptr(), scratch.data_ptr(), scr, sp)

        for _ in range(5):
            enc()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.iters):
            enc()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters  # includes the scratch memset (a few KB)
        nbytes = w * h * 3 + int(n.item())
        print(json.dumps({"kernel": "gs_ppm_kernel", "image": "%dx%d" % (w, h), "us": round(ms * 1e3, 2),
                          "text_bytes": int(n.item()), "algorithmic_bytes": nbytes,
                          "GBps": round(nbytes / (ms / 1e3) / 1e9, 1),
                          "frac": round(nbytes / (ms / 1e3) / 8.0e12, 3)}), flush=True)

        # unpack of one rank's packed byte tiles into the frame
        sc_cam = N.gs_camera()
        sc_cam.image_width, sc_cam.image_height = w, h
        part = N.gs_partition(0, 1, 64, 64)
        capp = N.lib.gs_partition_capacity(C.byref(sc_cam), C.byref(part))
        packed = torch.from_numpy(rng.integers(0, 256, size=capp * 3, dtype=np.uint8)).to(dev)
        frame = torch.empty(w * h * 3, dtype=torch.uint8, device=dev)

        def unp():
            N.check(N.lib.gs_unpack_tiles_u8_async(C.byref(sc_cam), 1, 64, 64, capp, C.c_void_p(packed.data_ptr()),
                                                   C.c_void_p(frame.data_ptr()), C.c_void_p(sp)))

        for _ in range(5):
            unp()
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(a.iters):
            unp()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        ub = capp * 3 + w * h * 3
        print(json.dumps({"kernel": "gs_unpack_kernel (u8)", "image": "%dx%d" % (w, h), "us": round(ms * 1e3, 2),
                          "algorithmic_bytes": ub, "GBps": round(ub / (ms / 1e3) / 1e9, 1),
                          "frac": round(ub / (ms / 1e3) / 8.0e12, 3)}), flush=True)

        packed32 = torch.rand(capp * 3, dtype=torch.float32, device=dev)
        frame32 = torch.empty(w * h * 3, dtype=torch.float32, device=dev)

        def unp32():
            N.check(N.lib.gs_unpack_tiles_async(C.byref(sc_cam), 1, 64, 64, capp, C.c_void_p(packed32.data_ptr()),
                                                C.c_void_p(frame32.data_ptr()), C.c_void_p(sp)))

        for _ in range(5):
            unp32()
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(a.iters):
            unp32()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        ub = capp * 12 + w * h * 12
        print(json.dumps({"kernel": "gs_unpack_kernel (f32)", "image": "%dx%d" % (w, h), "us": round(ms * 1e3, 2),
                          "algorithmic_bytes": ub, "GBps": round(ub / (ms / 1e3) / 1e9, 1),
                          "frac": round(ub / (ms / 1e3) / 8.0e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
