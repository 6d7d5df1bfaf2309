#!/usr/bin/env python3
"""Traversal traces for the wave-scheduler model (tools/wave_sim/wave_sim.cpp).

Builds a copy of the CPU oracle (oracle/oracle.cpp, test infrastructure) with trace hooks
patched in -- in a temporary directory; the checked-in oracle is untouched -- and renders
a config single-threaded on a pixel subset, writing one byte stream of events in the
reference's order:
  P  a sample's path starts            R  a ray (world.hit) starts
  N  a BVH node visit (BVHNode::hit)   a/o/g/h  a sphere test: disc < 0 / both roots out of
                                       range / second root taken / first root taken
  U k / W k  random_vector_in_unit_sphere / _disk took k candidates (k one byte)

    python tools/wave_sim/trace_oracle.py --config C4 --blocks 64 --out /tmp/c4.tr
    g++ -O2 -o /tmp/wave_sim tools/wave_sim/wave_sim.cpp && /tmp/wave_sim /tmp/c4.tr 52 12 8
"""
import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

PATCHES = [
    ("struct Sphere : Hittable {",
     "#include <cstdlib>\nstatic FILE* g_tr = nullptr;\n"
     "static inline void TR(char c){ if(!g_tr){ const char* p=getenv(\"GS_TRACE\"); if(!p) return; g_tr=fopen(p,\"wb\"); } fputc(c,g_tr); }\n"
     "static void TRX(char c, int k) { TR(c); TR((char)(k > 200 ? 200 : k)); }\n"
     "struct TrFlush { ~TrFlush(){ if(g_tr) fclose(g_tr);} } g_trflush;\n"
     "struct Sphere : Hittable {"),
    ("        if (discriminant < 0.0) return false;\n        double sqrt_d = std::sqrt(discriminant);\n"
     "        double t = (h - sqrt_d) / a;\n        if (!ray_t.surrounds(t)) {\n            t = (h + sqrt_d) / a;\n"
     "            if (!ray_t.surrounds(t)) return false;\n        }",
     "        if (discriminant < 0.0) { TR('a'); return false; }\n        double sqrt_d = std::sqrt(discriminant);\n"
     "        double t = (h - sqrt_d) / a;\n        if (!ray_t.surrounds(t)) {\n            t = (h + sqrt_d) / a;\n"
     "            if (!ray_t.surrounds(t)) { TR('o'); return false; }\n            TR('g');\n        } else TR('h');"),
    ("        tl_cnt.node_visits++;\n", "        tl_cnt.node_visits++; TR('N');\n"),
    ("        tl_cnt.rays++;\n", "        tl_cnt.rays++; TR('R');\n"),
    ("                tl_cnt.paths++;\n", "                tl_cnt.paths++; TR('P');\n"),
    ("static Vec3 random_vector_in_unit_sphere() { /* util.rs:18-25 */\n    for (;;) {\n        Vec3 v = random_vector(-1.0, 1.0);\n"
     "        if (v.length_squared() < 1.0) return v;",
     "static Vec3 random_vector_in_unit_sphere() { /* util.rs:18-25 */\n    for (int k = 1;; k++) {\n"
     "        Vec3 v = random_vector(-1.0, 1.0);\n        if (v.length_squared() < 1.0) { TRX('U', k); return v; }"),
    ("static Vec3 random_vector_in_unit_disk() { /* :36-46 */\n    for (;;) {",
     "static Vec3 random_vector_in_unit_disk() { /* :36-46 */\n    for (int k = 1;; k++) {"),
    ("        Vec3 v(x, y, 0.0);\n        if (v.length_squared() < 1.0) return v;",
     "        Vec3 v(x, y, 0.0);\n        if (v.length_squared() < 1.0) { TRX('W', k); return v; }"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--blocks", type=int, default=64, help="random 8x8 pixel blocks of the full frame")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import numpy as np
    src = open(os.path.join(ROOT, "oracle", "oracle.cpp")).read()
    # the random-unit-sphere patch has to precede TRX's definition: declare it first
    src = src.replace("static Vec3 random_vector_in_unit_sphere()", "static void TRX(char c, int k);\n"
                      "static Vec3 random_vector_in_unit_sphere()", 1)
    for old, new in PATCHES:
        if src.count(old) != 1:
            raise SystemExit("trace patch does not apply: %r" % old[:60])
        src = src.replace(old, new)
    d = tempfile.mkdtemp()
    cpp, so = os.path.join(d, "oracle_trace.cpp"), os.path.join(d, "liboracle_trace.so")
    open(cpp, "w").write(src)
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-I" + os.path.join(ROOT, "oracle"),
                    "-shared", "-pthread", "-o", so, cpp], check=True)
    import oracle
    oracle.LIB_PATH = so
    from grayshift_amd import scenes
    sc = scenes.config(a.config)
    W, H = sc.width, sc.height
    rng = np.random.default_rng(5)
    bx, by = rng.integers(0, W // 8, a.blocks), rng.integers(0, H // 8, a.blocks)
    pix = np.array([(y0 * 8 + (l >> 3)) * W + x0 * 8 + (l & 7) for x0, y0 in zip(bx, by) for l in range(64)], np.int32)
    os.environ["GS_TRACE"] = a.out
    _, c = oracle.render(sc, seed=7, threads=1, subset=pix)
    print(a.out, c["rays"], "rays", c["node_visits"], "node visits")


if __name__ == "__main__":
    main()
