#!/usr/bin/env python3
"""Generate the committed golden frames from the CPU oracle.

The reference has no tests or golden images, so these fixtures are
build-authored: tiny frames of every catalog scene and BASELINE config, rendered by
oracle/ (the C++ restatement) at seed 1.  They pin the oracle against regressions
and are what the GPU parity tests compare to.  Regenerate only when the oracle is
deliberately changed:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

SEED = 1

# name -> (builder, kwargs, width, spp or None for the scene's own adaptive settings)
GOLDEN = {
    "C1": ("config", {"name": "C1"}, 32, 8),
    "C2": ("config", {"name": "C2"}, 32, 8),
    "C3": ("config", {"name": "C3"}, 32, 8),
    "C4": ("config", {"name": "C4"}, 32, 8),
    "C5": ("config", {"name": "C5"}, 32, 8),
    "earth": ("earth", {}, 32, 8),
    "quads": ("quads", {}, 24, 8),
    "triangles": ("triangles", {}, 24, 8),
    "checkered_spheres": ("checkered_spheres", {}, 32, 8),
    "hdri_adaptive": ("hdri", {}, 32, None),
    "cornell_adaptive": ("cornell_box", {}, 24, None),
    "bouncing_adaptive": ("bouncing_spheres", {"grid": 11}, 32, None),
    "cornell_smoke": ("cornell_smoke", {}, 24, 8),
    "smoke_adaptive": ("cornell_smoke", {}, 16, None),
    "perlin_spheres": ("perlin_spheres", {}, 32, 8),
    "simple_light": ("simple_light", {}, 32, 8),
    "final_scene": ("final_scene", {}, 24, 8),
    "final_adaptive": ("final_scene", {}, 12, None),
}


def build(name):
    from grayshift_amd import scenes
    from grayshift_amd.scene import fixed_spp
    kind, kw, width, spp = GOLDEN[name]
    if kind == "config":
        return scenes.config(kw["name"], width=width, spp=spp)
    settings = fixed_spp(spp) if spp else None
    return scenes.SCENES[kind](width=width, settings=settings, **kw)


def main():
    import oracle
    frames, counters = {}, {}
    for name in GOLDEN:
        sc = build(name)
        rgb, c = oracle.render(sc, seed=SEED)
        frames[name] = rgb
        counters[name] = c
        print(name, rgb.shape, c["rays"], flush=True)
    np.savez_compressed(os.path.join(HERE, "frames.npz"), **frames)
    with open(os.path.join(HERE, "counters.json"), "w") as f:
        json.dump({"seed": SEED, "counters": counters}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
