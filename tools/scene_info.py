#!/usr/bin/env python3
"""gs_device_scene_info for the BASELINE configs and the reference's scenes (needs a GPU:
the device scene is what reports it).

    python tools/scene_info.py [--scenes]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", action="store_true", help="also every scene of grayshift_amd.scenes.SCENES")
    a = ap.parse_args()
    import grayshift_amd as g
    from grayshift_amd import scenes
    items = [(c, scenes.config(c, width=64, spp=1)) for c in scenes.CONFIGS]
    if a.scenes:
        items += [(n, f(width=64)) for n, f in scenes.SCENES.items()]
    for name, sc in items:
        r = g.Renderer(sc, 0, 1, 64)
        i = r.scene_info()
        r.close()
        print("%-18s %s" % (name, " ".join("%s=%s" % (k, round(v, 3) if isinstance(v, float) else v)
                                           for k, v in i.items())), flush=True)


if __name__ == "__main__":
    main()
