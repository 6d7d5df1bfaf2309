#!/usr/bin/env python3
"""One parameterised sweep over bench.py runs (replaces round 1's sweep*.sh / ab_variants.sh).

Every combination of the given values runs `bench.py --steps S --warmup 1 --no-cpu` once,
each under its own time limit; one line per run is printed (and the JSON kept under
gpurun_out/sweep/).  A failing run ends the sweep.

    python tools/sweep.py --shade-batch 48 52 56 --leaf-batch 10 12
    python tools/sweep.py --lib base variants/x.so --config C3      # A/B library builds
"""
import argparse
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KNOBS = ["shade_batch", "leaf_batch", "sample_chunk", "blocks_per_cu", "tile", "node_steps", "camera_batch", "fine_chunk",
         "tail_pct"]


def main():
    ap = argparse.ArgumentParser()
    for k in KNOBS:
        ap.add_argument("--" + k.replace("_", "-"), nargs="+", type=int, default=[None])
    ap.add_argument("--lib", nargs="+", default=["base"],
                    help="library builds: 'base' (grayshift_amd/libgrayshift.so) or paths under grayshift_amd/")
    ap.add_argument("--config", nargs="+", default=["C4"])
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--timeout", type=int, default=200)
    ap.add_argument("--width", type=int, default=None, help="frame width (reference scenes; invalidates a metric config)")
    ap.add_argument("--spp", type=int, default=None)
    a = ap.parse_args()
    out_dir = os.path.join(ROOT, "gpurun_out", "sweep")
    os.makedirs(out_dir, exist_ok=True)
    axes = [a.lib, a.config] + [getattr(a, k) for k in KNOBS]
    for n, combo in enumerate(itertools.product(*axes)):
        lib, config, vals = combo[0], combo[1], combo[2:]
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(a.steps), "--warmup", "1", "--no-cpu",
               "--config", config]
        cmd += ["--width", str(a.width)] if a.width else []
        cmd += ["--spp", str(a.spp)] if a.spp else []
        for k, v in zip(KNOBS, vals):
            if v is not None:
                cmd += ["--" + k.replace("_", "-"), str(v)]
        env = dict(os.environ)
        if lib != "base":
            env["GS_LIB"] = os.path.join(ROOT, "grayshift_amd", lib)
        tag = "%s %s %s" % (lib, config, " ".join("%s=%s" % (k, v) for k, v in zip(KNOBS, vals) if v is not None))
        try:
            r = subprocess.run(["timeout", "-k", "10", str(a.timeout)] + cmd, env=env, capture_output=True, text=True)
        except OSError as e:
            raise SystemExit("%s: %s" % (tag, e))
        if r.returncode != 0:
            print("FAILED", tag, r.returncode, r.stderr[-800:], flush=True)
            raise SystemExit(1)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
        with open(os.path.join(out_dir, "run_%03d.json" % n), "w") as f:
            f.write(line + "\n")
        d = json.loads(line)
        print("%-48s %10.1f Msamples/s  %9.2f ms/frame  kernel %.2f ms" % (
            tag, d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"]), flush=True)


if __name__ == "__main__":
    main()
