"""Fold tools/pmc.sh's per-pass rocprofv3 CSVs into one JSON per kernel launch.

    python tools/pmc_summary.py gpurun_out profiles/pmc_C4_latest.json [--kernel gs_render_kernel]

Counter values are summed over the kernel's dispatches and divided by their number
(per-launch figures).  HBM bytes follow MI355X_MICROARCH.md's gfx950 correction:
FETCH_SIZE / WRITE_SIZE are KB and FETCH_SIZE counts half the bytes of wide reads, so
hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="gs_render_kernel")
    ap.add_argument("--config", default="C4")
    ap.add_argument("--round", type=int, default=1)
    a = ap.parse_args()
    vals = defaultdict(float)
    dispatches = defaultdict(set)
    dur = []
    for f in sorted(glob.glob(os.path.join(a.root, "pmc_*", "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if a.kernel not in row["Kernel_Name"]:
                continue
            name = row["Counter_Name"]
            vals[name] += float(row["Counter_Value"])
            dispatches[name].add((f, row["Dispatch_Id"]))
        kt = f.replace("run_counter_collection.csv", "run_kernel_trace.csv")
        if os.path.exists(kt):
            for row in csv.DictReader(open(kt)):
                if a.kernel in row["Kernel_Name"]:
                    dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    if not vals:
        raise SystemExit("no %s rows under %s/pmc_*" % (a.kernel, a.root))
    c = {k: vals[k] / len(dispatches[k]) for k in sorted(vals)}
    fetch, write = c.get("FETCH_SIZE", 0.0) * 1024, c.get("WRITE_SIZE", 0.0) * 1024
    out = {
        "config": a.config, "kernel": a.kernel, "round": a.round,
        "source": "tools/pmc.sh on MI355X: rocprofv3 --kernel-trace --pmc, one pass per counter group, "
                  "one frame per pass; folded by tools/pmc_summary.py",
        "kernel_duration_ms_profiled": sum(dur) / len(dur) if dur else None,
        "counters": c,
        "fetch_bytes_raw": fetch, "write_bytes_raw": write,
        "hbm_bytes_per_launch": 2 * fetch + write,
        "note": "FETCH_SIZE/WRITE_SIZE are KB; gfx950 FETCH_SIZE reads 1/2 of the bytes of wide reads "
                "(MI355X_MICROARCH.md), so hbm_bytes_per_launch = 2*FETCH + WRITE.  Infinity-Cache hits "
                "are included: this is L2->fabric traffic, an upper bound on HBM bytes.",
    }
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        out["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "SQ_WAVE_CYCLES" in c:
        out["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
        out["active_inst_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("hbm_bytes_per_launch", "kernel_duration_ms_profiled")}))


if __name__ == "__main__":
    main()
