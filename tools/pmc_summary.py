"""Fold tools/pmc.sh's per-pass rocprofv3 CSVs into one JSON per kernel launch.

    python tools/pmc_summary.py gpurun_out profiles/pmc [--config C4] [--kernel gs_render_kernel]

Writes <out_dir>/<config>_<code-object hash>.json: bench.py reads the summary of the very
code object it times (grayshift_amd/codeobj.py hashes libgrayshift.so's gfx950 code).

Counter values are summed over the kernel's dispatches and divided by their number
(per-launch figures).  HBM bytes follow MI355X_MICROARCH.md's gfx950 correction:
FETCH_SIZE / WRITE_SIZE are KB and FETCH_SIZE counts half the bytes of wide reads, so
hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
"""
import argparse
import re
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
    ap.add_argument("--exclude", default="",
                    help="comma-separated kernel-name substrings to skip as well (the placement pilot's "
                         "counting instantiations -- template argument with GS_FEAT_VISITS, 32: <55>, <183> "
                         "-- are always skipped)")
    ap.add_argument("--config", default="C4")
    ap.add_argument("--round", type=int, default=3)
    ap.add_argument("--lib", default=None, help="the library profiled (default: the in-tree libgrayshift.so)")
    a = ap.parse_args()
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from grayshift_amd.codeobj import code_object_hash
    lib = a.lib or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "grayshift_amd",
                                "libgrayshift.so")
    h = code_object_hash(lib)
    excl = [x for x in a.exclude.split(",") if x]

    def skipped(name):
        # the pilot's instantiations count every record's tests (GS_FEAT_VISITS = 32)
        m = re.search(r"gs_render_kernel<(\d+)>", name)
        if m and int(m.group(1)) & 32:
            return True
        return any(x in name for x in excl)

    vals = defaultdict(float)
    dispatches = defaultdict(set)
    dur = []
    for f in sorted(glob.glob(os.path.join(a.root, "pmc_*", "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if a.kernel not in row["Kernel_Name"] or skipped(row["Kernel_Name"]):
                continue
            name = row["Counter_Name"]
            vals[name] += float(row["Counter_Value"])
            dispatches[name].add((f, row["Dispatch_Id"]))
        kt = f.replace("run_counter_collection.csv", "run_kernel_trace.csv")
        if os.path.exists(kt):
            for row in csv.DictReader(open(kt)):
                if a.kernel in row["Kernel_Name"] and not skipped(row["Kernel_Name"]):
                    dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    if not vals:
        raise SystemExit("no %s rows under %s/pmc_*" % (a.kernel, a.root))
    c = {k: vals[k] / len(dispatches[k]) for k in sorted(vals)}
    fetch, write = c.get("FETCH_SIZE", 0.0) * 1024, c.get("WRITE_SIZE", 0.0) * 1024
    out = {
        "config": a.config, "kernel": a.kernel, "round": a.round, "code_object": h,
        "source": "tools/pmc.sh on MI355X: rocprofv3 --kernel-trace --pmc, one pass per counter group, "
                  "one frame per pass; folded by tools/pmc_summary.py",
        "kernel_duration_ms_profiled": sum(dur) / len(dur) if dur else None,
        # megakernel launches in one frame (one per batch round and sample-buffer segment for
        # adaptive settings; 1 otherwise): the counters above are per launch
        "dispatches_per_frame": len(dispatches.get("SQ_ACTIVE_INST_VALU", dispatches[next(iter(dispatches))])),
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
    if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0  # per-XCD cycles (rocprofv3 sums the 8 XCDs)
        out["valu_issue_frac"] = c["SQ_INSTS_VALU"] * 4 / (1024 * cyc)
        if "SQ_ACTIVE_INST_VALU" in c:
            out["valu_active_frac"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * cyc)
            if "SQ_ACTIVE_INST_VALU2" in c:  # the measured busy fraction bench.py reports
                out["valu_busy_frac"] = 4 * (c["SQ_ACTIVE_INST_VALU"] - c["SQ_ACTIVE_INST_VALU2"]) / (1024 * cyc)
        if "SQ_INSTS_SALU" in c:
            out["salu_issue_frac"] = c["SQ_INSTS_SALU"] / (1024 * cyc)
    if "SQ_LDS_IDX_ACTIVE" in c and "GRBM_GUI_ACTIVE" in c:
        out["lds_busy_frac"] = c["SQ_LDS_IDX_ACTIVE"] / (256 * c["GRBM_GUI_ACTIVE"] / 8.0)
    os.makedirs(a.out, exist_ok=True)
    path = os.path.join(a.out, "%s_%s.json" % (a.config, h))
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path)
    print(json.dumps({k: out[k] for k in ("hbm_bytes_per_launch", "kernel_duration_ms_profiled")}))


if __name__ == "__main__":
    main()
