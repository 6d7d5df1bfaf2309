#!/usr/bin/env python3
"""Instruction census of the traversal loop's node and leaf passes (static, from the ISA).

Compiles render.hip for gfx950 with -DGS_ISA_MARKS (assembler comments delimit the
regions; everything else is the product build's flags), extracts one kernel
instantiation (default FEAT=20: the C4 kernel, leaf runs + staged shading) and counts instructions by class:

* loop head: from the traversal loop's header label to the node-pass mark (ballots,
  shade-count and pass-kind tests, shared by both passes);
* node pass: node_begin .. node_end minus the f64 fallback block (taken only by lanes
  the certified f32 test leaves undecided) and the f64 path of waves holding a non-cert
  ray (both listed on their own);
* leaf pass: leaf_begin .. leaf_end minus the other-kind leaves (moving spheres, quads,
  triangles, lists, instances, media: listed on their own), i.e. the stationary-sphere
  path with its leaf run (a run's second sphere counted statically once);
* shade pass: shade_begin .. shade_end (hit record, scatter, throughput);
* advance + get_ray: adv_begin .. adv_end (a finished sample's sums, the next item's claim,
  the camera ray).

    python tools/isa_census.py [--feat 4] [--dump profiles/r02/isa_node_leaf.s]
"""
import argparse
import os
import re
import subprocess
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "grayshift_amd", "csrc", "device", "render.hip")


def classify(op):
    if op.startswith(("v_cmp", "v_cmpx")):
        return "VALU"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch", "s_endpgm", "s_setprio", "s_sleep")):
        return "ctrl"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "SMEM"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    return "other"


def census(lines):
    c = Counter()
    f64 = 0
    for l in lines:
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c[classify(op)] += 1
        if op.startswith("v_") and ("_f64" in op or op.startswith("v_div")):
            f64 += 1
    c["VALU_f64"] = f64
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--feat", type=int, default=20)
    ap.add_argument("--dump", default=None, help="write the marked regions' assembly here")
    ap.add_argument("--dump-kernel", default=None, help="write the whole instantiation's assembly here")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-x", "hip",
               "--offload-arch=gfx950", "-mllvm", "-disable-machine-licm", "-DGS_ISA_MARKS", "--save-temps", "-c", SRC,
               "-o", os.path.join(d, "r.o")]
        subprocess.run(cmd, check=True, cwd=d, stderr=subprocess.DEVNULL)
        s = open(os.path.join(d, "render-hip-amdgcn-amd-amdhsa-gfx950.s")).read().splitlines()
    name = "_Z16gs_render_kernelILi%dEEv5KArgs:" % a.feat
    i0 = next(i for i, l in enumerate(s) if l.startswith(name))
    i1 = next(i for i in range(i0, len(s)) if s[i].startswith(".Lfunc_end"))
    k = s[i0:i1]
    if a.dump_kernel:
        open(a.dump_kernel, "w").write("\n".join(k) + "\n")
    marks = {}
    for i, l in enumerate(k):
        m = re.search(r";; GS_MARK (\w+)", l)
        if m:
            marks.setdefault(m.group(1), []).append(i)
    nb, ne = marks["node_begin"][0], marks["node_end"][0]
    fb, fe = marks["fallback_begin"][0], marks["fallback_end"][0]
    lb, le = marks["leaf_begin"][0], marks["leaf_end"][-1]
    # sphere-only kernels (GS_FEAT_SPHLEAF) have no other-kind leaf region
    ob, oe = (marks["other_begin"][0], marks["other_end"][0]) if "other_begin" in marks else (le, le)
    # the traversal loop header: the last "Loop Header" label before node_begin
    hdr = max(i for i in range(nb) if "Loop Header" in k[i] or "This Loop Header" in k[i])
    # The compiler spreads the f64 test's code (fallback and non-cert waves) over several
    # basic blocks between the marks: the node pass of a cert wave is the region's blocks
    # that hold no f64 instruction, the f64 blocks are listed on their own.
    blocks, cur = [], []
    for l in k[nb:ne]:
        if re.match(r"^\.LBB\d+_\d+:|^; %bb\.\d+:", l) and cur:
            blocks.append(cur)
            cur = []
        cur.append(l)
    blocks.append(cur)
    has64 = lambda b: any(re.match(r"\s+v_\w*(_f64|div_)", l) for l in b)
    node = [l for b in blocks if not has64(b) for l in b]
    node64 = [l for b in blocks if has64(b) for l in b]
    sph_b, sph_e = marks["sphere_begin"][0], marks["sphere_end"][0]
    regions = {"loop head": k[hdr:nb], "node pass (cert wave)": node,
               "  f64 test blocks (rare paths)": node64,
               "leaf pass (head, links, run)": k[lb:sph_b] + k[sph_e:ob] + k[oe:le],
               "  stationary-sphere test": k[sph_b:sph_e], "  other leaf kinds": k[ob:oe]}
    # the shade pass (hit record, material scatter, throughput) and the sample advance
    # (chunk sums, refill, camera ray: get_ray) when the instantiation has their marks
    for nm, b, e in (("shade pass", "shade_begin", "shade_end"), ("advance + get_ray", "adv_begin", "adv_end")):
        if b in marks and e in marks:
            regions[nm] = k[marks[b][0]:marks[e][-1]]
    print("gs_render_kernel<%d> (gfx950, static instruction counts)" % a.feat)
    print("%-32s %6s %6s %6s %6s %6s %6s" % ("region", "VALU", "(f64)", "SALU", "VMEM", "LDS", "ctrl"))
    for n, r in regions.items():
        c = census(r)
        print("%-32s %6d %6d %6d %6d %6d %6d" % (n, c["VALU"], c["VALU_f64"], c["SALU"], c["VMEM"], c["LDS"], c["ctrl"]))
    if a.dump:
        with open(a.dump, "w") as f:
            for n, r in regions.items():
                f.write(";; ===== %s =====\n" % n)
                f.write("\n".join(r) + "\n")
        print("wrote", a.dump)


if __name__ == "__main__":
    main()
