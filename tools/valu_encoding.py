#!/usr/bin/env python3
"""VALU issue cost of the C4 kernel's hot regions by instruction encoding (static, from the
gfx950 ISA), for the roofline's issue-cycle estimate.

tools/ubench/valu_rate.hip measured (profiles/r03/valu_rate_ubench.txt, 8 waves/SIMD):
VOP1/VOP2/VOPC forms (the compiler's `_e32` mnemonics) with VGPR operands issue in ~2.2
cycles per wave64 instruction on a SIMD; VOP3 / VOP3P forms (`_e64`, three-operand and
packed instructions, SGPR or literal operands) in ~4.1; every f64 add / mul / fma in ~4.1;
v_sqrt_f32 / v_rcp_f32 class 8; f64 transcendentals 16.  This tool classifies every VALU
instruction of each marked region (GS_ISA_MARKS) of one instantiation and prints the mean
cost per instruction, which bench.py's PMC instruction classes cannot resolve.

    python tools/valu_encoding.py [--feat 84]
"""
import argparse
import os
import re
import subprocess
import tempfile
from collections import Counter, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "grayshift_amd", "csrc", "device", "render.hip")


def cost(op):
    base = op.split("_e32")[0].split("_e64")[0]
    if re.match(r"v_(sqrt|rsq|rcp|exp|log|sin|cos)_f64", base):
        return 16.0
    if re.match(r"v_(sqrt|rsq|rcp|exp|log|sin|cos|rcp_iflag)_f32", base):
        return 8.0
    if "f64" in base or "_u64" in base or "_i64" in base or base.startswith("v_pk_") or "b64" in base:
        return 4.1
    if op.endswith("_e32") or op in ("v_readfirstlane_b32", "v_nop"):
        return 2.2
    return 4.1  # VOP3 / VOP3P encodings (explicit _e64, three-operand, modifiers, literals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--feat", type=int, default=84)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "r.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
                        "-x", "hip", "--offload-arch=gfx950", "-mllvm", "-disable-machine-licm", "-DGS_ISA_MARKS",
                        "--save-temps", "-c", SRC, "-o", out], cwd=td, check=True, stderr=subprocess.DEVNULL)
        asm = open(os.path.join(td, "render-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    sym = "_Z16gs_render_kernelILi%dEEv5KArgs:" % a.feat
    body = asm[asm.index(sym):]
    body = body[:body.index("s_endpgm")]
    region = "entry"
    per = defaultdict(Counter)
    for line in body.split("\n"):
        m = re.search(r"GS_MARK (\w+)", line)
        if m:
            region = m.group(1)
            continue
        t = line.strip().split()
        if not t or not t[0].startswith("v_"):
            continue
        per[region][t[0]] += 1
    print("gs_render_kernel<%d>: VALU instructions per region (static), mean issue cycles per instruction" % a.feat)
    print("%-16s %6s %8s %8s %8s %8s" % ("region (after)", "VALU", "2.2-cyc", "4.1-cyc", "trans", "mean"))
    for r, c in per.items():
        n = sum(c.values())
        cy = sum(cost(op) * k for op, k in c.items())
        two = sum(k for op, k in c.items() if cost(op) == 2.2)
        tr = sum(k for op, k in c.items() if cost(op) >= 8)
        print("%-16s %6d %8d %8d %8d %8.2f" % (r, n, two, n - two - tr, tr, cy / max(1, n)))


if __name__ == "__main__":
    main()
