"""Build the in-tree native libraries.

* ``grayshift_amd/libgrayshift.so`` — the product: HIP megakernel for gfx950 plus
  the C++ host mirror, one shared library (hipcc; no torch, no JIT cache).
* ``oracle/liboracle.so`` — the CPU checker (test infrastructure; g++ via
  oracle/Makefile).

Both are compiled with ``-ffp-contract=off``: the reference's Rust f64 code
never fuses multiply-add, and neither may we.

Usage: python -m grayshift_amd.build [--force] [--no-oracle]
"""
import argparse
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libgrayshift.so")
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")

SOURCES = [
    os.path.join(HERE, "csrc", "device", "render.hip"),
    os.path.join(HERE, "csrc", "device", "output.hip"),
    os.path.join(HERE, "csrc", "host", "world.cpp"),
    os.path.join(HERE, "csrc", "host", "camera.cpp"),
    os.path.join(HERE, "csrc", "host", "host_capi.cpp"),
    os.path.join(HERE, "csrc", "host", "multi_gpu.cpp"),
]
DEPS = SOURCES + [
    os.path.join(HERE, "csrc", "device", "devmath.hpp"),
    os.path.join(HERE, "csrc", "device", "geometry.hpp"),
    os.path.join(HERE, "csrc", "device", "perlin.hpp"),
    os.path.join(HERE, "csrc", "host", "world.hpp"),
    os.path.join(ROOT, "include", "grayshift_gpu.h"),
    os.path.join(ROOT, "include", "grayshift_host.h"),
    os.path.join(ROOT, "include", "grayshift_scene.h"),
    os.path.abspath(__file__),  # the compiler flags
]

ARCH = os.environ.get("GS_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall",
          "-Wno-unused-parameter", "-Wno-unused-variable"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_product(force=False, verbose=False, extra=(), out=None):
    """Build libgrayshift.so (or a variant at `out` with extra compiler flags)."""
    lib = out or LIB
    if not force and not _stale(lib, DEPS):
        return lib
    objs = []
    tag = "" if out is None else "_" + os.path.basename(out).replace(".so", "")
    for src in SOURCES:
        obj = os.path.join(HERE, "csrc", "_obj" + tag, os.path.basename(src) + ".o")
        os.makedirs(os.path.dirname(obj), exist_ok=True)
        cmd = [HIPCC] + COMMON + list(extra)
        if src.endswith(".hip"):
            # Machine LICM hoists the f64 polynomial constants of OCML's asin/atan2/acos
            # out of the megakernel's loop, then spills them to per-lane scratch (344 B/lane)
            # and reloads each one with a dependent scratch load: measured on MI355X C4,
            # disabling it removes all scratch and runs +19% (1990 -> 2370 Msamples/s).
            cmd += ["-x", "hip", "--offload-arch=" + ARCH, "-mllvm", "-disable-machine-licm"]
            # A fixed compilation-unit id: clang's default hashes the command line, -o
            # included, into a symbol of the code object, so the same sources built into
            # another directory would hash differently (grayshift_amd/codeobj.py keys the
            # committed PMC summaries by the code objects' hash).
            cmd += ["-cuid=gs_" + os.path.basename(src).replace(".", "_")]
        cmd += ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = lib + ".tmp"
    cmd = [HIPCC, "-shared", "--offload-arch=" + ARCH, "-o", tmp] + objs + ["-lpthread", "-ldl"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    return lib


KAT_SRC = os.path.join(ROOT, "tests", "hip", "kat_device.hip")
KAT_LIB = os.path.join(ROOT, "tests", "hip", "libkat_device.so")


def build_kat(force=False, verbose=False):
    """Test-only HIP harness running the kernel's device functions on test arrays."""
    deps = [KAT_SRC] + DEPS
    if not force and not _stale(KAT_LIB, deps):
        return KAT_LIB
    cmd = [HIPCC] + COMMON + ["-x", "hip", "--offload-arch=" + ARCH, "-shared", "-o", KAT_LIB + ".tmp", KAT_SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(KAT_LIB + ".tmp", KAT_LIB)
    return KAT_LIB


def build_oracle(force=False, verbose=False):
    if force and os.path.exists(ORACLE_LIB):
        os.remove(ORACLE_LIB)
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)
    return ORACLE_LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--variant", action="append", metavar="NAME:FLAGS", default=[],
                    help="also build variants/NAME.so with extra FLAGS (A/B), e.g. --variant 'v4:-DGS_MIN_WAVES=4'")
    ap.add_argument("--resource-usage", action="store_true",
                    help="print per-kernel VGPR/SGPR/LDS/occupancy (hipcc remarks)")
    a = ap.parse_args(argv)
    extra = ["-Rpass-analysis=kernel-resource-usage"] if a.resource_usage else []
    import concurrent.futures as cf

    def variant(spec):
        name, _, flags = spec.partition(":")
        path = os.path.join(HERE, "variants", name + ".so")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        build_product(force=True, verbose=a.verbose, extra=extra + flags.split(), out=path)
        return "variant %s %s" % (path, flags)

    # the product and the variants side by side (each compile is one process; 4 at a time)
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        jobs = [ex.submit(build_product, force=a.force or a.resource_usage, verbose=a.verbose, extra=extra)]
        jobs += [ex.submit(variant, spec) for spec in a.variant]
        for j in jobs[1:]:
            print(j.result())
        jobs[0].result()
    if not a.no_oracle:
        build_oracle(force=a.force, verbose=a.verbose)
        build_kat(force=a.force, verbose=a.verbose)
    print("built", LIB, "" if a.no_oracle else ORACLE_LIB)


if __name__ == "__main__":
    sys.exit(main())
