#!/bin/bash
# Per-instantiation VGPRs / scratch of render.hip (gfx950, the product's flags + any extra
# flags given): "FEAT vgprs scratch-bytes-per-lane".  usage: bash tools/resource_usage.sh [-DX=1 ...]
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -x hip --offload-arch=gfx950 \
    -mllvm -disable-machine-licm -Rpass-analysis=kernel-resource-usage "$@" \
    -c "$R/grayshift_amd/csrc/device/render.hip" -o "$T/r.o" 2> "$T/ru.txt" || { tail -20 "$T/ru.txt"; exit 1; }
python3 - "$T/ru.txt" <<'PY'
import re, sys
cur = None
for l in open(sys.argv[1]):
    m = re.search(r"Function Name: _Z16gs_render_kernelILi(\d+)E", l)
    if m: cur = m.group(1); row = [cur]; continue
    if cur is None: continue
    m = re.search(r" VGPRs: (\d+)", l)
    if m: row.append(m.group(1))
    m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", l)
    if m: row.append(m.group(1)); print("feat %-3s vgprs %-4s scratch %s" % tuple(row)); cur = None
PY
rm -rf "$T"
