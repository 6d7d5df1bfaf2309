#!/usr/bin/env python3
"""Decode the reference's two image assets into committed data fixtures.

The GPU box has no /root/reference, so the scenes' texels travel as data:

* ``earthmap.jpg`` (1024x512 baseline JPEG, used by ``ImageTexture::new``
  texture.rs:77-81) is decoded once with PIL into RGB8.  The reference decodes
  it with the ``image`` 0.25.2 crate (zune-jpeg); IDCT rounding may differ by a
  few LSB, so texel parity against the Rust reference is *unpinned*.  The
  product and the oracle both read this same array.
* ``airport.hdr`` (Radiance RGBE, new-style RLE scanlines, header
  ``-Y 512 +X 1024``, loaded by ``radiant::load`` main.rs:806) is RLE-decoded
  here into its raw RGBE bytes (our own decoder; no third-party code).  The
  RGBE -> f32 step is done at load time by ``grayshift_amd.assets``.

Outputs go to ``grayshift_amd/assets/*.npz`` (compressed, no pickles) and a
``manifest.json`` with the sha256 of every source file and decoded array.

Run: python tools/make_assets.py [--reference /root/reference]
"""
import argparse
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "grayshift_amd", "assets")


def sha256(b):
    return hashlib.sha256(b).hexdigest()


def decode_rgbe_rle(data):
    """Radiance .hdr -> uint8 [H, W, 4] RGBE (top row first for -Y H +X W)."""
    pos = 0
    lines = []
    while True:
        end = data.index(b"\n", pos)
        line = data[pos:end].decode("ascii", "replace")
        pos = end + 1
        lines.append(line)
        if line.strip() == "" and len(lines) > 1:
            break
    if not lines[0].startswith("#?"):
        raise ValueError("not a Radiance file")
    if not any(l.startswith("FORMAT=32-bit_rle_rgbe") for l in lines):
        raise ValueError("unsupported FORMAT")
    end = data.index(b"\n", pos)
    res = data[pos:end].decode("ascii").split()
    pos = end + 1
    if len(res) != 4 or res[0] != "-Y" or res[2] != "+X":
        raise ValueError("unsupported orientation %r" % res)
    h, w = int(res[1]), int(res[3])
    out = np.zeros((h, w, 4), dtype=np.uint8)
    buf = memoryview(data)
    for y in range(h):
        b0, b1, b2, b3 = buf[pos], buf[pos + 1], buf[pos + 2], buf[pos + 3]
        if b0 == 2 and b1 == 2 and (b2 & 0x80) == 0 and 8 <= w < 32768:
            if ((b2 << 8) | b3) != w:
                raise ValueError("scanline width mismatch")
            pos += 4
            for c in range(4):
                x = 0
                while x < w:
                    n = buf[pos]
                    pos += 1
                    if n > 128:
                        n -= 128
                        out[y, x:x + n, c] = buf[pos]
                        pos += 1
                    else:
                        if n == 0:
                            raise ValueError("bad RLE count")
                        out[y, x:x + n, c] = np.frombuffer(buf[pos:pos + n], dtype=np.uint8)
                        pos += n
                    x += n
        else:  # flat scanline
            out[y] = np.frombuffer(buf[pos:pos + 4 * w], dtype=np.uint8).reshape(w, 4)
            pos += 4 * w
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    from PIL import Image  # only needed to regenerate the fixture

    jpg_path = os.path.join(a.reference, "earthmap.jpg")
    hdr_path = os.path.join(a.reference, "airport.hdr")
    jpg = open(jpg_path, "rb").read()
    hdr = open(hdr_path, "rb").read()

    earth = np.asarray(Image.open(jpg_path).convert("RGB"), dtype=np.uint8)
    rgbe = decode_rgbe_rle(hdr)
    np.savez_compressed(os.path.join(OUT, "earthmap_rgb8.npz"), rgb8=earth)
    np.savez_compressed(os.path.join(OUT, "airport_rgbe.npz"), rgbe=rgbe)
    manifest = {
        "earthmap.jpg": {"sha256": sha256(jpg), "decoded": "earthmap_rgb8.npz",
                          "shape": list(earth.shape), "decoded_sha256": sha256(earth.tobytes()),
                          "decoder": "PIL %s" % Image.__version__ if hasattr(Image, "__version__") else "PIL"},
        "airport.hdr": {"sha256": sha256(hdr), "decoded": "airport_rgbe.npz",
                         "shape": list(rgbe.shape), "decoded_sha256": sha256(rgbe.tobytes()),
                         "decoder": "tools/make_assets.py decode_rgbe_rle"},
    }
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=2)
    print(json.dumps(manifest, indent=2))


if __name__ == "__main__":
    main()
