"""The reference's two image assets, as committed data fixtures.

See tools/make_assets.py for how they were produced from /root/reference and
assets/manifest.json for the sha256 of sources and decoded arrays.
"""
import functools
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")


@functools.lru_cache(maxsize=None)
def earthmap_rgb8():
    """earthmap.jpg decoded to uint8 [512, 1024, 3] (ImageTexture::new, texture.rs:77-81)."""
    with np.load(os.path.join(HERE, "earthmap_rgb8.npz"), allow_pickle=False) as z:
        a = z["rgb8"]
    a.setflags(write=False)
    return a


def rgbe_to_f32(rgbe):
    """radiant 0.3.0 RGBE -> f32 RGB: m * 2^(e - 136), e == 0 -> black.

    Restated from the crate's published conversion (the crate is not in the
    container): every value is an exact power-of-two scaling of an 8-bit mantissa.
    """
    m = rgbe[..., :3].astype(np.float64)
    e = rgbe[..., 3].astype(np.int32)
    out = np.ldexp(m, (e - 136)[..., None]).astype(np.float32)  # exact for this file's exponents
    out[e == 0] = 0.0
    return out


@functools.lru_cache(maxsize=None)
def airport_hdr_f32():
    """airport.hdr as f32 [512, 1024, 3], top row first (radiant::Image layout)."""
    with np.load(os.path.join(HERE, "airport_rgbe.npz"), allow_pickle=False) as z:
        rgbe = z["rgbe"]
    a = np.ascontiguousarray(rgbe_to_f32(rgbe))
    a.setflags(write=False)
    return a
