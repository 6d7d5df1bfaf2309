"""Image-space partition of include/grayshift_gpu.h (gs_partition), in Python.

Tile k of the frame (row-major over tiles_x x tiles_y tiles of tile_w x tile_h)
belongs to rank k mod world_size.  A rank packs its tiles slot after slot, each
tile row-major inside and padded to whole tiles.  ``packed_pixel_ids`` gives, for
every packed slot, the frame pixel id (j*W + i) it holds, or -1 for padding —
the same mapping gs_render_tiles_async writes and gs_unpack_tiles_async reads.
"""
import numpy as np


def tiles(width, height, tile_w, tile_h):
    return (width + tile_w - 1) // tile_w, (height + tile_h - 1) // tile_h


def capacity(width, height, rank, world_size, tile_w, tile_h):
    tx, ty = tiles(width, height, tile_w, tile_h)
    nt = tx * ty
    mine = (nt - rank + world_size - 1) // world_size if nt > rank else 0
    return mine * tile_w * tile_h


def packed_pixel_ids(width, height, rank, world_size, tile_w, tile_h):
    tx, _ = tiles(width, height, tile_w, tile_h)
    cap = capacity(width, height, rank, world_size, tile_w, tile_h)
    k = np.arange(cap, dtype=np.int64)
    tp = tile_w * tile_h
    slot, w = k // tp, k % tp
    tile = rank + slot * world_size
    x = (tile % tx) * tile_w + w % tile_w
    y = (tile // tx) * tile_h + w // tile_w
    ids = y * width + x
    ids[(x >= width) | (y >= height)] = -1
    return ids


def unpack(gathered, width, height, world_size, tile_w, tile_h, cap):
    """numpy restatement of gs_unpack_tiles_async: [world*cap, 3] -> [H, W, 3]."""
    frame = np.zeros((height * width, 3), dtype=gathered.dtype)
    g = gathered.reshape(world_size, cap, 3)
    for r in range(world_size):
        ids = packed_pixel_ids(width, height, r, world_size, tile_w, tile_h)
        n = len(ids)
        ok = ids >= 0
        frame[ids[ok]] = g[r, :n][ok]
    return frame.reshape(height, width, 3)
