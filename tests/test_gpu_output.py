"""GPU parity of the output stage: write_color's bytes of the
f64 colour (color.rs:8-18) from the megakernel, and the PPM text of Camera::render
(camera.rs:101-103,116-118) formatted on the device.

Bar: byte-exact.  The oracle produces the same text from its own f64 colours
(oracle.render_ppm); random byte frames check the encoder alone at every size class
(one block, block boundaries, ragged tails, 4K), against the oracle's formatter.
"""
import ctypes as C

import numpy as np
import pytest

import grayshift_amd as g
from grayshift_amd import _native as N
from grayshift_amd import scenes
import oracle

from tests.test_gpu_volumes import fog_scene

pytestmark = pytest.mark.gpu


def _encode(b8):
    """Device PPM text of an [H,W,3] u8 frame."""
    import torch
    dev = torch.device("cuda", 0)
    h, w = b8.shape[0], b8.shape[1]
    cap = N.lib.gs_ppm_max_bytes(w, h)
    scr = N.lib.gs_ppm_scratch_bytes(w, h)
    src = torch.from_numpy(np.ascontiguousarray(b8).reshape(-1)).to(dev)
    text = torch.full((cap,), 0xAA, dtype=torch.uint8, device=dev)  # poison: no gaps may survive
    n = torch.zeros(1, dtype=torch.int64, device=dev)
    scratch = torch.full(((scr + 7) // 8,), -1, dtype=torch.int64, device=dev)  # encoder must clear it
    stream = torch.cuda.current_stream(dev).cuda_stream
    g.ppm_encode_async(src.data_ptr(), w, h, text.data_ptr(), cap, n.data_ptr(), scratch.data_ptr(), scr, stream)
    torch.cuda.synchronize()
    ln = int(n.item())
    assert 0 < ln <= cap
    return text[:ln].cpu().numpy().tobytes()


@pytest.mark.parametrize("w,h", [(1, 1), (3, 7), (2048, 1), (2049, 1), (45, 91), (2047, 3), (333, 100),
                                 (1920, 1080), (3840, 2160)])
def test_ppm_encoder_matches_oracle_text(w, h):
    rng = np.random.default_rng(w + 7 * h)
    # mix of 1-, 2- and 3-digit values so line lengths vary inside every block
    b8 = rng.choice(np.array([0, 5, 9, 10, 42, 99, 100, 200, 255], np.uint8), size=(h, w, 3))
    assert _encode(b8) == oracle.ppm_text(b8)


@pytest.mark.parametrize("fill", [0, 255])
def test_ppm_encoder_extreme_line_lengths(fill):
    b8 = np.full((37, 301, 3), fill, np.uint8)  # shortest ("0 0 0\n") and longest lines
    assert _encode(b8) == oracle.ppm_text(b8)


def test_ppm_encoder_reuses_scratch_and_is_repeatable():
    rng = np.random.default_rng(5)
    b8 = rng.integers(0, 256, size=(200, 300, 3), dtype=np.uint8)
    assert _encode(b8) == _encode(b8) == oracle.ppm_text(b8)


@pytest.mark.parametrize("name", ["C1", "C3", "C4", "C5"])
def test_render_ppm_matches_oracle(name):
    """Camera::render end to end: device bytes of the f64 colour + device text."""
    sc = scenes.config(name, width=48, spp=8)
    text, gc = g.render_ppm(sc, seed=11)
    ref, rc = oracle.render_ppm(sc, seed=11)
    assert text == ref
    assert gc["paths"] == rc["paths"] and gc["pixels"] == rc["pixels"]


def test_render_ppm_adaptive_and_media():
    sc = scenes.cornell_smoke(width=32, settings=None)  # the reference's adaptive settings
    text, _ = g.render_ppm(sc, seed=3)
    ref, _ = oracle.render_ppm(sc, seed=3)
    assert text == ref
    sc = fog_scene(width=40, spp=8)
    assert g.render_ppm(sc, seed=5)[0] == oracle.render_ppm(sc, seed=5)[0]


def _render_bytes_partitioned(sc, world, tile, seed):
    import torch
    dev = torch.device("cuda", 0)
    cam = g.camera(sc.camera)
    cap0 = N.lib.gs_partition_capacity(C.byref(cam), C.byref(N.gs_partition(0, world, tile, tile)))
    gathered = torch.zeros(world * cap0 * 3, dtype=torch.uint8, device=dev)
    rgb = torch.zeros(world * cap0 * 3, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for r in range(world):
        rr = g.Renderer(sc, rank=r, world_size=world, tile=tile)
        rr.render_ex_async(d_rgb=rgb.data_ptr() + r * cap0 * 12, d_rgb8=gathered.data_ptr() + r * cap0 * 3,
                           stream=stream, seed=seed)
        torch.cuda.synchronize()
        rr.close()
    frame8 = torch.zeros(cam.image_height * cam.image_width * 3, dtype=torch.uint8, device=dev)
    frame = torch.zeros(cam.image_height * cam.image_width * 3, dtype=torch.float32, device=dev)
    rr = g.Renderer(sc, rank=0, world_size=world, tile=tile)
    rr.unpack_u8_async(gathered.data_ptr(), frame8.data_ptr(), world, stream)
    rr.unpack_async(rgb.data_ptr(), frame.data_ptr(), world, stream)
    torch.cuda.synchronize()
    rr.close()
    shp = (cam.image_height, cam.image_width, 3)
    return frame.view(*shp).cpu().numpy(), frame8.view(*shp).cpu().numpy()


@pytest.mark.parametrize("world,tile", [(1, 64), (3, 16), (8, 8)])
def test_rgb8_output_is_partition_invariant(world, tile):
    """Both outputs of one launch: the f32 frame equals gs_render's, the byte frame
    equals the oracle's write_color bytes, for every partition (gathered + unpacked)."""
    sc = scenes.config("C5", width=80, spp=8)
    full, _ = g.render(sc, seed=3)
    rgb, b8 = _render_bytes_partitioned(sc, world, tile, seed=3)
    assert np.array_equal(full, rgb)
    _, _, ref8 = oracle.render(sc, seed=3, bytes_out=True)
    assert np.array_equal(b8, ref8)


def test_rgb8_only_output():
    """rgb may be NULL when rgb8 is set (bytes only, no f32 traffic)."""
    import torch
    sc = scenes.config("C3", width=32, spp=4)
    r = g.Renderer(sc)
    b = torch.zeros(r.capacity * 3, dtype=torch.uint8, device="cuda")
    r.render_ex_async(d_rgb8=b.data_ptr(), stream=torch.cuda.current_stream().cuda_stream, seed=2)
    frame8 = torch.zeros(r.height * r.width * 3, dtype=torch.uint8, device="cuda")
    r.unpack_u8_async(b.data_ptr(), frame8.data_ptr(), 1, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    r.close()
    _, _, ref8 = oracle.render(sc, seed=2, bytes_out=True)
    assert np.array_equal(frame8.view(sc.height, sc.width, 3).cpu().numpy(), ref8)
