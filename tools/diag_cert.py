"""Diagnostic (variants/certcheck.so, -DGS_CERT_CHECK): certified f32 node decisions that
disagree with the f64 test, on a scene."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import grayshift_amd as g
from grayshift_amd import _native as N, scenes
from grayshift_amd.scene import fixed_spp
name = sys.argv[1] if len(sys.argv) > 1 else "final_scene"
# a BASELINE config at its full size and spp (or width / spp given after it), else a scene
# at 40 px, 8 spp
if name in scenes.CONFIGS or len(sys.argv) > 3:
    kw = {"width": int(sys.argv[2]), "spp": int(sys.argv[3])} if len(sys.argv) > 3 else {}
    sc = scenes.config(name, **kw)
else:
    sc = scenes.SCENES[name](width=40, settings=fixed_spp(8))
r = g.Renderer(sc)
dev = torch.device("cuda", 0)
packed = torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev)
cnt = torch.zeros(16, dtype=torch.int64, device=dev)
dbg = torch.zeros(max(64 * 16 * 2, r.capacity), dtype=torch.float64, device=dev)
N.check(N.lib.gs_render_tiles_debug_async(r.dev, C.byref(r.cam), C.byref(r.settings), 21, C.byref(r.part),
                                          C.c_void_p(packed.data_ptr()), C.c_void_p(cnt.data_ptr()),
                                          C.c_void_p(dbg.data_ptr()), None))
torch.cuda.synchronize()
n = int(cnt[15].item())
print(name, "mismatches", n, "node visits", int(cnt[1].item()))
rec = dbg[:64 * 16].view(64, 16).cpu().numpy()
np.set_printoptions(precision=17, linewidth=200)
for k in range(min(n, 5)):
    print(rec[k].tolist())
