#!/usr/bin/env python3
"""Phase split of the megakernel (diagnostic build variants/stamps.so, -DGS_STAMPS).
GS_LIB=grayshift_amd/variants/stamps.so python tools/stamps.py [--config C4] [tuning] [--json DIR]

--json DIR writes the lane-efficiency summary bench.py reads into its roofline
(DIR/<config>_<product code-object hash>.json): each phase's wave clock and active lanes
of 64, and lane_frac, their clock-weighted mean.  The stamps build is a
different binary than the product (its clock reads perturb scheduling, so only shares are
meaningful); the summary is keyed by the product library built from the same sources."""
import argparse, ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--shade-batch", type=int, default=0, help="0: the scene's own")
    ap.add_argument("--leaf-batch", type=int, default=0, help="0: the scene's choice")
    ap.add_argument("--sample-chunk", type=int, default=-1)
    ap.add_argument("--node-steps", type=int, default=0, help="0: the scene's own")
    ap.add_argument("--json", default=None, help="write the lane-efficiency summary into this directory")
    ap.add_argument("--tag", default=None, help="the summary's config name (default: --config, or "
                                                   "<config>_w<width>_s<spp> for an overridden size)")
    a = ap.parse_args()
    import torch
    import grayshift_amd as g
    from grayshift_amd import _native as N, scenes
    g.set_tuning(a.shade_batch, 0, a.leaf_batch, a.sample_chunk)
    N.check(N.lib.gs_set_node_steps(a.node_steps))
    sc = scenes.config(a.config, width=a.width, spp=a.spp)
    r = g.Renderer(sc, 0, 1, 64)
    dev = torch.device("cuda", 0)
    packed = torch.zeros(r.capacity * 3, dtype=torch.float32, device=dev)
    dbg = torch.zeros(max(40, r.capacity // 2 + 2), dtype=torch.int64, device=dev)
    N.check(N.lib.gs_render_tiles_debug_async(r.dev, C.byref(r.cam), C.byref(r.settings), 1, C.byref(r.part),
                                              C.c_void_p(packed.data_ptr()), None, C.c_void_p(dbg.data_ptr()), None))
    torch.cuda.synchronize()
    v = dbg[:3].cpu().tolist()
    tot = sum(v)
    print("refill %.1f%%  traverse %.1f%%  shade %.1f%%  (wave-clock totals %s)" % (
        100 * v[0] / tot, 100 * v[1] / tot, 100 * v[2] / tot, v))
    it_all, it_node, it_leaf, ln_node, ln_leaf, it_shade, ln_shade = dbg[3:10].cpu().tolist()
    print("traversal iterations %d: node passes %d (%.1f active lanes), leaf passes %d (%.1f lanes); "
          "shade passes %d (%.1f lanes)" % (it_all, it_node, ln_node / max(1, it_node), it_leaf,
                                           ln_leaf / max(1, it_leaf), it_shade, ln_shade / max(1, it_shade)))
    node_clk, leaf_clk, dist_ref, dist_kind = dbg[15:19].cpu().tolist()
    print("traversal split (wave clock, per-iteration stamps): node passes %.1f%%  leaf passes %.1f%%" % (
        100.0 * node_clk / max(1, node_clk + leaf_clk), 100.0 * leaf_clk / max(1, node_clk + leaf_clk)))
    print("leaf passes: %.2f distinct refs, %.2f distinct ref kinds per pass" % (
        dist_ref / max(1, it_leaf), dist_kind / max(1, it_leaf)))
    gvis, wsteps, wsteps_g, wlanes = dbg[19:23].cpu().tolist()
    print("node steps: %d wave steps (%.1f active lanes), %.1f%% with a lane reading global memory; "
          "%.1f%% of lane node visits from global memory" % (
              wsteps, wlanes / max(1, wsteps), 100.0 * wsteps_g / max(1, wsteps), 100.0 * gvis / max(1, wlanes)))
    bad = int(dbg[23].item())
    if bad:
        print("WARNING: %d leaf passes whose exec mask held lanes outside the ballot (their distinct-ref / kind counts are not trusted)" % bad)
    kinds = dbg[24:32].cpu().tolist()
    if sum(kinds):
        names = ["node", "sphere", "msphere", "quad", "triangle", "list", "instance", "medium"]
        print("leaf-kind clock (%% of leaf-pass clock; a pass's non-sphere branch by its first lane's ref kind): " +
              "  ".join("%s %.1f%%" % (n, 100.0 * x / max(1, leaf_clk)) for n, x in zip(names, kinds) if x))
    rc_clk, ret_clk = dbg[34:36].cpu().tolist()
    if rc_clk or ret_clk:
        print("leaf passes of nested / media-run kernels: cert constants recomputed %.1f%%, return passes %.1f%% "
              "of the leaf-pass clock" % (100.0 * rc_clk / max(1, leaf_clk), 100.0 * ret_clk / max(1, leaf_clk)))
    reg = dbg[10:15].cpu().tolist()
    # split shading (no GS_FEAT_MIXED) stamps background / reconstruct / scatter on their own;
    # staged shading (GS_FEAT_MIXED, media, nested) stamps all of it as region 2
    print("shade regions (%% of shade clock): " + "  ".join(
        "%s %.1f%%" % (n, 100.0 * x / max(1, v[2])) for n, x in
        zip(["background", "reconstruct", "scatter (staged: all shading)", "-", "add_sample + chunk end"], reg)))
    # camera rays (advance) and begin_ray run at the loop head since r02: inside "refill"
    it_adv, ln_adv = dbg[32:34].cpu().tolist()
    phases = {  # wave clock, mean active lanes of 64
        "node passes (per node step)": (node_clk, wlanes / max(1, wsteps)),
        "leaf passes": (leaf_clk, ln_leaf / max(1, it_leaf)),
        "shade passes": (v[2], ln_shade / max(1, it_shade)),
    }
    if it_adv:
        phases["refill + camera rays (per get_ray)"] = (v[0], ln_adv / it_adv)
    tot_clk = sum(p[0] for p in phases.values())
    lane_frac = sum(p[0] * p[1] / 64.0 for p in phases.values()) / max(1, tot_clk)
    print("lanes of 64 by phase: " + "  ".join("%s %.1f" % (k, p[1]) for k, p in phases.items()) +
          "  -> clock-weighted lane_frac %.3f" % lane_frac)
    if a.json:
        from grayshift_amd.codeobj import code_object_hash
        prod = os.path.join(ROOT, "grayshift_amd", "libgrayshift.so")
        h = code_object_hash(prod)
        tag = a.tag or (a.config if a.width is None and a.spp is None else "%s_w%s_s%s" % (a.config, a.width, a.spp))
        os.makedirs(a.json, exist_ok=True)
        out = {"config": tag, "code_object": h, "stamps_library": os.environ.get("GS_LIB", ""),
               "source": "tools/stamps.py on MI355X: the -DGS_STAMPS build's per-wave phase clocks and active-lane counts, one frame",
               "phases": {k: {"wave_clock": int(p[0]), "active_lanes": round(p[1], 2)} for k, p in phases.items()},
               "wave_clock_split": {"refill": v[0], "traverse": v[1], "shade": v[2]},
               "lane_frac": round(lane_frac, 4),
               "definition": "sum over phases of wave_clock x active_lanes / 64, over the phases' wave clock"}
        path = os.path.join(a.json, "%s_%s.json" % (tag, h))
        json.dump(out, open(path, "w"), indent=1)
        print("wrote", path)


if __name__ == "__main__":
    main()
