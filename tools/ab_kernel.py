#!/usr/bin/env python3
"""A/B of render-kernel option sets on one GPU, interleaved rounds in one process (cdna guide §5.4
rule 24), each variant checked bit for bit against the production option set.

usage: python tools/ab_kernel.py [--config c2] [--rounds 5] [--spp 64] [--stats]
"""
import argparse
import ctypes as C
import json
import statistics
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "path-tracer-and-rasterizer-engine_amd"))

import numpy as np  # noqa: E402

from iqpt import _build, _lib  # noqa: E402

OPT = {"cam": 1, "acc": 2, "pair": 4, "sincos": 32, "stats": 128}
DEFAULT = 0   # the library's production mask (iqpt_debug_default_options), set after loading it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="", help="run one variant for --frames frames (profiling)")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--stats-opt", type=int, default=-1, help="option mask of the stats run (default: production)")
    ap.add_argument("--crop", default="", help="x0,x1,y0,ystep,nrows pixel set")
    ap.add_argument("--variants", default="", help="comma list of name=optmask")
    ap.add_argument("--scene", default="", help="empty | walls (cornell without spheres) | preset name")
    ap.add_argument("--timeline-npy", default="", help="save the stats run's raw per-wave records (.npy)")
    ap.add_argument("--lib", default="", help="load this prebuilt A/B library (compiler-option runs)")
    args = ap.parse_args()
    lib_path = Path(args.lib) if args.lib else _build.build_lib(stats=True)
    _lib.LIB_PATH = lib_path                    # load the instrumented build instead of the production one
    lib = _lib.load()
    global DEFAULT
    DEFAULT = lib.iqpt_debug_default_options()
    if args.stats_opt < 0:
        args.stats_opt = DEFAULT
    lib.iqpt_debug_set_kernel_options.argtypes = [C.c_void_p, C.c_int]
    lib.iqpt_debug_read_stats.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    import iqpt
    from iqpt.scene import CONFIGS
    cfg = CONFIGS[args.config]
    spp = args.spp or cfg.spp
    sc = iqpt.Scene()
    if args.scene == "empty":
        pass
    elif args.scene == "walls":
        sc.add_mesh_quad("quad")
        wall = (2.0, 2.0, 1.0, 1.0)
        sc.add_model("back", "quad", wall, 0.0, (0.0, 0.5, 1.0))
        sc.add_model("floor", "quad", wall, (1.5707963267948966, 0, 0), (0.0, -0.5, 0.0))
        sc.add_model("ceiling", "quad", wall, (-1.5707963267948966, 0, 0), (0.0, 1.5, 0.0))
        sc.add_model("left", "quad", wall, (0, 1.5707963267948966, 0), (-1.0, 0.5, 0.0))
        sc.add_model("right", "quad", wall, (0, -1.5707963267948966, 0), (1.0, 0.5, 0.0))
    else:
        sc.add_preset(args.scene or cfg.preset)
    pk = sc.build_packet()
    cam = iqpt.make_camera(cfg.width, cfg.height)
    variants = {"default": DEFAULT, "none": 0, "-cull": DEFAULT & ~512, "-fastdiv": DEFAULT & ~256,
                "-pair": DEFAULT & ~4, "-sincos": DEFAULT & ~32,
                "-bvh": DEFAULT & ~2048}
    if args.variants:
        # name=optmask (option sets the loaded library builds)
        variants = {}
        for kv in args.variants.split(","):
            name, val = kv.split("=")
            variants[name] = int(val, 0)
    ps = None
    if args.crop:
        x0, x1, y0, ys, nr = (int(v) for v in args.crop.split(","))
        ps = iqpt.pixel_set(cfg.width, cfg.height, x0, x1, y0, ys, nr)
    if args.only:
        opt = variants[args.only] if args.only in variants else int(args.only, 0)
        pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth)
        assert lib.iqpt_debug_set_kernel_options(pt.handle, opt) == 0, lib.iqpt_last_error()
        pt.set_camera(cam)
        pt.upload_packet(pk)
        for _ in range(args.frames):
            pt.render(spp)
        pt.sync()
        ms, n = pt.kernel_time()
        print(json.dumps({"only": args.only, "opt": opt, "frames": n, "avg_ms": ms / max(1, n), "rays": pt.rays()}))
        return
    ctxs = {}
    for name, opt in list(variants.items()):
        pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth)
        st = lib.iqpt_debug_set_kernel_options(pt.handle, opt)
        if st != 0:
            print(f"skip {name}: {lib.iqpt_last_error().decode()}", file=sys.stderr)
            pt.close()
            variants.pop(name)
            continue
        pt.set_camera(cam)
        pt.upload_packet(pk)
        ctxs[name] = pt
    # correctness first: one frame each from fresh states must be bit-identical
    ref = None
    exact = {}
    for name, pt in ctxs.items():
        pt.render(spp)
        lin, bgra = pt.read()
        if ref is None:
            ref = (lin, bgra, pt.rays())
        exact[name] = bool(np.array_equal(lin.view(np.uint32), ref[0].view(np.uint32))
                           and np.array_equal(bgra, ref[1]) and pt.rays() == ref[2])
    times = {n: [] for n in ctxs}
    names = list(ctxs)
    for r in range(args.rounds):
        # alternate the order every round (position effects: clocks, caches)
        for name in (names if r % 2 == 0 else names[::-1]):
            pt = ctxs[name]
            pt.sync()
            pt.kernel_time()
            pt.render(spp)
            ms, n = pt.kernel_time()
            times[name].append(ms)
    res = {}
    base = statistics.median(times[next(iter(ctxs))])
    for name in ctxs:
        med = statistics.median(times[name])
        res[name] = {"median_ms": round(med, 4), "min_ms": round(min(times[name]), 4),
                     "vs_default": round(med / base, 4), "bitexact": exact[name],
                     "times_ms": [round(t, 4) for t in times[name]]}
    # stats variant (counters; slower, diagnostic only)
    stats = None
    pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth)
    stats_opt = args.stats_opt | 128
    if lib.iqpt_debug_set_kernel_options(pt.handle, stats_opt) == 0:
        pt.set_camera(cam)
        pt.upload_packet(pk)
        try:
            pt.render(spp)
        except iqpt.IqptError as e:
            print("stats variant unavailable:", e, file=sys.stderr)
            spp = 0
    timeline = None
    if spp:
        cap = 65536
        wt = (C.c_ulonglong * (3 * cap))()
        nw = C.c_uint32(0)
        lib.iqpt_debug_read_wave_times.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_uint32,
                                                   C.POINTER(C.c_uint32)]
        if lib.iqpt_debug_read_wave_times(pt.handle, wt, cap, C.byref(nw)) == 0 and nw.value:
            raw = np.array(wt[:3 * nw.value], dtype=np.uint64).reshape(-1, 3)
            if args.timeline_npy:
                np.save(args.timeline_npy, raw)
            a = (raw & np.uint64(0xffffffffffff)).astype(np.float64)    # 48-bit times (wave id above)
            a[:, 2] = (raw[:, 2] & np.uint64(0xffffffff)).astype(np.float64)
            t0 = a[:, 0].min()
            start_us, end_us = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0     # 100 MHz ticks
            kern = end_us.max()
            timeline = {"waves": int(nw.value), "kernel_us": round(kern, 1),
                        "start_us_max": round(start_us.max(), 1),
                        "end_us_pct": {str(q): round(float(np.percentile(end_us, q)), 1)
                                       for q in (0, 1, 5, 10, 25, 50, 75, 90, 95, 99, 100)},
                        "mean_lifetime_frac": round(float((end_us - start_us).mean() / kern), 4),
                        "iters_pct": {str(q): int(np.percentile(a[:, 2], q)) for q in (0, 50, 100)}}
        s = (C.c_ulonglong * 24)()
        lib.iqpt_debug_read_stats(pt.handle, s)
        it, ready, active, sc_ex, sc_l, t_ex, t_l, waves = list(s)[:8]
        tri_tests, sph_tests, full_iters = list(s)[8:11]
        refills, refill_lanes = list(s)[12:14]
        tri_rays, tri_nodes, tri_pairs, sph_rays, sph_nodes, sph_tests = list(s)[14:20]
        stats = {"opt": stats_opt, "waves": waves, "iterations": it, "ready_lane_frac": ready / max(1, it * 64),
                 "active_lane_frac": active / max(1, it * 64), "scatter_exec_per_iter": sc_ex / max(1, it),
                 "scatter_lanes_per_exec": sc_l / max(1, sc_ex), "term_exec_per_iter": t_ex / max(1, it),
                 "term_lanes_per_exec": t_l / max(1, t_ex), "rays": pt.rays(),
                 "tri_pair_tests_per_iter": tri_tests / max(1, it), "sph_pair_tests_per_iter": sph_tests / max(1, it),
                 "full_loop_iter_frac": full_iters / max(1, it),
                 "refills_per_iter": refills / max(1, it), "pixels_per_refill": refill_lanes / max(1, refills),
                 "tri_bvh": {"rays": tri_rays, "nodes_per_ray": tri_nodes / max(1, tri_rays),
                             "leaf_pairs_per_ray": tri_pairs / max(1, tri_rays)},
                 "sph_bvh": {"rays": sph_rays, "nodes_per_ray": sph_nodes / max(1, sph_rays),
                             "spheres_per_ray": sph_tests / max(1, sph_rays)}}
    out = {"config": cfg.name, "spp": spp, "rounds": args.rounds, "variants": res, "stats_default": stats,
           "wave_timeline": timeline}
    print(json.dumps(out, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
