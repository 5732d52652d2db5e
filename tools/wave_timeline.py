#!/usr/bin/env python3
"""Per-wave timeline of the plain kernel on the C2 frame: the kOptStats build of the production
option set (one ray or two rays per lane, kOptPipe), every wave's start / end (s_memrealtime, 100 MHz) and loop
iterations, and the launch's counters: iterations, active lanes per iteration (exec population), iterations that
ran an Oren-Nayar scatter or a path end, iterations forced onto every pair by a secondary ray.

    wave_timeline.py [--two-ray 1] [--overlap 1] [--crop x0,x1,y0,rows] [--out f.json]

Waves are sorted by iteration count; the longest ones are the sphere tiles' chains that set the launch. With
--overlap 1 two launches run at once (the production form); the timeline is the last launch's."""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "path-tracer-and-rasterizer-engine_amd"))
import iqpt  # noqa: E402
from iqpt import _build, _lib  # noqa: E402
from iqpt.scene import CONFIGS, Scene, make_camera  # noqa: E402

K_STATS, K_PIPE, K_OVERLAP, K_CAMAXIS, K_PRIO = 1 << 7, 1 << 21, 1 << 19, 1 << 14, 1 << 17

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--spp", type=int, default=0, help="samples per launch (default: the config's)")
ap.add_argument("--two-ray", type=int, default=1)
ap.add_argument("--overlap", type=int, default=1)
ap.add_argument("--crop", default="", help="x0,x1,y0,rows: a pixel set instead of the full frame")
ap.add_argument("--warm", type=int, default=3)
ap.add_argument("--out", default="")
args = ap.parse_args()

_lib.LIB_PATH = _build.build_lib(stats=True)
lb = _lib.load()
lb.iqpt_debug_set_kernel_options.argtypes = [C.c_void_p, C.c_int]
lb.iqpt_debug_default_options.restype = C.c_int
lb.iqpt_debug_read_stats.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
lb.iqpt_debug_read_wave_times.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_uint32, C.POINTER(C.c_uint32)]
cfg = CONFIGS[args.config]
spp = args.spp or cfg.spp
sc = Scene()
sc.add_preset(cfg.preset)
pk = sc.build_packet()
cam = make_camera(cfg.width, cfg.height)
ps = None
if args.crop:
    x0, x1, y0, rows = (int(v) for v in args.crop.split(","))
    ps = iqpt.pixel_set(cfg.width, cfg.height, x0, x1, y0, 1, rows)
pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth)
pt.set_split(_lib.SPLIT_OFF)
pt.set_overlap(_lib.OVERLAP_AUTO if args.overlap else _lib.OVERLAP_OFF)
pt.set_camera(cam)
pt.upload_packet(pk)
if args.config == "c2":
    opt = lb.iqpt_debug_default_options() | K_PRIO | K_STATS | (K_PIPE if args.two_ray else 0)
    if args.overlap:
        opt |= K_OVERLAP | K_CAMAXIS        # the production overlapped form (its stats variants are built)
else:
    # other configs: the production launch's own option set (its first launches tune the camera-ray path), + stats
    lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    for _ in range(6):
        pt.render(spp)
    o = C.c_int(0)
    _lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(o)), "last options")
    opt = (o.value & ~((1 << 30) | (1 << 29))) | K_STATS
_lib.check(lb.iqpt_debug_set_kernel_options(pt._h, opt), "kernel options")
for _ in range(args.warm):
    pt.render(spp)
pt.sync()
s = (C.c_ulonglong * 24)()
lb.iqpt_debug_read_stats(pt._h, s)                  # clears the counters and the wave slots
pt.render(spp)
pt.sync()
cap = 1 << 16
wt = (C.c_ulonglong * (3 * cap))()
nw = C.c_uint32(0)
_lib.check(lb.iqpt_debug_read_wave_times(pt._h, wt, cap, C.byref(nw)), "wave times")
ph = (C.c_ulonglong * (4 * cap))()
lb.iqpt_debug_read_wave_phases.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_uint32]
_lib.check(lb.iqpt_debug_read_wave_phases(pt._h, ph, cap), "wave phases")
phases = np.array(ph[:4 * nw.value], dtype=np.float64).reshape(-1, 4)
lb.iqpt_debug_read_stats(pt._h, s)
v = [int(x) for x in s]
t, k = pt.kernel_time()
a = np.array(wt[:3 * nw.value], dtype=np.uint64).reshape(-1, 3)
start = (a[:, 0] & np.uint64(0xffffffffffff)).astype(np.float64)
end = a[:, 1].astype(np.float64)
iters = (a[:, 2] & np.uint64(0xffffffff)).astype(np.int64)
busy = iters > 0
t0 = start[busy].min()
dur = (end - start) / 100.0                          # us
us_iter = dur[busy] / iters[busy]


def pct(x):
    return {str(q): round(float(np.percentile(x, q)), 2) for q in (0, 10, 50, 90, 99, 100)}


order = np.argsort(-iters)
top = order[:max(1, int(0.05 * busy.sum()))]           # the longest 5 % of the waves: the chains that set the launch
res = {"config": args.config, "spp": spp, "two_ray": args.two_ray, "overlap": args.overlap, "crop": args.crop or None, "options": hex(opt),
       "kernel_ms": round(t / max(k, 1), 4), "waves": int(busy.sum()),
       "launch_iterations": v[0], "active_lanes_per_iteration": round(v[1] / max(v[0], 1), 2),
       "exec_population": round(v[1] / max(v[0], 1) / 64.0, 3),
       "scatter_iteration_frac": round(v[3] / max(v[0], 1), 3), "scatter_lanes_per_scatter_iteration": round(v[4] / max(v[3], 1), 2),
       "end_iteration_frac": round(v[5] / max(v[0], 1), 3), "end_lanes_per_end_iteration": round(v[6] / max(v[5], 1), 2),
       "full_loop_iteration_frac": round(v[10] / max(v[0], 1), 3),
       "iters_per_wave": pct(iters[busy]), "wave_us": pct(dur[busy]), "us_per_iter": pct(us_iter),
       "end_us": pct((end[busy] - t0) / 100.0),
       "longest_5pct": {"waves": int(len(top)), "iters": pct(iters[top]), "us_per_iter": pct(dur[top] / np.maximum(iters[top], 1)),
                        "start_us": pct((start[top] - t0) / 100.0), "end_us": pct((end[top] - t0) / 100.0),
                        # shader-clock cycles per loop iteration in the closest hits, the shading, the next rays (two-ray
                        # kernel; the one-ray kernel's path end is in its shading) and the rest of the loop
                        "cycles_per_iter": {nm: pct(phases[top, i] / np.maximum(iters[top], 1))
                                            for i, nm in enumerate(("closest_hits", "shading", "next_rays", "rest"))}}}
print(json.dumps(res), flush=True)
if args.out:
    Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
pt.close()
