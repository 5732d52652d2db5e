#!/usr/bin/env python3
"""Distribution of the sphere pixels' chain lengths (slots per sample of their last chain, the spec kernel's
history) on rank 0's share of C2 (the spread of chain lengths the spec plan works from).

    spec_rho_hist.py [--share 1]"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "path-tracer-and-rasterizer-engine_amd"))
import iqpt  # noqa: E402
from iqpt import _lib  # noqa: E402
from iqpt import dist as iqdist  # noqa: E402
from iqpt.scene import CONFIGS, Scene, make_camera  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--share", type=int, default=1)
args = ap.parse_args()
cfg = CONFIGS["c2"]
sc = Scene()
sc.add_preset(cfg.preset)
pk = sc.build_packet()
ps = iqdist.pixel_set_for_rank(cfg.width, cfg.height, 0, args.share)
pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth)
pt.set_split(_lib.SPLIT_SPEC)
lb = _lib.load()
lb.iqpt_debug_spec_plan.argtypes = [C.c_void_p, C.c_int]
_lib.check(lb.iqpt_debug_spec_plan(pt.handle, 2), "iqpt_debug_spec_plan")     # a plan before every launch
pt.set_camera(make_camera(cfg.width, cfg.height))
pt.upload_packet(pk)
for _ in range(3):
    pt.render(cfg.spp)
pt.sync()
cap = 1 << 22
order = (C.c_uint32 * cap)()
blocks = (C.c_uint32 * (2 * cap))()
rho = (C.c_uint32 * cap)()
n, nb = C.c_uint32(0), C.c_uint32(0)
lb.iqpt_debug_read_spec_plan.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
_lib.check(lb.iqpt_debug_read_spec_plan(pt.handle, order, blocks, rho, cap, C.byref(n), C.byref(nb)),
           "iqpt_debug_read_spec_plan")
r = np.frombuffer(rho, dtype=np.uint32, count=n.value).astype(np.float64) / 256.0
out = {"share": args.share, "sphere_pixels": int(n.value), "owned_pixels": int(pt.npix),
       "slots_per_sample_pct": {str(q): round(float(np.percentile(r, q)), 3) for q in (0, 10, 25, 50, 75, 90, 95, 99, 100)},
       "frac_at_or_above": {str(t): round(float(np.mean(r >= t)), 4) for t in (1.25, 1.5, 1.75, 2.0, 2.25, 2.5, 2.75, 3.0)}}
print(json.dumps(out))
