#!/usr/bin/env python3
"""Candidate-list sizes of a config's frame (streamed scenes): tiles with per-pixel masks, whether every tile has
them, the longest triangle list (iqpt_debug_pixel_mask_info), and the launch form the default render took.

    list_stats.py [--config c4] [--spp 1]"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "path-tracer-and-rasterizer-engine_amd"))
import iqpt  # noqa: E402
from iqpt import _lib  # noqa: E402
from iqpt.scene import CONFIGS, Scene, make_camera  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--spp", type=int, default=1)
args = ap.parse_args()
cfg = CONFIGS[args.config]
sc = Scene()
sc.add_preset(cfg.preset)
pk = sc.build_packet()
pt = iqpt.PathTracer(cfg.width, cfg.height, max_depth=cfg.max_depth)
pt.set_camera(make_camera(cfg.width, cfg.height))
pt.upload_packet(pk)
pt.render(args.spp)
pt.sync()
lb = _lib.load()
lb.iqpt_debug_pixel_mask_info.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_int), C.POINTER(C.c_uint32)]
n, every, mx = C.c_uint32(0), C.c_int(0), C.c_uint32(0)
_lib.check(lb.iqpt_debug_pixel_mask_info(pt._h, C.byref(n), C.byref(every), C.byref(mx)), "pixel mask info")
lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
o = C.c_int(0)
_lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(o)), "last options")
print(json.dumps({"config": args.config, "masked_tiles": n.value, "every_tile": bool(every.value),
                  "list_max": mx.value, "anyhit_kernel": bool(o.value & (1 << 29)), "options": hex(o.value)}))
pt.close()
