#!/usr/bin/env python3
"""Map of the certain tiles (kparams::certain, iq_interval.h tri_certain) of a config's frame: per 8x8 tile
'#' every pixel certain, '+' at least half, '-' some, '.' none. Prints the counts
and a character map, and writes them to --out.

    certain_map.py [--config c2] [--share 1] [--out f.json]"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "path-tracer-and-rasterizer-engine_amd"))
import iqpt  # noqa: E402
from iqpt import _lib  # noqa: E402
from iqpt import dist as iqdist  # noqa: E402
from iqpt.scene import CONFIGS, Scene, make_camera  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--share", type=int, default=1)
ap.add_argument("--out", default="")
args = ap.parse_args()
cfg = CONFIGS[args.config]
sc = Scene()
sc.add_preset(cfg.preset)
pk = sc.build_packet()
ps = iqdist.pixel_set_for_rank(cfg.width, cfg.height, 0, args.share)
pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth)
pt.set_camera(make_camera(cfg.width, cfg.height))
pt.upload_packet(pk)
pt.prepare()
lb = _lib.load()
lb.iqpt_debug_certain_tiles.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint32]
n, nt, ntx = C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
_lib.check(lb.iqpt_debug_certain_tiles(pt._h, C.byref(n), C.byref(nt), C.byref(ntx), None, 0), "certain")
flags = (C.c_uint32 * (2 * nt.value))()
_lib.check(lb.iqpt_debug_certain_tiles(pt._h, C.byref(n), C.byref(nt), C.byref(ntx), flags, nt.value), "certain")
info = (C.c_ulonglong * 8)()
lb.iqpt_debug_split_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
res = {"config": cfg.name, "share": args.share, "tiles": nt.value, "certain_pixels": n.value,
       "pixels": ps.nrows * (ps.x1 - ps.x0), "tiles_x": ntx.value}
rows = []
w = ntx.value
full = 0


def cnt(t):
    return bin(flags[2 * t]).count("1") + bin(flags[2 * t + 1]).count("1")


for r in range(nt.value // w):
    line = ""
    for x in range(w):
        k = cnt(r * w + x)
        full += k == 64
        line += "#" if k == 64 else ("+" if k >= 32 else ("-" if k > 0 else "."))
    rows.append(line)
res["full_tiles"] = full
res["map"] = rows
print(json.dumps({k: v for k, v in res.items() if k != "map"}))
for line in rows[:: max(1, len(rows) // 40)]:
    print(line[:: max(1, w // 120)])
if args.out:
    Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
