#!/usr/bin/env python3
"""Does overlapping consecutive C2 launches hide the launch tail? Two independent contexts (two HIP streams)
render full C2 frames alternately without host synchronisation, against one context rendering the same
number of launches back to back. Wall time per launch; no correctness claim (independent frames)."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "path-tracer-and-rasterizer-engine_amd"))
import iqpt  # noqa: E402
from iqpt import _lib  # noqa: E402
from iqpt.scene import CONFIGS, Scene, make_camera  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
n = 20
sc = Scene()
sc.add_preset(cfg.preset)
pk = sc.build_packet()
cam = make_camera(cfg.width, cfg.height)
pts = []
for k in range(2):
    pt = iqpt.PathTracer(cfg.width, cfg.height, max_depth=cfg.max_depth, seed=1984 + k)
    pt.set_split(_lib.SPLIT_OFF)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    for _ in range(3):
        pt.render(cfg.spp)
    pt.sync()
    pts.append(pt)
out = {}
for rnd in range(3):
    t0 = time.perf_counter()
    for _ in range(n):
        pts[0].render(cfg.spp)
    pts[0].sync()
    seq = (time.perf_counter() - t0) / n * 1e3
    t0 = time.perf_counter()
    for _ in range(n // 2):
        pts[0].render(cfg.spp)
        pts[1].render(cfg.spp)
    pts[0].sync()
    pts[1].sync()
    ovl = (time.perf_counter() - t0) / n * 1e3
    out[f"round{rnd}"] = {"sequential_ms_per_launch": round(seq, 4), "two_streams_ms_per_launch": round(ovl, 4),
                          "ratio": round(ovl / seq, 4)}
    print(json.dumps(out[f"round{rnd}"]), flush=True)
if len(sys.argv) > 2:
    Path(sys.argv[2]).write_text(json.dumps(out, indent=1))
