#!/usr/bin/env python3
"""Does overlapping consecutive launches hide the launch tail? Two independent contexts (two HIP streams)
render the same pixel set alternately without host synchronisation, against one context rendering the
same number of launches back to back. Wall time per launch; no correctness claim (independent frames).

    overlap_probe.py [--config c2] [--share N] [--mode plain|spec|auto] [--out f.json]

--share N: rank 0's rows of an N-way C3 split (one GPU's share); the ratio then says how much of a
share launch is tail (latency) rather than throughput."""
import argparse
import json
import sys
import time
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
ap.add_argument("--mode", default="plain", choices=["plain", "spec", "auto"])
ap.add_argument("--launches", type=int, default=20)
ap.add_argument("--out", default="")
args = ap.parse_args()
mode = {"plain": _lib.SPLIT_OFF, "spec": _lib.SPLIT_SPEC, "auto": _lib.SPLIT_AUTO}[args.mode]

cfg = CONFIGS[args.config]
n = args.launches
sc = Scene()
sc.add_preset(cfg.preset)
pk = sc.build_packet()
cam = make_camera(cfg.width, cfg.height)
ps = iqdist.pixel_set_for_rank(cfg.width, cfg.height, 0, args.share)
pts = []
for k in range(2):
    pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth, seed=1984 + k)
    pt.set_split(mode)
    pt.set_overlap(_lib.OVERLAP_OFF)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    for _ in range(3):
        pt.render(cfg.spp)
    pt.sync()
    pts.append(pt)
out = {"config": cfg.name, "share": args.share, "mode": args.mode, "launch_mode": pts[0].launch_mode()}
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
    print(json.dumps({"share": args.share, "mode": args.mode, **out[f"round{rnd}"]}), flush=True)
if args.out:
    Path(args.out).write_text(json.dumps(out, indent=1))
