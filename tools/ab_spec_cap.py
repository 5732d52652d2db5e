#!/usr/bin/env python3
"""A/B of the spec plan's lane cap (iqpt_debug_set_spec_cap): rank 0's row share of C2
at N = 8 / 4 / 2, pipelined 64-spp launches as bench.py runs them (no join between launches), wall time
and kernel span per launch for each cap, rounds interleaved; every cap's frame, RNG states and ray count
must equal the default cap's (a plan only orders work).

    python tools/ab_spec_cap.py [--ns 8,4,2] [--caps 0.97,0.75,1.5] [--launches 20] [--rounds 2] [--out f.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "path-tracer-and-rasterizer-engine_amd"))

import numpy as np  # noqa: E402

import iqpt  # noqa: E402
from iqpt import _lib  # noqa: E402
from iqpt import dist as iqdist  # noqa: E402
from iqpt.scene import CONFIGS, Scene, make_camera  # noqa: E402


def run(n: int, cap: float, launches: int, warm: int) -> dict:
    cfg = CONFIGS["c2"]
    sc = Scene()
    sc.add_preset(cfg.preset)
    pk = sc.build_packet()
    ps = iqdist.pixel_set_for_rank(cfg.width, cfg.height, 0, n)
    pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth)
    lb = _lib.load()
    lb.iqpt_debug_set_spec_cap.argtypes = [C.c_void_p, C.c_double]
    _lib.check(lb.iqpt_debug_set_spec_cap(pt._h, cap), "iqpt_debug_set_spec_cap")
    pt.set_camera(make_camera(cfg.width, cfg.height))
    pt.upload_packet(pk)
    pt.prepare()
    for _ in range(warm):
        pt.render(cfg.spp)
    pt.sync()
    pt.kernel_time()
    r0 = pt.rays()
    t0 = time.perf_counter()
    for _ in range(launches):
        pt.render(cfg.spp)
    pt.sync()
    wall = (time.perf_counter() - t0) * 1e3 / launches
    pt.kernel_time()
    span = pt.kernel_span() / launches
    mode = pt.launch_mode()
    rays = pt.rays() - r0
    lin, bgra = pt.read()
    st = pt.read_rng()
    pt.close()
    return {"wall_ms": wall, "span_ms": span, "mode": mode, "rays": rays, "lin": lin, "bgra": bgra, "rng": st}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="8,4,2")
    ap.add_argument("--caps", default="0.97,0.75,1.5")
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--warm", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    caps = [float(x) for x in args.caps.split(",")]
    out = {"what": "spec plan lane cap A/B, rank 0's C2 row share, pipelined 64-spp launches", "rows": []}
    for n in [int(x) for x in args.ns.split(",")]:
        row = {"n": n}
        ref = None
        for r in range(args.rounds):
            for cap in caps:
                res = run(n, cap, args.launches, args.warm)
                if ref is None:
                    ref = res
                same = bool(np.array_equal(ref["lin"].view(np.uint32), res["lin"].view(np.uint32)) and
                            np.array_equal(ref["bgra"], res["bgra"]) and np.array_equal(ref["rng"], res["rng"]) and
                            ref["rays"] == res["rays"])
                k = f"cap{cap}"
                row.setdefault(k + "_wall_ms", []).append(round(res["wall_ms"], 4))
                row.setdefault(k + "_span_ms", []).append(round(res["span_ms"], 4))
                row[k + "_identical"] = row.get(k + "_identical", True) and same
                row[k + "_mode"] = res["mode"]
        print(json.dumps(row), flush=True)
        out["rows"].append(row)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
