#!/usr/bin/env python3
"""Strong-scaling share emulation on one GPU: rank 0's cyclic row share of the C2 frame
(rows 0, N, 2N, ...) for N = 1, 2, 4, 8, rendered with the plain kernel and with sample-parallel chains
(kOptSplit), 64 spp per launch. Reports the per-launch time (HIP events around the launch sequence),
the projected speed-up over N = 1 and checks that both modes give the same bits.

    python tools/split_share.py [--launches 10] [--ns 1,2,4,8] [--out profiles/...json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "path-tracer-and-rasterizer-engine_amd"))

import numpy as np  # noqa: E402

import iqpt  # noqa: E402
from iqpt import _lib  # noqa: E402
from iqpt import dist as iqdist  # noqa: E402
from iqpt.scene import CONFIGS, Scene, make_camera  # noqa: E402


OPT = 0


def run(n: int, mode: int, launches: int, warm: int, spp: int, knobs=None, chain_waves: int = 0,
        fan: bool = True, spec_run: int = 0, specfan=None) -> dict:
    cfg = CONFIGS["c2"]
    sc = Scene()
    sc.add_preset(cfg.preset)
    pk = sc.build_packet()
    cam = make_camera(cfg.width, cfg.height)
    ps = iqdist.pixel_set_for_rank(cfg.width, cfg.height, 0, n)
    pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth)
    pt.set_split(mode)
    if OPT:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_kernel_options.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_kernel_options(pt._h, OPT), "iqpt_debug_set_kernel_options")
    if knobs:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_split_knobs.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        _lib.check(lb.iqpt_debug_set_split_knobs(pt._h, knobs[0], knobs[1]), "iqpt_debug_set_split_knobs")
    if spec_run:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_spec.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        _lib.check(lb.iqpt_debug_set_spec(pt._h, 0, spec_run), "iqpt_debug_set_spec")   # margin divisor
    if specfan is not None:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_specfan.argtypes = [C.c_void_p, C.c_int, C.c_uint32]
        _lib.check(lb.iqpt_debug_set_specfan(pt._h, specfan[0], specfan[1]), "iqpt_debug_set_specfan")
    if not fan:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_fan.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_fan(pt._h, 0), "iqpt_debug_set_fan")
    if chain_waves:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_chain_waves.argtypes = [C.c_void_p, C.c_uint32]
        _lib.check(lb.iqpt_debug_set_chain_waves(pt._h, chain_waves), "iqpt_debug_set_chain_waves")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    pt.prepare()
    for _ in range(warm):
        pt.render(spp)
    pt.sync()
    pt.kernel_time()
    r0 = pt.rays()
    times = []
    for _ in range(launches):
        pt.render(spp)
        ms, k = pt.kernel_time()
        times.append(ms / max(k, 1))
    rays = pt.rays() - r0
    import ctypes as C
    lb = _lib.load()
    info = (C.c_ulonglong * 8)()
    lb.iqpt_debug_split_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    _lib.check(lb.iqpt_debug_split_info(pt._h, info), "iqpt_debug_split_info")
    info = list(info)
    spec = (C.c_ulonglong * 8)()
    lb.iqpt_debug_spec_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    _lib.check(lb.iqpt_debug_spec_info(pt._h, spec), "iqpt_debug_spec_info")
    spec = list(spec)
    lin, bgra = pt.read()
    st = pt.read_rng()
    pt.close()
    return {"ms": times, "rays": rays, "lin": lin, "bgra": bgra, "rng": st,
            "info": {"split_tiles": info[0], "anchor_tiles": info[1], "leftovers": info[3],
                     "split_pixels": info[6], "mean_window": info[4] / max(info[6], 1),
                     "mean_slots_per_sample": info[5] / 256 / max(info[6], 1), "ran_split": info[7],
                     "sphere_pixels": spec[0], "fan_tiles": spec[1], "spec_runs": spec[4], "spec_window_slots": spec[5],
                     "spec_slots_per_sample": spec[6] / 256 / max(spec[0], 1), "spec_leftovers": spec[7] & 0xffffffff,
                     "spec_fixup_chains": spec[7] >> 32}}


def wave_timeline(n: int, spp: int, warm: int, knobs=None) -> dict:
    """kOptStats build of the split variant (A/B library): per-wave start / end / iterations of one
    launch's round 1 (the first waves recorded after the counters are cleared)."""
    import ctypes as C
    cfg = CONFIGS["c2"]
    sc = Scene()
    sc.add_preset(cfg.preset)
    pk = sc.build_packet()
    cam = make_camera(cfg.width, cfg.height)
    ps = iqdist.pixel_set_for_rank(cfg.width, cfg.height, 0, n)
    lb = _lib.load()
    pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth)
    lb.iqpt_debug_set_kernel_options.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lb.iqpt_debug_set_kernel_options(pt._h, lb.iqpt_debug_default_options() | 128), "set options (stats)")
    pt.set_split(_lib.SPLIT_ON)
    if knobs:
        lb.iqpt_debug_set_split_knobs.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        _lib.check(lb.iqpt_debug_set_split_knobs(pt._h, knobs[0], knobs[1]), "knobs")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    for _ in range(warm):
        pt.render(spp)
    s = (C.c_ulonglong * 24)()
    lb.iqpt_debug_read_stats.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    lb.iqpt_debug_read_stats(pt._h, s)                      # clears
    pt.render(spp)
    cap = 65536
    wt = (C.c_ulonglong * (3 * cap))()
    nw = C.c_uint32(0)
    lb.iqpt_debug_read_wave_times.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_uint32,
                                              C.POINTER(C.c_uint32)]
    _lib.check(lb.iqpt_debug_read_wave_times(pt._h, wt, cap, C.byref(nw)), "wave times")
    raw = np.array(wt[:3 * nw.value], dtype=np.uint64).reshape(-1, 3)
    a = (raw & np.uint64(0xffffffffffff)).astype(np.float64)     # 48-bit times (wave id above)
    a[:, 2] = (raw[:, 2] & np.uint64(0xffffffff)).astype(np.float64)
    spec = (raw[:, 2] >> np.uint64(32)).astype(np.float64)
    pt.close()
    half = a.shape[0] // 2                                  # round 1, then round 2 (same grid)
    out = {}
    for name, b, sl in (("round1", a[:half], spec[:half]), ("round2", a[half:], spec[half:])):
        if not len(b):
            continue
        t0 = b[:, 0].min()
        st, en = (b[:, 0] - t0) / 100.0, (b[:, 1] - t0) / 100.0
        it = b[:, 2]
        out[name] = {"waves": int(len(b)), "kernel_us": round(float(en.max()), 1),
                     "end_us_pct": {str(q): round(float(np.percentile(en, q)), 1) for q in (0, 10, 50, 90, 99, 100)},
                     "iters_pct": {str(q): int(np.percentile(it, q)) for q in (0, 10, 50, 90, 99, 100)},
                     "us_per_iter_pct": {str(q): round(float(np.percentile((en - st) / np.maximum(it, 1), q)), 2)
                                         for q in (0, 50, 100)},
                     "slowest": [[round(float(en[i]), 1), int(it[i]), int(sl[i])] for i in np.argsort(-en)[:12]],
                     "spec_waves": int((sl > 0).sum()),
                     "end_us_pct_spec": {str(q): round(float(np.percentile(en[sl > 0], q)), 1)
                                         for q in (0, 50, 100)} if (sl > 0).any() else None,
                     "end_us_pct_anchor_only": {str(q): round(float(np.percentile(en[sl == 0], q)), 1)
                                                for q in (0, 50, 100)} if (sl == 0).any() else None}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--out", default="")
    ap.add_argument("--modes", default="plain,split", help="plain, split, chain (IQPT_SPLIT_CHAIN, anchored tiles in "
                    "the fan kernel), chainplain (the same, anchored tiles in the plain kernel), fan (IQPT_SPLIT_FAN)")
    ap.add_argument("--chain-waves", default="", help="extra chain rows at these chain-kernel waves per CU")
    ap.add_argument("--spec-runs", default="", help="extra spec rows at these window margin divisors")
    ap.add_argument("--specfan", default="", help="extra spec rows mode:lead[,...] (iqpt_debug_set_specfan: 0 two "
                    "streams, 1 one stream, 2 one grid; lead 'all' or a block count)")
    ap.add_argument("--knobs", default="", help="split knob sets heavy_rho:refill_min[,...] (extra split rows)")
    ap.add_argument("--stats", action="store_true", help="wave timelines of the split variant (instrumented library)")
    ap.add_argument("--opt", type=lambda v: int(v, 0), default=0, help="kernel option set (instrumented library; 0 = production)")
    ap.add_argument("--lib", default="", help="load this prebuilt library (compile-time knob A/B)")
    args = ap.parse_args()
    if args.lib:
        _lib.LIB_PATH = Path(args.lib)
    out = {"config": "c2 rank-0 row share, 64 spp per launch", "launches": args.launches, "rows": []}
    if args.opt:
        global OPT
        from iqpt import _build
        _lib.LIB_PATH = _build.build_lib(stats=True)
        OPT = args.opt
    if args.stats:
        from iqpt import _build
        _lib.LIB_PATH = _build.build_lib(stats=True)
        for n in [int(x) for x in args.ns.split(",")]:
            tl = wave_timeline(n, args.spp, args.warm)
            print(json.dumps({"n": n, "timeline": tl}), flush=True)
            out["rows"].append({"n": n, "timeline": tl})
        if args.out:
            Path(args.out).write_text(json.dumps(out, indent=1) + "\n")
        return
    base = None
    for n in [int(x) for x in args.ns.split(",")]:
        row = {"n": n}
        res = {}
        modes = [m for m in (("plain", _lib.SPLIT_OFF, 0), ("split", _lib.SPLIT_ON, 0),
                             ("chain", _lib.SPLIT_CHAIN, 0), ("chainplain", _lib.SPLIT_CHAIN, 0),
                             ("fan", _lib.SPLIT_FAN, 0), ("splitplain", _lib.SPLIT_ON, 0),
                             ("spec", _lib.SPLIT_SPEC, 0))
                 if m[0] in args.modes.split(",")]
        # "16" = 16 chain-kernel waves per CU; "16a" = the same with every tile in the split set (all chains);
        # "16l4" = 4 lanes per pixel
        def cw(w):
            v = w.rstrip("a")
            return int(v.split("l")[0]) | ((int(v.split("l")[1]) << 8) if "l" in v else 0)
        modes += [(f"chain_w{w}", _lib.SPLIT_CHAIN, cw(w)) for w in args.chain_waves.split(",") if w]
        modes += [(f"spec_r{r}", _lib.SPLIT_SPEC, int(r)) for r in args.spec_runs.split(",") if r]
        sfs = {}
        for v in args.specfan.split(","):
            if v:
                m, _, ld = v.partition(":")
                sfs[f"spec_sf{m}_{ld or 'all'}"] = (int(m), 0xffffffff if ld in ("", "all") else int(ld))
                modes.append((f"spec_sf{m}_{ld or 'all'}", _lib.SPLIT_SPEC, 0))
        for name, mode, cw in modes:
            kn = (0, 16 | (1 << 16)) if name.endswith("a") else None
            r = run(n, mode, args.launches, args.warm, args.spp, knobs=kn, chain_waves=0 if name.startswith("spec") else cw,
                    fan=name not in ("chainplain", "splitplain"), spec_run=cw if name.startswith("spec_r") else 0,
                    specfan=sfs.get(name))
            res[name] = r
            row[name + "_ms_median"] = float(np.median(r["ms"]))
            row[name + "_ms_min"] = float(np.min(r["ms"]))
            row[name + "_mrays_per_s"] = r["rays"] / (sum(r["ms"]) * 1e-3) / 1e6
            if name == "split":
                row["split_info"] = r["info"]
            if name.startswith(("chain", "spec")):
                row[name + "_sphere_pixels"] = r["info"]["sphere_pixels"]
            if name.startswith("spec"):
                row[name + "_runs"] = r["info"]["spec_runs"]
                row[name + "_window_slots"] = r["info"]["spec_window_slots"]
                row[name + "_leftovers"] = r["info"]["spec_leftovers"]
                row[name + "_slots_per_sample"] = round(r["info"]["spec_slots_per_sample"], 3)
            if name.startswith(("chain", "fan", "split", "spec")):
                row[name + "_ran"] = {0: "plain", 1: "split", 2: "chain", 3: "fan", 4: "chain+fan", 5: "split+fan", 6: "spec"}.get(
                    int(r["info"]["ran_split"]), "?")
            if name != "plain" and "plain" in res:
                a = res["plain"]
                row[name + "_identical"] = bool(
                    np.array_equal(a["lin"].view(np.uint32), r["lin"].view(np.uint32)) and
                    np.array_equal(a["bgra"], r["bgra"]) and np.array_equal(a["rng"], r["rng"]) and
                    a["rays"] == r["rays"])
        for kn in [k for k in args.knobs.split(",") if k]:
            rl, rm = (int(x) for x in kn.split(":"))
            r = run(n, _lib.SPLIT_ON, args.launches, args.warm, args.spp, (rl, rm))
            row[f"split_h{rl}_m{rm}_ms_median"] = float(np.median(r["ms"]))
            row[f"split_h{rl}_m{rm}_ran"] = int(r["info"]["ran_split"])
            if "plain" in res:
                a = res["plain"]
                row[f"split_h{rl}_m{rm}_identical"] = bool(
                    np.array_equal(a["lin"].view(np.uint32), r["lin"].view(np.uint32)) and
                    np.array_equal(a["rng"], r["rng"]) and a["rays"] == r["rays"])
        if "plain" in res and "split" in res:
            a, b = res["plain"], res["split"]
            row["identical"] = bool(np.array_equal(a["lin"].view(np.uint32), b["lin"].view(np.uint32)) and
                                    np.array_equal(a["bgra"], b["bgra"]) and np.array_equal(a["rng"], b["rng"]) and
                                    a["rays"] == b["rays"])
        best = min(row[k + "_ms_median"] for k in res)
        if n == 1:
            base = best
        if base:
            row["speedup_vs_n1_best"] = base / best
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
