#!/usr/bin/env python3
"""Per-block timeline of iqpt_spec_kernel on rank 0's row share of C2: for every spec
block the s_memrealtime stamps (100 MHz) at its start, after round 0's slot pass, after round 0's walk (with a
parity pixel's fix-up pass and second walk) and at its end (iqpt_debug_spec_timeline). Prints percentiles of the block start, the phases and the end, and
the blocks that needed more than one round.

    spec_timeline.py [--share 8] [--specfan 1] [--plan 1] [--parity R] [--out f.json]

--specfan: 1 = the spec kernel alone on the stream (the fan kernel after it), 0 = beside the fan kernel
on a second stream. (Round 6 archived queue mode and the plan-cap / priority / parity-bound knobs.)"""
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
ap.add_argument("--share", type=int, default=8)
ap.add_argument("--specfan", type=int, default=1)
ap.add_argument("--warm", type=int, default=3)
ap.add_argument("--plan", type=int, default=1, help="iqpt_debug_spec_plan mode (0 none, 1 asynchronous)")
ap.add_argument("--parity", type=float, default=None, help="iqpt_debug_set_spec_parity in slots per sample (0: off)")
ap.add_argument("--two-ray", type=int, default=None, help="iqpt_debug_set_two_ray (kOptPipe: 1 on, 0 off)")
ap.add_argument("--out", default="")
args = ap.parse_args()

cfg = CONFIGS["c2"]
sc = Scene()
sc.add_preset(cfg.preset)
pk = sc.build_packet()
cam = make_camera(cfg.width, cfg.height)
ps = iqdist.pixel_set_for_rank(cfg.width, cfg.height, 0, args.share)
pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, max_depth=cfg.max_depth)
pt.set_split(_lib.SPLIT_SPEC)
lb = _lib.load()
lb.iqpt_debug_set_specfan.argtypes = [C.c_void_p, C.c_int, C.c_uint32]
_lib.check(lb.iqpt_debug_set_specfan(pt._h, args.specfan, 0xffffffff), "iqpt_debug_set_specfan")
lb.iqpt_debug_spec_plan.argtypes = [C.c_void_p, C.c_int]
_lib.check(lb.iqpt_debug_spec_plan(pt._h, args.plan), "iqpt_debug_spec_plan")
if args.parity is not None:
    lb.iqpt_debug_set_spec_parity.argtypes = [C.c_void_p, C.c_uint32]
    _lib.check(lb.iqpt_debug_set_spec_parity(pt._h, int(round(args.parity * 256))), "iqpt_debug_set_spec_parity")
if args.two_ray is not None:
    lb.iqpt_debug_set_two_ray.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lb.iqpt_debug_set_two_ray(pt._h, args.two_ray), "iqpt_debug_set_two_ray")
pt.set_camera(cam)
pt.upload_packet(pk)
for _ in range(args.warm):
    pt.render(cfg.spp)
pt.sync()
lb.iqpt_debug_spec_timeline.argtypes = [C.c_void_p, C.c_int]
_lib.check(lb.iqpt_debug_spec_timeline(pt._h, 1), "iqpt_debug_spec_timeline")
info = (C.c_ulonglong * 8)()
lb.iqpt_debug_spec_info.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
_lib.check(lb.iqpt_debug_spec_info(pt._h, info), "iqpt_debug_spec_info")      # clears the statistics
pt.render(cfg.spp)
pt.sync()
_lib.check(lb.iqpt_debug_spec_info(pt._h, info), "iqpt_debug_spec_info")
spec_stats = {"sphere_pixels": int(info[0]), "windows_sum": int(info[5]), "past_window_chains": int(info[7] & 0xffffffff),
              "fixup_chains": int(info[7] >> 32)}
cap = 1 << 16
buf = (C.c_ulonglong * (8 * cap))()
n = C.c_uint32(0)
lb.iqpt_debug_read_spec_timeline.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_uint32, C.POINTER(C.c_uint32)]
_lib.check(lb.iqpt_debug_read_spec_timeline(pt._h, buf, cap, C.byref(n)), "iqpt_debug_read_spec_timeline")
raw8 = np.array(buf[:8 * n.value], dtype=np.uint64).reshape(-1, 8)


def pct(a):
    return {str(q): round(float(np.percentile(a, q)), 1) for q in (0, 10, 50, 90, 99, 100)}


raw = raw8[:, :3]
# per wave (round 5: the waves of a block run their rounds on their own): end | slot-loop iterations << 48
wave_iters = (raw8[:, 4:] >> np.uint64(48)).astype(np.int64)
wave_end = (raw8[:, 4:] & np.uint64(0xffffffffffff)).astype(np.float64)
rounds = (raw8[:, 3] >> np.uint64(48)).astype(np.int64)
iters = wave_iters.max(axis=1)                            # the block's slowest wave's slot-loop iterations
t = (raw & np.uint64(0xffffffffffff)).astype(np.float64)
t0 = t[:, 0].min()
us = (t - t0) / 100.0                     # 100 MHz ticks -> us
wave_us = (wave_end - t0) / 100.0
# wave 0's start, its round-0 slot pass end and round-0 end; the block's end (its latest wave)
start, slots_end, walk_end, end = us[:, 0], us[:, 1], us[:, 2], wave_us.max(axis=1)


res = {"share": args.share, "two_ray": args.two_ray, "specfan": args.specfan, "plan": args.plan, "parity": args.parity,
       "blocks": int(n.value), "spec_stats": spec_stats,
       "kernel_us": round(float(end.max()), 1),
       "start_us": pct(start), "slots_us": pct(slots_end - start), "walk_us": pct(walk_end - slots_end),
       "later_rounds_us": pct(end - walk_end), "end_us": pct(end),
       "iters_max_wave": pct(iters), "iters_spread_in_block": pct(wave_iters.max(axis=1) - wave_iters.min(axis=1)),
       "wave_end_us": pct(wave_us.reshape(-1)), "wave_end_spread_in_block_us": pct(wave_us.max(axis=1) - wave_us.min(axis=1)),
       "rounds_hist": {str(int(k)): int(v) for k, v in zip(*np.unique(rounds, return_counts=True))},
       "slowest": [[int(i), round(float(start[i]), 1), round(float(slots_end[i] - start[i]), 1),
                    round(float(walk_end[i] - slots_end[i]), 1), round(float(end[i] - walk_end[i]), 1),
                    int(rounds[i])] for i in np.argsort(-end)[:16]]}
# the plan behind the blocks and the history: per block its lanes per pixel, pixels, and its pixels' largest
# work estimate (window x slots per sample) and window, to fit the slot phase against
nb = C.c_uint32(0)
npx = C.c_uint32(0)
order = (C.c_uint32 * cap)()
blk = (C.c_uint32 * (2 * cap))()
rho = (C.c_uint32 * cap)()
lb.iqpt_debug_read_spec_plan.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                         C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
_lib.check(lb.iqpt_debug_read_spec_plan(pt._h, order, blk, rho, cap, C.byref(npx), C.byref(nb)), "iqpt_debug_read_spec_plan")
if npx.value and nb.value == n.value:
    spp, mcap = cfg.spp, (3 * cfg.spp + 15) & ~15
    rho_a = np.array(rho[:npx.value], dtype=np.float64)
    r = np.where(rho_a > 0, rho_a, 576.0)
    m = r * spp / 256.0
    m = np.minimum(mcap, np.maximum(spp, m + np.maximum(4, (m - spp) / 16) + 4))   # spec_window (margin 1/16)
    w = m * np.maximum(r, 256.0) / 256.0
    rows = []
    for b in range(nb.value):
        first, word = blk[2 * b], blk[2 * b + 1]
        cnt, lanes = word & 0xff, word >> 8                  # count | lanes per pixel << 8
        qs = [order[first + i] for i in range(cnt)]
        rows.append([lanes, cnt, float(w[qs].max()), float(m[qs].max()), float(slots_end[b] - start[b]), float(iters[b])])
    a = np.array(rows)
    res["per_block"] = {"lanes_hist": {str(int(k)): int(v) for k, v in zip(*np.unique(a[:, 0], return_counts=True))}}
    # every block: lanes, pixels, max work, max window, slot pass (us), walk + fix-up (us), end (us), rounds, the
    # slowest wave's iterations, its waves' ends (us): for offline analysis of what sets the kernel's tail
    res["blocks"] = [[int(a[b, 0]), int(a[b, 1]), round(float(a[b, 2]), 1), round(float(a[b, 3]), 1),
                      round(float(slots_end[b] - start[b]), 1), round(float(walk_end[b] - slots_end[b]), 1),
                      round(float(end[b]), 1), int(rounds[b]), int(iters[b]),
                      [round(float(x), 1) for x in wave_us[b]], [int(x) for x in wave_iters[b]]]
                     for b in range(nb.value)]
    # slot phase ~ alpha * max w / lanes + beta * max window + gamma (least squares)
    X = np.stack([a[:, 2] / a[:, 0], a[:, 3], np.ones(len(a))], axis=1)
    coef, *_ = np.linalg.lstsq(X, a[:, 4], rcond=None)
    pred = X @ coef
    res["per_block"]["fit_us"] = {"per_work_per_lane": float(coef[0]), "per_window_slot": float(coef[1]),
                                  "const": float(coef[2]),
                                  "r2": float(1 - ((a[:, 4] - pred) ** 2).sum() / ((a[:, 4] - a[:, 4].mean()) ** 2).sum())}
    for L in (8, 16, 32, 64):
        sel = a[:, 0] == L
        if sel.any():
            res["per_block"][f"lanes{L}"] = {"blocks": int(sel.sum()), "slots_us": pct(a[sel, 4]), "iters_max_wave": pct(a[sel, 5]),
                                             "us_per_iter": pct(a[sel, 4] / np.maximum(a[sel, 5], 1)),
                                             "w_per_lane": pct(a[sel, 2] / L), "window": pct(a[sel, 3])}
print(json.dumps(res), flush=True)
if args.out:
    Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
