#!/usr/bin/env python3
"""Instruction mix and wave-time breakdown of the render kernel from rocprofv3 PMC passes.

Pass A: SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32
Pass B: SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
(each in its own run with --kernel-trace only). SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count
quad-cycles; WAIT_ANY (parked on s_waitcnt / barrier) + WAIT_INST_ANY (ready, not issued) +
ACTIVE_INST_ANY ~= WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots). GRBM_GUI_ACTIVE is summed
over the 8 XCDs: kernel cycles = GRBM_GUI_ACTIVE / 8. valu_busy_frac = the SIMDs' VALU issue cycles over the
kernel's cycles (1024 SIMDs): a wave64 VALU instruction holds a SIMD-32 for 2 cycles, a transcendental one for 4
(MI355X_MICROARCH.md, constants table), so this cannot exceed 1. valu_active_per_simd is the older measure,
SQ_ACTIVE_INST_VALU summed over waves per SIMD-cycle: waves' VALU instructions in flight overlap, so it can exceed
1 (round 5's sky kernel read 1.025) and is not a utilisation.

usage: pmc_mix.py <passA.csv> <passB.csv> <config> <wave_iterations_per_launch> <out.json> [label] [kernel]

kernel: a substring of the kernel name to select (default iqpt_render_kernel; e.g. iqpt_spec_kernel,
iqpt_fan_kernel, iqpt_chain_kernel).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "path-tracer-and-rasterizer-engine_amd"))
from iqpt._build import kernel_source_sha16  # noqa: E402  (the kernels the profile describes; bench.py keys on it)

SIMDS = 256 * 4


KERNEL = "iqpt_render_kernel"


def last_dispatch(path):
    agg = defaultdict(lambda: defaultdict(float))
    dur = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if KERNEL not in r.get("Kernel_Name", ""):
                continue
            agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    if not agg:
        raise SystemExit(f"no {KERNEL} rows in {path}")
    d = sorted(agg, key=int)[-1]
    return dict(agg[d]), dur[d]


def main():
    a_csv, b_csv, config, iters, out = sys.argv[1:6]
    label = sys.argv[6] if len(sys.argv) > 6 else ""
    global KERNEL
    if len(sys.argv) > 7:
        KERNEL = sys.argv[7]
    iters = float(iters)
    a, _ = last_dispatch(a_csv)
    b, dur = last_dispatch(b_csv)
    kcycles = b["GRBM_GUI_ACTIVE"] / 8.0
    wave = b["SQ_WAVE_CYCLES"]
    res = {
        "config": config,
        "kernel": label or KERNEL,
        "kernel_sha16": kernel_source_sha16(),
        "wave_iterations_per_launch": iters,
        "counters": {**a, **b},
        "per_iteration": {k: round(v / iters, 2) for k, v in a.items() if k.startswith("SQ_INSTS")},
        "kernel_ms_profiled": round(dur * 1e3, 4),
        "clock_ghz": round(kcycles / dur / 1e9, 3),
        "valu_busy_frac": round((2.0 * a["SQ_INSTS_VALU"] + 2.0 * a.get("SQ_INSTS_VALU_TRANS_F32", 0.0)) / SIMDS / kcycles, 3),
        "valu_active_per_simd": round(b["SQ_ACTIVE_INST_VALU"] * 4 / SIMDS / kcycles, 3),
        "wave_time_split": {"issuing": round(b["SQ_ACTIVE_INST_ANY"] / wave, 3),
                            "ready_not_issued": round(b["SQ_WAIT_INST_ANY"] / wave, 3),
                            "parked_on_waitcnt": round(b["SQ_WAIT_ANY"] / wave, 3)},
        "mean_waves_per_simd": round(wave * 4 / SIMDS / kcycles, 2),
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
