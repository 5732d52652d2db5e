#!/usr/bin/env python3
"""Frame-level distance between the parity target and two other floating-point flavours of the
reference kernel, on the CPU oracle (test infrastructure):

* B (the target, what the HIP kernel reproduces bit for bit): iq_fp.h transcendentals, contraction off;
* A: glibc libm transcendentals, contraction off;
* FMA: glibc libm with FMA contraction on (-ffp-contract=fast -mfma): the closest this image gets to
  nvcc's default build of the reference (contraction on, libdevice; IoniqRE.vcxproj:58-64,82-86).

Per-pixel RMSE over RGB, bit-identical pixel fraction and ray counts, written as JSON.

    python tools/fp_flavours.py [--full] [--out profiles/r02/fp_flavours.json]
"""
import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
for p in (REPO / "tests", REPO / "oracle", REPO / "path-tracer-and-rasterizer-engine_amd"):
    sys.path.insert(0, str(p))

import oracle  # noqa: E402  (test infrastructure)
from helpers import compare, scene_for  # noqa: E402
from iqpt import make_camera, pixel_set  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true", help="the whole C2 frame (1920x1080, 64 spp)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    cases = [("c2_crop", "cornell", 1920, 1080, 64, 8, (880, 1000, 470, 1, 48)),
             ("app_default", "app_default", 320, 180, 64, 5, None)]
    if args.full:
        cases.append(("c2_full", "cornell", 1920, 1080, 64, 8, None))
    out = {"flavours": {"B": "iq_fp.h, contraction off (parity target)", "A": "glibc libm, contraction off",
                        "FMA": "glibc libm, -ffp-contract=fast -mfma"}, "cases": {}}
    for name, preset, w, h, spp, depth, crop in cases:
        sc, pk = scene_for(preset)
        cam = make_camera(w, h)
        ps = pixel_set(w, h, *crop) if crop else None
        frames = {}
        for fl in ("b", "glibc", "fma"):
            t0 = time.time()
            f = oracle.OracleFrame(w, h, pixels=ps, max_depth=depth, flavour=fl)
            f.render(pk, cam, spp)
            frames[fl] = (f, time.time() - t0)
        row = {"preset": preset, "size": [w, h], "spp": spp, "max_depth": depth, "crop": crop}
        for fl, key in (("glibc", "A_vs_B"), ("fma", "FMA_vs_B")):
            c = compare(frames["b"][0].lin, frames[fl][0].lin)
            row[key] = {"rmse": c["rmse"], "bitexact_frac": c["bitexact"] / c["npix"], "maxabs": c["maxabs"],
                        "rays": int(frames[fl][0].rays.sum()), "rays_B": int(frames["b"][0].rays.sum())}
        out["cases"][name] = row
        print(name, json.dumps(row), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
