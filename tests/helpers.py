"""Helpers shared by the parity tests: build a config's scene, render it on both sides."""
from __future__ import annotations

import numpy as np

import oracle
from iqpt import PathTracer, Scene, make_camera
from iqpt.render import pixel_set


def scene_for(preset: str):
    sc = Scene()
    sc.add_preset(preset)
    return sc, sc.build_packet()


def oracle_render(preset, width, height, spp, max_depth, pixels=None, seed=1984, launches=None, glibc=False):
    sc, pk = scene_for(preset)
    cam = make_camera(width, height)
    fr = oracle.OracleFrame(width, height, pixels=pixels, seed=seed, max_depth=max_depth, glibc=glibc)
    for s in (launches or [spp]):
        fr.render(pk, cam, s)
    return fr


def gpu_render(preset, width, height, spp, max_depth, pixels=None, seed=1984, launches=None, split=None):
    sc, pk = scene_for(preset)
    cam = make_camera(width, height)
    pt = PathTracer(width, height, pixels=pixels, seed=seed, max_depth=max_depth)
    if split is not None:
        pt.set_split(split)
    pt.set_camera(cam)
    pt.upload_packet(pk)
    for s in (launches or [spp]):
        pt.render(s)
    lin, bgra = pt.read()
    return pt, lin, bgra


def compare(lin_a: np.ndarray, lin_b: np.ndarray) -> dict:
    """Per-pixel RMSE over RGB and the count of bit-identical pixels."""
    a = lin_a[:, :3].astype(np.float64)
    b = lin_b[:, :3].astype(np.float64)
    both_nan = np.isnan(a) & np.isnan(b)
    d = np.where(both_nan, 0.0, a - b)
    rmse = float(np.sqrt(np.mean(d * d))) if d.size else 0.0
    # bit-identical per component; a NaN matches a NaN of any payload/sign (IEEE leaves the payload
    # of a generated NaN to the implementation: x86 SSE yields 0xffc00000, gfx950 0x7fc00000, CUDA
    # 0x7fffffff — the reference itself has no fixed NaN bits)
    same = np.all((lin_a[:, :3].view(np.uint32) == lin_b[:, :3].view(np.uint32)) | both_nan, axis=1)
    return {"rmse": rmse, "bitexact": int(same.sum()), "npix": int(lin_a.shape[0]),
            "maxabs": float(np.max(np.abs(d))) if d.size else 0.0}


__all__ = ["scene_for", "oracle_render", "gpu_render", "compare", "pixel_set"]
