"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (oracle/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The oracle restates the reference hot path on the CPU (oracle/iqpt_oracle.c); parity against the
reference binary itself is UNPINNED (the reference cannot be built here and ships no golden data).
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_PROJ = _HERE.parent / "path-tracer-and-rasterizer-engine_amd"
if str(_PROJ) not in sys.path:
    sys.path.insert(0, str(_PROJ))

from iqpt._lib import Camera, PacketDesc, PixelSet  # noqa: E402  (ctypes layouts of include/iqpt.h)

LIB = _HERE / "liboracle.so"
LIB_GLIBC = _HERE / "liboracle_glibc.so"
LIB_FMA = _HERE / "liboracle_fma.so"     # informational flavour: FMA contraction on, glibc libm
# bench.py's CPU baseline: flavour B built on the host that runs it with -O3 -march=native (iqpt._build.
# build_oracle_native), so it matches that host's CPU
LIB_NATIVE = _HERE / "_native" / "liboracle_native.so"

_cache: dict[str, C.CDLL] = {}
_FP = C.POINTER(C.c_float)
_UP = C.POINTER(C.c_uint32)


def load(glibc: bool = False, flavour: str | None = None) -> C.CDLL:
    """flavour: None / "b" (the parity target), "glibc", "fma" (see DESIGN.md §4), "native" (flavour B with
    -march=native, built on this host: bench.py's CPU baseline)."""
    flavour = flavour or ("glibc" if glibc else "b")
    path = {"b": LIB, "glibc": LIB_GLIBC, "fma": LIB_FMA, "native": LIB_NATIVE}[flavour]
    key = str(path)
    if key in _cache:
        return _cache[key]
    if not path.exists():
        raise ImportError(f"{path} missing: run __graft_entry__.build()")
    lib = C.CDLL(str(path))
    lib.iqo_rng_init.argtypes = [C.c_uint32, C.POINTER(PixelSet), C.c_uint64, _UP]
    lib.iqo_render.argtypes = [C.POINTER(PacketDesc), C.POINTER(Camera), C.c_int, C.POINTER(PixelSet), C.c_uint64,
                               C.c_uint32, _UP, _FP, C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.c_int]
    lib.iqo_get_ray.argtypes = [C.POINTER(Camera), C.c_uint32, C.c_uint32, _UP, _FP, _FP]
    lib.iqo_triangle_intersect.argtypes = [_FP] * 8 + [C.c_float, C.c_float, _FP, _FP, _FP, C.POINTER(C.c_int)]
    lib.iqo_sphere_intersect.argtypes = [_FP, C.c_float, _FP, _FP, C.c_float, C.c_float, _FP, _FP, _FP,
                                         C.POINTER(C.c_int)]
    lib.iqo_onb.argtypes = [_FP, _FP, _FP, _FP]
    lib.iqo_cosine_weighted.argtypes = [_UP, _FP]
    lib.iqo_oren_nayar.argtypes = [_FP, _FP, _FP, _UP, _FP, _FP, _FP, _FP, _FP]
    lib.iqo_normal_matrix.argtypes = [_FP, _FP]
    lib.iqo_transform_point.argtypes = [_FP, _FP, _FP]
    for fn in ("iqo_sinf", "iqo_cosf", "iqo_tanf", "iqo_acosf", "iqo_asinf"):
        getattr(lib, fn).argtypes = [C.c_float]
        getattr(lib, fn).restype = C.c_float
    lib.iqo_atan2f.argtypes = [C.c_float, C.c_float]
    lib.iqo_atan2f.restype = C.c_float
    lib.iqo_libm_batch.argtypes = [C.c_int, _FP, _FP, _FP, C.c_int64]
    lib.iqo_xorwow_tables.argtypes = [_UP, C.c_int]
    lib.iqo_xorwow_seed.argtypes = [C.c_uint64, _UP]
    lib.iqo_xorwow_next.argtypes = [_UP]
    lib.iqo_xorwow_next.restype = C.c_uint32
    _cache[key] = lib
    return lib


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_FP)


def _up(a: np.ndarray):
    return a.ctypes.data_as(_UP)


def pixel_set(width: int, height: int, x0=0, x1=None, y0=0, ystep=1, nrows=None) -> PixelSet:
    x1 = width if x1 is None else x1
    if nrows is None:
        nrows = (height - y0 + ystep - 1) // ystep
    return PixelSet(x0, x1, y0, ystep, nrows)


class OracleFrame:
    """Per-pixel state of one pixel set, advanced on the CPU exactly like the reference kernel."""

    def __init__(self, width: int, height: int, pixels: PixelSet | None = None, seed: int = 1984,
                 max_depth: int = 5, glibc: bool = False, flavour: str | None = None):
        self.lib = load(glibc, flavour)
        self.width, self.height = width, height
        self.pixels = pixels if pixels is not None else pixel_set(width, height)
        self.npix = (self.pixels.x1 - self.pixels.x0) * self.pixels.nrows
        self.max_depth = max_depth
        self.states = np.zeros((self.npix, 6), dtype=np.uint32)
        self.lin = np.zeros((self.npix, 4), dtype=np.float32)
        self.bgra = np.zeros((self.npix, 4), dtype=np.uint8)
        self.rays = np.zeros(self.npix, dtype=np.uint64)
        self.frame = 0
        st = self.lib.iqo_rng_init(width, C.byref(self.pixels), seed, _up(self.states))
        assert st == 0

    def render(self, packet: PacketDesc, camera: Camera, spp: int, threads: int | None = None) -> int:
        """spp consecutive reference launches; returns the closest-hit queries traced."""
        nthreads = threads if threads is not None else int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
        rays = np.zeros(self.npix, dtype=np.uint64)
        st = self.lib.iqo_render(C.byref(packet), C.byref(camera), self.max_depth, C.byref(self.pixels),
                                 self.frame, spp, _up(self.states), _fp(self.lin),
                                 self.bgra.ctypes.data_as(C.POINTER(C.c_uint8)),
                                 rays.ctypes.data_as(C.POINTER(C.c_uint64)), nthreads)
        if st != 0:
            raise RuntimeError(f"iqo_render failed with status {st}")
        self.frame += spp
        self.rays += rays
        return int(rays.sum())

    def reset(self):
        """path_tracer.cu:394-400: clear the BGRA frame and restart the mean (lin and RNG kept)."""
        self.bgra[:] = 0
        self.frame = 0
