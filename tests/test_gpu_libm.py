"""The device build of the shared math (csrc/iq_fp.h + csrc/iq_fastdiv.h, as the render kernel
compiles it) against the host build the oracle runs, bit for bit.

The GPU pass uses the short exact reciprocal / division / sqrt forms of iq_fastdiv.h inside the
transcendentals (tools/fastdiv_check.hip proves the forms on all reciprocals and roots); this test
checks the composed functions on the argument ranges the kernel produces, the special values and
wide random ranges. A NaN matches a NaN of any payload (tests/helpers.py).
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from iqpt import _lib

pytestmark = pytest.mark.gpu

FP = C.POINTER(C.c_float)
ORACLE_FN = {"sin": 0, "cos": 1, "tan": 2, "acos": 3, "atan2": 4, "asin": 5, "atan": 6}
GPU_FN = dict(ORACLE_FN, sincos_sin=7, sincos_cos=8, sqrt=9, rcp=10, div=11,
              atan2_x2_lo=12, atan2_x2_hi=13, acos_x2_lo=14, acos_x2_hi=15, sin_x2=16, cos_x2=17, tan_bf=18,
              sqrt_x2=19)

SPECIAL = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 0.5, -0.5, 1e-45, -1e-45, 1e-38, 3.4e38,
                    -3.4e38, np.pi / 2, np.pi, 2 * np.pi, 1e-4, 1.0001e-4, 0.4142135, 0.41421357, 2.4142137,
                    2.4142134, 8192.0, 8193.5, 1e18, 1.1e18, 2.0 ** 126, 2.0 ** -126, 2.0 ** -127],
                   dtype=np.float32)


def gpu(fn, a, b=None):
    lib = _lib.load()
    f = lib.iqpt_debug_libm
    f.argtypes = [C.c_int, FP, FP, FP, C.c_uint64]
    f.restype = C.c_int
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b if b is not None else np.zeros_like(a), dtype=np.float32)
    out = np.empty_like(a)
    assert f(GPU_FN[fn], a.ctypes.data_as(FP), b.ctypes.data_as(FP), out.ctypes.data_as(FP), a.size) == 0, \
        lib.iqpt_last_error()
    return out


def host(fn, a, b=None):
    lib = oracle.load()
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b if b is not None else np.zeros_like(a), dtype=np.float32)
    out = np.empty_like(a)
    lib.iqo_libm_batch(ORACLE_FN[fn], a.ctypes.data_as(FP), b.ctypes.data_as(FP), out.ctypes.data_as(FP), a.size)
    return out


def same_bits(x, y):
    return (x.view(np.uint32) == y.view(np.uint32)) | (np.isnan(x) & np.isnan(y))


def check(got, want, *inputs):
    ok = same_bits(got, want)
    if not ok.all():
        i = int(np.flatnonzero(~ok)[0])
        raise AssertionError(f"{(~ok).sum()} mismatches, first at inputs {[float(v[i]) for v in inputs]}: "
                             f"got {got[i]!r} ({got[i:i+1].view(np.uint32)[0]:08x}) want {want[i]!r} "
                             f"({want[i:i+1].view(np.uint32)[0]:08x})")


rng = np.random.default_rng(2024)


def args(lo, hi, n=1 << 20):
    return np.concatenate([rng.uniform(lo, hi, n).astype(np.float32), SPECIAL])


def random_bits(n=1 << 20):
    return rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)


@pytest.mark.parametrize("fn,lo,hi", [
    ("sin", 0.0, 2 * np.pi), ("cos", -2 * np.pi, 2 * np.pi), ("tan", 0.0, np.pi / 2), ("tan", -1e4, 1e4),
    ("acos", -1.0, 1.0), ("asin", -1.0, 1.0), ("atan", -50.0, 50.0), ("atan", -1e30, 1e30),
    ("sin", -1e6, 1e6), ("cos", -1e6, 1e6),
])
def test_transcendentals_device_equals_host(require_gpu, fn, lo, hi):
    a = args(lo, hi)
    check(gpu(fn, a), host(fn, a), a)


@pytest.mark.parametrize("fn", ["sin", "cos", "tan", "acos", "asin", "atan"])
def test_transcendentals_random_bit_patterns(require_gpu, fn):
    a = np.concatenate([random_bits(), SPECIAL])
    check(gpu(fn, a), host(fn, a), a)


def test_atan2_all_quadrants_and_extreme_ratios(require_gpu):
    n = 1 << 20
    f32 = np.float32
    y = np.concatenate([rng.uniform(-1, 1, n).astype(f32), (rng.uniform(-1, 1, n) * 1e-30).astype(f32), random_bits(n)])
    x = np.concatenate([rng.uniform(-1, 1, n).astype(f32), rng.uniform(-1, 1, n).astype(f32), random_bits(n)])
    sy, sx = np.meshgrid(SPECIAL, SPECIAL)
    y = np.concatenate([y, sy.ravel()])
    x = np.concatenate([x, sx.ravel()])
    check(gpu("atan2", y, x), host("atan2", y, x), y, x)


def test_sincos_equals_sin_and_cos(require_gpu):
    a = np.concatenate([args(0.0, 2 * np.pi), random_bits()])
    check(gpu("sincos_sin", a), host("sin", a), a)
    check(gpu("sincos_cos", a), host("cos", a), a)


def test_short_sqrt_rcp_div_are_ieee(require_gpu):
    a = np.concatenate([random_bits(), SPECIAL])
    with np.errstate(all="ignore"):
        check(gpu("sqrt", a), np.sqrt(a), a)
        check(gpu("rcp", a), np.float32(1.0) / a, a)
        b = np.concatenate([random_bits(), SPECIAL[::-1]])
        check(gpu("div", a, b), a / b, a, b)


# iq_fp2.h: the packed, branch-free pairs of the Oren-Nayar scatter (kOptScatter2). Each lane evaluates
# element i in one slot of the pair and the mirrored element n-1-i in the other; "_lo"/"_hi" read the
# two slots, so every input is checked in both.
def pair_inputs(n=1 << 20):
    f32 = np.float32
    sy, sx = np.meshgrid(SPECIAL, SPECIAL)
    y = np.concatenate([rng.uniform(-1, 1, n).astype(f32), (rng.uniform(-1, 1, n) * 1e-30).astype(f32),
                        random_bits(n), sy.ravel()])
    x = np.concatenate([rng.uniform(-1, 1, n).astype(f32), rng.uniform(-1, 1, n).astype(f32), random_bits(n),
                        sx.ravel()])
    return y, x


def test_atan2_pairs_equal_scalar(require_gpu):
    y, x = pair_inputs()
    want = host("atan2", y, x)
    check(gpu("atan2_x2_lo", y, x), want, y, x)
    check(gpu("atan2_x2_hi", y, x), want, y, x)


@pytest.mark.parametrize("lo,hi", [(0.0, 1.0), (-1.0, 1.0), (-1.1, 1.1)])
def test_acos_pairs_equal_scalar(require_gpu, lo, hi):
    a = np.concatenate([args(lo, hi), random_bits()])
    want = host("acos", a)
    check(gpu("acos_x2_lo", a), want, a)
    check(gpu("acos_x2_hi", a), want, a)


@pytest.mark.parametrize("lo,hi", [(0.0, 2 * np.pi), (-2 * np.pi, 2 * np.pi), (-1e4, 1e4)])
def test_sin_cos_pairs_and_tan_equal_scalar(require_gpu, lo, hi):
    a = np.concatenate([args(lo, hi), random_bits()])
    check(gpu("sin_x2", a), host("sin", a), a)
    check(gpu("cos_x2", a), host("cos", a), a)
    check(gpu("tan_bf", a), host("tan", a), a)


def test_sqrt_pair_is_ieee_on_its_domain(require_gpu):
    a = np.concatenate([random_bits(), SPECIAL])
    a = a[(np.abs(a) >= 2.0 ** -96) | (a == 0) | np.isnan(a)]
    with np.errstate(all="ignore"):
        want = np.sqrt(a)
    got = gpu("sqrt_x2", a)
    pos = ~(a < 0)
    check(got[pos], want[pos], a[pos])
