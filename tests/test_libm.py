"""The shared transcendentals of csrc/iq_fp.h (FP policy).

They replace CUDA libdevice's sinf/cosf/tanf/acosf/atan2f (material.cu:28-37, random.cu:100-102),
which cannot run here. Accuracy is checked against float64 numpy on the argument ranges the
kernel produces; CUDA documents 2-4 ulp for the functions the reference calls.
"""
import ctypes as C

import numpy as np
import pytest

import oracle

FN = {"sin": 0, "cos": 1, "tan": 2, "acos": 3, "atan2": 4, "asin": 5, "atan": 6}


def run(fn, a, b=None):
    lib = oracle.load()
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b if b is not None else np.zeros_like(a), dtype=np.float32)
    out = np.empty_like(a)
    lib.iqo_libm_batch(FN[fn], a.ctypes.data_as(C.POINTER(C.c_float)), b.ctypes.data_as(C.POINTER(C.c_float)),
                       out.ctypes.data_as(C.POINTER(C.c_float)), a.size)
    return out


def ulp_err(got, exact):
    exact32 = exact.astype(np.float32)
    sp = np.spacing(np.abs(exact32)).astype(np.float64)
    sp = np.maximum(sp, np.float64(np.spacing(np.float32(0))))
    return np.abs(got.astype(np.float64) - exact) / sp


def _rng(tag: str) -> np.random.Generator:
    """A generator per test, so a sample does not depend on which tests ran before (pytest -n)."""
    return np.random.default_rng(sum(map(ord, tag)) + 7)


@pytest.mark.parametrize("fn,lo,hi,ref,max_ulp", [
    ("sin", 0.0, 2 * np.pi, np.sin, 2.0),            # cosine_weighted phi in [0, 2pi]
    ("cos", 0.0, 2 * np.pi, np.cos, 2.0),
    ("sin", 0.0, np.pi / 2, np.sin, 2.0),            # sinf(alpha), alpha in [0, pi/2]
    ("cos", -2 * np.pi, 2 * np.pi, np.cos, 2.0),     # cosf(phi_i - phi_o)
    ("tan", 0.0, np.pi / 2 - 1e-3, np.tan, 3.0),     # tanf(beta)
    ("acos", 0.0, 1.0, np.arccos, 2.0),              # acosf(costheta)
    ("acos", -1.0, 1.0, np.arccos, 2.0),
    ("asin", -1.0, 1.0, np.arcsin, 2.5),
    ("atan", -50.0, 50.0, np.arctan, 3.0),
    ("sin", -100.0, 100.0, np.sin, 2.0),
    ("cos", -100.0, 100.0, np.cos, 2.0),
])
def test_accuracy(fn, lo, hi, ref, max_ulp):
    x = _rng(f"{fn}{lo}{hi}").uniform(lo, hi, 200_000).astype(np.float32)
    got = run(fn, x)
    e = ulp_err(got, ref(x.astype(np.float64)))
    assert e.max() <= max_ulp, (fn, float(e.max()), float(x[np.argmax(e)]))


def test_atan2_accuracy_all_quadrants():
    # measured maximum over 10^7 uniform (y, x) in [-1, 1]^2: 3.13 ulp (atan of the quotient, <= 2.5 ulp,
    # plus the rounding of y / x and of the quadrant offset)
    r = _rng("atan2")
    y = r.uniform(-1, 1, 200_000).astype(np.float32)
    x = r.uniform(-1, 1, 200_000).astype(np.float32)
    got = run("atan2", y, x)
    e = ulp_err(got, np.arctan2(y.astype(np.float64), x.astype(np.float64)))
    assert e.max() <= 3.25, float(e.max())


def test_atan2_special_cases_c99():
    inf, nan = np.float32(np.inf), np.float32(np.nan)
    cases = [(0.0, 1.0), (-0.0, 1.0), (0.0, -1.0), (-0.0, -1.0), (0.0, 0.0), (0.0, -0.0), (-0.0, -0.0),
             (1.0, 0.0), (-1.0, 0.0), (inf, 1.0), (-inf, 1.0), (inf, inf), (inf, -inf), (1.0, inf),
             (1.0, -inf), (-1.0, -inf), (1e-30, -1.0)]
    y = np.array([c[0] for c in cases], dtype=np.float32)
    x = np.array([c[1] for c in cases], dtype=np.float32)
    got = run("atan2", y, x)
    exact = np.arctan2(y.astype(np.float64), x.astype(np.float64))
    assert np.all(np.signbit(got) == np.signbit(exact)), (got, exact)
    assert np.all(ulp_err(got, exact) <= 1.0), (got, exact)
    assert np.isnan(run("atan2", np.array([nan]), np.array([1.0]))[0])


def test_special_values():
    nan_in = np.array([np.nan, np.inf, -np.inf], dtype=np.float32)
    for fn in ("sin", "cos", "tan"):
        assert np.all(np.isnan(run(fn, nan_in)))
    assert np.all(np.isnan(run("acos", np.array([1.5, -1.5, np.nan], dtype=np.float32))))
    assert run("acos", np.array([1.0], dtype=np.float32))[0] == 0.0
    assert run("sin", np.array([0.0], dtype=np.float32))[0] == 0.0
    assert np.signbit(run("sin", np.array([-0.0], dtype=np.float32))[0])
    assert run("cos", np.array([0.0], dtype=np.float32))[0] == 1.0


def test_glibc_flavour_is_close():
    """Flavour A (glibc libm) vs flavour B (iq_fp.h): the substitution is within a few ulp."""
    ga = oracle.load(glibc=True)
    assert ga.iqo_has_glibc_libm() == 1
    x = _rng("glibc").uniform(0, 2 * np.pi, 10_000).astype(np.float32)
    a = np.array([ga.iqo_sinf(float(v)) for v in x[:2000]], dtype=np.float32)
    b = run("sin", x[:2000])
    assert np.max(ulp_err(b, a.astype(np.float64))) <= 3.0
