"""cuRAND XORWOW restatement (csrc/iq_xorwow.h): step, seeding, subsequence jumps.

The jump matrices are pinned against the independent tables ROCm ships
(/opt/rocm/include/rocrand/rocrand_xorwow_precomputed.h: A^(4^i * 2^67)). The seeding constants
are cuRAND's published ones; no reference output pins them (parity with real cuRAND unpinned).
"""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

import oracle

ROCRAND = Path("/opt/rocm/include/rocrand/rocrand_xorwow_precomputed.h")
UP = C.POINTER(C.c_uint32)


def seed_state(seed):
    st = np.zeros(6, dtype=np.uint32)
    oracle.load().iqo_xorwow_seed(seed, st.ctypes.data_as(UP))
    return st


def step(st):
    return oracle.load().iqo_xorwow_next(st.ctypes.data_as(UP))


def py_next(s):
    v0, v1, v2, v3, v4, d = [int(x) for x in s]
    t = (v0 ^ (v0 >> 2)) & 0xffffffff
    v4n = ((v4 ^ ((v4 << 4) & 0xffffffff)) ^ (t ^ ((t << 1) & 0xffffffff))) & 0xffffffff
    d = (d + 362437) & 0xffffffff
    return [v1, v2, v3, v4, v4n, d], (v4n + d) & 0xffffffff


def test_seed_kat_curand_init_1984():
    """curand_init(1984, 0, 0) (path_tracer.cu:45) — the KAT recorded in SURVEY.md §8c."""
    st = seed_state(1984)
    assert st[5] == 237688853
    assert list(st[:5]) == [999278866, 564768280, 4171507460, 3705206908, 881605398]
    assert step(st) == 841754470


def test_step_matches_python_recurrence():
    st = seed_state(12345)
    s = list(st)
    for _ in range(1000):
        s, r = py_next(s)
        assert step(st) == r
    assert list(st) == s


def tables(count):
    out = np.zeros((count, 800), dtype=np.uint32)
    oracle.load().iqo_xorwow_tables(out.ctypes.data_as(UP), count)
    return out


def matvec(m, v):
    r = np.zeros(5, dtype=np.uint32)
    for i in range(5):
        for j in range(32):
            if (int(v[i]) >> j) & 1:
                r ^= m[(i * 32 + j) * 5:(i * 32 + j) * 5 + 5]
    return r


def matmul(a, b):
    out = np.zeros(800, dtype=np.uint32)
    for c in range(160):
        out[c * 5:c * 5 + 5] = matvec(a, b[c * 5:c * 5 + 5])
    return out


@pytest.mark.skipif(not ROCRAND.exists(), reason="rocRAND headers absent")
def test_jump_tables_match_rocrand_sequence_tables():
    text = ROCRAND.read_text()
    m = re.search(r"h_xorwow_sequence_jump_matrices\[XORWOW_JUMP_MATRICES\]\[XORWOW_SIZE\]\s*=\s*\{(.*?)\};",
                  text, re.S)
    assert m
    nums = [int(x, 0) for x in re.findall(r"0x[0-9a-fA-F]+|\d+", m.group(1).replace("U", ""))]
    roc = np.array(nums, dtype=np.uint64).astype(np.uint32).reshape(-1, 800)
    ours = tables(7)                                         # A^(2^(67+i)), i < 7
    assert np.array_equal(ours[0], roc[0])                   # A^(2^67)
    assert np.array_equal(ours[2], roc[1])                   # A^(4 * 2^67)
    assert np.array_equal(ours[4], roc[2])                   # A^(16 * 2^67)
    assert np.array_equal(ours[6], roc[3])                   # A^(64 * 2^67)
    assert np.array_equal(matmul(ours[0], ours[0]), ours[1]) # squaring composes


def test_subsequence_init_composes():
    """curand_init(seed, p) for p = 0..5 and bigger ids equals successive 2^67 jumps."""
    lib = oracle.load()
    ps = oracle.pixel_set(7, 1)
    st = np.zeros((7, 6), dtype=np.uint32)
    lib.iqo_rng_init(7, C.byref(ps), 1984, st.ctypes.data_as(UP))
    t = tables(3)
    v = seed_state(1984)
    for p in range(7):
        assert np.array_equal(st[p, :5], v[:5]), p
        assert st[p, 5] == v[5]
        v[:5] = matvec(t[0], v[:5])


def test_rng_states_keyed_by_global_pixel_id():
    """A crop's states equal the same pixels of the full frame (path_tracer.cu:43, 338)."""
    lib = oracle.load()
    W, H = 64, 32
    full = np.zeros((W * H, 6), dtype=np.uint32)
    lib.iqo_rng_init(W, C.byref(oracle.pixel_set(W, H)), 1984, full.ctypes.data_as(UP))
    ps = oracle.pixel_set(W, H, 10, 30, 3, 4, 7)
    crop = np.zeros((20 * 7, 6), dtype=np.uint32)
    lib.iqo_rng_init(W, C.byref(ps), 1984, crop.ctypes.data_as(UP))
    rows = 3 + 4 * np.arange(7)
    expect = full.reshape(H, W, 6)[rows][:, 10:30].reshape(-1, 6)
    assert np.array_equal(crop, expect)
