"""Golden fixtures (tests/golden/*.npz, written by tests/golden/make_golden.py from the oracle).

CPU: the oracle reproduces them bit for bit (regression pin of the restatement).
GPU: the HIP kernel reproduces them bit for bit without running the oracle.
"""
import ctypes as C
import hashlib
import sys
from pathlib import Path

import numpy as np
import pytest

HERE = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(HERE))
import make_golden  # noqa: E402
import oracle  # noqa: E402


def load(name):
    return np.load(HERE / f"{name}.npz", allow_pickle=False)


def check(g, lin, bgra, rays, states):
    assert np.array_equal(lin.view(np.uint32), g["lin"].view(np.uint32))
    assert np.array_equal(bgra, g["bgra"])
    assert np.array_equal(rays.astype(np.uint16), g["rays"])
    assert hashlib.sha256(np.ascontiguousarray(states).tobytes()).digest() == g["states_sha256"].tobytes()


@pytest.mark.parametrize("name", list(make_golden.CASES))
def test_oracle_matches_golden(name):
    fr = make_golden.render(*make_golden.CASES[name])
    check(load(name), fr.lin, fr.bgra, fr.rays, fr.states)


def test_rng_kat():
    lib = oracle.load()
    for row in np.load(HERE / "rng_kat.npz")["kat"]:
        w, h, pid = int(row[0]), int(row[1]), int(row[2])
        ps = oracle.pixel_set(w, h, pid % w, pid % w + 1, pid // w, 1, 1)
        st = np.zeros((1, 6), dtype=np.uint32)
        lib.iqo_rng_init(w, C.byref(ps), 1984, st.ctypes.data_as(C.POINTER(C.c_uint32)))
        assert st[0].tolist() == [int(v) for v in row[3:]]


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(make_golden.CASES))
def test_gpu_matches_golden(require_gpu, name):
    import iqpt
    preset, w, h, launches, depth, crop = make_golden.CASES[name]
    sc = iqpt.Scene()
    sc.add_preset(preset)
    pk = sc.build_packet()
    ps = iqpt.pixel_set(w, h, *crop) if crop else None
    pt = iqpt.PathTracer(w, h, pixels=ps, max_depth=depth)
    pt.set_camera(iqpt.make_camera(w, h))
    pt.upload_packet(pk)
    for s in launches:
        pt.render(s)
    lin, bgra = pt.read()
    g = load(name)
    assert np.array_equal(lin.view(np.uint32), g["lin"].view(np.uint32))
    assert np.array_equal(bgra, g["bgra"])
    assert hashlib.sha256(pt.read_rng().tobytes()).digest() == g["states_sha256"].tobytes()
    assert pt.rays() == int(g["rays"].astype(np.uint64).sum())
