"""The C++ path_tracer facade (csrc/path_tracer.hpp) and the headless CLI, on the GPU.

test_facade drives the facade like IoniqRE's application loop (cadence, deferred reset, present)
and prints checksums that must equal the C-ABI path, which the parity tests tie to the oracle.
"""
import json
import subprocess

import numpy as np
import pytest

from iqpt import _build

pytestmark = pytest.mark.gpu


def test_facade_program(require_gpu, tmp_path):
    exe = _build.FACADE_TEST_PATH
    assert exe.exists()
    res = subprocess.run([str(exe), str(tmp_path / "facade.ppm")], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["ok"] is True
    assert out["sharded_equal"] is True          # the facade's sharded present path (RCCL gather, world 1)
    # the same four 1-spp launches through the Python C-ABI binding, then oracle
    import oracle
    from helpers import scene_for
    from iqpt import make_camera
    sc, pk = scene_for("cornell")
    cam = make_camera(96, 64)
    fr = oracle.OracleFrame(96, 64, max_depth=8)
    for _ in range(4):
        fr.render(pk, cam, 1)
    s4 = float(np.sum(fr.lin[:, :3].astype(np.float64)))
    assert abs(out["sum_after_4"] - s4) <= 1e-6 * max(1.0, s4)
    fr.reset()
    fr.render(pk, cam, 1)
    s5 = float(np.sum(fr.lin[:, :3].astype(np.float64)))
    assert abs(out["sum_after_reset"] - s5) <= 1e-6 * max(1.0, s5)
    assert (tmp_path / "facade.ppm").read_bytes().startswith(b"P6\n96 64\n255\n")


def test_cli_headless_dump(require_gpu, tmp_path):
    out = tmp_path / "cornell.ppm"
    res = subprocess.run([str(_build.CLI_PATH), "--preset", "cornell", "--width", "64", "--height", "36",
                          "--spp", "8", "--launches", "2", "--out", str(out)], capture_output=True, text=True,
                         timeout=300)
    assert res.returncode == 0, res.stderr
    info = json.loads(res.stdout.strip().splitlines()[-1])
    assert info["frames"] == 16
    data = out.read_bytes()
    assert data.startswith(b"P6\n64 36\n255\n") and len(data) == len(b"P6\n64 36\n255\n") + 64 * 36 * 3
