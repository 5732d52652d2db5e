"""The product's multi-rank path end to end (C3 of BASELINE.json): bench.py --gpus 2 starts its two rank
processes itself, each renders its cyclic row share through libiqpt, every step gathers the frame to
rank 0, and the float accumulators gathered after timing must equal a 1-rank render bit for bit
(RNG streams are keyed by the global pixel id, path_tracer.cu:36-46/336-339). One GPU: both ranks on
device 0 with gloo collectives (RCCL refuses two ranks on one device); the driver's runs use RCCL.
"""
import json
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _bench(tmp_path, gpus, name, extra=(), timeout=240):
    out = tmp_path / f"{name}.npy"
    cmd = [sys.executable, str(REPO / "bench.py"), "--gpus", str(gpus), "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--verify-rows", "2", "--save-frame", str(out), *extra]
    if gpus > 1:
        cmd += ["--backend", "gloo", "--one-device"]
    proc = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    assert proc.returncode == 0, proc.stderr[-3000:]
    line = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line), np.load(out)


@pytest.mark.parametrize("gather", ["frame", "accum"])
def test_two_rank_strong_frame_equals_one_rank(require_gpu, tmp_path, gather):
    one, f1 = _bench(tmp_path, 1, "one")
    two, f2 = _bench(tmp_path, 2, "two", ("--gather", gather))
    assert two["n_gpus"] == 2 and two["n_ranks_seen"] == 2 and two["scaling"] == "strong"
    assert two["bitexact_frac_vs_oracle"] == 1.0 and one["bitexact_frac_vs_oracle"] == 1.0
    assert f1.shape == f2.shape == (1920 * 1080, 4)
    assert np.array_equal(f1.view(np.uint32), f2.view(np.uint32))
    # same work: the rays of two half frames add up to the rays of the whole frame
    assert two["rays_per_sample"] == one["rays_per_sample"]


@pytest.mark.parametrize("share,split,mode", [(2, "auto", "spec"), (2, "off", "plain"), (4, "auto", "spec"),
                                              (8, "auto", "spec")])
def test_stream_ordered_gather_on_one_gpu(require_gpu, tmp_path, share, split, mode):
    """The RCCL path the driver's N-GPU runs take, on one GPU: a one-rank nccl process group, rank 0's
    rows of an N-way split, the stream-ordered frame copy + gather every step, 8 hardware queues: the
    pipelined spec launches AUTO takes (copies on a third stream behind both kernels), overlapped plain
    launches at N = 2 (copies on the last launch's stream; the RCCL kernels share the CUs with launches
    that wait per tile for the one before)."""
    res, _ = _bench(tmp_path, 1, f"self{share}{split}", ("--self-gather", "--share-of", str(share), "--split", split))
    assert res["gather"] == "stream-ordered" and res["gather_check"] is True
    assert res["hw_queues"] == 8 and res["n_ranks_seen"] == 1
    assert res["config"]["launch_mode"] == mode
    assert res["bitexact_frac_vs_oracle"] == 1.0


@pytest.mark.parametrize("gpus", [4, 8])
def test_c3_assembly_at_4_and_8_ranks(require_gpu, tmp_path, gpus):
    """C3 as the driver's N-GPU runs split it, at N = 4 and 8: bench.py --gpus N starts N fresh rank
    processes (here all on GPU 0, gloo through host memory), each renders its cyclic rows through the
    sample-parallel launches of small shares, every step gathers the BGRA frame to rank 0, and the float
    accumulators gathered after timing must equal the 1-rank frame bit for bit."""
    one, f1 = _bench(tmp_path, 1, "one")
    res, fn = _bench(tmp_path, gpus, f"n{gpus}", timeout=600)
    assert res["n_gpus"] == gpus and res["n_ranks_seen"] == gpus and res["scaling"] == "strong"
    assert res["gather_check"] is True
    assert res["config"]["launch_mode"] != "plain", res["config"]
    assert res["bitexact_frac_vs_oracle"] == 1.0
    assert fn.shape == f1.shape == (1920 * 1080, 4)
    assert np.array_equal(f1.view(np.uint32), fn.view(np.uint32))
    assert res["rays_per_sample"] == one["rays_per_sample"]
