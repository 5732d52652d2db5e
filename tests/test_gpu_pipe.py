"""Two rays per lane (kOptPipe): the plain kernel traces a lane's path ray and the camera ray of
its pixel's next sample in one iteration; the second ray is used only when the path ends without drawing again
(path_tracer.cu:338-339). Every result must be the oracle's bits — accumulator, BGRA8, XORWOW states and ray
counts — with the two-ray variants actually launched, and equal to the one-ray kernel (iqpt_debug_set_two_ray 0)."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import scene_for
from iqpt import PathTracer, _lib, make_camera
from iqpt.render import pixel_set

pytestmark = pytest.mark.gpu

K_OPT_PIPE = 1 << 21
K_OPT_OVERLAP = 1 << 19


def last_options(pt):
    lb = _lib.load()
    lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    o = C.c_int(0)
    _lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(o)), "iqpt_debug_last_options")
    return o.value


def set_two_ray(pt, on):
    lb = _lib.load()
    lb.iqpt_debug_set_two_ray.argtypes = [C.c_void_p, C.c_int]
    _lib.check(lb.iqpt_debug_set_two_ray(pt._h, 1 if on else 0), "iqpt_debug_set_two_ray")


def run(preset, w, h, launches, depth=8, pixels=None, two_ray=True, overlap=True, frame=None):
    _, pk = scene_for(preset)
    cam = make_camera(w, h)
    pt = PathTracer(w, h, pixels=pixels, max_depth=depth)
    pt.set_split(_lib.SPLIT_OFF)
    pt.set_overlap(_lib.OVERLAP_AUTO if overlap else _lib.OVERLAP_OFF)
    set_two_ray(pt, two_ray)
    if frame is not None:
        lb = _lib.load()
        lb.iqpt_debug_set_frame.argtypes = [C.c_void_p, C.c_uint64]
        _lib.check(lb.iqpt_debug_set_frame(pt._h, frame), "iqpt_debug_set_frame")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    opts = []
    for s in launches:
        pt.render(s)
        opts.append(last_options(pt))
    pt.sync()
    lin, bgra = pt.read()
    out = (lin, bgra, pt.read_rng(), pt.rays())
    pt.close()
    return out, opts


def oracle_frame(preset, w, h, launches, depth=8, pixels=None, frame=None):
    _, pk = scene_for(preset)
    fr = oracle.OracleFrame(w, h, pixels=pixels, max_depth=depth)
    if frame is not None:
        fr.frame = frame
    cam = make_camera(w, h)
    for s in launches:
        fr.render(pk, cam, s)
    return fr


def same_as_oracle(out, fr):
    lin, bgra, rng, rays = out
    a, b = lin[:, :3], fr.lin[:, :3]
    both_nan = np.isnan(a) & np.isnan(b)
    assert np.all((a.view(np.uint32) == b.view(np.uint32)) | both_nan)
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(rng, fr.states)
    assert rays == int(fr.rays.sum())


def same(a, b):
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    assert np.array_equal(a[1], b[1])
    assert np.array_equal(a[2], b[2])
    assert a[3] == b[3]


@pytest.mark.parametrize("overlap", [True, False])
def test_sphere_crop_launches(require_gpu, overlap):
    """A crop through both spheres (secondary rays, 1- 2- and 3-slot samples), launches of 1, 2, 3 and 64
    samples: every launch takes the two-ray variant, the frame is the oracle's."""
    w, h = 1920, 1080
    ps = pixel_set(w, h, 720, 1200, 500, 1, 96)
    launches = [1, 2, 3, 64]
    out, opts = run("cornell", w, h, launches, pixels=ps, overlap=overlap)
    assert all(o & K_OPT_PIPE for o in opts), [hex(o) for o in opts]
    if overlap:
        assert any(o & K_OPT_OVERLAP for o in opts)
    same_as_oracle(out, oracle_frame("cornell", w, h, launches, pixels=ps))


@pytest.mark.parametrize("depth", [1, 2, 3, 16])
def test_depths(require_gpu, depth):
    """max_depth 1 (every sphere hit ends the path on its scatter, drawing), 2, 3 and 16 (the MAXD-16 variant)."""
    w, h = 1920, 1080
    ps = pixel_set(w, h, 760, 1160, 520, 1, 64)
    out, opts = run("cornell", w, h, [5, 7], depth=depth, pixels=ps)
    assert all(o & K_OPT_PIPE for o in opts)
    same_as_oracle(out, oracle_frame("cornell", w, h, [5, 7], depth=depth, pixels=ps))


def test_two_ray_equals_one_ray_full_share(require_gpu):
    """Rank 0's rows of a 3-way split of the C2 frame, two launches: the two-ray kernel equals the one-ray kernel
    bit for bit (accumulators, frame, RNG states, ray counts)."""
    w, h = 1920, 1080
    ps = pixel_set(w, h, 0, w, 0, 3, (h + 2) // 3)
    on, o1 = run("cornell", w, h, [64, 16], pixels=ps)
    off, o0 = run("cornell", w, h, [64, 16], pixels=ps, two_ray=False)
    assert all(o & K_OPT_PIPE for o in o1) and not any(o & K_OPT_PIPE for o in o0)
    same(on, off)


def test_other_presets(require_gpu):
    """The application scene (lamp sphere of triangles, Oren-Nayar ball) and the small C1 scene, ragged frames."""
    for preset, (w, h), depth in (("app_default", (317, 181), 5), ("c1_plumbing", (250, 250), 2)):
        out, opts = run(preset, w, h, [3, 4], depth=depth)
        assert all(o & K_OPT_PIPE for o in opts)
        same_as_oracle(out, oracle_frame(preset, w, h, [3, 4], depth=depth))


def test_large_frame_counter(require_gpu):
    """Frame counters beyond 2^32 (the running mean's large-n table values and thresholds)."""
    w, h = 1920, 1080
    ps = pixel_set(w, h, 800, 1000, 560, 1, 40)
    frame = (1 << 33) + 5
    out, opts = run("cornell", w, h, [6, 3], pixels=ps, frame=frame)
    assert all(o & K_OPT_PIPE for o in opts)
    same_as_oracle(out, oracle_frame("cornell", w, h, [6, 3], pixels=ps, frame=frame))
