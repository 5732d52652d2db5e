"""kOptCamAxis on the GPU (an opt-in variant): the device builds of camera_ndc and camera_ray_axis give
the same bits (zero signs included) on random and adversarial NDC inputs, renders with pitch-only
cameras run the short transform and match the oracle bit for bit, other cameras keep the general
one, and the default selection does not use it."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare
from iqpt import PathTracer, Scene, _lib, make_camera
from test_camera_axis import cam_axis, general, mats, ndc_samples, pitch_camera

pytestmark = pytest.mark.gpu

K_OPT_CAM_AXIS = 1 << 14


def device_rays(cam, x, y):
    lb = _lib.load()
    lb.iqpt_debug_camera_rays.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_uint64, C.POINTER(C.c_float),
                                          C.POINTER(C.c_float)]
    lb.iqpt_debug_camera_rays.restype = C.c_int
    n = x.size
    ndc = np.ascontiguousarray(np.stack([x, y], axis=-1).astype(np.float32))
    gen = np.zeros((n, 6), np.float32)
    ax = np.zeros((n, 6), np.float32)
    fp = C.POINTER(C.c_float)
    r = lb.iqpt_debug_camera_rays(C.byref(cam), ndc.ctypes.data_as(fp), n, gen.ctypes.data_as(fp),
                                  ax.ctypes.data_as(fp))
    assert r in (0, 1), _lib.load().iqpt_last_error()
    return bool(r), gen, ax


def last_options(pt):
    lb = _lib.load()
    lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    o = C.c_int(0)
    _lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(o)), "iqpt_debug_last_options")
    return o.value


@pytest.mark.parametrize("which", ["reference", "pitch_up", "origin", "degenerate"])
def test_device_camera_transforms_bit_identical(require_gpu, which):
    if which == "reference":
        cam = make_camera(1920, 1080)
    elif which == "pitch_up":
        cam = pitch_camera(320, 200, 1.7, (0.0, -2.0, 4.0), fovh=60.0)
    elif which == "origin":
        cam = pitch_camera(320, 200, 0.0, (0.0, 0.0, 0.0))
    else:
        cam = make_camera(64, 48)
        cam.inv_view[0] = 0.0
    x, y = ndc_samples()
    ok, gen, ax = device_rays(cam, x, y)
    assert ok
    assert np.array_equal(gen.view(np.uint32), ax.view(np.uint32))
    # and the device's general transform is the host restatement's (the oracle's chain)
    P, V = mats(cam)
    k = cam_axis(cam)[1]
    host = general(P, V, k[4], k[5], x, y)
    assert np.array_equal(gen.view(np.uint32), host.view(np.uint32))


K_OPT_MATERIALS = 1 << 10


def render_both(cam, w, h, spp, depth=8, preset="cornell", axis=True):
    sc = Scene()
    sc.add_preset(preset)
    pk = sc.build_packet()
    pt = PathTracer(w, h, max_depth=depth)
    if axis:   # opt-in variant (the runtime drops the bit when the camera does not qualify)
        lb = _lib.load()
        lb.iqpt_debug_set_kernel_options.argtypes = [C.c_void_p, C.c_int]
        opt = lb.iqpt_debug_default_options() | K_OPT_CAM_AXIS | (K_OPT_MATERIALS if preset == "cornell_lit" else 0)
        _lib.check(lb.iqpt_debug_set_kernel_options(pt._h, opt), "iqpt_debug_set_kernel_options")
    pt.set_camera(cam)
    pt.upload_packet(pk)
    pt.render(spp)
    lin, bgra = pt.read()
    fr = oracle.OracleFrame(w, h, max_depth=depth)
    fr.render(pk, cam, spp)
    c = compare(lin, fr.lin)
    assert c["bitexact"] == c["npix"], c
    assert np.array_equal(bgra, fr.bgra)
    assert np.array_equal(pt.read_rng(), fr.states)
    assert pt.rays() == int(fr.rays.sum())
    opt = last_options(pt)
    pt.close()
    return opt


@pytest.mark.parametrize("pitch,pos", [(-0.5, (0.0, 0.5, -3.0)), (0.2, (0.0, 0.3, -2.5)), (0.0, (0.0, 0.5, -2.0))])
def test_pitch_camera_renders_match_oracle(require_gpu, pitch, pos):
    opt = render_both(pitch_camera(96, 64, pitch, pos), 96, 64, 4)
    assert opt & K_OPT_CAM_AXIS


def test_lit_scene_with_material_table_short_camera(require_gpu):
    opt = render_both(make_camera(96, 64), 96, 64, 3, preset="cornell_lit")
    assert opt & K_OPT_CAM_AXIS


def test_yawed_camera_keeps_general_transform(require_gpu):
    cam = make_camera(96, 64, position=(0.3, 0.5, -3.0, 0.0), forward=(-0.2, -0.5, 3.0, 0.0))
    opt = render_both(cam, 96, 64, 4)
    assert not opt & K_OPT_CAM_AXIS


def test_default_selection_takes_short_camera(require_gpu):
    """The runtime's own choice: a pitch-only camera gets the short transform (same bits as the oracle)."""
    opt = render_both(make_camera(96, 64), 96, 64, 2, axis=False)
    assert opt & K_OPT_CAM_AXIS


def test_default_selection_yawed_camera_general(require_gpu):
    """The runtime's own choice for a yawed camera: the general transform."""
    cam = make_camera(96, 64, position=(0.3, 0.5, -3.0, 0.0), forward=(-0.2, -0.5, 3.0, 0.0))
    opt = render_both(cam, 96, 64, 3, axis=False)
    assert not opt & K_OPT_CAM_AXIS
