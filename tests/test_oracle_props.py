"""Size-independent properties of the reference semantics, checked on the oracle (CPU)."""
import ctypes as C

import numpy as np
import pytest

import oracle
from helpers import compare, oracle_render, scene_for
from iqpt import Scene, make_camera


def test_thread_count_does_not_change_results():
    sc, pk = scene_for("app_default")
    cam = make_camera(96, 54)
    a = oracle.OracleFrame(96, 54, max_depth=5)
    b = oracle.OracleFrame(96, 54, max_depth=5)
    a.render(pk, cam, 3, threads=1)
    b.render(pk, cam, 3, threads=8)
    assert np.array_equal(a.lin.view(np.uint32), b.lin.view(np.uint32))
    assert np.array_equal(a.states, b.states)


def test_crop_equals_the_same_pixels_of_the_full_frame():
    full = oracle_render("cornell", 160, 90, 4, 8)
    ps = oracle.pixel_set(160, 90, 40, 120, 20, 3, 15)
    crop = oracle_render("cornell", 160, 90, 4, 8, pixels=ps)
    rows = 20 + 3 * np.arange(15)
    expect = full.lin.reshape(90, 160, 4)[rows][:, 40:120].reshape(-1, 4)
    assert compare(crop.lin, expect)["bitexact"] == crop.npix


def test_launch_split_is_equivalent():
    a = oracle_render("app_default", 64, 36, 0, 5, launches=[1] * 5)
    b = oracle_render("app_default", 64, 36, 0, 5, launches=[2, 3])
    assert np.array_equal(a.lin.view(np.uint32), b.lin.view(np.uint32))
    assert np.array_equal(a.states, b.states)


def test_sky_only_scene_is_the_gradient_of_the_camera_ray():
    """Empty packet: every path misses; lin after frame 1 = clamp(sky(dir)) (path_tracer.cu:307-316)."""
    sc = Scene()
    pk = sc.build_packet()
    w, h = 32, 16
    cam = make_camera(w, h)
    fr = oracle.OracleFrame(w, h, max_depth=8)
    states0 = fr.states.copy()
    fr.render(pk, cam, 1)
    lib = oracle.load()
    f32 = np.float32
    for pix in range(fr.npix):
        st = states0[pix].copy()
        o, d = np.zeros(4, np.float32), np.zeros(4, np.float32)
        lib.iqo_get_ray(C.byref(cam), pix % w, pix // w, st.ctypes.data_as(C.POINTER(C.c_uint32)),
                        o.ctypes.data_as(C.POINTER(C.c_float)), d.ctypes.data_as(C.POINTER(C.c_float)))
        a = (d[1] + f32(1)) * f32(0.5)
        sky = [(f32(1) - a) + a * f32(0.5), (f32(1) - a) + a * f32(0.7), (f32(1) - a) + a * f32(1.0)]
        sky = [min(max(s, f32(0)), f32(1)) for s in sky]
        assert [fr.lin[pix, k] for k in range(3)] == sky
        assert np.array_equal(st, fr.states[pix])
    assert int(fr.rays.sum()) == fr.npix


def test_emissive_only_scene_traces_one_ray_per_path():
    """C4 semantics: every triangle is emissive (path_tracer.cu:278), so each path is 1 ray."""
    ps = oracle.pixel_set(1920, 1080, 940, 980, 500, 1, 4)
    fr = oracle_render("mesh10k", 1920, 1080, 2, 8, pixels=ps)
    assert int(fr.rays.sum()) == fr.npix * 2


def test_rays_per_path_of_the_app_scene_matches_the_survey_probe():
    """the reference's own source, compiled verbatim as a host loop, traced 1.61
    rays per path on the application's default scene (max_depth 5)."""
    fr = oracle_render("app_default", 320, 180, 4, 5)
    assert abs(fr.rays.sum() / (320 * 180 * 4) - 1.61) < 0.02


def test_max_depth_paths_end_on_a_scatter_record():
    """Camera inside a huge Oren–Nayar sphere: no path ever escapes or hits a light, so every path
    traces exactly max_depth rays and its colour is the product of scatter records (biased, :252)."""
    sc = Scene()
    sc.add_mesh_uv_sphere("sphere")
    sc.add_model("shell", "sphere", scale=50.0)
    pk = sc.build_packet()
    cam = make_camera(16, 8)
    for depth in (1, 2, 5):
        fr = oracle.OracleFrame(16, 8, max_depth=depth)
        fr.render(pk, cam, 2)
        assert int(fr.rays.sum()) == 16 * 8 * 2 * depth
        assert np.all(fr.lin[:, 0] == fr.lin[:, 1]) and np.all(fr.lin[:, 1] == fr.lin[:, 2])
        assert np.all(fr.lin[:, :3] > 0) and np.all(fr.lin[:, :3] <= 1)


def test_reset_restarts_the_mean_and_keeps_nan_sticky():
    sc, pk = scene_for("app_default")
    cam = make_camera(32, 18)
    fr = oracle.OracleFrame(32, 18, max_depth=5)
    fr.render(pk, cam, 3)
    fr.lin[0, 0] = np.nan                       # a NaN in the accumulator survives (NaN * 0 = NaN)
    fr.reset()
    fr.render(pk, cam, 1)
    assert np.isnan(fr.lin[0, 0])
    ref = oracle.OracleFrame(32, 18, max_depth=5)
    ref.states[:] = 0
    # frame 1 after reset: lin = c/1 + lin * 0 — equal to a fresh 1-spp render from the same RNG
    st_after3 = oracle_render("app_default", 32, 18, 3, 5).states
    ref.states[:] = st_after3
    ref.render(pk, cam, 1)
    same = np.all(fr.lin[1:, :3].view(np.uint32) == ref.lin[1:, :3].view(np.uint32), axis=1)
    assert same.all()


def test_bgra8_is_truncated_sqrt_of_the_accumulator():
    fr = oracle_render("app_default", 48, 27, 2, 5)
    f = np.float32(255) * np.sqrt(fr.lin[:, :3].astype(np.float32))
    q = np.clip(np.floor(f), 0, 255).astype(np.uint8)
    assert np.array_equal(fr.bgra[:, 2], q[:, 0]) and np.array_equal(fr.bgra[:, 1], q[:, 1])
    assert np.array_equal(fr.bgra[:, 0], q[:, 2]) and np.all(fr.bgra[:, 3] == 255)
