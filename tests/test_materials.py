"""Material table on the CPU: the scene builder's packet fields and the oracle's
semantics.

* A table that spells out the reference's own materials (emissive(white, 10) on every triangle,
  oren_nayar(0.5, sigma 1) on every sphere, path_tracer.cu:248-249) renders bit-identically to a
  packet without a table — the generalised ray_color reduces to the reference.
* Oren–Nayar roughness is clamped to [0, 1] like the constructor (material.h:25-29).
* Emissive spheres end the path on their first hit (one ray per path); an all-Oren–Nayar closed box
  traces exactly max_depth rays per path.
"""
import numpy as np
import pytest

import oracle
from iqpt import MAT_EMISSIVE, MAT_OREN_NAYAR, IqptError, Scene, make_camera


def cornell(materials=None):
    sc = Scene()
    sc.add_preset("cornell")
    if materials:
        for model, (kind, albedo, param) in materials.items():
            sc.set_model_material(model, sc.add_material(kind, albedo, param))
    return sc


def render(sc, w=48, h=32, spp=3, depth=8, seed=1984):
    pk = sc.build_packet()
    fr = oracle.OracleFrame(w, h, seed=seed, max_depth=depth)
    fr.render(pk, make_camera(w, h), spp, threads=4)
    return fr


def test_builder_fills_the_table_and_defaults():
    sc = Scene()
    sc.add_preset("cornell")
    assert sc.build_packet().materials is None or not bool(sc.build_packet().materials)
    k = sc.add_material(MAT_OREN_NAYAR, (0.7, 0.1, 0.1), 0.3)
    sc.set_model_material("left", k)
    pk = sc.build_packet()
    assert pk.num_materials == 3                      # the entry + the two reference defaults
    tri = [pk.tri_dc_material[i] for i in range(pk.num_drawcalls[0])]
    sph = [pk.sphere_dc_material[i] for i in range(pk.num_drawcalls[1])]
    assert sorted(set(tri)) == [0, 1] and tri.count(0) == 1     # "left" uses the table entry
    assert sph == [2, 2]
    assert pk.materials[1].type == MAT_EMISSIVE and pk.materials[1].param == 10.0
    assert pk.materials[2].type == MAT_OREN_NAYAR and list(pk.materials[2].albedo) == [0.5, 0.5, 0.5, 0.0]
    with pytest.raises(IqptError):
        sc.set_model_material("nope", 0)
    with pytest.raises(IqptError):
        sc.set_model_material("left", 9)
    with pytest.raises(IqptError):
        sc.add_material(7, (1, 1, 1), 1.0)


def test_explicit_reference_materials_equal_no_table():
    base = render(cornell())
    walls = {m: (MAT_EMISSIVE, (1.0, 1.0, 1.0, 1.0), 10.0) for m in ("back", "floor", "ceiling", "left", "right")}
    balls = {m: (MAT_OREN_NAYAR, (0.5, 0.5, 0.5, 0.0), 1.0) for m in ("sphere_big", "sphere_small")}
    tab = render(cornell({**walls, **balls}))
    assert np.array_equal(tab.lin.view(np.uint32), base.lin.view(np.uint32))
    assert np.array_equal(tab.states, base.states)
    assert np.array_equal(tab.rays, base.rays)


def test_roughness_is_clamped_like_the_constructor():
    a = render(cornell({"sphere_big": (MAT_OREN_NAYAR, (0.5, 0.5, 0.5, 0.0), 7.0)}))
    b = render(cornell({"sphere_big": (MAT_OREN_NAYAR, (0.5, 0.5, 0.5, 0.0), 1.0)}))
    assert np.array_equal(a.lin.view(np.uint32), b.lin.view(np.uint32))
    c = render(cornell({"sphere_big": (MAT_OREN_NAYAR, (0.5, 0.5, 0.5, 0.0), -3.0)}))
    d = render(cornell({"sphere_big": (MAT_OREN_NAYAR, (0.5, 0.5, 0.5, 0.0), 0.0)}))
    assert np.array_equal(c.lin.view(np.uint32), d.lin.view(np.uint32))


def test_emissive_spheres_end_paths_and_diffuse_walls_bounce():
    emissive_all = {m: (MAT_EMISSIVE, (0.2, 0.4, 0.8, 1.0), 3.0) for m in ("sphere_big", "sphere_small")}
    fr = render(cornell(emissive_all), spp=2)
    assert fr.rays.max() == 2                          # emissive everywhere: one ray per sample
    # closed Oren-Nayar shell: every path is cut at max_depth
    sc = Scene()
    sc.add_mesh_uv_sphere("shell", False, 24, 12, 0)   # triangle mesh around the camera
    sc.add_model("shell", "shell", 20.0, 0.0, 0.0)
    sc.set_model_material("shell", sc.add_material(MAT_OREN_NAYAR, (0.9, 0.9, 0.9, 0.0), 0.5))
    fr = render(sc, spp=2, depth=5)
    assert np.all(fr.rays == 2 * 5)


def test_colored_lit_box_is_not_the_reference_box():
    lit = Scene()
    lit.add_preset("cornell_lit")
    fr = render(lit, spp=4)
    ref = render(cornell(), spp=4)
    assert not np.array_equal(fr.lin, ref.lin)
    rgb = fr.lin[:, :3]
    assert np.isfinite(rgb).all()
    # the red and green walls tint their halves of the frame
    left, right = rgb.reshape(32, 48, 3)[:, :8].mean(axis=(0, 1)), rgb.reshape(32, 48, 3)[:, -8:].mean(axis=(0, 1))
    assert left[0] > left[1] and right[1] > right[0]
