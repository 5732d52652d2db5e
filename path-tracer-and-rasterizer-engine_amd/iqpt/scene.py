"""Scene, camera and benchmark configurations over the native scene builder (iqpt_scene_*).

Mirrors IoniqRE's scene/mesh/model/camera host classes (scene.h, mesh.h, model.h, camera.h);
the arithmetic runs in libiqpt.so (csrc/iq_scene.cpp).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import Camera, PacketDesc, check, farr


class Scene:
    """Name-keyed meshes and models; ``build_packet()`` returns a ``PacketDesc`` (scene.cu:104-181)."""

    def __init__(self):
        self._lib = _lib.load()
        h = C.c_void_p()
        check(self._lib.iqpt_scene_create(C.byref(h)), "iqpt_scene_create")
        self._h = h
        self._keep = []

    def close(self):
        if getattr(self, "_h", None):
            self._lib.iqpt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # procedural meshes (mesh.cu)
    def add_mesh_tri(self, name: str):
        check(self._lib.iqpt_scene_add_mesh_tri(self._h, name.encode()), "add_mesh_tri")

    def add_mesh_quad(self, name: str):
        check(self._lib.iqpt_scene_add_mesh_quad(self._h, name.encode()), "add_mesh_quad")

    def add_mesh_reg_polygon(self, name: str, vertices: int):
        check(self._lib.iqpt_scene_add_mesh_reg_polygon(self._h, name.encode(), vertices), "add_mesh_reg_polygon")

    def add_mesh_cube(self, name: str):
        check(self._lib.iqpt_scene_add_mesh_cube(self._h, name.encode()), "add_mesh_cube")

    def add_mesh_uv_sphere(self, name: str, flat: bool = False, segments: int = 32, rings: int = 16,
                           mesh_type: int = _lib.MESH_SPHERES):
        check(self._lib.iqpt_scene_add_mesh_uv_sphere(self._h, name.encode(), int(flat), segments, rings,
                                                      mesh_type), "add_mesh_uv_sphere")

    def add_mesh(self, name: str, vertices: np.ndarray, indices: np.ndarray, mesh_type: int = _lib.MESH_TRIANGLES):
        v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 6)
        i = np.ascontiguousarray(indices, dtype=np.uint32).reshape(-1)
        check(self._lib.iqpt_scene_add_mesh(self._h, name.encode(), mesh_type,
                                            v.ctypes.data_as(C.POINTER(_lib.Vertex)), v.shape[0],
                                            i.ctypes.data_as(C.POINTER(C.c_uint32)), i.shape[0]), "add_mesh")

    def add_model(self, name: str, mesh_name: str, scale=1.0, rotation=0.0, translation=0.0):
        def v4(x):
            if np.isscalar(x):
                return [float(x)] * 4
            x = list(x)
            return x + [0.0] * (4 - len(x))
        check(self._lib.iqpt_scene_add_model(self._h, name.encode(), mesh_name.encode(), farr(v4(scale), 4),
                                             farr(v4(rotation), 4), farr(v4(translation), 4)), "add_model")

    def add_preset(self, preset: str):
        check(self._lib.iqpt_scene_add_preset(self._h, preset.encode()), "add_preset")

    def add_material(self, kind: int, albedo, param: float) -> int:
        """Material table entry (iqpt.h): kind MAT_EMISSIVE (param = strength) or MAT_OREN_NAYAR
        (param = roughness sigma). Returns its index."""
        m = _lib.Material()
        m.type = kind
        a = list(albedo) + [0.0] * (4 - len(albedo))
        for k in range(4):
            m.albedo[k] = a[k]
        m.param = param
        idx = C.c_uint32()
        check(self._lib.iqpt_scene_add_material(self._h, C.byref(m), C.byref(idx)), "add_material")
        return idx.value

    def set_model_material(self, model: str, material: int):
        check(self._lib.iqpt_scene_set_model_material(self._h, model.encode(), material), "set_model_material")

    def num_meshes(self) -> int:
        n = C.c_uint32()
        check(self._lib.iqpt_scene_num_meshes(self._h, C.byref(n)), "num_meshes")
        return n.value

    def build_packet(self) -> PacketDesc:
        pk = PacketDesc()
        check(self._lib.iqpt_scene_build_packet(self._h, C.byref(pk)), "build_packet")
        return pk


def make_camera(width: int, height: int, fovh: float = 45.0, znear: float = 0.01, zfar: float = 100.0,
                position=None, forward=None) -> Camera:
    """camera::camera (camera.cu:5-18) with the reference defaults (camera.h:11, 26-27)."""
    lib = _lib.load()
    cam = Camera()
    pos = farr(position, 4) if position is not None else None
    fwd = farr(forward, 4) if forward is not None else None
    check(lib.iqpt_camera_init(C.byref(cam), width, height, fovh, znear, zfar, pos, fwd), "iqpt_camera_init")
    return cam


def packet_stats(pk: PacketDesc) -> dict:
    """T (triangle instances, Σ over drawcalls of num_indices/3) and S (sphere drawcalls)."""
    t = 0
    for i in range(pk.num_drawcalls[_lib.MESH_TRIANGLES]):
        m = pk.tri_meshes[pk.tri_mesh_dcs[i].mesh_id]
        t += m.num_indices // 3
    return {"triangles": t, "spheres": int(pk.num_drawcalls[_lib.MESH_SPHERES])}


@dataclass(frozen=True)
class Config:
    """One of BASELINE.json's configs."""
    name: str
    preset: str
    width: int
    height: int
    spp: int
    max_depth: int
    description: str

    @property
    def flops_per_ray(self) -> int:
        """F_ray = 52 T + 19 S: MT (shape.cu:65-92) and sphere (shape.cu:16-25) FLOPs."""
        return 52 * TRIANGLES[self.preset] + 19 * SPHERES[self.preset]


TRIANGLES = {"c1_plumbing": 224, "cornell": 10, "mesh10k": 10_000, "mixed": 50_000, "app_default": 12}
SPHERES = {"c1_plumbing": 1, "cornell": 2, "mesh10k": 0, "mixed": 1000, "app_default": 2}

CONFIGS = {
    "c1": Config("c1", "c1_plumbing", 256, 256, 1, 2, "1 emissive + 1 diffuse sphere, 256x256, 1 spp, 2 bounces"),
    "c2": Config("c2", "cornell", 1920, 1080, 64, 8, "Cornell box (5 quads + 2 spheres), 1920x1080, 64 spp, 8 bounces"),
    "c3": Config("c3", "cornell", 1920, 1080, 64, 8, "C2 row-tiled across GPUs, RCCL gather"),
    "c4": Config("c4", "mesh10k", 1920, 1080, 256, 8, "10k-triangle mesh, 1920x1080, 256 spp"),
    "c5": Config("c5", "mixed", 3840, 2160, 1024, 8, "1k spheres + 50k triangles, 3840x2160, 1024 spp"),
    "app": Config("app", "app_default", 1280, 720, 1, 5, "IoniqRE application default scene (application.cu:25-34)"),
}


def config_scene(cfg: Config) -> tuple[Scene, PacketDesc, Camera]:
    scene = Scene()
    scene.add_preset(cfg.preset)
    pk = scene.build_packet()
    cam = make_camera(cfg.width, cfg.height)
    return scene, pk, cam
