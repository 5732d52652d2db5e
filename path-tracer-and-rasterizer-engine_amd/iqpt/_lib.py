"""ctypes mirror of include/iqpt.h and the loader of the in-tree libiqpt.so.

The product path is native: this module only binds the C ABI. If the library is missing or does
not load, importing the render API raises — there is no Python or CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "libiqpt.so"

IQPT_OK = 0
STATUS_NAMES = {
    0: "IQPT_OK", 1: "IQPT_ERR_INVALID_ARG", 2: "IQPT_ERR_HIP", 3: "IQPT_ERR_OUT_OF_MEMORY",
    4: "IQPT_ERR_NO_DEVICE", 5: "IQPT_ERR_NOT_READY", 6: "IQPT_ERR_UNSUPPORTED",
}
MESH_TRIANGLES = 0
MESH_SPHERES = 1
DEFAULT_SEED = 1984
DEFAULT_MAX_DEPTH = 5
SPLIT_AUTO, SPLIT_OFF, SPLIT_ON, SPLIT_CHAIN, SPLIT_FAN, SPLIT_SPEC = -1, 0, 1, 2, 3, 4   # IQPT_SPLIT_* (iqpt_set_split;
# CHAIN and FAN are refused with IQPT_ERR_UNSUPPORTED since round 6)
OVERLAP_OFF, OVERLAP_AUTO = 0, 1               # IQPT_OVERLAP_* (iqpt_set_overlap)
COMM_ID_BYTES = 128                            # IQPT_COMM_ID_BYTES (iqpt_comm_unique_id)
GATHER_ACCUM = 1                               # IQPT_GATHER_ACCUM / IQPT_GATHER_FRAME (iqpt_gather_read_select)
GATHER_FRAME = 2


class IqptError(RuntimeError):
    """A non-zero iqpt_status, with the library's iqpt_last_error() detail."""

    def __init__(self, status: int, detail: str, call: str):
        super().__init__(f"{call} -> {STATUS_NAMES.get(status, status)}: {detail}")
        self.status = status
        self.detail = detail


class Vertex(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("normal", C.c_float * 3)]


class TriMesh(C.Structure):
    _fields_ = [("vertices", C.POINTER(Vertex)), ("indices", C.POINTER(C.c_uint32)),
                ("num_indices", C.c_uint32), ("num_vertices", C.c_uint32)]


class TriMeshDrawcall(C.Structure):
    _fields_ = [("transform", C.c_float * 16), ("mesh_id", C.c_uint32)]


class SphereDrawcall(C.Structure):
    _fields_ = [("center", C.c_float * 4), ("radius", C.c_float)]


class Material(C.Structure):
    """iqpt_material (include/iqpt.h): IQPT_MAT_EMISSIVE (param = strength) or IQPT_MAT_OREN_NAYAR
    (param = roughness sigma)."""
    _fields_ = [("type", C.c_uint32), ("albedo", C.c_float * 4), ("param", C.c_float)]


MAT_EMISSIVE = 0
MAT_OREN_NAYAR = 1


class PacketDesc(C.Structure):
    _fields_ = [("num_drawcalls", C.c_uint32 * 2), ("num_tri_meshes", C.c_uint32),
                ("tri_meshes", C.POINTER(TriMesh)), ("tri_mesh_dcs", C.POINTER(TriMeshDrawcall)),
                ("sphere_dcs", C.POINTER(SphereDrawcall)),
                ("materials", C.POINTER(Material)), ("num_materials", C.c_uint32),
                ("tri_dc_material", C.POINTER(C.c_uint32)), ("sphere_dc_material", C.POINTER(C.c_uint32))]


class Camera(C.Structure):
    _fields_ = [("width", C.c_uint16), ("height", C.c_uint16), ("fovh", C.c_float),
                ("position", C.c_float * 4), ("forward", C.c_float * 4),
                ("view", C.c_float * 16), ("projection", C.c_float * 16),
                ("inv_view", C.c_float * 16), ("inv_proj", C.c_float * 16)]


class PixelSet(C.Structure):
    _fields_ = [("x0", C.c_uint32), ("x1", C.c_uint32), ("y0", C.c_uint32),
                ("ystep", C.c_uint32), ("nrows", C.c_uint32)]


# (name, restype, argtypes) of every entry point declared in include/iqpt.h
_P = C.c_void_p
_FP = C.POINTER(C.c_float)
SIGNATURES = [
    ("iqpt_camera_init", C.c_int, [C.POINTER(Camera), C.c_uint16, C.c_uint16, C.c_float, C.c_float, C.c_float, _FP, _FP]),
    ("iqpt_create", C.c_int, [C.c_int, C.c_uint32, C.c_uint32, C.POINTER(PixelSet), C.c_uint64, C.c_int, C.POINTER(_P)]),
    ("iqpt_destroy", C.c_int, [_P]),
    ("iqpt_set_camera", C.c_int, [_P, C.POINTER(Camera)]),
    ("iqpt_upload_packet", C.c_int, [_P, C.POINTER(PacketDesc)]),
    ("iqpt_render", C.c_int, [_P, C.c_uint32]),
    ("iqpt_sync", C.c_int, [_P]),
    ("iqpt_reset", C.c_int, [_P]),
    ("iqpt_read", C.c_int, [_P, _FP, C.POINTER(C.c_uint8)]),
    ("iqpt_read_rng", C.c_int, [_P, C.POINTER(C.c_uint32)]),
    ("iqpt_copy_accum_device", C.c_int, [_P, _P, C.c_size_t]),
    ("iqpt_copy_frame_device", C.c_int, [_P, _P, C.c_size_t]),
    ("iqpt_copy_frame_device_async", C.c_int, [_P, _P, C.c_size_t]),
    ("iqpt_stream", C.c_int, [_P, C.POINTER(C.c_void_p)]),
    ("iqpt_frame_stream", C.c_int, [_P, C.POINTER(C.c_void_p)]),
    ("iqpt_set_split", C.c_int, [_P, C.c_int]),
    ("iqpt_set_overlap", C.c_int, [_P, C.c_int]),
    ("iqpt_kernel_span", C.c_int, [_P, C.POINTER(C.c_double)]),
    ("iqpt_prepare", C.c_int, [_P]),
    ("iqpt_num_pixels", C.c_int, [_P, C.POINTER(C.c_uint64)]),
    ("iqpt_frame_count", C.c_int, [_P, C.POINTER(C.c_uint64)]),
    ("iqpt_rays_traced", C.c_int, [_P, C.POINTER(C.c_uint64)]),
    ("iqpt_kernel_time", C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    ("iqpt_kernel_name", C.c_char_p, []),
    ("iqpt_checkpoint_save", C.c_int, [_P, C.c_char_p]),
    ("iqpt_checkpoint_load", C.c_int, [_P, C.c_char_p]),
    ("iqpt_write_ppm", C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8)]),
    ("iqpt_error_string", C.c_char_p, [C.c_int]),
    ("iqpt_last_error", C.c_char_p, []),
    ("iqpt_abi_version", C.c_int, []),
    ("iqpt_comm_unique_id", C.c_int, [_P, C.c_size_t]),
    ("iqpt_comm_init", C.c_int, [_P, C.c_int, C.c_int, _P, C.c_size_t]),
    ("iqpt_gather_frame_async", C.c_int, [_P, C.c_int, _P, C.c_size_t]),
    ("iqpt_gather_accum", C.c_int, [_P, C.c_int, _P, C.c_size_t]),
    ("iqpt_gather_read", C.c_int, [_P, C.c_int, _FP, C.POINTER(C.c_uint8)]),
    ("iqpt_gather_read_select", C.c_int, [_P, C.c_int, C.c_int, _FP, C.POINTER(C.c_uint8)]),
    ("iqpt_comm_stream", C.c_int, [_P, C.POINTER(C.c_void_p)]),
    ("iqpt_comm_time", C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    ("iqpt_scene_create", C.c_int, [C.POINTER(_P)]),
    ("iqpt_scene_destroy", C.c_int, [_P]),
    ("iqpt_scene_add_mesh_tri", C.c_int, [_P, C.c_char_p]),
    ("iqpt_scene_add_mesh_quad", C.c_int, [_P, C.c_char_p]),
    ("iqpt_scene_add_mesh_reg_polygon", C.c_int, [_P, C.c_char_p, C.c_uint32]),
    ("iqpt_scene_add_mesh_cube", C.c_int, [_P, C.c_char_p]),
    ("iqpt_scene_add_mesh_uv_sphere", C.c_int, [_P, C.c_char_p, C.c_int, C.c_uint32, C.c_uint32, C.c_int]),
    ("iqpt_scene_add_mesh", C.c_int, [_P, C.c_char_p, C.c_int, C.POINTER(Vertex), C.c_uint32, C.POINTER(C.c_uint32), C.c_uint32]),
    ("iqpt_scene_add_model", C.c_int, [_P, C.c_char_p, C.c_char_p, _FP, _FP, _FP]),
    ("iqpt_scene_num_meshes", C.c_int, [_P, C.POINTER(C.c_uint32)]),
    ("iqpt_scene_add_preset", C.c_int, [_P, C.c_char_p]),
    ("iqpt_scene_add_material", C.c_int, [_P, C.POINTER(Material), C.POINTER(C.c_uint32)]),
    ("iqpt_scene_set_model_material", C.c_int, [_P, C.c_char_p, C.c_uint32]),
    ("iqpt_scene_build_packet", C.c_int, [_P, C.POINTER(PacketDesc)]),
]

_lib = None


ABI_VERSION = 6      # IQPT_ABI_VERSION of include/iqpt.h these bindings mirror
LOADED_ABI = None    # the ABI of the library load() bound (an A/B library may be older; bench.py reports it)


def load() -> C.CDLL:
    """Load libiqpt.so from the package directory (raises if it is absent: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() "
                          "(the HIP extension is required; there is no CPU fallback)")
    global LOADED_ABI
    lib = C.CDLL(str(LIB_PATH))
    # an A/B library of an earlier round (bench.py --lib, another path) may lack the newest entry points: those
    # are left unbound there; the package's own library must export every one. A library of a newer ABI than
    # these bindings is refused whatever its path (its signatures may differ from the ones bound here).
    own = LIB_PATH.resolve() == (_PKG / "libiqpt.so").resolve()
    abi = lib.iqpt_abi_version() if getattr(lib, "iqpt_abi_version", None) is not None else None
    if abi is not None and abi > ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI {abi}, newer than these bindings' {ABI_VERSION}")
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name, None)
        if fn is None:
            if own:
                raise ImportError(f"{LIB_PATH} does not export {name}: rebuild with __graft_entry__.build()")
            continue
        fn.restype = res
        fn.argtypes = args
    if own and abi != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI {abi}, the bindings expect {ABI_VERSION}: "
                          "rebuild with __graft_entry__.build()")
    LOADED_ABI = abi
    _lib = lib
    return lib


def check(status: int, call: str) -> None:
    if status != IQPT_OK:
        lib = load()
        detail = lib.iqpt_last_error().decode(errors="replace")
        raise IqptError(status, detail, call)


def farr(values, n: int):
    arr = (C.c_float * n)(*[float(v) for v in values])
    return arr
