"""iqpt — MI355X-native path tracer for IoniqRE's path-tracing hot path (Python bindings).

The product is native (libiqpt.so: HIP kernels for gfx950 + a C ABI, include/iqpt.h). This package
binds it with ctypes for the tests and the benchmark; it raises if the library is missing.
"""
from ._lib import (DEFAULT_MAX_DEPTH, DEFAULT_SEED, MAT_EMISSIVE, MAT_OREN_NAYAR, MESH_SPHERES,  # noqa: F401
                   MESH_TRIANGLES, IqptError, Material, load)
from .render import PathTracer, comm_unique_id, kernel_name, pixel_set, write_ppm  # noqa: F401
from .scene import CONFIGS, Config, Scene, config_scene, make_camera, packet_stats  # noqa: F401
