# r06 run 28: pixel-mask tests with a 3-way row share (every third row)
mkdir -p gpurun_out
O=gpurun_out
R=r06_28
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pixel_masks.py -m gpu -v --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
grep -c PASSED $O/${R}_tests.log; tail -1 $O/${R}_tests.log
timeout -k 10 120 python3 - <<'PY'
import sys, ctypes as C
sys.path.insert(0, "path-tracer-and-rasterizer-engine_amd")
from iqpt import PathTracer, Scene, _lib, make_camera, pixel_set
sc = Scene(); sc.add_preset("mesh10k"); pk = sc.build_packet()
pt = PathTracer(1920, 1080, pixels=pixel_set(1920, 1080, 0, 1920, 500, 3, 16), max_depth=8)
pt.set_camera(make_camera(1920, 1080)); pt.upload_packet(pk); pt.render(2); pt.sync()
lb = _lib.load(); lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
o = C.c_int(0); _lib.check(lb.iqpt_debug_last_options(pt._h, C.byref(o)), "last")
print("ystep 3 band: iqpt_anyhit_kernel", bool(o.value & (1 << 29)))
PY
