"""The HIP frame against the glibc-flavour oracle (flavour A: glibc libm, contraction off) on a C2
crop and the application scene: RMSE < 1e-5 (north_star), with the bit-exact fraction reported. The
HIP frame equals flavour B bit for bit (tests/test_gpu_parity.py); this pins the libm substitution
at frame level."""
import pytest

from helpers import compare, gpu_render, oracle_render, pixel_set

pytestmark = pytest.mark.gpu
RMSE_TOL = 1e-5


@pytest.mark.parametrize("preset,w,h,spp,depth,crop", [
    ("cornell", 1920, 1080, 64, 8, (880, 1000, 470, 1, 48)),
    ("app_default", 320, 180, 64, 5, None),
])
def test_hip_vs_glibc_flavour(require_gpu, preset, w, h, spp, depth, crop):
    ps = pixel_set(w, h, *crop) if crop else None
    pt, lin, _ = gpu_render(preset, w, h, spp, depth, pixels=ps)
    fa = oracle_render(preset, w, h, spp, depth, pixels=ps, glibc=True)
    c = compare(lin, fa.lin)
    print(f"{preset}: RMSE {c['rmse']:.3g}, bit-exact {c['bitexact']}/{c['npix']}")
    assert c["rmse"] < RMSE_TOL, c
    assert c["bitexact"] > 0.5 * c["npix"], c
