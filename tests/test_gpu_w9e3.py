"""W9E3 (res/shaders/w9e3.wgsl; scenes.rs "W9 E3 Teapot"): the sun-lit
lambertian, the holdout plane shaded by an occlusion ray and a sun ray, the
transparent teapot at selection 3 (ior 1.5: total internal reflection, NaN
rays), and the back-face-culled triangle test with ETA-weighted normals, which
the kernel threads through both walks as a template flag.  HIP kernel vs the
CPU oracle; bar: bit-exact radiance and ids, equal ray counts."""
import numpy as np
import pytest

from conftest import model
from parity_util import TEAPOT_CAM, Scene
from test_gpu_parity import check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["BSP", "BVH"])
def teapot(request, rt, gpu):
    return Scene(rt, rt.Mesh.from_obj(model("teapot.obj")), request.param)


@pytest.mark.parametrize("sel", [0, 2, 3, 5, 6, 7])
def test_w9e3_selection(teapot, sel):
    region = (150, 120, 500, 260)
    g = teapot.render_gpu("W9E3", TEAPOT_CAM, 800, 450, region, 0, 2, selection1=sel)
    o = teapot.render_oracle("W9E3", TEAPOT_CAM, 800, 450, region, 0, 2, selection1=sel)
    check(g, o)


def test_w9e3_progressive_and_texture(rt, teapot):
    rng = np.random.default_rng(9)
    tex = rng.integers(0, 256, size=(31, 57, 4), dtype=np.uint8)
    teapot.ctx.set_environment_map(tex)
    try:
        teapot.oscene = teapot.oscene.__class__(teapot.om, teapot.obsp, teapot.obvh, teapot.env, env_tex=tex)
        a = teapot.render_gpu("W9E3", TEAPOT_CAM, 400, 225, (0, 0, 400, 225), 0, 2)
        b = teapot.render_gpu("W9E3", TEAPOT_CAM, 400, 225, (0, 0, 400, 225), 2, 2, accum_in=a[0])
        o = teapot.render_oracle("W9E3", TEAPOT_CAM, 400, 225, (0, 0, 400, 225), 2, 2, accum_in=a[0].copy())
        check(b, o)
    finally:
        teapot.ctx.set_environment_map(None)
        teapot.oscene = teapot.oscene.__class__(teapot.om, teapot.obsp, teapot.obvh, teapot.env)
