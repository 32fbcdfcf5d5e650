"""The BSP walk's plane divisions in a scene whose planes leave rt_div_by_recip's
exact range (rt_kernels.hip bsp_decide's chk; rt_bsp_build.hip k_plane_range): the
bunny stand-in plus one degenerate triangle at (2^101, 2^101, 2^101), so the root
splits at 2^100 > 2^99 and the scene's flag keeps every decision's range check.  The
W9E1 frame (k_path) equals the oracle's bit for bit, as does the same frame without
the far triangle (the unchecked divisions)."""
import numpy as np
import pytest

from parity_util import BUNNY_CAM, Scene, compare

pytestmark = pytest.mark.gpu

W, H, SPP = 256, 144, 4
ENV = (0.8, 0.9, 1.0)


def _frame(rt, mesh):
    s = Scene(rt, mesh, "BSP", env=ENV)
    try:
        g = s.render_gpu("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 0, SPP)
        o = s.render_oracle("W9E1", BUNNY_CAM, W, H, (0, 0, W, H), 0, SPP)
    finally:
        s.ctx.close()
    return g, o


@pytest.mark.parametrize("far", [False, True])
def test_w9e1_frame_with_and_without_out_of_range_planes_equals_oracle(rt, gpu, far):
    base = rt.Mesh.synth_bunny()
    mesh = base
    if far:
        V, N, I, M, L = base.arrays()
        n = V.shape[0]
        p = np.float32(2.0 ** 101)
        V2 = np.concatenate([V, np.array([[p, p, p, 1.0]] * 3, np.float32)])
        N2 = np.concatenate([N, np.array([[0.0, 0.0, 1.0, 0.0]] * 3, np.float32)])
        I2 = np.concatenate([I, np.array([[n, n + 1, n + 2, 0]], np.uint32)])
        mesh = rt.Mesh.from_arrays(V2, I2, N2, M)
        tree, planes, ids, aabb, D = mesh.bsp_tree().arrays()
        leaf = (np.asarray(tree).reshape(-1, 4)[:, 0] & 3) == 3
        assert (np.abs(np.asarray(planes)[~leaf]) > 2.0 ** 99).any()   # the flag's condition holds
    g, o = _frame(rt, mesh)
    linf, bits, idm = compare(g, o)
    hit = float((g[1] != 0xFFFFFFFF).mean())
    print(f"far={far}: {hit:.3f} of the pixels hit, L-inf {linf}, {bits} words and {idm} ids differ")
    assert hit > 0.1
    assert bits == 0 and idm == 0
