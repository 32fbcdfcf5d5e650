"""GPU side of the reference-JS pin (tests/test_js_walk.py): the reference's own
BSP arrays (build_bsp_tree of js/bsp_tree/modules/BspTree_interleaved.js, equal to
the oracle's f64 build by SHA-256) uploaded through rt_upload_bsp, rendered by the
W6E1/PROJECT primary-ray kernel (root-AABB clip + BSP walk + triangle test) at
64x64: every pixel's primary-hit triangle id equals the id the reference's
intersect_min_max + intersect_bsp_array produced under node for the same camera
ray -- except the listed edge rays, where the f32 test rejects an exactly-on-edge
hit that the f64 JS accepts; there the kernel must equal the f32 oracle."""
import numpy as np
import pytest

from conftest import model
from parity_util import compare
from test_js_walk import EXCEPTIONS, SCENES, load_fixture

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", SCENES)
def test_primary_ids_match_reference_js_walk(rt, oracle, name):
    meta, z = load_fixture(name)
    cam = tuple(tuple(c) if isinstance(c, list) else c for c in meta["camera"])
    R = meta["res"]
    m = oracle.load_obj(model(f"{name}.obj"))
    b = oracle.build_bsp(m, 20, 4, js64=True)
    ctx = rt.Context(0)
    try:
        ctx.upload_mesh_arrays(m.pos, m.nrm, m.idx, m.mats, m.lights)
        ctx.upload_bsp_arrays(b.aabb, b.tree, b.planes, b.ids, b.max_depth)
        ctx.set_uniforms(rt.make_uniform(*cam, R, R, selection1=0))
        acc = ctx.alloc(R * R * 16)
        ids = ctx.alloc(R * R * 4)
        acc.zero()
        cnt = ctx.render("PROJECT", "BSP", (0, 0, R, R), 0, 1, acc.ptr, ids.ptr, counts=True)
        g = (acc.to_numpy(np.float32, (R, R, 4)), ids.to_numpy(np.uint32, (R, R)), cnt)
    finally:
        ctx.close()
    # the kernel == the f32 oracle on the same (reference-built) tree, bit for bit
    o = oracle.render(oracle.SceneRef(m, b), oracle.make_uniform(*cam, R, R), "PROJECT", "BSP", (0, 0, R, R), 0, 1)
    linf, bits, idm = compare(g, o)
    assert idm == 0 and bits == 0, (idm, bits, linf)
    # ... and == the reference's own walk, ray for ray
    gi = g[1].reshape(-1).astype(np.int64)
    js = np.where(z["status"][:R * R] == 1, z["tri"][:R * R], 0xFFFFFFFF)
    differ = set(np.nonzero(gi != js)[0].tolist())
    listed = {i for i, c in EXCEPTIONS[name].items() if i < R * R and c in ("edge", "tie")}
    assert differ == listed, (sorted(differ), sorted(listed))
    assert (gi != 0xFFFFFFFF).sum() > 500
