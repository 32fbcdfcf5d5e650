"""GPU parity of the BVH walk's stack edge cases (bvh.wgsl:130-191) on
hand-made node arrays uploaded through rt_upload_bvh, against the oracle on
the same arrays:
  * the 50-entry stack with WGSL index clamping (pushes past entry 49 overwrite
    slot 49, pops read it back),
  * the 1000-pop cap (a truncated walk keeps the hits found so far),
  * runs of missed boxes, which the device handles two pops per trip.
The reference's HLBVH never gets deep enough for the first two, but the C ABI
takes any node array, so the walk must follow the shader there too."""
import numpy as np
import pytest

import oracle_ffi as O
from conftest import model
from parity_util import TEAPOT_CAM, Scene, compare

pytestmark = pytest.mark.gpu

FAR = ((1.0e6, 1.0e6, 1.0e6), (1.0e6 + 1.0, 1.0e6 + 1.0, 1.0e6 + 1.0))


def _node(box, offset, nprims):
    f = np.array(list(box[0]) + [0.0] + list(box[1]) + [0.0], dtype=np.float32).view(np.uint32)
    f[3], f[7] = offset, nprims
    return f


def chain_bvh(ntris, depth, shape, seed, p_leaf_hit=0.6, interior_miss_at=None, scene_box=None):
    """shape "A": interior k's left child is a leaf, its right child the next
    interior (the stack grows by one per level); shape "B": the left child is
    the next interior and the right child a leaf (popped first, so a missed
    leaf is followed by an interior pop)."""
    rng = np.random.default_rng(seed)
    hit_box = scene_box
    ids = []

    nleaves = depth + 1
    blk = max(1, 3 * ntris // nleaves)   # each triangle sits in about three leaves

    def leaf(force_hit=False):
        n = ntris if force_hit else int(rng.integers(1, 2 * blk + 1))
        first = 0 if force_hit else int(rng.integers(0, ntris))
        off = len(ids)
        ids.extend((first + j) % ntris for j in range(n))
        return _node(hit_box if (rng.random() < p_leaf_hit or force_hit) else FAR, off, n)

    def interior(k, right):
        return _node(FAR if k == interior_miss_at else hit_box, right, 0)

    nodes = []
    if shape == "A":
        for k in range(depth):                    # I_k at 2k, L_k at 2k + 1
            nodes.append(interior(k, 2 * k + 2))
            nodes.append(leaf())
        nodes.append(leaf(True))                  # right child of the last interior (popped again and
                                                  # again from the clamped slot 49)
    else:
        for k in range(depth):                    # I_k at k; right leaf R_k at depth + 1 + k
            nodes.append(interior(k, depth + 1 + k))
        nodes.append(leaf())                      # left child of the last interior
        for k in range(depth):
            nodes.append(leaf())
    return np.stack(nodes), np.array(ids, dtype=np.uint32)


@pytest.fixture(scope="module")
def teapot(rt, gpu):
    s = Scene(rt, rt.Mesh.from_obj(model("teapot.obj")), "BVH", env=(0.8, 0.9, 1.0))
    pos = s.mesh.arrays()[0][:, :3]
    lo, hi = pos.min(axis=0) - 0.1, pos.max(axis=0) + 0.1
    s.scene_box = (tuple(float(v) for v in lo), tuple(float(v) for v in hi))
    s.ntris = s.mesh.ntris
    return s


@pytest.mark.parametrize("shape,depth,miss_at,seed", [
    ("A", 70, None, 1),       # stack past 50 entries: clamped slot 49
    ("A", 520, None, 2),      # 1000-pop cap
    ("A", 90, 60, 3),         # an interior miss ends the chain below the clamp
    ("B", 40, None, 4),       # missed right leaves followed by interior pops
    ("B", 700, None, 5),      # 1000-pop cap in the shallow shape
])
@pytest.mark.parametrize("mode,spp", [("PROJECT", 1), ("W9E1", 2)])
def test_bvh_stack_clamp_and_pop_cap(rt, teapot, shape, depth, miss_at, seed, mode, spp):
    nodes, ids = chain_bvh(teapot.ntris, depth, shape, seed, interior_miss_at=miss_at, scene_box=teapot.scene_box)
    teapot.ctx.upload_bvh_arrays(nodes, ids)
    teapot.oscene = O.SceneRef(teapot.om, None, O.OracleBvh(nodes, ids), teapot.env)
    region = (336, 170, 96, 64)
    g = teapot.render_gpu(mode, TEAPOT_CAM, 800, 450, region, 0, spp)
    o = teapot.render_oracle(mode, TEAPOT_CAM, 800, 450, region, 0, spp)
    linf, bits, idm = compare(g, o)
    assert idm == 0, f"{idm} primary-hit ids differ"
    assert bits == 0, f"{bits} radiance words differ (L-inf {linf})"
    for k in ("samples", "primary", "shadow", "bounce"):
        assert g[2][k] == o[2][k], (k, g[2][k], o[2][k])
    assert (g[1] != 0xFFFFFFFF).any()
