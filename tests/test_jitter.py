"""compute_jitters (src/bindings/uniform.rs:254-277) restated in
02562_raytracer_amd/jitter.py.  The PCG32 generator is pinned by its published
reference vector; the strata properties follow from the reference's formula."""
import importlib

import numpy as np
import pytest

J = importlib.import_module("02562_raytracer_amd.jitter")


def test_pcg32_reference_vector():
    # PCG32 (pcg-c pcg32-demo, rand_pcg's Lcg64Xsh32 reference test): seed 42, stream 54
    rng = J.Lcg64Xsh32(42, 54)
    assert [rng.next_u32() for _ in range(6)] == [0xa15c02b7, 0x7b47f409, 0xba1d3330, 0x83d2f293, 0xbfa4784b,
                                                  0xcbed606e]


def test_subdiv1_is_zero():
    assert np.array_equal(J.compute_jitters(1 / 512, 1), np.zeros((1, 2), np.float32))


@pytest.mark.parametrize("n", [2, 3, 7, 10])
def test_strata(n):
    ps = 1.0 / 450
    jt = J.compute_jitters(ps, n)
    assert jt.shape == (n * n, 2) and jt.dtype == np.float32
    step = ps / n
    for k, (x, y) in enumerate(jt.astype(np.float64)):
        i, j = divmod(k, n)
        # x in column j's stratum, y in row i's, both inside [-ps/2, ps/2]
        assert -ps / 2 + j * step - 1e-9 <= x <= -ps / 2 + (j + 1) * step + 1e-9
        assert -ps / 2 + i * step - 1e-9 <= y <= -ps / 2 + (i + 1) * step + 1e-9
    assert np.array_equal(jt, J.compute_jitters(ps, n))   # a fixed seed: the same table every frame


def test_bounds():
    with pytest.raises(ValueError):
        J.compute_jitters(1 / 512, 11)
    with pytest.raises(ValueError):
        J.compute_jitters(1 / 512, 0)
