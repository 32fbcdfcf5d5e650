"""Register-allocation guard for the bench kernel (CPU only: hipcc
cross-compiles gfx950 here).  A spill reload inside k_path's traversal trip
loop cost 18 % of the config-3 frame when an unrelated shading change moved
the allocator's choices.  The default instantiations'
trip loops may hold only the spill stores of the accept path they hold today,
and the whole kernel's spill footprint (scratch bytes per lane, spill
instructions) may not grow: the shading-phase spills are most of the kernel's
HBM traffic ("HBM traffic")."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

# kernel -> allowed scratch instructions in its trip loop (today's values)
BUDGET = {
    # W9E1, BSP: the bench kernel, eight traversal steps per trip
    # (RT_TRIPS_PER_CHECK); none of them spills
    "k_pathILi4ELi0ELb0ELi1": 0,
    "k_pathILi4ELi0ELb0ELi0": 0,   # W9E1, BSP, the fast-margin instantiation
    "k_pathILi4ELi0ELb0ELi2": 0,   # W9E1, BSP, the silhouette bound
    "k_pathILi4ELi1ELb0ELi1": 0,   # W9E1, BVH at 8 waves/SIMD (4 before the round-2 spill cuts)
    "k_pathILi3ELi0ELb0ELi1": 0,
    "k_pathILi3ELi0ELb0ELi0": 0,   # W7E3, BSP, the fast-margin instantiation   # W7E3, BSP at 7 waves/SIMD
}


@pytest.fixture(scope="module")
def device_asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "rt_kernels.s"
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "--offload-arch=gfx950", "-ffp-contract=off",
           "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wno-bitwise-instead-of-logical",
           "-fno-slp-vectorize",   # as the Makefile builds rt_kernels.o
           "-x", "hip", "--cuda-device-only", "-S", os.path.join(ROOT, "02562_raytracer_amd", "csrc", "rt_kernels.hip"),
           "-o", str(out)]
    if not os.path.exists(cmd[0]):
        pytest.skip("hipcc not available")
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return str(out)


# kernel -> (scratch bytes per lane, scratch instructions in the whole kernel), today's values
WHOLE_BUDGET = {
    # (round 2: 148/133, 152/116 and 8/2 before the kernel arguments were
    # re-read in the shading phase and the shading state was trimmed)
    # round 3: the per-wave threshold choice, the 80-B treelets' fifth load and the
    # subtree cull added shading-phase spills (W9E1 BSP 68 B / 70 ops, W7E3 52 B / 30
    # ops before); the exact and clipped decisions took some back (final: 72/67,
    # 80/77, 44/43); the trip loops stay spill-free (BUDGET above).  At 6 waves/SIMD
    # (make WPE=6) the W9E1 BSP kernel spills 16 B / 9 ops.
    # round 4: the certified culling margin keeps three per-ray terms of the box
    # test in registers across the trip loop (w1 x 20u, w1 x k1, the origin
    # margin) and the 96-B treelets a sixth load: 104/90 and 64/59 (from 72/67, 44/43);
    # the camera bound (eye compare, |w|inf, the eye term) 108/93 and 68/58; its
    # per-treelet precomputed form 108/93 and 64/56.
    # round 5: the zero-component slab of the cull (an infinite reciprocal, the
    # capped gap tolerance) and bsp_inv1's flag: 108/99 (W7E3 64/56 and 64/53 with
    # the one-load hit resolve); the silhouette bound's instantiation 128/118.
    # round 6: the box test's min / max without canonicalising instructions and the
    # treelet offset without v_mul_lo_u32 (W7E3 certified 60/50; the fast-margin
    # W9E1 instantiation 92/106, in its shading phase), the VERT leaf tests of
    # W9E1's shadow rays (no change); the plane divisions' range check behind a
    # wave-uniform flag (bsp_decide chk): W7E3 certified 72/59, its fast margin 60/43,
    # the silhouette instantiation 128/119, all in the shading phase
    "k_pathILi4ELi0ELb0ELi1": (108, 99),    # W9E1, BSP
    "k_pathILi4ELi0ELb0ELi2": (128, 119),   # W9E1, BSP, RT_BSP_CULL_SILHOUETTE (auto picks it on config 4)
    "k_pathILi4ELi0ELb0ELi0": (92, 106),    # W9E1, BSP, the fast-margin instantiation
    "k_pathILi4ELi1ELb0ELi1": (80, 77),     # W9E1, BVH
    "k_pathILi3ELi0ELb0ELi1": (72, 59),     # W7E3, BSP at 7 waves/SIMD
    "k_pathILi3ELi0ELb0ELi0": (60, 43),     # W7E3, BSP, the fast-margin instantiation (0/0 at 5)
}


def kernel_spills(path, ksub):
    import re
    s = open(path).read()
    name = next(l.split(":")[0] for l in s.splitlines() if re.match(r"^_Z\S*:", l) and ksub in l)
    i = s.index(name + ":")
    body = s[i:s.index(".Lfunc_end", i)]
    k = s.index(".amdhsa_kernel " + name)
    meta = s[k:s.index(".end_amdhsa_kernel", k)]
    scratch = int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", meta).group(1))
    return scratch, len(re.findall(r"\bscratch_(?:load|store)", body))


@pytest.mark.parametrize("kernel", sorted(WHOLE_BUDGET))
def test_whole_kernel_spills_within_budget(device_asm, kernel):
    scratch, ops = kernel_spills(device_asm, kernel)
    b_scratch, b_ops = WHOLE_BUDGET[kernel]
    assert scratch <= b_scratch, f"{kernel}: {scratch} B of scratch per lane (budget {b_scratch})"
    assert ops <= b_ops, f"{kernel}: {ops} spill instructions (budget {b_ops})"


@pytest.mark.parametrize("kernel", sorted(BUDGET))
def test_trip_loop_spills_within_budget(device_asm, kernel):
    from trip_loop_scratch import trip_loop_scratch
    n = trip_loop_scratch(device_asm, kernel)
    assert n <= BUDGET[kernel], f"{kernel}: {n} scratch ops in the trip loop (budget {BUDGET[kernel]})"
