"""Register-allocation guard for the bench kernel (CPU only: hipcc
cross-compiles gfx950 here).  A spill reload inside k_path's traversal trip
loop cost 18 % of the config-3 frame when an unrelated shading change moved
the allocator's choices.  The default instantiations'
trip loops may hold only the spill stores of the accept path they hold today."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

# kernel -> allowed scratch instructions in its trip loop (today's values)
BUDGET = {
    "k_pathILi4ELi0ELb0": 2,   # W9E1, BSP: the bench kernel (two stores on a triangle accept)
    "k_pathILi4ELi1ELb0": 6,   # W9E1, BVH (two pops per trip)
}


@pytest.fixture(scope="module")
def device_asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "rt_kernels.s"
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "--offload-arch=gfx950", "-ffp-contract=off",
           "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wno-bitwise-instead-of-logical",
           "-x", "hip", "--cuda-device-only", "-S", os.path.join(ROOT, "02562_raytracer_amd", "csrc", "rt_kernels.hip"),
           "-o", str(out)]
    if not os.path.exists(cmd[0]):
        pytest.skip("hipcc not available")
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return str(out)


@pytest.mark.parametrize("kernel", sorted(BUDGET))
def test_trip_loop_spills_within_budget(device_asm, kernel):
    from trip_loop_scratch import trip_loop_scratch
    n = trip_loop_scratch(device_asm, kernel)
    assert n <= BUDGET[kernel], f"{kernel}: {n} scratch ops in the trip loop (budget {BUDGET[kernel]})"
