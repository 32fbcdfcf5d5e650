"""The certified culling margin (rt_kernels.hip bsp_box_miss, DESIGN.md section 4
"Certified culling") against adversarial rays on the CPU: tests/native/cert_bound.c
runs the reference's f32 triangle test (w7e3.wgsl:286-332) on random triangles
(sizes 1e-4 .. 3, slivers included) and rays aimed near them from up to 10x the
scene size away, half of them at elevations that put |denom| just above the
shader's 1e-10 reject -- where the f32 hit point strays furthest from the
triangle -- and checks that every accepted hit point o + dist*w lies within the
margin of the triangle's box (the proof's claim; the bound is not tight: the
worst point seen sits at under 2 % of it).  With the camera bound (rays from the
eye the treelets' camera terms are computed for), every ray's origin plays the
eye: a third of the accepts then have their margin set by the camera bound."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("cert") / "cert_bound")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(ROOT, "tests", "native", "cert_bound.c"),
                    "-lm"], check=True, timeout=120)
    return exe


@pytest.mark.parametrize("seed,camera", [(1, 0), (7, 0), (3, 1), (11, 1)])
def test_every_f32_accept_lies_within_the_certified_margin(harness, seed, camera):
    # camera 1: the margin also takes the camera-ray bound (each ray's origin as the eye,
    # H = |(v0 - o) . n*| / E^2 as the repack stores it)
    out = subprocess.run([harness, "1500000", str(seed), str(camera)], check=True, capture_output=True, text=True,
                         timeout=300)
    acc, worst, floor_acc, cam_binds = out.stdout.split()
    acc, worst, floor_acc, cam_binds = int(acc), float(worst), int(floor_acc), int(cam_binds)
    print(f"seed {seed} camera {camera}: {acc} accepts ({floor_acc} with |denom| < 1e-9, {cam_binds} with the "
          f"camera bound the tighter), worst distance / margin {worst:.4g}")
    assert acc > 200_000 and floor_acc > 50_000
    assert cam_binds > (50_000 if camera else -1)
    assert worst < 1.0
