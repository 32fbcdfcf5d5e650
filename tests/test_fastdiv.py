"""The BSP walk's exact division from a per-ray reciprocal
(include/rt_detmath.h rt_div_by_recip, Markstein's theorem) must equal IEEE
binary32 division bit for bit on its operand range: a host check over 2*10^7
operand pairs (the device side is covered by rt_selftest_math on the GPU)."""
import os
import subprocess

from conftest import ROOT


def test_div_by_recip_matches_ieee_division(tmp_path):
    exe = str(tmp_path / "fastdiv_check")
    src = os.path.join(ROOT, "tests", "native", "fastdiv_check.c")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-o", exe, src, "-lm"], check=True)
    for seed in (1, 2):
        out = subprocess.run([exe, "10000000", str(seed)], capture_output=True, text=True)
        assert out.returncode == 0, out.stdout
        assert "mismatches 0" in out.stdout
