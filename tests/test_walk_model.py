"""The trip model of the BSP walk (tools/walk_sim.c) that
priced subtree culling and the clipped decisions before they were built: on
the config-3 scene's camera, shadow and bounce rays, the culled walk (content
boxes grown by 2^-10 of the scene), with and without decisions against the
box's interval, returns the same hit -- triangle and distance -- as the
reference walk (bsp.wgsl:10-81) for every ray, and needs far fewer trips.
The model checks the algorithm in f32 on the CPU; the kernel's own equality
(culling on vs off) is tests/test_gpu_cull*.py."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(clip):
    env = dict(os.environ, WALK_BOXES="1", WALK_MARGIN_LG="10", WALK_CLIP=str(clip))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "walk_sim.py"), "3", "1500"], env=env,
                         capture_output=True, text=True, timeout=600, check=True).stdout
    rows = {}
    for line in out.splitlines():
        m = re.match(r"^(v\d) \{(.*)\} trips/ray ([0-9.]+)", line)
        if m:
            d = dict(re.findall(r"'(\w+)': (?:np\.float64\()?([0-9.]+)", m.group(2)))
            rows[m.group(1)] = {k: float(v) for k, v in d.items()} | {"trips": float(m.group(3))}
    return rows


def test_culled_and_clipped_walks_return_the_reference_hits():
    plain = _run(0)
    clipped = _run(1)
    for rows in (plain, clipped):
        assert {"v0", "v3", "v4"} <= set(rows)
        for v in ("v3", "v4"):
            assert rows[v]["mismatch"] == 0, (v, rows[v])
    # the model's case for building them: culling, then clipping, cut the trips
    assert plain["v4"]["trips"] < 0.45 * plain["v0"]["trips"]
    assert clipped["v4"]["trips"] < 0.95 * plain["v4"]["trips"]
    assert clipped["v4"]["pushes"] < plain["v4"]["pushes"]
