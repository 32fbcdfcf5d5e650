"""The five workloads BASELINE.json names, as concrete
synthetic scenes: geometry, camera, resolution, spp, shading mode and
traversal.  bench.py measures config 3 by default; the others are parity and
scale cases (``bench.py --config N``, tests/test_gpu_configs.py).

Cameras follow src/scenes.rs where the reference has the scene (configs 1-3);
configs 4 and 5 have no reference scene, so the camera is stated here.
"""
import os
from dataclasses import dataclass

from .core import Mesh

ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets", "models")


@dataclass(frozen=True)
class Workload:
    number: int
    name: str
    mode: str            # rt_mode: W1E6 / W6E1 / PROJECT / W7E3 / W9E1
    traversal: str       # BSP / BVH / NONE
    width: int
    height: int
    spp: int
    camera: tuple        # (eye, target, up, camera_constant)
    env: tuple = (1.0, 1.0, 1.0)
    ntris: int = 0       # nominal triangle count (0: analytic / asset)

    def mesh(self, ntris=None):
        """Build the scene geometry (None for the analytic W1E6 scene)."""
        n = ntris or self.ntris
        if self.number == 1:
            return None
        if self.number == 2:
            return Mesh.from_obj(os.path.join(ASSETS, "CornellBoxWithBlocks.obj"))
        if self.number == 3:
            return Mesh.synth_bunny(n)
        if self.number == 4:
            return Mesh.grid(Mesh.synth_bunny(n // 100 if n else 69451), 10, 10, 0.2)
        if self.number == 5:
            return Mesh.synth_soup(n)
        raise KeyError(self.number)


WORKLOADS = {
    # scenes.rs:47-53 worksheet 1 camera; w1e6.wgsl analytic triangle/sphere/plane
    1: Workload(1, "W1E6 analytic sphere/plane/triangle", "W1E6", "NONE", 512, 512, 1,
                ((2.0, 1.5, 2.0), (0.0, 0.5, 0.0), (0.0, 1.0, 0.0), 1.0)),
    # scenes.rs:63-69 Cornell camera; CornellBoxWithBlocks.obj (36 tris), W7E3 BSP
    2: Workload(2, "Cornell box with blocks (36 tris) W7E3 path trace", "W7E3", "BSP", 1024, 1024, 64,
                ((277.0, 275.0, -570.0), (277.0, 275.0, 0.0), (0.0, 1.0, 0.0), 1.0), ntris=36),
    # scenes.rs:71-77 bunny camera; deterministic 69,451 +- 1 % tri stand-in, W9E1 constant env
    3: Workload(3, "bunny stand-in W9E1 path trace", "W9E1", "BSP", 1920, 1080, 256,
                ((-0.02, 0.11, 0.6), (-0.02, 0.11, 0.0), (0.0, 1.0, 0.0), 3.5), ntris=69451),
    # 10 x 10 grid of bunny copies (spacing 0.2, centred at the origin), camera pulled back
    4: Workload(4, "bunny x100 grid W9E1 path trace", "W9E1", "BSP", 1920, 1080, 256,
                ((0.0, 1.0, 2.6), (0.0, 0.1, 0.0), (0.0, 1.0, 0.0), 1.5), ntris=6945100),
    # 10M random triangles, centres U[-1,1]^3, half-size 0.01 (PCG32 seed 0x5EED)
    5: Workload(5, "10M random-triangle soup W9E1 path trace", "W9E1", "BSP", 3840, 2160, 1024,
                ((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 1.5), ntris=10_000_000),
}
