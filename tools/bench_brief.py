"""One-line digest of a bench.py JSON line (stdin)."""
import json
import sys

d = json.loads(sys.stdin.read().strip().splitlines()[-1])
t = d["traversal_per_launch"]
trips = max(1, t["trips"])
cyc = max(1, t.get("trav_cycles", 0) + t.get("shade_cycles", 0))
print(f'{d["value"]} Mrays/s  {d["ms_per_step"]} ms/step  kernel {d["roofline"]["kernel_ms"]} ms  '
      f'frac {d["roofline"]["frac"]}  lane_util {d["simd_lane_util"]}  '
      f'leaf_iters/trip {t["leaf_iters"] / trips:.3f}  trips {trips:.3e}  '
      f'shade_passes/trip {t.get("shade_passes", 0) / trips:.3f}  '
      f'shade_lanes/pass {t.get("shade_lanes", 0) / max(1, t.get("shade_passes", 0)):.1f}  '
      f'trav_cycle_frac {t.get("trav_cycles", 0) / cyc:.3f}  '
      f'cycles/trip {t.get("trav_cycles", 0) / trips:.0f}')
