"""One-line digest of a bench.py JSON line (stdin)."""
import json
import sys

d = json.loads(sys.stdin.read().strip().splitlines()[-1])
t = d.get("traversal_per_step") or d["traversal_per_launch"]
trips = max(1, t["trips"])
cyc = max(1, t.get("trav_cycles", 0) + t.get("shade_cycles", 0))
print(f'{d["value"]} Mrays/s  {d["ms_per_step"]} ms/step  kernel {d["roofline"]["kernel_ms"]} ms  '
      f'frac {d["roofline"]["frac"]}  lane_util {d["simd_lane_util"]}  '
      f'trips {trips:.3e}  node_trips {t.get("node_trips", 0) / trips:.3f}  '
      f'leaf_trips {t.get("leaf_trips", 0) / trips:.3f}  '
      f'node_lanes/trip {(t["lane_steps"] - t.get("leaf_lane_steps", 0)) / trips:.1f}  '
      f'leaf_lanes/trip {t.get("leaf_lane_steps", 0) / trips:.1f}  '
      f'exact_tests/test {t.get("exact_tests", 0) / max(1, t["tri_tests"]):.3f}  '
      f'exact_nodes/node {t.get("exact_nodes", 0) / max(1, t["node_interior"]):.3f}  '
      f'shade_passes/trip {t.get("shade_passes", 0) / trips:.3f}  '
      f'shade_lanes/pass {t.get("shade_lanes", 0) / max(1, t.get("shade_passes", 0)):.1f}  '
      f'trav_cycle_frac {t.get("trav_cycles", 0) / cyc:.3f}  '
      f'cycles/trip {t.get("trav_cycles", 0) / trips:.0f}  memwait/trip {t.get("memwait_cycles", 0) / trips:.0f}  '
      f'wave_Gcycles {cyc / 1e9:.1f}')
