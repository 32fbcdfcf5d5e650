"""Scratch (spill) instructions inside k_path's traversal trip loop.

The trip loop is the innermost loop that issues the treelet / record loads
(>= 3 buffer_load_dwordx4 in one block); a spill reload there costs ~18 % of the BSP frame
(kernel-source rule).  usage:
  python tools/trip_loop_scratch.py <device .s> [kernel-substring ...]
prints one line per kernel: <kernel> <scratch ops in the trip loop>."""
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_blocks import blocks   # noqa: E402


def trip_loop_scratch(path, ksub):
    bl = blocks(path, ksub)
    headers = {b["loop"] for b in bl if b["loop"] and b["kinds"].get("buffer", 0) >= 3}
    if not headers:
        raise RuntimeError(f"{ksub}: no loop with the treelet loads")
    # the innermost such loop (deepest)
    h = max(headers, key=lambda x: x[1])
    return sum(b["kinds"].get("scratch", 0) for b in bl if b["loop"] == h)


if __name__ == "__main__":
    for k in sys.argv[2:] or ["k_pathILi4ELi0ELb0ELb1", "k_pathILi4ELi1ELb0ELb1"]:
        print(k, trip_loop_scratch(sys.argv[1], k))
