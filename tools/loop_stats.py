"""Static instruction counts of k_path's trip loop (the innermost loop with the
treelet / record loads), per instruction class: a quick A/B of kernel source
changes before timing them.  usage: python tools/loop_stats.py <device .s> [kernel-substring ...]"""
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_blocks import blocks   # noqa: E402


def loop_stats(path, ksub):
    bl = blocks(path, ksub)
    headers = {b["loop"] for b in bl if b["loop"] and b["kinds"].get("buffer", 0) >= 3}
    h = max(headers, key=lambda x: x[1])
    tot = {}
    for b in bl:
        if b["loop"] == h:
            for k, v in b["kinds"].items():
                tot[k] = tot.get(k, 0) + v
    return tot


if __name__ == "__main__":
    for k in sys.argv[2:] or ["k_pathILi4ELi0ELb0ELb1"]:
        t = loop_stats(sys.argv[1], k)
        print(k, sum(t.values()), dict(sorted(t.items(), key=lambda x: -x[1])))
