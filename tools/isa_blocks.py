"""Per-basic-block instruction counts of one kernel in an amdgcn .s dump,
with the loop nesting the compiler annotates.
usage: isa_blocks.py <file.s> <kernel-symbol-substring> [--loop BBx_y]"""
import re
import sys


def blocks(path, ksub):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and ksub in l)
    out, cur = [], None
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):(.*)$", l) or re.match(r"^; %(bb\.\d+):(.*)$", l)
        if m:
            cur = {"name": m.group(1), "loop": None, "ins": 0, "kinds": {}}
            out.append(cur)
            rest = m.group(2)
            h = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", rest)
            if h:
                cur["loop"] = (h.group(1), int(h.group(2)))
            h2 = re.search(r"Loop Header: Depth=(\d+)", rest)
            if h2:
                cur["loop"] = (m.group(1).lstrip("."), int(h2.group(1)))
            continue
        if cur is None:
            cur = {"name": "entry", "loop": None, "ins": 0, "kinds": {}}
            out.append(cur)
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        if cur["loop"] is None:
            h = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", l)
            if h:
                cur["loop"] = (h.group(1), int(h.group(2)))
        op = s.split()[0]
        cur["ins"] += 1
        k = op.split("_")[0]
        cur["kinds"][k] = cur["kinds"].get(k, 0) + 1
    return out


if __name__ == "__main__":
    bl = blocks(sys.argv[1], sys.argv[2])
    loop = sys.argv[4] if len(sys.argv) > 4 and sys.argv[3] == "--loop" else None
    tot = {}
    for b in bl:
        if loop and (b["loop"] is None or b["loop"][0] != loop):
            continue
        print(f'{b["name"]:>12} {str(b["loop"]):>18} {b["ins"]:5d}  {b["kinds"]}')
        for k, v in b["kinds"].items():
            tot[k] = tot.get(k, 0) + v
    print("total", sum(tot.values()), tot)
