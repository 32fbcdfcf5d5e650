"""Summarise rocprofv3 --pmc CSVs: per kernel, the mean per dispatch of every
counter (summed over the counter's dimensions), plus derived figures.

  pmc_summary.py <dir> [kernel-substring] [--out FILE] [--traffic KEY]

--summary KEY records the kernel's per-launch counter figures in
profiles/pmc_summary.json under KEY (bench.py's roofline reads them): HBM bytes,
VALU wave-instructions, L2 hit rate, VALU lane utilisation, wait fraction, and
`source` = the directory of the passes (commit it under profiles/).
HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB units): MI355X_MICROARCH.md
"HBM / rocprofv3": on gfx950 FETCH_SIZE reports half the bytes of wide reads.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(root, ksub=None):
    per = defaultdict(lambda: defaultdict(float))   # kernel -> counter -> sum over dispatches
    disp = defaultdict(set)
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"]
                if ksub and ksub not in k:
                    continue
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[(k, r["Counter_Name"])].add((f, r["Dispatch_Id"]))
    return {k: {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()} for k, cs in per.items()}


def derived(c):
    d = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        d["hbm_bytes_per_launch"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        d["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "TCP_TCC_READ_REQ_sum" in c and "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
        d["l1_hit_rate"] = 1.0 - c["TCP_TCC_READ_REQ_sum"] / max(1.0, c["TCP_TOTAL_CACHE_ACCESSES_sum"])
    if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
        d["valu_lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / max(1.0, 64.0 * c["SQ_ACTIVE_INST_VALU"])
    if "SQ_INSTS_VALU" in c and "SQ_INSTS_SALU" in c:
        d["salu_per_valu"] = c["SQ_INSTS_SALU"] / max(1.0, c["SQ_INSTS_VALU"])
    if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
        d["wait_frac"] = c["SQ_WAIT_ANY"] / max(1.0, c["SQ_WAVE_CYCLES"])
    return d


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel", nargs="?")
    ap.add_argument("--out")
    ap.add_argument("--summary")
    ap.add_argument("--source", help="profiles/ path recorded as the summary's source")
    ap.add_argument("--bench-json", help="the bench line of the same build: its roofline.fatbin_sha16 is recorded")
    a = ap.parse_args()
    res = load(a.dir, a.kernel)
    out = {k: {"counters": c, "derived": derived(c)} for k, c in res.items()}
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    if a.summary:
        if len(res) != 1:
            raise SystemExit(f"--summary needs exactly one kernel, got {list(res)}")
        (kname, c), = res.items()
        d = derived(c)
        ent = {"kernel": kname, "source": a.source or a.dir,
               "hbm_bytes_per_launch": int(d["hbm_bytes_per_launch"]),
               "fetch_bytes_per_launch": int(2.0 * c["FETCH_SIZE"] * 1024.0),
               "write_bytes_per_launch": int(c["WRITE_SIZE"] * 1024.0),
               "valu_insts_per_launch": int(c["SQ_INSTS_VALU"])}
        if "SQ_INSTS_SALU" in c:
            ent["salu_insts_per_launch"] = int(c["SQ_INSTS_SALU"])
        if a.bench_json:
            line = [l for l in open(a.bench_json) if l.startswith("{")][-1]
            ent["fatbin_sha16"] = json.loads(line)["roofline"].get("fatbin_sha16")
        for k in ("l2_hit_rate", "valu_lane_util", "wait_frac", "salu_per_valu", "l1_hit_rate"):
            if k in d:
                ent[k] = round(d[k], 4)
        path = os.path.join(ROOT, "profiles", "pmc_summary.json")
        cur = json.load(open(path)) if os.path.exists(path) else {}
        cur[a.summary] = ent
        with open(path, "w") as f:
            json.dump(cur, f, indent=1, sort_keys=True)
            f.write("\n")
