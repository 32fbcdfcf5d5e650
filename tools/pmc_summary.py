"""Summarise rocprofv3 --pmc CSVs: per kernel, the mean per dispatch of every
counter (summed over the counter's dimensions).  usage: pmc_summary.py <dir> [kernel-substring]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(root, ksub=None):
    per = defaultdict(lambda: defaultdict(float))   # (kernel) -> counter -> sum over dispatches
    disp = defaultdict(set)
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"]
                if ksub and ksub not in k:
                    continue
                did = (f, r["Dispatch_Id"])
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[(k, r["Counter_Name"])].add(did)
    out = {}
    for k, cs in per.items():
        out[k] = {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()}
    return out


if __name__ == "__main__":
    res = load(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
    print(json.dumps(res, indent=1))
