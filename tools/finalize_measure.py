"""Commit one measured workload of a GPU session (tools/session.sh m<C>...): its PMC
passes summarised into profiles/pmc_summary.json under the bench's key (tied to the
build's fatbin hash), the per-kernel PMC and kernel-trace summaries and the bench
line copied under profiles/<round>/final/, and the bench line's roofline recomputed
from that summary (the run itself printed "unmeasured": its summary did not exist yet).

  python tools/finalize_measure.py <session tag>/<workload dir> <name> <pmc key> <kernel substring> [--round r05]
e.g. python tools/finalize_measure.py f1/c3 c3 1920x1080x256_BSP_n1 "k_path<4, 0, false, 1>"
"""
import argparse
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tagdir")
    ap.add_argument("name")
    ap.add_argument("key")
    ap.add_argument("kernel")
    ap.add_argument("--round", default="r05")
    a = ap.parse_args()
    run = os.path.join(ROOT, "gpurun_out", a.tagdir)
    prof = os.path.join(ROOT, "gpurun_out", "prof", a.tagdir)
    dst = os.path.join(ROOT, "profiles", a.round, "final")
    os.makedirs(dst, exist_ok=True)
    pmc_out = os.path.join(dst, f"k_path_bsp_{a.name}_pmc.json")
    rel = os.path.relpath(pmc_out, ROOT)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), prof, a.kernel, "--out", pmc_out,
                    "--summary", a.key, "--source", rel, "--bench-json", os.path.join(run, "bench.json")],
                   check=True, stdout=subprocess.DEVNULL)
    shutil.copy(os.path.join(run, "kernel_stats.csv"), os.path.join(dst, f"kernel_stats_{a.name}.csv"))
    import bench
    line = json.loads([l for l in open(os.path.join(run, "bench.json")) if l.startswith("{")][-1])
    r = line["roofline"]
    bench.LIB_FOR_SHA = os.path.join(ROOT, "02562_raytracer_amd", "lib02562rt.so")
    cfg = int(line["config"]["workload"].split()[1].rstrip(":"))
    new = bench.roofline(a.key, r["kernel_ms"], r["algorithmic"]["bytes_per_launch"], cfg, r["kernel"])
    if new.get("fatbin_sha16") != r.get("fatbin_sha16"):
        raise SystemExit(f"the in-tree library ({new.get('fatbin_sha16')}) is not the measured build ({r.get('fatbin_sha16')})")
    for k in ("launches_per_step", "render_ms", "kernel_ms_max_over_ranks"):
        if k in r:
            new[k] = r[k]
    new["note"] = ("recomputed after the run from the PMC summary of the same build and workload "
                   f"(profiles/pmc_summary.json[{a.key}], {rel}); the run's own line said 'unmeasured'")
    line["roofline"] = new
    with open(os.path.join(dst, f"bench_{a.name}.json"), "w") as f:
        f.write(json.dumps(line) + "\n")
    print(a.name, line["value"], new["bound"], new["frac"], {k: new[k]["frac"] for k in ("hbm", "valu_issue") if k in new})


if __name__ == "__main__":
    main()
