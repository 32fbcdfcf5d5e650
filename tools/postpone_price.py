"""Prices "postpone the minority half" for k_path's BSP trip on the walk model's trip
sequences (the same traces and cost model as tools/two_ray_price.py, one ray per lane):
a trip whose walking and leaf halves both have lanes skips the half with at most P lanes
(those lanes advance in a later trip), so the wave pays one half instead of two.  Round
2 measured this policy slower when the scalar ALU was the kernel's limit (DESIGN.md
section 4, "Trip-half postponement"); this prices its VALU on the round-6 trip.  The
per-trip scalar cost of the choice (two ballots, popcounts, compares) is not in the
VALU model.  Tool code, not part of the product.
usage: python tools/postpone_price.py trace.npz [T] [P,...] [rays]"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__file__))
from two_ray_price import CB, CL, CSHADE, CW, paths_of  # noqa: E402


def simulate(paths, T, P, lanes=64, postpone_leaf=True, postpone_walk=True):
    qpos = 0
    path = [None] * lanes
    ray = np.zeros(lanes, np.int64)
    pos = np.zeros(lanes, np.int64)
    state = np.zeros(lanes, np.int8)
    cost = 0.0
    trips = hw = hl = lw = ll = passes = skipped = 0

    def shade():
        nonlocal cost, passes, qpos
        n = 0
        for l in range(lanes):
            if state[l]:
                continue
            p = path[l]
            if p is not None and ray[l] + 1 < len(p):
                ray[l] += 1
            else:
                p = paths[qpos] if qpos < len(paths) else None
                qpos += 1 if p is not None else 0
                path[l] = p
                ray[l] = 0
                if p is None:
                    continue
            pos[l] = 0
            state[l] = 1
            n += 1
        if n:
            cost += CSHADE
            passes += 1

    shade()
    while state.any():
        aw = [l for l in range(lanes) if state[l] and path[l][ray[l]][pos[l]] == 0]
        al = [l for l in range(lanes) if state[l] and path[l][ray[l]][pos[l]] == 1]
        trips += 1
        cost += CB
        if aw and al and P > 0:
            if postpone_walk and len(aw) <= P and len(aw) <= len(al):
                skipped += 1
                aw = []
            elif postpone_leaf and len(al) <= P:
                skipped += 1
                al = []
        if aw:
            cost += CW
            hw += 1
            lw += len(aw)
        if al:
            cost += CL
            hl += 1
            ll += len(al)
        for l in aw + al:
            pos[l] += 1
            if pos[l] >= len(path[l][ray[l]]):
                state[l] = 0
        if int(state.sum()) <= T:
            shade()
            while not state.any() and qpos < len(paths):
                shade()
    rays = sum(len(p) for p in paths)
    return {"T": T, "P": P, "valu_per_ray": round(cost / rays, 2), "wave_trips_per_ray": round(trips / rays, 4),
            "walk_half_frac": round(hw / trips, 3), "leaf_half_frac": round(hl / trips, 3),
            "walk_lanes": round(lw / max(1, hw), 1), "leaf_lanes": round(ll / max(1, hl), 1),
            "skipped_frac": round(skipped / trips, 3), "shade_passes_per_trip": round(passes / trips, 4)}


def main():
    d = np.load(sys.argv[1])
    paths = paths_of(d["trace"], d["off"].astype(np.int64), d["kind"])
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    Ps = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "0,2,4,8,12,16").split(",")]
    n = int(sys.argv[4]) if len(sys.argv) > 4 else len(paths)
    paths = paths[:n]
    base = None
    for P in Ps:
        r = simulate(paths, T, P)
        base = base or r["valu_per_ray"]
        r["valu_vs_P0"] = round(r["valu_per_ray"] / base, 4)
        print(r, flush=True)


if __name__ == "__main__":
    main()
