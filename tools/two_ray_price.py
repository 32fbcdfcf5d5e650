"""Prices "two rays per lane" for k_path's BSP walk on the walk
model's trip sequences (tools/walk_sim.py with WALK_TRACE=<npz> WALK_COHERENT=64:
per ray its walking (0) and leaf (1) trips in the certified walk; rays in
generation order -- each sample's camera ray, then its W9E1 shadow ray and bounce
-- with 64 consecutive samples per pixel, as k_path's pixel-major units hand
them out).  Tool code, not part of the product.

One wave of 64 lanes replays the kernel's trip loop:
  * K = 1 (today): each lane holds one path sample; a trip runs the walking half if
    any lane walks and the leaf half if any lane is in a leaf; a lane whose ray ended
    waits until at most T lanes still trace, then every waiting lane shades (its
    next ray, or the next sample from the queue) in one shading pass.
  * K = 2: each lane holds two samples; a trip's walking half advances one walking
    ray per lane and its leaf half one ray in a leaf, so a lane whose rays are in
    different phases does two trips' work in one; a lane whose two rays are in the
    same phase advances one.  Each half first selects the chosen ray's state into
    its registers and writes it back (per-lane v_cndmask: `sel` VALU per trip), and
    the wave shades when at most T2 of the 128 slots trace.  Slots draw either from
    one queue (both slots: consecutive samples of the same pixel, "same") or slot k
    from its own half of the queue (two pixels per lane, "split").
Cost per wave-trip (VALU wave-instructions, from the trip's ISA, DESIGN.md "where a
trip's instructions go"): walking half 150, leaf half 105, the check/loop 14; a
shading pass 340 per sample a lane shades in it (a lane shading two samples runs
the shading code twice).
usage: python tools/two_ray_price.py trace.npz [T] [T2,...] [sel,...] [rays]"""
import sys

import numpy as np

CW, CL, CB, CSHADE = 150.0, 105.0, 14.0, 340.0


def paths_of(trace, off, kind):
    """[[trip sequence of each ray of the sample's path], ...] in generation order."""
    paths, cur = [], None
    for i in range(len(off) - 1):
        if kind[i] == 0:
            cur = []
            paths.append(cur)
        cur.append(trace[off[i]:off[i + 1]])
    return paths


def simulate(paths, K, T, sel=0.0, split=False, lanes=64):
    queues = [paths[k::K] if split else None for k in range(K)] if split else [paths]
    qpos = [0] * len(queues)
    path = [[None] * K for _ in range(lanes)]    # the slot's path (list of ray sequences)
    ray = np.zeros((lanes, K), np.int64)          # which ray of the path
    pos = np.zeros((lanes, K), np.int64)          # next trip of that ray
    state = np.zeros((lanes, K), np.int8)         # 0 idle/waiting, 1 tracing
    cost = 0.0
    trips = halves_w = halves_l = lanes_w = lanes_l = passes = 0

    def take(k):
        q = queues[k if split else 0]
        i = qpos[k if split else 0]
        if i >= len(q):
            return None
        qpos[k if split else 0] += 1
        return q[i]

    def shade():
        nonlocal cost, passes
        most = 0
        for l in range(lanes):
            n = 0
            for k in range(K):
                if state[l, k]:
                    continue
                p = path[l][k]
                if p is not None and ray[l, k] + 1 < len(p):
                    ray[l, k] += 1
                else:
                    p = take(k)
                    path[l][k] = p
                    ray[l, k] = 0
                    if p is None:
                        continue
                pos[l, k] = 0
                state[l, k] = 1
                n += 1
            most = max(most, n)
        if most:
            cost += CSHADE * most
            passes += 1

    shade()
    while True:
        if not state.any():
            if all(qpos[i] >= len(queues[i]) for i in range(len(queues))) and \
                    all(path[l][k] is None or ray[l, k] + 1 >= len(path[l][k]) for l in range(lanes) for k in range(K)):
                break
            shade()
            continue
        adv_w, adv_l = [], []
        for l in range(lanes):
            w = lf = None
            for k in range(K):
                if not state[l, k]:
                    continue
                ph = path[l][k][ray[l, k]][pos[l, k]]
                if ph == 0 and w is None:
                    w = k
                elif ph == 1 and lf is None:
                    lf = k
            if w is not None:
                adv_w.append((l, w))
            if lf is not None:
                adv_l.append((l, lf))
        trips += 1
        cost += CB + (sel if K > 1 else 0.0)
        if adv_w:
            cost += CW
            halves_w += 1
            lanes_w += len(adv_w)
        if adv_l:
            cost += CL
            halves_l += 1
            lanes_l += len(adv_l)
        for l, k in adv_w + adv_l:
            pos[l, k] += 1
            if pos[l, k] >= len(path[l][k][ray[l, k]]):
                state[l, k] = 0
        if int(state.sum()) <= T:
            shade()
    rays = sum(len(p) for p in paths)
    lane_work = CW * lanes_w + CL * lanes_l
    return {"K": K, "T": T, "sel": sel, "split": split, "valu_per_ray": round(cost / rays, 2),
            "wave_trips_per_ray": round(trips / rays, 4),
            "walk_half_frac": round(halves_w / trips, 3), "leaf_half_frac": round(halves_l / trips, 3),
            "walk_lanes": round(lanes_w / max(1, halves_w), 1), "leaf_lanes": round(lanes_l / max(1, halves_l), 1),
            "lane_use_halves": round(lane_work / (lanes * (CW * halves_w + CL * halves_l)), 3),
            "shade_passes_per_trip": round(passes / trips, 4)}


def main():
    d = np.load(sys.argv[1])
    trace, off, kind = d["trace"], d["off"].astype(np.int64), d["kind"]
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    T2s = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "16,32,48").split(",")]
    sels = [float(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "0,32,64").split(",")]
    paths = paths_of(trace, off, kind)
    n = int(sys.argv[5]) if len(sys.argv) > 5 else len(paths)
    paths = paths[:n]
    print(f"{len(paths)} samples, {sum(len(p) for p in paths)} rays, "
          f"{sum(len(r) for p in paths for r in p) / sum(len(p) for p in paths):.2f} trips per ray")
    base = simulate(paths, 1, T)
    print("K=1", base)
    for split in (False, True):
        for T2 in T2s:
            for sel in sels:
                r = simulate(paths, 2, T2, sel, split)
                r["valu_vs_K1"] = round(r["valu_per_ray"] / base["valu_per_ray"], 4)
                print("K=2", r)


if __name__ == "__main__":
    main()
