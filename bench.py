"""Benchmark: Mrays/s (primary + shadow) of the BSP traversal + shading hot
path at 1920x1080, 256 spp (BASELINE.json configs[2]: ~70k-tri bunny, W9E1
path tracer), on N GPUs of one node.

One step = one complete progressive frame (iterations 0..spp-1, the
reference's spp RenderState::render() calls fused into one launch per GPU)
with the framebuffer tiled across ranks (interleaved 8x8 tiles) and the
finished tiles all-gathered over RCCL to assemble the frame on rank 0.
Total work is fixed as N grows ("strong" scaling).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2..5]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

--config selects another BASELINE.json workload (02562_raytracer_amd/configs.py);
the default, 3, is the headline.  Prints ONE JSON line on rank 0.  See
DESIGN.md "Measurement".
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
L2_PEAK_GBS = 34500.0   # aggregate L2 (8 XCDs x 4 MiB), MI355X_MICROARCH.md "L2 (per XCD)"
# VALU issue: a wave64 VALU instruction issues over 2 cycles on its SIMD
# (MI355X_MICROARCH.md "issues each VALU instruction over 2 cycles"): 256 CUs x 4
# SIMDs x 2.4 GHz (max clock) / 2 = wave-instructions per second, chip-wide
NUM_CUS, SIMDS_PER_CU, MAX_CLOCK_GHZ = 256, 4, 2.4
VALU_PEAK_GINSTS = NUM_CUS * SIMDS_PER_CU * MAX_CLOCK_GHZ / 2.0
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")
LIB_FOR_SHA = None   # the loaded lib02562rt.so (set in main once the package is imported)
# SALU issue: the scalar ALU is one per-CU resource; tools/probes/issue_probe.hip
# measured it saturating at 0.758 wave-instructions per shader cycle per CU
# (profiles/r02/issue_probe.txt; the microarchitecture guide gives no figure)
SALU_PEAK_GINSTS = NUM_CUS * 0.758 * MAX_CLOCK_GHZ
METRIC = "Mrays/sec primary+shadow at 1920x1080; achieved HBM GB/s vs peak"


def algorithmic_bytes(c, trav):
    """reference-layout useful bytes of the traversal work,
    plus the output bytes k_path writes: one 16-B sample record (radiance +
    primary id) per pixel-iteration (the fold kernel that averages them is
    not part of k_path and is timed apart)."""
    if trav == "BSP":
        t = 20 * c["node_interior"] + 16 * c["node_leaf"]
    else:
        t = 32 * c["bvh_pops"]
    t += 4 * c["ids_read"] + 52 * c["tri_tests"] + 36 * c["tri_accepts"]
    return t + 16 * c["samples"]


def cpu_baseline(wl, trav, mesh, accel, spp, W, H, budget_s):
    """The CPU oracle (a restatement of the reference WGSL path; the reference
    itself needs Rust + Vulkan, absent here) on the host cores, over a bounded
    sample of the same workload: the full frame, 1 spp per pass, passes
    (iterations 0, 1, 2, ...) repeated until ~budget_s of CPU time.  The oracle
    renders from the product builder's arrays (bit-identical to the oracle's own
    builders: tests/test_host_builders.py), which spares its single-threaded
    BSP build on the 7M/10M-triangle configs."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    V, N, I, M, L = mesh.arrays()
    om = O.OracleMesh(V, N, I, M, L)
    if trav == "BSP":
        tree, planes, ids, aabb, md = accel.arrays()
        osc = O.SceneRef(om, O.OracleBsp(tree, planes, ids, aabb, md), None, env=wl.env)
    else:
        nodes, tids = accel.arrays()
        osc = O.SceneRef(om, None, O.OracleBvh(nodes, tids), env=wl.env)
    u = O.make_uniform(*wl.camera, W, H)
    # the threads this process may use: the GPU box gives each GPU a 16-thread
    # share of the host (it sets OMP_NUM_THREADS=16; os.cpu_count() there reports
    # the whole machine, which other jobs share); here, every core of the container
    cores = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    region = (0, 0, W, H)
    acc = None
    rays = 0
    it = 0
    t0 = time.perf_counter()
    while True:
        acc, _, c = O.render(osc, u, wl.mode, trav, region, it, 1, accum=acc, nthreads=cores)
        rays += c["primary"] + c["shadow"]
        it += 1
        el = time.perf_counter() - t0
        if el >= budget_s or it >= spp:
            break
    return {"value": rays / el / 1e6, "unit": "Mrays/s", "cores": cores, "kind": "port",
            "sample": f"CPU oracle (C restatement of {wl.mode.lower()}.wgsl+{trav.lower()}.wgsl, pthreads), the same "
                      f"{W}x{H} frame, first {it} of its {spp} spp, {el:.1f} s"}


def pmc_key(W, H, spp, trav, world, config, cull=1):
    return (f"{W}x{H}x{spp}_{trav}_n{world}" + ("" if config == 3 else f"_c{config}") +
            {0: "_off", 1: "", 2: "_fast", 3: "_sil"}[cull if trav == "BSP" else 1])


def fatbin_sha16(path):
    """SHA-256 (16 hex digits) of the library's device code (.hip_fatbin section):
    ties a committed PMC summary to the kernel build it was measured on."""
    import hashlib
    import struct
    with open(path, "rb") as f:
        b = f.read()
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    sec = [struct.unpack_from("<IIQQQQ", b, shoff + i * shentsize) for i in range(shnum)]
    stroff = sec[shstrndx][4]
    for name, _t, _f, _a, off, size in sec:
        end = b.index(b"\0", stroff + name)
        if b[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(b[off:off + size]).hexdigest()[:16]
    return None


def roofline(key, kern_ms, alg_bytes, config, kernel):
    """Roofline of the dominant kernel.  Counter figures per launch (HBM bytes,
    VALU wave-instructions) come from the committed PMC summary of the same
    workload (profiles/pmc_summary.json, tools/pmc_summary.py; its `source` names
    the rocprofv3 passes); the time is this run's HIP-event kernel time.
      * hbm: counter HBM bytes / time / 8 TB/s;
      * valu-issue: VALU wave-instructions / time / the chip's VALU issue rate;
      * salu-issue: SALU instructions / time / the probe-measured SALU ceiling.
    `bound` is whichever of these is largest for this launch (DESIGN.md "What
    bounds it"); all three are given.
    The SURVEY 8(d) algorithmic bytes (reference layout) over the kernel time is a
    diagnostic ("algorithmic"): the bytes stay in L2/MALL, so against HBM it can
    exceed 1 and is never reported as the HBM fraction."""
    s = kern_ms / 1e3
    pmc = None
    if os.path.exists(PMC_SUMMARY):
        with open(PMC_SUMMARY) as f:
            pmc = json.load(f).get(key)
    sha = fatbin_sha16(LIB_FOR_SHA) if LIB_FOR_SHA else None
    alg = {"bytes_per_launch": int(alg_bytes), "achieved": round(alg_bytes / s / 1e9, 1), "unit": "GB/s",
           "l2_peak": L2_PEAK_GBS, "l2_frac": round(alg_bytes / s / 1e9 / L2_PEAK_GBS, 4)}
    r = {"kernel": kernel, "kernel_ms": round(kern_ms, 3), "algorithmic": alg, "pmc": None, "traffic": None}
    r["fatbin_sha16"] = sha
    if pmc is None or (pmc.get("fatbin_sha16") and sha and pmc["fatbin_sha16"] != sha):
        r.update({"bound": "unmeasured", "achieved": None, "peak": None, "unit": None, "frac": None,
                  "note": (f"no PMC summary for {key} in profiles/pmc_summary.json" if pmc is None else
                           f"the PMC summary for {key} was measured on another kernel build "
                           f"({pmc['fatbin_sha16']}, this one {sha})")})
        return r
    hbm_gbs = pmc["hbm_bytes_per_launch"] / s / 1e9
    valu = pmc["valu_insts_per_launch"] / s / 1e9
    r["traffic"] = int(pmc["hbm_bytes_per_launch"])
    r["hbm"] = {"achieved": round(hbm_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(hbm_gbs / HBM_PEAK_GBS, 4)}
    r["valu_issue"] = {"achieved": round(valu, 1), "peak": round(VALU_PEAK_GINSTS, 1),
                       "unit": "G wave64 VALU instr/s", "frac": round(valu / VALU_PEAK_GINSTS, 4)}
    if "salu_insts_per_launch" in pmc:
        salu = pmc["salu_insts_per_launch"] / s / 1e9
        r["salu_issue"] = {"achieved": round(salu, 1), "peak": round(SALU_PEAK_GINSTS, 1),
                           "unit": "G wave SALU instr/s", "frac": round(salu / SALU_PEAK_GINSTS, 4),
                           "peak_source": "measured ceiling, tools/probes/issue_probe.hip"}
    r["pmc"] = {k: pmc[k] for k in ("source", "kernel_ms_profiled", "l2_hit_rate", "valu_lane_util", "wait_frac",
                                    "write_bytes_per_launch", "fetch_bytes_per_launch") if k in pmc}
    # the bound is the limit the counters put closest to its peak, whatever the config
    fr = {"hbm": r["hbm"], "valu-issue": r["valu_issue"]}
    if "salu_issue" in r:
        fr["salu-issue"] = r["salu_issue"]
    bound = max(fr, key=lambda k: fr[k]["frac"])
    prim = fr[bound]
    r.update({"bound": bound, "achieved": prim["achieved"], "peak": prim["peak"], "unit": prim["unit"],
              "frac": prim["frac"]})
    if max(v["frac"] for v in fr.values()) > 1.0:
        # a summary of another kernel build
        r.update({"bound": "unmeasured", "frac": None, "note": f"PMC summary for {key} does not match this kernel"})
    return r


class DeviceAccel:
    """The context's device-built BSP / HLBVH, downloaded on demand (the CPU
    baseline's oracle renders from the same arrays), with BspTree's / Bvh's
    arrays() shape."""

    def __init__(self, ctx, trav):
        self.ctx, self.trav = ctx, trav

    def arrays(self):
        if self.trav == "BSP":
            tree, planes, ids, aabb = self.ctx.download_bsp()
            return tree, planes, ids, aabb, 20
        return self.ctx.download_bvh()


def all_reduce(dist, t, op):
    """In place on the device under RCCL; through host memory under gloo."""
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=op)
        return t
    h = t.cpu()
    dist.all_reduce(h, op=op)
    return h.to(t.device)


def all_gather(dist, t, world):
    """world x len(t) array of every rank's t (RCCL on the device, gloo through host memory)."""
    import torch
    src = t if dist.get_backend() == "nccl" else t.cpu()
    out = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(out, src)
    return torch.stack(out).cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 4, 5])
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--trav", default=None, choices=["BSP", "BVH"])
    ap.add_argument("--ntris", type=int, default=None)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shade-threshold", type=lambda x: int(x, 0), default=None,
                    help="RT_OPT_SHADE_THRESHOLD: 0..64, or 0x10000 | hi << 8 | lo (a per-wave choice)")
    ap.add_argument("--waves-per-cu", type=int, default=None)
    ap.add_argument("--sample-chunk", type=int, default=None)
    ap.add_argument("--unit-order", type=int, default=None)
    ap.add_argument("--host-build", action="store_true",
                    help="build the BSP / HLBVH on the host (rt_bsp_build / rt_bvh_build) instead of on the "
                         "device (rt_build_bsp_device / rt_build_bvh_device: the same arrays bit for bit, "
                         "tests/test_gpu_bsp_build.py, test_gpu_build.py; 27 ms against 3.3 s for config 5)")
    ap.add_argument("--bsp-cull", type=int, default=None,
                    help="RT_OPT_BSP_CULL: 0 off, 1 certified, 2 fast margin, 3 certified + silhouette bound, "
                         "4 the faster of 1 and 3 by a timed probe (the library default)")
    ap.add_argument("--async-fold", action="store_true",
                    help="pipelined frames (RT_OPT_ASYNC_FOLD 1): a frame's fold and gather overlap the next "
                         "frame's traversal kernel (measured slower on config 3: profiles/r04/ab_async_fold.txt)")
    ap.add_argument("--dump-frame", default=None,
                    help="rank 0 saves the last step's assembled frame (accum + ids) to this .npz")
    ap.add_argument("--progress", action="store_true",
                    help="a stderr line after every timed step (a host synchronisation per step)")
    ap.add_argument("--rank-share", type=int, default=None,
                    help="profiling: one process renders only rank 0's share of an N-rank split (the work one GPU "
                         "of the N-GPU bench does); its roofline is looked up under the _nN PMC key")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # launched by torch.distributed.run (the driver's N-GPU form): the process
    # group and the gather to rank 0 run for any N, so `--nproc-per-node 1`
    # executes the RCCL path on one GPU
    use_dist = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    share = args.rank_share or 1   # tile split: world ranks, or rank 0 of a --rank-share split
    if args.rank_share and use_dist:
        raise SystemExit("--rank-share is a single-process profiling mode")
    nsplit = world if use_dist else share
    # rehearsal knob: RT_BENCH_DEVICE pins every rank to one device (N ranks
    # sharing a single GPU exercise the N>1 path where only one GPU exists)
    if os.environ.get("RT_BENCH_DEVICE") is not None:
        local = int(os.environ["RT_BENCH_DEVICE"])
    # RCCL (backend "nccl"); RT_BENCH_DIST_BACKEND=gloo is the rehearsal path
    # with RT_BENCH_DEVICE (RCCL refuses two ranks on one GPU): host gathers
    backend = os.environ.get("RT_BENCH_DIST_BACKEND", "nccl")
    if use_dist:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # a real (non-null) stream shared by our kernels, torch's events and RCCL
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    rt = importlib.import_module("02562_raytracer_amd")   # after torch: shares its HIP runtime
    global LIB_FOR_SHA
    LIB_FOR_SHA = rt._ffi.LIB_PATH
    tiling = importlib.import_module("02562_raytracer_amd.tiling")
    wl = importlib.import_module("02562_raytracer_amd.configs").WORKLOADS[args.config]
    W, H = args.width or wl.width, args.height or wl.height
    spp = args.spp or wl.spp
    trav = args.trav or wl.traversal
    cam = wl.camera

    t0 = t_start = time.perf_counter()
    mesh = wl.mesh(args.ntris)
    ctx = rt.Context(local)
    ctx.set_stream(stream.cuda_stream)
    if args.shade_threshold is not None:
        ctx.set_option(rt._ffi.RT_OPT_SHADE_THRESHOLD, args.shade_threshold)
    if args.waves_per_cu is not None:
        ctx.set_option(rt._ffi.RT_OPT_WAVES_PER_CU, args.waves_per_cu)
    if args.sample_chunk is not None:
        ctx.set_option(rt._ffi.RT_OPT_SAMPLE_CHUNK, args.sample_chunk)
    if args.unit_order is not None:
        ctx.set_option(rt._ffi.RT_OPT_UNIT_ORDER, args.unit_order)
    if args.bsp_cull is not None:
        ctx.set_option(rt._ffi.RT_OPT_BSP_CULL, args.bsp_cull)
    if args.async_fold:
        ctx.set_option(rt._ffi.RT_OPT_ASYNC_FOLD, 1)
    t_mesh = time.perf_counter() - t0
    ctx.upload_mesh(mesh)
    # every rank builds its own replica of the scene's acceleration structure on its
    # GPU (replicas per GPU): no host build per rank on a shared host
    t1 = time.perf_counter()
    if args.host_build:
        accel = mesh.bsp_tree() if trav == "BSP" else mesh.bvh()
        ctx.upload_bsp(accel) if trav == "BSP" else ctx.upload_bvh(accel)
    else:
        accel = DeviceAccel(ctx, trav)
        ctx.build_bsp_device(20, 4) if trav == "BSP" else ctx.build_bvh_device(4)
    ctx.set_environment(wl.env)
    ctx.set_uniforms(rt.make_uniform(*cam, W, H, selection1=0))
    torch.cuda.synchronize(dev)
    t_accel = time.perf_counter() - t1
    setup_s = time.perf_counter() - t0

    lt = rt.local_tiles(W, H, nsplit)
    acc_local = torch.empty((lt * 64, 4), dtype=torch.float32, device=dev)
    ids_local = torch.empty((lt * 64,), dtype=torch.int32, device=dev)
    acc_all = ids_all = None
    # the tile gather: over RCCL through the library's C ABI (rt_comm_init /
    # rt_gather_tiles; torch.distributed only hands the communicator id around
    # and times the run), or, on the gloo rehearsal path, torch's gather
    native_gather = use_dist and backend == "nccl"
    if native_gather:
        uid = [rt.Context.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(world, rank, uid[0])
    elif use_dist and rank == 0:   # gather-to-root: only rank 0 receives the packed tiles
        acc_all = torch.empty((world * lt * 64, 4), dtype=torch.float32, device=dev)
        ids_all = torch.empty((world * lt * 64,), dtype=torch.int32, device=dev)
    frame = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
    frame_ids = torch.empty((H, W), dtype=torch.int32, device=dev)

    host_gather_s = [0.0]   # gloo rehearsal: the host-blocking torch gather, wall time per timed step

    def step(events=None):
        if events is not None:
            events[0].record(stream)
        ctx.render_tiles(wl.mode, trav, rank, nsplit, 0, spp, acc_local.data_ptr(), ids_local.data_ptr())
        if events is not None:
            events[1].record(stream)
        if native_gather:   # one grouped RCCL receive per peer on rank 0, then the unpack
            ctx.gather_tiles(W, H, acc_local.data_ptr(), ids_local.data_ptr(),
                             frame.data_ptr() if rank == 0 else None, frame_ids.data_ptr() if rank == 0 else None)
        elif use_dist:
            stream.synchronize()   # (the gather's .cpu() would wait for the render anyway)
            tg = time.perf_counter()
            tiling.gather_tiles(dist, acc_local, ids_local, acc_all, ids_all)   # (blocks the host: .cpu())
            if events is not None:
                host_gather_s[0] += time.perf_counter() - tg
            if rank == 0:
                ctx.unpack_tiles(W, H, world, acc_all.data_ptr(), ids_all.data_ptr(), frame.data_ptr(),
                                 frame_ids.data_ptr())
        elif share > 1:
            pass   # rank 0's share alone: no frame to assemble
        else:
            ctx.unpack_tiles(W, H, 1, acc_local.data_ptr(), ids_local.data_ptr(), frame.data_ptr(),
                             frame_ids.data_ptr())

    def progress(msg):   # stderr heartbeat: a long configuration (config 5 at 1024 spp) is not silent for minutes
        print(f"[bench rank {rank}] {msg} ({time.perf_counter() - t_start:.1f} s)", file=sys.stderr, flush=True)

    progress(f"setup done in {setup_s:.1f} s")
    # counted step (also the first warm-up): rays per step, deterministic
    step()
    counts = ctx.last_counts()
    progress("counted step done")
    # counting instantiation: traversal counters for the algorithmic bytes
    ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 1)
    step()
    detail = ctx.last_counts()
    ctx.set_option(rt._ffi.RT_OPT_DETAIL_COUNTERS, 0)
    progress("counting-instantiation step done")
    for _ in range(max(0, args.warmup - 1)):
        step()
        torch.cuda.synchronize(dev)
        progress("warm-up step done")

    rays = torch.tensor([counts["primary"] + counts["shadow"], counts["primary"], counts["shadow"],
                         counts["bounce"], algorithmic_bytes(detail, trav)],
                        dtype=torch.float64, device=dev)
    if use_dist:
        rays = all_reduce(dist, rays, dist.ReduceOp.SUM)
    rays = rays.cpu().numpy()

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    # HIP events around each k_path launch, on the stream it runs on (the
    # step's other kernels -- fold, unpack -- and the gather are excluded)
    ctx.set_option(rt._ffi.RT_OPT_KERNEL_TIMING, 1)
    ctx.kernel_time(reset=True)
    gather_timing = hasattr(rt._ffi.lib(), "rt_gather_time")   # (an A/B variant of an earlier tree has none)
    if gather_timing:
        ctx.gather_time(reset=True)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
        if args.progress:   # (a host sync per step: off unless asked, the steps stay back to back)
            torch.cuda.synchronize(dev)
            progress(f"timed step {k + 1}/{args.steps} done")
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_total, launches = ctx.kernel_time(reset=True)
    # the frame's assembly, per rank: rt_gather_tiles' RCCL transfers (HIP events;
    # under gloo the host-timed torch gather) and the unpack kernel (rank 0)
    xfer_total, unpack_total, _ = ctx.gather_time(reset=True) if gather_timing else (0.0, 0.0, 0)
    if use_dist and not native_gather:
        xfer_total = host_gather_s[0] * 1e3
    ctx.set_option(rt._ffi.RT_OPT_KERNEL_TIMING, 0)
    launches_per_step = launches // args.steps
    kern_ms = kern_total / max(1, launches)   # average k_path launch
    render_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    kern_ms_own = kern_ms   # this rank's own launches: the roofline pairs them with this rank's counters
    t = torch.tensor([elapsed, kern_ms, render_ms], dtype=torch.float64, device=dev)
    if use_dist:
        t = all_reduce(dist, t, dist.ReduceOp.MAX)
    elapsed, kern_ms, render_ms = [float(x) for x in t.cpu().numpy()]
    # per-rank step breakdown (ms per step): k_path, the gather's transfers, the unpack
    mine = torch.tensor([kern_total / args.steps, xfer_total / args.steps, unpack_total / args.steps],
                        dtype=torch.float64, device=dev)
    # every rank's culling kernel (RT_BSP_CULL_*; each rank probes its own share) and probes
    cull_mine = ctx.bsp_cull_in_use()
    probes_mine = ctx.bsp_cull_probes()
    cm = torch.tensor([cull_mine[0], cull_mine[1], cull_mine[2], probes_mine[0], probes_mine[1]],
                      dtype=torch.float64, device=dev)
    if use_dist:
        per_rank = all_gather(dist, mine, world)
        cull_ranks = all_gather(dist, cm, world)
    else:
        per_rank = mine.cpu().numpy()[None, :]
        cull_ranks = cm.cpu().numpy()[None, :]

    value = rays[0] * args.steps / elapsed / 1e6
    if rank == 0:
        # roofline of the dominant kernel (k_path<mode, traversal>): one launch on
        # one GPU -- rank 0's, with rank 0's own kernel time and the PMC summary of
        # rank 0's share (profiles/pmc_summary.json key _n<N>, measured with --rank-share N)
        bytes_per_launch = rays[4] / (world if use_dist else 1) / max(1, launches_per_step)
        # the culling mode the kernel ran (RT_BSP_CULL_AUTO: its probe's choice, made in
        # the first warm-up step) picks the instantiation and the PMC summary
        names = {0: "off", 1: "certified", 2: "fast", 3: "silhouette"}
        cull, probe_c, probe_s = cull_mine
        cull_name = names[cull] if trav == "BSP" else None
        if trav == "BSP" and probe_c > 0:
            cull_name = (f"auto: {cull_name} (probe: certified {probe_c:.3f}, silhouette {probe_s:.3f} ms per "
                         f"2^20 samples)")
        cull_per_rank = [names[int(r[0])] for r in cull_ranks] if trav == "BSP" else None
        probes_per_rank = [[int(r[3]), int(r[4])] for r in cull_ranks] if trav == "BSP" else None
        roof = roofline(pmc_key(W, H, spp, trav, nsplit, args.config, cull), kern_ms_own, bytes_per_launch, args.config,
                        f"k_path<{wl.mode},{trav}>")
        roof["launches_per_step"] = launches_per_step
        roof["render_ms"] = round(render_ms, 3)
        roof["kernel_ms_max_over_ranks"] = round(kern_ms, 3)
        cpu = None
        if not args.no_cpu_baseline and not use_dist and share == 1:
            cpu = cpu_baseline(wl, trav, mesh, accel, spp, W, H, args.cpu_budget)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"config {wl.number}: {wl.name} ({mesh.ntris} tris), "
                                   f"{trav}{' D20/leaf4' if trav == 'BSP' else ' leaf4'}, {W}x{H}, {spp} spp/step",
                       "resolution": [W, H], "spp": spp, "traversal": trav, "ntris": mesh.ntris, "mode": wl.mode,
                       "parallelism": f"tiles8x8/{nsplit}",
                       # RT_OPT_BSP_CULL: the subtree culling (a different k_path instantiation per mode)
                       "bsp_cull": cull_name,
                       # every rank's kernel and its probes (started, launches): each rank
                       # decides on its own share of the frame
                       "bsp_cull_per_rank": cull_per_rank,
                       "bsp_cull_probes_per_rank": probes_per_rank,
                       "accel_build": "host" if args.host_build else "device",
                       "world_size": dist.get_world_size() if use_dist else 1,
                       "backend": dist.get_backend() if use_dist else None,
                       "fold": "async (RT_OPT_ASYNC_FOLD)" if args.async_fold else "sync",
                       "gather": ("rt_gather_tiles (RCCL via the C ABI)" if native_gather else
                                  "torch.distributed.gather (gloo)" if use_dist else None),
                       **({"share": f"rank 0 of {share} (profiling: this GPU's part of the {share}-GPU frame)"}
                          if share > 1 else {})},
            "roofline": roof,
            "cpu_baseline": cpu,
            # where each rank's step goes (ms per step, HIP events on the stream the work
            # runs on; the gloo rehearsal's gather is host wall time): its k_path
            # launches, the tile gather's transfers, the unpack (rank 0); the rest of
            # ms_per_step is k_fold, the barrier and launch gaps
            "step_breakdown": {
                "k_path_ms": [round(float(x), 3) for x in per_rank[:, 0]],
                "gather_ms": [round(float(x), 3) for x in per_rank[:, 1]],
                "unpack_ms": [round(float(x), 3) for x in per_rank[:, 2]],
                "gather_timer": ("rt_gather_time (HIP events around the RCCL transfers)" if native_gather else
                                 "host wall time of torch.distributed.gather (gloo)" if use_dist else None),
            },
            "rays_per_step": {"primary": int(rays[1]), "shadow": int(rays[2]), "bounce": int(rays[3])},
            # this rank's counting step: every launch of one step summed (config 5
            # at 1024 spp is 8 launches of 128 spp, roofline.launches_per_step)
            "traversal_per_step": {k: detail[k] for k in ("node_interior", "node_leaf", "bvh_pops", "tri_tests",
                                                            "tri_accepts", "trips", "lane_steps",
                                                            "leaf_lane_steps", "node_trips", "leaf_trips",
                                                            "exact_tests", "exact_nodes", "shade_passes",
                                                            "shade_lanes", "trav_cycles", "shade_cycles",
                                                            "memwait_cycles", "subtree_culls")},
            "simd_lane_util": round(detail["lane_steps"] / max(1, 64 * detail["trips"]), 4),
            "setup_s": round(setup_s, 3),
            # setup_s split: the synthetic mesh (generated on the host), the acceleration
            # structure's build + the uniforms (on the device unless --host-build)
            "setup_breakdown_s": {"mesh": round(t_mesh, 3), "accel": round(t_accel, 3)},
        }
        print(json.dumps(line), flush=True)
        if args.dump_frame:
            np.savez(args.dump_frame, accum=frame.cpu().numpy(), ids=frame_ids.cpu().numpy().view(np.uint32))
    ctx.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
