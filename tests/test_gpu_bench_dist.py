"""The N>1 path of bench.py on the one GPU of the box: two ranks launched by
torch.distributed.run exactly as the driver launches the 8-GPU bench, pinned to
device 0 (RT_BENCH_DEVICE=0) with the gloo backend (RCCL refuses two ranks on one
GPU).  Each rank renders its interleaved 8x8 tiles (rt_render_tiles), the packed
tiles are gathered to rank 0 (tiling.gather_tiles), rank 0 unpacks them
(rt_unpack_tiles): the assembled frame equals the 1-rank frame bit for bit, and
both equal the CPU oracle.  With RCCL (one rank on the box's GPU) the gather is
the library's own (rt_gather_tiles, through the C ABI).  Only RCCL between
GPUs is left to the 8-GPU node."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from parity_util import compare

pytestmark = pytest.mark.gpu

W, H, SPP = 200, 136, 2   # 25 x 17 tiles: ragged split between the ranks


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(nproc, out, launcher=None, backend="gloo"):
    args = ["bench.py", "--gpus", str(nproc), "--steps", "1", "--warmup", "1", "--config", "2", "--spp", str(SPP),
            "--width", str(W), "--height", str(H), "--no-cpu-baseline", "--dump-frame", out]
    if nproc > 1 if launcher is None else launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, RT_BENCH_DEVICE="0", RT_BENCH_DIST_BACKEND=backend, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0]), np.load(out)


def _check_breakdown(line, world):
    # the per-rank step breakdown the N>1 line carries: every rank's
    # k_path time, its part of the gather, the unpack on rank 0; none exceeds the step
    b = line["step_breakdown"]
    assert len(b["k_path_ms"]) == len(b["gather_ms"]) == len(b["unpack_ms"]) == world
    for r in range(world):
        assert b["k_path_ms"][r] > 0
        assert b["k_path_ms"][r] + b["gather_ms"][r] + b["unpack_ms"][r] <= line["ms_per_step"] * 1.05 + 0.5, b
        if r > 0:
            assert b["gather_ms"][r] > 0 and b["unpack_ms"][r] == 0, b
    assert b["unpack_ms"][0] > 0
    # rank 0's k_path launches are the line's roofline kernel time x launches per step
    roof = line["roofline"]
    assert abs(b["k_path_ms"][0] - roof["kernel_ms"] * roof["launches_per_step"]) <= 0.01 + 1e-3 * b["k_path_ms"][0]


def test_two_rank_bench_frame_equals_one_rank(tmp_path, rt, oracle):
    one, f1 = _bench(1, str(tmp_path / "n1.npz"))
    two, f2 = _bench(2, str(tmp_path / "n2.npz"))
    _check_breakdown(one, 1)
    _check_breakdown(two, 2)
    assert two["step_breakdown"]["gather_timer"].startswith("host wall time")
    assert one["config"]["bsp_cull"] == "certified"
    # every rank's culling kernel and probes in the line (W7E3 has no silhouette form:
    # certified, no probe), and the ranks' BSPs built on the device
    assert one["config"]["bsp_cull_per_rank"] == ["certified"]
    assert two["config"]["bsp_cull_per_rank"] == ["certified"] * 2
    assert two["config"]["bsp_cull_probes_per_rank"] == [[0, 0]] * 2
    assert two["config"]["accel_build"] == "device"
    assert two["n_gpus"] == 2 and two["config"]["world_size"] == 2 and two["config"]["backend"] == "gloo"
    assert one["config"]["world_size"] == 1
    # every ray counted once across the ranks
    assert two["rays_per_step"] == one["rays_per_step"]
    assert np.array_equal(f1["ids"], f2["ids"])
    assert np.array_equal(f1["accum"].view(np.uint32), f2["accum"].view(np.uint32))
    # and the frame is the reference path's (CPU oracle)
    wl = __import__("importlib").import_module("02562_raytracer_amd.configs").WORKLOADS[2]
    m = oracle.load_obj(os.path.join(ROOT, "assets", "models", "CornellBoxWithBlocks.obj"))
    sc = oracle.SceneRef(m, oracle.build_bsp(m))
    o = oracle.render(sc, oracle.make_uniform(*wl.camera, W, H), wl.mode, "BSP", (0, 0, W, H), 0, SPP)
    linf, bits, idm = compare((f2["accum"], f2["ids"], None), o)
    assert idm == 0 and bits == 0, (idm, bits, linf)


def test_eight_rank_bench_frame_equals_one_rank(tmp_path):
    # the driver's largest launch (8 ranks), rehearsed on the one GPU: 425 tiles
    # dealt to 8 ranks (53 or 54 each), gathered to rank 0 and unpacked
    one, f1 = _bench(1, str(tmp_path / "n1.npz"))
    eight, f8 = _bench(8, str(tmp_path / "n8.npz"))
    assert eight["n_gpus"] == 8 and eight["config"]["world_size"] == 8
    assert eight["config"]["bsp_cull_per_rank"] == ["certified"] * 8
    assert len(eight["config"]["bsp_cull_probes_per_rank"]) == 8
    _check_breakdown(eight, 8)
    assert eight["rays_per_step"] == one["rays_per_step"]
    assert np.array_equal(f1["ids"], f8["ids"])
    assert np.array_equal(f1["accum"].view(np.uint32), f8["accum"].view(np.uint32))


def test_one_rank_rccl_bench_frame_equals_plain_run(tmp_path):
    # the driver's launch form with one process: torch.distributed.run opens an
    # RCCL ("nccl") process group on device 0 (bench.py init_process_group with
    # device_id), which hands rank 0's communicator id to the library
    # (rt_comm_unique_id / rt_comm_init); the packed tiles go through the C ABI's
    # RCCL gather and unpack (rt_gather_tiles); the counters and times go
    # through torch's RCCL all_reduce.  The frame equals the plain 1-process run's.
    one, f1 = _bench(1, str(tmp_path / "n1.npz"))
    nc, fn = _bench(1, str(tmp_path / "nccl1.npz"), launcher=True, backend="nccl")
    assert nc["config"]["backend"] == "nccl" and nc["config"]["world_size"] == 1
    _check_breakdown(nc, 1)
    assert nc["step_breakdown"]["gather_timer"].startswith("rt_gather_time")
    assert nc["step_breakdown"]["gather_ms"][0] > 0   # rank 0's copy of its own tiles
    assert nc["config"]["gather"].startswith("rt_gather_tiles")
    assert one["config"]["backend"] is None
    assert nc["rays_per_step"] == one["rays_per_step"]
    assert np.array_equal(f1["ids"], fn["ids"])
    assert np.array_equal(f1["accum"].view(np.uint32), fn["accum"].view(np.uint32))


def test_rank_share_renders_rank0_tiles(tmp_path):
    # --rank-share N: one process renders rank 0's share of an N-rank split (the
    # profiling form of one GPU's work in the N-GPU bench); its rays are rank 0's
    # part of the 1-rank total
    one, _ = _bench(1, str(tmp_path / "n1.npz"))
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "1", "--config", "2", "--spp",
                        str(SPP), "--width", str(W), "--height", str(H), "--no-cpu-baseline", "--rank-share", "4"],
                       cwd=ROOT, env=dict(os.environ, OMP_NUM_THREADS="2"), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert line["config"]["parallelism"] == "tiles8x8/4" and "share" in line["config"]
    assert 0 < line["rays_per_step"]["primary"] < one["rays_per_step"]["primary"]
    # 25 x 17 = 425 whole tiles (200 and 136 are multiples of 8); rank 0 of 4
    # holds tiles 0, 4, ..., 424: 107 tiles, one primary ray per pixel-iteration
    assert line["rays_per_step"]["primary"] == 107 * 64 * SPP


def test_config5_setup_under_a_second_and_per_rank_cull(tmp_path):
    """config 5's 10M-triangle BSP is built on the device
    (rt_build_bsp_device; the host build took 3.3 s per rank), and the W9E1 line
    reports each rank's auto-culling choice.  Two ranks over gloo on the one GPU,
    a small frame of the real config-5 scene."""
    env = dict(os.environ, RT_BENCH_DEVICE="0", RT_BENCH_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "2",
           "--config", "5", "--spp", "16", "--width", "1920", "--height", "1080", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    print(json.dumps({k: line[k] for k in ("setup_s", "setup_breakdown_s", "value")}),
          line["config"]["bsp_cull_per_rank"], line["config"]["bsp_cull_probes_per_rank"])
    assert line["config"]["accel_build"] == "device"
    assert line["setup_breakdown_s"]["accel"] < 1.0
    assert len(line["config"]["bsp_cull_per_rank"]) == 2
    assert all(c in ("certified", "silhouette") for c in line["config"]["bsp_cull_per_rank"])
    # each rank probed once (the first step's four launches) and decided by the timed step
    assert line["config"]["bsp_cull_probes_per_rank"] == [[1, 4], [1, 4]]
