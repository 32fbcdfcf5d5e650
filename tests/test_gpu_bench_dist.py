"""The N>1 path of bench.py on the one GPU of the box: two ranks launched by
torch.distributed.run exactly as the driver launches the 8-GPU bench, pinned to
device 0 (RT_BENCH_DEVICE=0) with the gloo backend (RCCL refuses two ranks on one
GPU).  Each rank renders its interleaved 8x8 tiles (rt_render_tiles), the packed
tiles are gathered to rank 0 (tiling.gather_tiles), rank 0 unpacks them
(rt_unpack_tiles): the assembled frame equals the 1-rank frame bit for bit, and
both equal the CPU oracle.  Only the RCCL transport itself is left to the 8-GPU
node."""
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


def _bench(nproc, out):
    args = ["bench.py", "--gpus", str(nproc), "--steps", "1", "--warmup", "1", "--config", "2", "--spp", str(SPP),
            "--width", str(W), "--height", str(H), "--no-cpu-baseline", "--dump-frame", out]
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, RT_BENCH_DEVICE="0", RT_BENCH_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0]), np.load(out)


def test_two_rank_bench_frame_equals_one_rank(tmp_path, rt, oracle):
    one, f1 = _bench(1, str(tmp_path / "n1.npz"))
    two, f2 = _bench(2, str(tmp_path / "n2.npz"))
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
    assert eight["rays_per_step"] == one["rays_per_step"]
    assert np.array_equal(f1["ids"], f8["ids"])
    assert np.array_equal(f1["accum"].view(np.uint32), f8["accum"].view(np.uint32))
