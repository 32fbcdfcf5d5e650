"""Multi-rank framebuffer tiling on CPU (gloo, world_size 2 and 3): every rank
renders its interleaved 8x8 tiles (the CPU oracle stands in for
rt_render_tiles here), the packed tiles go through the same gather bench.py
uses, and rank 0's unpacked frame equals the single-rank frame bit for bit --
PRNG seeds use global pixel coordinates, so the image does not depend on the
rank count."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import model

W, H, SPP = 42, 26, 2   # ragged: 6 x 4 tiles, partial right column and bottom row
CAM = ((277.0, 275.0, -570.0), (277.0, 275.0, 0.0), (0.0, 1.0, 0.0), 1.0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    import oracle_ffi as O
    m = O.load_obj(model("CornellBoxWithBlocks.obj"))
    return O, O.SceneRef(m, O.build_bsp(m))


def _render_rank(rank, nranks, lt):
    """Render this rank's tiles into the packed layout with the oracle."""
    O, sc = _scene()
    tiling = importlib.import_module("02562_raytracer_amd.tiling")
    u = O.make_uniform(*CAM, W, H)
    x, y, valid = tiling.packed_pixel_coords(W, H, rank, nranks, lt)
    acc = np.zeros((lt * 64, 4), np.float32)
    ids = np.full((lt * 64,), 0xFFFFFFFF, np.uint32)
    tx_n, _ = tiling.tile_grid(W, H)
    for l in range(lt):
        tx, ty = tiling.tile_of_seq(l * nranks + rank, tx_n)
        x0, y0 = tx * 8, ty * 8
        if y0 >= H:
            continue
        w, h = min(8, W - x0), min(8, H - y0)
        a, i, _ = O.render(sc, u, "W7E3", "BSP", (x0, y0, w, h), 0, SPP, nthreads=1)
        sl = slice(l * 64, l * 64 + 64)
        v = valid[sl]
        acc[sl][v] = a.reshape(-1, 4)
        ids[sl][v] = i.reshape(-1)
    return acc, ids


def _worker(rank, nranks, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=nranks)
    try:
        tiling = importlib.import_module("02562_raytracer_amd.tiling")
        lt = (tiling.tile_grid(W, H)[0] * tiling.tile_grid(W, H)[1] + nranks - 1) // nranks
        acc, ids = _render_rank(rank, nranks, lt)
        acc_l = torch.from_numpy(acc)
        ids_l = torch.from_numpy(ids.view(np.int32))
        acc_all = ids_all = None   # gather-to-root: only rank 0 receives
        if rank == 0:
            acc_all = torch.empty((nranks * lt * 64, 4), dtype=torch.float32)
            ids_all = torch.empty((nranks * lt * 64,), dtype=torch.int32)
        tiling.gather_tiles(dist, acc_l, ids_l, acc_all, ids_all)
        if rank == 0:
            frame, fids = tiling.unpack_numpy(W, H, nranks, lt, acc_all.numpy(), ids_all.numpy().view(np.uint32))
            np.save(os.path.join(outdir, "frame.npy"), frame)
            np.save(os.path.join(outdir, "ids.npy"), fids)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nranks", [2, 3])
def test_tiled_gather_equals_single_rank(nranks, tmp_path, oracle):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    mp.spawn(_worker, args=(nranks, _free_port(), str(tmp_path)), nprocs=nranks, join=True)
    frame = np.load(tmp_path / "frame.npy")
    fids = np.load(tmp_path / "ids.npy")
    O, sc = _scene()
    ref, rids, _ = O.render(sc, O.make_uniform(*CAM, W, H), "W7E3", "BSP", (0, 0, W, H), 0, SPP, nthreads=4)
    assert np.array_equal(fids, rids.reshape(H, W))
    assert np.array_equal(frame.view(np.uint32), ref.reshape(H, W, 4).view(np.uint32))


def test_local_tiles_matches_library(rt):
    tiling = importlib.import_module("02562_raytracer_amd.tiling")
    for (w, h, n) in [(1920, 1080, 1), (1920, 1080, 8), (42, 26, 3), (7, 5, 2), (3840, 2160, 7)]:
        tx, ty = tiling.tile_grid(w, h)
        assert rt.local_tiles(w, h, n) == (tx * ty + n - 1) // n
        # every in-frame pixel is owned by exactly one (rank, slot)
        seen = np.zeros((h, w), np.int32)
        lt = rt.local_tiles(w, h, n)
        for r in range(n):
            x, y, v = tiling.packed_pixel_coords(w, h, r, n, lt)
            np.add.at(seen, (y[v], x[v]), 1)
        assert (seen == 1).all()
