"""Framebuffer tiling across ranks: one process per GPU, each
renders the interleaved 8x8 tiles t = l*nranks + rank (rt_render_tiles), the
packed tiles are all-gathered, and rank 0 scatters them into the frame
(rt_unpack_tiles).  The gather is the only collective of the path.

The packed layout (include/rt.h rt_render_tiles): local tile l occupies pixels
[l*64, l*64+64), row-major inside the tile; every rank holds
rt_tileset_local_tiles(W, H, nranks) tiles (padding tiles past the frame are
left untouched by the kernel and dropped by the unpack).
"""
import numpy as np

TILE = 8


def tile_grid(width, height):
    return (width + TILE - 1) // TILE, (height + TILE - 1) // TILE


def packed_pixel_coords(width, height, rank, nranks, local_tiles):
    """Global (x, y) of every packed pixel of `rank`, and whether it is inside
    the frame -- the mapping k_path / k_primary use in tileset mode."""
    tx_n, ty_n = tile_grid(width, height)
    lane = np.arange(64)
    l = np.arange(local_tiles)[:, None]
    t = l * nranks + rank
    x = (t % tx_n) * TILE + (lane & 7)[None, :]
    y = (t // tx_n) * TILE + (lane >> 3)[None, :]
    valid = (t < tx_n * ty_n) & (x < width) & (y < height)
    return x.reshape(-1), y.reshape(-1), valid.reshape(-1)


def unpack_numpy(width, height, nranks, local_tiles, packed_accum, packed_ids):
    """Host restatement of rt_unpack_tiles (for CPU tests of the protocol)."""
    frame = np.zeros((height, width, 4), np.float32)
    ids = np.zeros((height, width), np.uint32)
    for r in range(nranks):
        x, y, v = packed_pixel_coords(width, height, r, nranks, local_tiles)
        base = r * local_tiles * 64
        sl = slice(base, base + local_tiles * 64)
        frame[y[v], x[v]] = packed_accum[sl][v]
        ids[y[v], x[v]] = packed_ids[sl][v]
    return frame, ids


def gather_tiles(dist, acc_local, ids_local, acc_all, ids_all):
    """All-gather the ranks' packed tiles into rank-major buffers (every rank
    receives all; the frame is assembled on rank 0).  RCCL (backend "nccl")
    gathers straight into the flat tensors; gloo (CPU tests) through a list."""
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(acc_all, acc_local)
        dist.all_gather_into_tensor(ids_all, ids_local)
        return
    world = dist.get_world_size()
    if acc_local.is_cuda:   # gloo rehearsal of the device path: through host memory
        ha, hi = acc_all.cpu(), ids_all.cpu()
        dist.all_gather(list(ha.chunk(world)), acc_local.cpu())
        dist.all_gather(list(hi.chunk(world)), ids_local.cpu())
        acc_all.copy_(ha)
        ids_all.copy_(hi)
        return
    dist.all_gather(list(acc_all.chunk(world)), acc_local)
    dist.all_gather(list(ids_all.chunk(world)), ids_local)
