"""Framebuffer tiling across ranks: one process per GPU, each
renders the interleaved 8x8 tiles at sequence positions s = l*nranks + rank
(rt_render_tiles; tile_of_seq: rows rotated by their index mod 8), the
packed tiles are gathered to rank 0, and rank 0 scatters them into the frame
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


def tile_of_seq(s, tx_n):
    """Tile (tx, ty) at sequence position s (include/rt.h rt_tileset): row-major,
    each row rotated by its index mod 8 (frames under 8 tiles wide: not rotated),
    so the ranks' tiles (s % nranks) form diagonal stripes instead of whole
    columns when nranks divides 8 and the tile columns."""
    ty = s // tx_n
    r = (ty & 7) if tx_n >= 8 else 0 * ty
    return (s % tx_n + r) % tx_n, ty


def packed_pixel_coords(width, height, rank, nranks, local_tiles):
    """Global (x, y) of every packed pixel of `rank`, and whether it is inside
    the frame -- the mapping k_path / k_primary use in tileset mode."""
    tx_n, ty_n = tile_grid(width, height)
    lane = np.arange(64)
    l = np.arange(local_tiles)[:, None]
    t = l * nranks + rank
    tx, ty = tile_of_seq(t, tx_n)
    x = tx * TILE + (lane & 7)[None, :]
    y = ty * TILE + (lane >> 3)[None, :]
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
    """Gather the ranks' packed tiles to rank 0, rank-major into acc_all /
    ids_all (None on the other ranks): SURVEY.md 8(e)'s gather-to-root -- only
    the rank that assembles the frame receives.  RCCL (backend "nccl") gathers
    device tensors in place (point-to-point over xGMI); gloo through host memory
    (the CPU tests, and the one-GPU rehearsal of the device path)."""
    world = dist.get_world_size()
    root = dist.get_rank() == 0
    if dist.get_backend() == "nccl":
        dist.gather(acc_local, list(acc_all.chunk(world)) if root else None, dst=0)
        dist.gather(ids_local, list(ids_all.chunk(world)) if root else None, dst=0)
        return
    if acc_local.is_cuda:   # gloo rehearsal of the device path: through host memory
        ha = acc_all.cpu() if root else None
        hi = ids_all.cpu() if root else None
        dist.gather(acc_local.cpu(), list(ha.chunk(world)) if root else None, dst=0)
        dist.gather(ids_local.cpu(), list(hi.chunk(world)) if root else None, dst=0)
        if root:
            acc_all.copy_(ha)
            ids_all.copy_(hi)
        return
    dist.gather(acc_local, list(acc_all.chunk(world)) if root else None, dst=0)
    dist.gather(ids_local, list(ids_all.chunk(world)) if root else None, dst=0)

