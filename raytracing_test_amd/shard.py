"""Frame sharding across GPUs: interleaved 8-pixel tile rows, hit records gathered to
rank 0 over torch.distributed (RCCL on GPUs, gloo in the CPU tests), then de-interleaved.

Row r of 8-pixel tiles belongs to rank r mod N: sky / horizon rows cost more than ground rows, so
contiguous bands would load-imbalance.  Every rank's buffer is padded to the largest shard so the
collective sees equal sizes.
"""
import numpy as np

TILE = 8


def tile_rows(height, rank, world):
    return list(range(rank, (height + TILE - 1) // TILE, world))


def shard_pixel_rows(height, rank, world):
    """global pixel rows (from the bottom) of this rank's records, in record order"""
    rows = [np.arange(t * TILE, min(height, t * TILE + TILE)) for t in tile_rows(height, rank, world)]
    return np.concatenate(rows) if rows else np.zeros(0, np.int64)


def shard_count(width, height, rank, world):
    return len(shard_pixel_rows(height, rank, world)) * width


def max_shard_count(width, height, world):
    return max(shard_count(width, height, r, world) for r in range(world))


def alloc_flat(n_pad, device):
    """one flat int32 record buffer laid out as pack() makes it, plus the hit views the kernel writes"""
    import torch

    flat = torch.zeros(6 * n_pad, dtype=torch.int32, device=device)
    return flat, unpack(flat, n_pad, n_pad)


def pack(hits, n_pad):
    """hit buffers {pos_steps (n,4) i32, t (n,) f32, info (n,) i32} -> one flat int32 tensor of 6*n_pad"""
    import torch

    ps, t, info = hits["pos_steps"], hits["t"], hits["info"]
    n = ps.shape[0]
    flat = torch.zeros(6 * n_pad, dtype=torch.int32, device=ps.device)
    flat[: 4 * n] = ps.reshape(-1)
    flat[4 * n_pad: 4 * n_pad + n] = t.view(torch.int32)
    flat[5 * n_pad: 5 * n_pad + n] = info.view(torch.int32)
    return flat


def unpack(flat, n_pad, n):
    import torch

    return {"pos_steps": flat[: 4 * n].view(n, 4), "t": flat[4 * n_pad: 4 * n_pad + n].view(torch.float32),
            "info": flat[5 * n_pad: 5 * n_pad + n]}


def gather_to_root(flat, rank, world, bufs=None):
    """torch.distributed.gather of equal-size flat records to rank 0 (returns the list on rank 0)"""
    import torch
    import torch.distributed as dist

    if world == 1:
        return [flat]
    if rank == 0 and bufs is None:
        bufs = [torch.empty_like(flat) for _ in range(world)]
    dist.gather(flat, bufs if rank == 0 else None, dst=0)
    return bufs if rank == 0 else None


def reassemble(flats, width, height, world):
    """rank 0: gathered flat records -> full-frame {pos_steps, t, info} in pixel order (row*width+px)"""
    import torch

    n_pad = max_shard_count(width, height, world)
    dev = flats[0].device
    full = {"pos_steps": torch.empty((width * height, 4), dtype=torch.int32, device=dev),
            "t": torch.empty(width * height, dtype=torch.float32, device=dev),
            "info": torch.empty(width * height, dtype=torch.int32, device=dev)}
    for r, flat in enumerate(flats):
        rows = torch.from_numpy(shard_pixel_rows(height, r, world)).to(dev)
        n = len(rows) * width
        part = unpack(flat, n_pad, n)
        idx = (rows[:, None] * width + torch.arange(width, device=dev)[None, :]).reshape(-1)
        for k in full:
            full[k][idx] = part[k]
    return full
