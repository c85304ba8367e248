"""Multi-rank sharding path on CPU (gloo, world_size 2 and 3): each rank produces its tile rows'
hit records (from the oracle — no GPU here), packs them, gathers to rank 0 and de-interleaves;
the result must equal the single-rank frame record for record."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _records(ref, pixel_idx):
    import torch

    axis = ref["axis"][pixel_idx]
    step = ref["pos"][pixel_idx] - ref["last"][pixel_idx]  # the last step (one axis, +-1)
    neg = (axis < 3) & (step[np.arange(len(axis)), np.minimum(axis, 2)] < 0)
    info = (ref["hit"][pixel_idx].astype(np.uint32) << 31) | (axis.astype(np.uint32) & 3) << 16 | (neg.astype(np.uint32) << 18)
    info |= (ref["flags"][pixel_idx] & 0xFFF).astype(np.uint32)
    ps = np.concatenate([ref["pos"][pixel_idx], ref["steps"][pixel_idx, None]], 1).astype(np.int32)
    return {"pos_steps": torch.from_numpy(ps), "t": torch.from_numpy(ref["t"][pixel_idx].astype(np.float32)),
            "info": torch.from_numpy(info.view(np.int32))}


def _worker(rank, world, port, W, H, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from oracle import oracle as O
    from raytracing_test_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T = O.Tree.reference_world()
    cam = O.normalize([1, -0.45, 1])
    rows = shard.shard_pixel_rows(H, rank, world)
    pix = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1)
    ref = T.cast_frame((4, 90, 4), cam, W, H, 300, pixels=pix, nthreads=2)
    n_pad = shard.max_shard_count(W, H, world)
    flat = shard.pack(_records(ref, np.arange(len(pix))), n_pad)
    got = shard.gather_to_root(flat, rank, world)
    if rank == 0:
        full = shard.reassemble(got, W, H, world)
        q.put({k: v.numpy().copy() for k, v in full.items()})
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tile_row_shard_gather_reassemble(world):
    import multiprocessing as mp

    sys.path.insert(0, ROOT)
    from oracle import oracle as O

    W, H = 96, 70  # 9 tile rows, the last one partial
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in ps:
        p.start()
    full = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    T = O.Tree.reference_world()
    ref = T.cast_frame((4, 90, 4), O.normalize([1, -0.45, 1]), W, H, 300)
    want = _records(ref, np.arange(W * H))
    for k in want:
        assert np.array_equal(full[k], want[k].numpy()), k


def _wire_worker(rank, world, port, W, H, origins, q, all_to_all=False, compact=False):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist

    import wire_ref
    from oracle import oracle as O
    from raytracing_test_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T = O.Tree.reference_world()
    cam = O.normalize([1, -0.45, 1])
    rows = shard.shard_pixel_rows(H, rank, world)
    pix = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1)
    # one multi-frame record buffer per rank: its tile rows of every frame, frame after frame
    parts = []
    for org in origins:
        ref = T.cast_frame(org, cam, W, H, 300, pixels=pix, nthreads=2)
        r = _records(ref, np.arange(len(pix)))
        cell = np.trunc(np.asarray(org, np.float32)).astype(np.int32)
        if compact:
            parts.append(wire_ref.pack_compact(r["pos_steps"].numpy(), r["info"].numpy().view(np.uint32), cell[None, :]))
        else:
            parts.append(wire_ref.pack(r["pos_steps"].numpy(), r["t"].numpy(), r["info"].numpy().view(np.uint32), cell[None, :]))
    mine = np.concatenate(parts)
    wb = mine.shape[1]
    if all_to_all:
        # frame f displayed by rank f (frames = ranks): my rows of frame f go to rank f
        counts = [shard.shard_count(W, H, r, world) for r in range(world)]
        recv = torch.zeros((W * H, wb), dtype=torch.uint8)
        dist.all_to_all_single(recv, torch.from_numpy(mine), output_split_sizes=counts, input_split_sizes=[len(pix)] * world)
        q.put((rank, recv.numpy().copy()))
    else:
        n_pad = shard.max_shard_count(W, H, world) * len(origins)
        wire = torch.zeros((n_pad, 12), dtype=torch.uint8)
        wire[: len(mine)] = torch.from_numpy(mine)
        got = shard.gather_to_root(wire, rank, world)
        if rank == 0:
            q.put([g.numpy().copy() for g in got])
    dist.destroy_process_group()


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("world", [2, 3])
def test_wire_all_to_all_frame_per_rank(world, compact):
    """bench.py's N>1 exchange: N frames per step, frame f displayed by rank f — one all-to-all of
    wire records (12 B, or the 8-B compact records of integral camera positions, whose receiver rebuilds
    each pixel's ray: tests/wire_ref.py); every rank's frame, unpacked, equals its single-rank cast."""
    import multiprocessing as mp

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import wire_ref
    from oracle import oracle as O
    from raytracing_test_amd import shard

    W, H = 64, 44
    origins = [(4.0 + 64.0 * f, 90.0, 4.0 + 64.0 * f) for f in range(world)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_wire_worker, args=(r, world, port, W, H, origins, q, True, compact)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    T = O.Tree.reference_world()
    cam = O.normalize([1, -0.45, 1])
    counts = [shard.shard_count(W, H, r, world) for r in range(world)]
    offs = np.concatenate([[0], np.cumsum(counts)])
    for f, org in enumerate(origins):
        want = _records(T.cast_frame(org, cam, W, H, 300), np.arange(W * H))
        cell = np.trunc(np.asarray(org, np.float32)).astype(np.int32)[None, :]
        for r in range(world):
            rows = shard.shard_pixel_rows(H, r, world)
            idx = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1)
            if compact:
                ppx, ppy = O.proj_plane(W, H)
                dirs = np.array([O.pixel_dir(cam, ppx, ppy, W, H, int(i % W), int(i // W)) for i in idx], np.float32)
                ps_, t_, info_ = wire_ref.unpack_compact(got[f][offs[r]:offs[r + 1]], np.repeat(np.asarray([org], np.float32), len(idx), 0),
                                                         dirs, 300)
            else:
                ps_, t_, info_ = wire_ref.unpack(got[f][offs[r]:offs[r + 1]], cell, 300)
            assert np.array_equal(ps_, want["pos_steps"].numpy()[idx]), (f, r)
            assert np.array_equal(t_, want["t"].numpy()[idx]), (f, r)
            assert np.array_equal(info_.view(np.int32), want["info"].numpy()[idx]), (f, r)


@pytest.mark.parametrize("world", [2, 3])
def test_wire_gather_multi_frame(world):
    """The N>1 step: each rank packs its tile rows of several frames into 12-B wire records, rank 0
    gathers and unpacks them; every frame equals its single-rank cast record for record."""
    import multiprocessing as mp

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import wire_ref
    from oracle import oracle as O
    from raytracing_test_amd import shard

    W, H = 64, 44  # 6 tile rows, the last one partial
    origins = [(4.0, 90.0, 4.0), (68.0, 90.0, 68.0), (-30.5, 70.25, 12.75)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_wire_worker, args=(r, world, port, W, H, origins, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    T = O.Tree.reference_world()
    cam = O.normalize([1, -0.45, 1])
    for f, org in enumerate(origins):
        ref = T.cast_frame(org, cam, W, H, 300)
        want = _records(ref, np.arange(W * H))
        cell = np.trunc(np.asarray(org, np.float32)).astype(np.int32)[None, :]
        full = {k: np.zeros_like(v.numpy()) for k, v in want.items()}
        for r in range(world):
            rows = shard.shard_pixel_rows(H, r, world)
            n = len(rows) * W
            ps_, t_, info_ = wire_ref.unpack(got[r][f * n:(f + 1) * n], cell, 300)
            idx = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1)
            full["pos_steps"][idx], full["t"][idx], full["info"][idx] = ps_, t_, info_.view(np.int32)
        for k in want:
            assert np.array_equal(full[k], want[k].numpy()), (f, k)


def test_shard_geometry():
    sys.path.insert(0, ROOT)
    from raytracing_test_amd import shard

    for H in (1080, 70, 8, 3):
        for world in (1, 2, 3, 8):
            rows = np.concatenate([shard.shard_pixel_rows(H, r, world) for r in range(world)])
            assert np.array_equal(np.sort(rows), np.arange(H))
