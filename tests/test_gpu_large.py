"""Node addressing beyond 4 GiB: a tree of more than 2^28 nodes (the 32-bit buffer-offset reach of the
narrow kernel instance) must be cast through 64-bit node addresses and give the oracle's results
bit for bit (castRayFromCam / getBlock semantics, src/ray_caster.cpp:54-87,
src/voxel_data/tetrahexa_tree.cpp:113-157, at any tree size).

The tree: 7 levels (16384^3), 4096^2 columns with random tops in [1, 1300) built on the GPU
(svo_build_heightfield_gpu): ~3.3e8 nodes, ~5 GB of nodes.  Rays fall steeply onto the high-x,
high-z corner, whose bricks sit at the end of the breadth-first array (node indices above 2^28).
The oracle holds only a 128^2-column window around them (its reference-format tree of the whole
field would not fit its pools); rays are shifted into the window by whole voxels, which leaves
every DDA quantity unchanged (dda_axis depends on origin - trunc(origin) only)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C, R, WIN = 4096, 1300, 128


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def wide_setup(rt, oracle_mod, torch_cuda):
    h = np.random.default_rng(28).integers(1, R, size=(C, C)).astype(np.int32)
    t = rt.Tree.heightfield_gpu(7, h, 0)
    x0 = z0 = C - WIN - 16
    T = oracle_mod.Tree.heightfield(7, np.ascontiguousarray(h[x0:x0 + WIN, z0:z0 + WIN]), native=False)
    yield t, T, x0, z0
    del t


def test_tree_exceeds_narrow_reach(rt, wide_setup):
    t, _, _, _ = wide_setup
    info = t.info()
    assert info.n_nodes > 2 ** 28, info.n_nodes  # beyond 32-bit byte offsets of 16-B nodes


def test_wide_tree_rays_vs_oracle(rt, torch_cuda, wide_setup):
    torch = torch_cuda
    t, T, x0, z0 = wide_setup
    rng = np.random.default_rng(5)
    n = 3000
    org = np.stack([rng.uniform(x0 + 40, x0 + WIN - 40, n), rng.uniform(1310.0, 1390.0, n), rng.uniform(z0 + 40, z0 + WIN - 40, n)],
                   1).astype(np.float32)
    d = np.stack([rng.uniform(-0.03, 0.03, n), -np.ones(n), rng.uniform(-0.03, 0.03, n)], 1).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[::9, 0] = 0.0  # exact zero components (NaN deltaPos for integral origins on that axis)
    org[::13, 0] = np.round(org[::13, 0])
    go, gd = torch.from_numpy(org).cuda(), torch.from_numpy(d).cuda()
    shift = np.array([x0, 0, z0], np.int32)
    ref = {k: [] for k in ("pos", "last", "steps", "hit", "flags", "color", "t")}
    for o, dd in zip(org - shift.astype(np.float32), d):
        r = T.cast_ray(o, dd, 16384)
        assert r.err == 0
        ref["pos"].append(np.array(r.pos) + shift)
        ref["last"].append(np.array(r.last) + shift)
        ref["steps"].append(r.steps)
        ref["hit"].append(r.hit)
        ref["flags"].append(r.flags)
        ref["color"].append(r.color)
        ref["t"].append(r.t)
    pal = t.palette()
    pf = np.array([p[0] for p in pal], np.uint32)
    pc = np.array([p[1] for p in pal], np.uint64)
    for flags in (0, rt.CAST_ITERATIVE):
        g = rt.decode_hits(t.cast_rays(gd, go, steps=16384, flags=flags))
        assert np.array_equal(g["pos"], np.array(ref["pos"])), flags
        assert np.array_equal(g["last_pos"], np.array(ref["last"])), flags
        assert np.array_equal(g["steps"], np.array(ref["steps"])), flags
        assert np.array_equal(g["hit"], np.array(ref["hit"]) != 0), flags
        mid = np.where(g["hit"], g["material"], 0)
        assert np.array_equal(pf[mid], np.array(ref["flags"], np.uint32)) and np.array_equal(pc[mid], np.array(ref["color"], np.uint64))
        assert np.array_equal(g["t"], np.array(ref["t"]).astype(np.float32)), flags
    assert g["hit"].all()  # every ray lands on a column top
    # the rays ended in bricks addressed beyond 2^28 nodes (4 GiB of 16-B nodes)
    idx = t.node_indices(g["pos"])
    assert (idx >= 2 ** 28).mean() > 0.9, np.percentile(idx, [0, 50, 100])
