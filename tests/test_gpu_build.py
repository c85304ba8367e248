"""On-device world generation + tree build: svo_build_terrain_gpu /
svo_build_heightfield_gpu must emit the host builder's node and material arrays byte for byte."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _same(a, b, label):
    na, ma = a.export()
    nb, mb = b.export()
    assert na.shape == nb.shape, "%s: %d vs %d nodes" % (label, len(na), len(nb))
    assert np.array_equal(na, nb), "%s: node arrays differ at %d records" % (label, int((na != nb).any(1).sum()))
    assert np.array_equal(ma, mb), label
    ia, ib = a.info(), b.info()
    assert list(ia.nodes_per_level) == list(ib.nodes_per_level) and ia.n_bricks == ib.n_bricks, label


@pytest.mark.parametrize("view", [0, 1])
@pytest.mark.parametrize("levels,W,L", [(3, 64, 64), (4, 200, 200), (5, 1000, 700), (6, 1024, 1024)])
def test_terrain_gpu_equals_host(rt, torch_cuda, levels, W, L, view):
    g, h = rt.Tree.terrain_gpu(levels, W, L, 0, view=view), rt.Tree.terrain(levels, W, L, view=view)
    assert g.info().view == view
    _same(g, h, "terrain L%d %dx%d view %d" % (levels, W, L, view))
    # the column-ceiling tables the casts read (ceilings, pairs, per-level quads) are the same for both builders
    h.upload(0)
    lg, cg, pg = g.device_ceilings()
    lh, ch, ph = h.device_ceilings()
    assert lg == lh and np.array_equal(cg, ch) and np.array_equal(pg, ph)
    assert np.array_equal(g.device_ceiling_quads(), h.device_ceiling_quads())


def test_heightfield_gpu_equals_host(rt, torch_cuda):
    rng = np.random.default_rng(4)
    for levels, shape, hi in ((3, (64, 64), 62), (4, (256, 100), 254), (4, (33, 250), 40)):
        h = rng.integers(0, hi + 1, size=shape).astype(np.int32)
        h[: shape[0] // 2, : shape[1] // 3] = rng.integers(20, 24)  # flat plateaus: uniform regions
        _same(rt.Tree.heightfield_gpu(levels, h, 0), rt.Tree.heightfield(levels, h), "heightfield %s" % (shape,))
    with pytest.raises(RuntimeError):
        rt.Tree.heightfield_gpu(3, np.full((8, 8), 63, np.int32), 0)  # top + 1 reaches the extent


def test_terrain_gpu_casts_and_c3_build_time(rt, torch_cuda):
    """the GPU-built C3 tree is already uploaded: casting it equals casting the host-built tree"""
    t0 = time.perf_counter()
    g = rt.Tree.terrain_gpu(6, 4096, 4096, 0)
    torch_cuda.cuda.synchronize()
    dt = time.perf_counter() - t0
    h = rt.Tree.terrain(6, 4096, 4096).upload(0)
    _same(g, h, "C3")
    cam = rt.normalize((1.0, -0.45, 1.0))
    a, b = g.cast_frame((4.0, 90.0, 4.0), cam, 960, 540, 16384), h.cast_frame((4.0, 90.0, 4.0), cam, 960, 540, 16384)
    for k in ("pos_steps", "t", "info"):
        assert torch_cuda.equal(a[k], b[k]), k
    print("C3 GPU build %.3f s" % dt)


def test_checkpoint_of_gpu_tree_casts_the_same(rt, torch_cuda, tmp_path):
    """a GPU-built tree saved (svo_tree_save) and loaded back (svo_tree_load) casts bit for bit like the
    original once uploaded (the checkpoint replaces a rebuild at start-up)"""
    g = rt.Tree.terrain_gpu(6, 2048, 2048, 0)
    p = str(tmp_path / "c3.svo")
    g.save(p)
    h = rt.Tree.load(p).upload(0)
    cam = rt.normalize((1.0, -0.45, 1.0))
    a, b = g.cast_frame((4.0, 90.0, 4.0), cam, 640, 360, 16384), h.cast_frame((4.0, 90.0, 4.0), cam, 640, 360, 16384)
    for k in ("pos_steps", "t", "info"):
        assert torch_cuda.equal(a[k], b[k]), k
