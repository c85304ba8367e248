"""Small trees at the edges of the column-ceiling table: a 3-level (64^3) tree has one ceiling level (16-column blocks),
so the primary casts' second level is a copy of the first (set_ceilings; the kernel reads both unconditionally), and
a 2-level (16^3) tree has none.  Frames from integral, half-integral and fractional cameras against the oracle's
castRayFromCam, with and without ceilings (every field bit-exact, tests/test_gpu_parity.py compare)."""
import numpy as np
import pytest

from test_gpu_parity import compare

pytestmark = pytest.mark.gpu

CAMS = [((4.0, 60.0, 4.0), (1.0, -0.45, 1.0)),     # integral: the octant linear instance
        ((30.5, 40.5, 2.5), (-0.3, -0.6, 1.0)),    # half-integral, mixed signs
        ((7.3, 50.9, 60.1), (0.8, -0.7, -1.0)),    # fractional: the segment instance
        ((20.0, 20.0, 20.0), (1.0, 0.001, 0.4))]   # inside the terrain band, rising slowly (wraps in x / z)


@pytest.fixture(scope="module")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _world(rt, oracle_mod, levels):
    """64^3: genWorld terrain (both builders); 16^3: 300 random voxels put block by block on both sides"""
    if levels == 3:
        return rt.Tree.terrain(3, 64, 64).upload(0), oracle_mod.Tree.terrain(3, 64, 64)
    rng = np.random.default_rng(5)
    pts = rng.integers(0, 16, (300, 3))
    cols = rng.integers(1, 1 << 40, 300).astype(np.uint64)
    w = rt.World(2)
    w.put_blocks(pts, np.zeros(300, np.uint32), cols)
    T = oracle_mod.Tree(2)
    oracle_mod.lib().orc_init_clean_root(T.h)
    for p, c in zip(pts, cols):
        assert T.put_block(int(p[0]), int(p[1]), int(p[2]), 0, int(c), 0.0, 3) == 0
    return w.build().upload(0), T


@pytest.mark.parametrize("levels", [3, 2])
@pytest.mark.parametrize("cam", range(len(CAMS)))
def test_small_tree_frames(rt, oracle_mod, cuda, levels, cam):
    tree, T = _world(rt, oracle_mod, levels)
    k0 = rt.ceiling_layout()[0]
    assert len(tree.ceilings()) == max(0, min(levels - k0, 4))  # blocks of 4^k columns, k0 <= k < levels
    org, d = CAMS[cam]
    dn = rt.normalize(d)
    ref = T.cast_frame(org, dn, 160, 96, 300)
    assert ref["rc"] == 0
    for flags in (0, rt.CAST_NO_CEILINGS, rt.CAST_ITERATIVE):
        out = tree.cast_frame(org, dn, 160, 96, 300, flags=flags)
        compare(rt, tree, out, ref, "levels=%d cam%d flags=%d" % (levels, cam, flags))
