"""Trees whose root is not an ordinary interior node, and near-empty worlds.  Every trace seeds its first parent from
the root (round 6: node 0 read once, uniform); a root that is not interior — a uniform world (the root itself a SOLID
block, putBlock at level 1), a one-level 4^3 tree (the root is the only brick) — keeps the virtual parent above it
(svo_cast.hip trace()).  Frames on such trees, on an empty world and on a world of one far block, against the oracle's
castRayFromCam (ray_caster.cpp:54-87 over tetrahexa_tree.cpp:113-157), every field bit-exact, with and without
ceilings and with voxel stepping (tests/test_gpu_parity.py compare)."""
import numpy as np
import pytest

from test_gpu_parity import compare

pytestmark = pytest.mark.gpu

CAMS = [((1.0, 2.0, 3.0), (0.6, -0.45, 0.66)),     # integral: the octant linear instance
        ((2.5, 1.5, 0.5), (-0.3, 0.6, 1.0)),       # half-integral, mixed signs
        ((3.3, 0.9, 2.1), (0.8, -0.7, -1.0)),      # fractional: the segment instance
        ((0.0, 0.0, 0.0), (1.0, 0.001, 0.4))]      # a corner, rising slowly (wraps in x / z)


@pytest.fixture(scope="module")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _pair(rt, oracle_mod, levels, blocks, level=None):
    """the same blocks put on both sides: (x, y, z, colour) at `level` (None: voxels; 1: the root itself)"""
    w = rt.World(levels)
    T = oracle_mod.Tree(levels)
    oracle_mod.lib().orc_init_clean_root(T.h)
    for x, y, z, c in blocks:
        if level is None:
            w.put_block(x, y, z, 0, c)
        else:
            w.put_block(x, y, z, 0, c, level=level)
        assert T.put_block(x, y, z, 0, c, 0.0, levels + 1 if level is None else level) == 0
    return w.build().upload(0), T


def _frames(rt, tree, T, label, steps=300, cams=CAMS):
    for ci, (org, d) in enumerate(cams):
        dn = rt.normalize(d)
        ref = T.cast_frame(org, dn, 64, 32, steps)
        assert ref["rc"] == 0
        for flags in (0, rt.CAST_NO_CEILINGS, rt.CAST_ITERATIVE):
            out = tree.cast_frame(org, dn, 64, 32, steps, flags=flags)
            compare(rt, tree, out, ref, "%s cam%d flags=%d" % (label, ci, flags))
    return ref


@pytest.mark.parametrize("levels", [1, 2, 3])
def test_uniform_solid_world(rt, oracle_mod, cuda, levels):
    """the root itself a SOLID block: every ray hits the first voxel it steps into"""
    tree, T = _pair(rt, oracle_mod, levels, [(0, 0, 0, 77)], level=1)
    ref = _frames(rt, tree, T, "uniform levels=%d" % levels)
    assert ref["hit"].all() and (ref["steps"] == 299).all()


def test_one_level_tree(rt, oracle_mod, cuda):
    """a 4^3 world: the root is the only brick (its voxel mask tested in registers, no parent above it)"""
    rng = np.random.default_rng(11)
    pts = {tuple(p) for p in rng.integers(0, 4, (9, 3)).tolist()}
    tree, T = _pair(rt, oracle_mod, 1, [(x, y, z, 1 + i) for i, (x, y, z) in enumerate(sorted(pts))])
    ref = _frames(rt, tree, T, "one-level")
    assert ref["hit"].any() and not ref["hit"].all()


@pytest.mark.parametrize("levels", [2, 4])
def test_empty_world(rt, oracle_mod, cuda, levels):
    """nothing stored: every ray spends its budget (a miss, steps 0) and ends where the DDA leaves it"""
    tree, T = _pair(rt, oracle_mod, levels, [])
    ref = _frames(rt, tree, T, "empty levels=%d" % levels, steps=200)
    assert not ref["hit"].any() and (ref["steps"] == 0).all()


def test_one_far_block(rt, oracle_mod, cuda):
    """one voxel in a 256^3 world: the root's mask has one bit, every other region is empty down to it"""
    tree, T = _pair(rt, oracle_mod, 4, [(200, 1, 130, 5)])
    aimed = [((190.5, 1.5, 120.5), (1.0, 0.0, 1.0)), ((180.0, 10.0, 110.0), (1.0, -0.45, 1.0))]
    ref = _frames(rt, tree, T, "one block", steps=1000, cams=CAMS + aimed)
    assert ref["hit"].any() and (ref["pos"][ref["hit"] != 0] == [200, 1, 130]).all()


@pytest.mark.parametrize("case", ["uniform", "one_level", "one_block"])
def test_shade_degenerate(rt, oracle_mod, cuda, case):
    """the shading pass on the same trees: its straight trace and the shadow rays (75 steps towards the sun, each
    seeded from the root of the solid tree) against the oracle's shading restatement (low_res.frag's colour model)"""
    from test_gpu_shade import _check

    if case == "uniform":
        tree, T = _pair(rt, oracle_mod, 3, [(0, 0, 0, 77)], level=1)
        cams = CAMS
    elif case == "one_level":
        rng = np.random.default_rng(11)
        pts = {tuple(p) for p in rng.integers(0, 4, (9, 3)).tolist()}
        tree, T = _pair(rt, oracle_mod, 1, [(x, y, z, 1 + i) for i, (x, y, z) in enumerate(sorted(pts))])
        cams = CAMS
    else:
        tree, T = _pair(rt, oracle_mod, 4, [(200, 1, 130, 5), (201, 1, 130, 6), (200, 2, 131, 7)])
        cams = [((190.5, 1.5, 120.5), (1.0, 0.0, 1.0)), ((180.0, 10.0, 110.0), (1.0, -0.45, 1.0))]
    sun = rt.sun_dir()
    for ci, (org, d) in enumerate(cams):
        dn = rt.normalize(d)
        rgba, hits = tree.shade_frame(org, dn, 64, 32, 300, sun=sun, with_hits=True)
        ref = T.shade_frame(org, dn, 64, 32, 300, sun)
        _check(rgba, ref, rt.decode_hits(hits)["hit"], "%s cam%d" % (case, ci))
