"""Incremental edits: putBlock / deleteBlock on the world, then svo_tree_update
patches the linearised tree in place.  Its content must equal a fresh svo_build of the edited
world at every position (host lookups here; GPU casts in test_gpu_edits)."""
import numpy as np
import pytest

LIQUID, REFLECTIVE, REFRACTIVE = 0x10, 0x2, 0x4


def _probe_points(rng, edits, extent, n_random=20000):
    """edited voxels, their 3^3 neighbourhoods and random points (some far outside: wrap)"""
    e = np.asarray(edits, np.int64).reshape(-1, 3)
    nb = (e[:, None, :] + np.stack(np.meshgrid([-1, 0, 1], [-1, 0, 1], [-1, 0, 1]), -1).reshape(1, -1, 3)).reshape(-1, 3)
    r = rng.integers(-extent, 2 * extent, size=(n_random, 3))
    r[: n_random // 2, 1] = rng.integers(0, 128, size=n_random // 2)  # the terrain band
    return np.concatenate([e, nb, r]).astype(np.int32)


def _same_as_fresh(rt, world, tree, pts):
    fresh = world.build()
    got, want = tree.get_blocks(pts), fresh.get_blocks(pts)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, "%d positions differ, first %s: patched %s fresh %s" % (len(bad), pts[bad[:3]], got[bad[:3]], want[bad[:3]])


def _random_edits(rng, n, lo, hi):
    return np.stack([rng.integers(lo[0], hi[0], n), rng.integers(lo[1], hi[1], n), rng.integers(lo[2], hi[2], n)], 1)


def test_voxel_edits_match_rebuild(rt):
    rng = np.random.default_rng(7)
    w = rt.World.reference()
    tree = w.build()
    extent = 1 << (2 * w.levels)
    n0 = tree.info().n_nodes
    all_edits = []
    for batch in range(6):
        pts = _random_edits(rng, 60, (0, 0, 0), (220, 70, 220))  # terrain surface and below: carve / fill
        if batch % 2 == 0:
            colors = rng.integers(1, 1 << 60, size=len(pts)).astype(np.uint64)
            flags = rng.choice([0, LIQUID | REFRACTIVE, REFLECTIVE, REFRACTIVE], size=len(pts)).astype(np.uint32)
            w.put_blocks(pts, flags, colors)
        else:
            for p in pts:
                w.delete_block(*[int(v) for v in p])
        tree.update(w, pts)
        all_edits.append(pts)
        _same_as_fresh(rt, w, tree, _probe_points(rng, np.concatenate(all_edits), extent))
    assert tree.info().n_nodes > n0  # patched in place (appended blocks), not rebuilt from scratch


def test_block_level_edits_and_sky(rt):
    """level-5 (4^3) puts / deletes, edits in empty sky and far away (wrap), a solid 16^3 carved"""
    rng = np.random.default_rng(11)
    w = rt.World.reference()
    tree = w.build()
    lv = w.levels  # one 4^3 block
    pts = np.array([[40, 30, 40], [44, 30, 40], [600, 600, 600], [-5, 900, 3000], [128, 64, 128]], np.int32)
    w.put_blocks(pts, np.zeros(len(pts), np.uint32), np.full(len(pts), 12345, np.uint64), level=lv)
    tree.update(w, pts, level=lv)
    _same_as_fresh(rt, w, tree, _probe_points(rng, pts, 1 << (2 * w.levels)))
    w.delete_block(40, 30, 40, level=lv)
    tree.update(w, [[40, 30, 40]], level=lv)
    # a whole 16^3 region (level 4) made solid, then single voxels carved out of it
    w.put_block(160, 16, 160, 0, 777, level=lv - 1)
    tree.update(w, [[160, 16, 160]], level=lv - 1)
    carve = _random_edits(rng, 40, (160, 16, 160), (176, 32, 176))
    for p in carve:
        w.delete_block(*[int(v) for v in p])
    tree.update(w, carve)
    _same_as_fresh(rt, w, tree, _probe_points(rng, np.concatenate([pts, carve]), 1 << (2 * w.levels)))


def test_many_edits_trigger_rebuild(rt):
    """superseded blocks above half the array: the tree is rebuilt from the world (still equal)"""
    rng = np.random.default_rng(3)
    w = rt.World(levels=3)  # 64^3 world: a few edits outweigh it
    w.put_block(1, 1, 1, 0, 5)
    tree = w.build()
    for _ in range(30):
        pts = _random_edits(rng, 20, (0, 0, 0), (64, 64, 64))
        w.put_blocks(pts, np.zeros(len(pts), np.uint32), rng.integers(1, 9, len(pts)).astype(np.uint64))
        tree.update(w, pts)
    _same_as_fresh(rt, w, tree, _probe_points(rng, pts, 64))
    assert tree.info().n_nodes <= 4 * w.build().info().n_nodes


def test_whole_world_edit(rt):
    w = rt.World(levels=3)
    w.put_block(1, 1, 1, 0, 5)
    tree = w.build()
    w.put_block(0, 0, 0, 0, 9, level=1)  # the root itself: a uniform world
    tree.update(w, [[0, 0, 0]], level=1)
    _same_as_fresh(rt, w, tree, np.array([[0, 0, 0], [63, 63, 63], [5, 70, 1]], np.int32))
    w.delete_block(3, 3, 3)
    tree.update(w, [[3, 3, 3]])
    _same_as_fresh(rt, w, tree, np.array([[3, 3, 3], [2, 3, 3], [3, 2, 3]], np.int32))


def test_update_errors(rt):
    w = rt.World(levels=3)
    tree = w.build()
    other = rt.World(levels=4)
    with pytest.raises(RuntimeError):
        tree.update(other, [[0, 0, 0]])
    with pytest.raises(RuntimeError):
        tree.update(w, [[0, 0, 0]], level=9)
    with pytest.raises(RuntimeError):
        tree.sync()  # not uploaded
