"""Incremental edits on the GPU: after world edits, svo_tree_update + svo_tree_sync
must give the same casts as a freshly built and uploaded tree (bit-exact hit records)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _frames_equal(rt, a, b, label):
    ga, gb = rt.decode_hits(a), rt.decode_hits(b)
    for k in ("pos", "steps", "hit", "material", "axis"):
        assert np.array_equal(ga[k], gb[k]), "%s: %s differs at %d rays" % (label, k, int((ga[k] != gb[k]).reshape(len(ga[k]), -1).any(1).sum()))
    assert np.array_equal(ga["t"].view(np.uint32), gb["t"].view(np.uint32)), label


def test_edits_then_sync_match_fresh_upload(rt, torch_cuda):
    rng = np.random.default_rng(21)
    w = rt.World.reference()
    tree = w.build().upload(0)
    cams = [((35.0, 50.0, 35.0), (1.0, 0.0, 1.0)), ((4.0, 90.0, 4.0), (1.0, -0.45, 1.0))]
    for step in range(4):
        # carve the terrain in view, drop blocks (some reflective) in the sky, fill a 4^3 block
        carve = np.stack([rng.integers(30, 120, 80), rng.integers(20, 50, 80), rng.integers(30, 120, 80)], 1)
        for p in carve:
            w.delete_block(*[int(v) for v in p])
        tree.update(w, carve)
        sky = np.stack([rng.integers(20, 150, 40), rng.integers(50, 90, 40), rng.integers(20, 150, 40)], 1)
        w.put_blocks(sky, rng.choice([0, 2], size=len(sky)).astype(np.uint32), rng.integers(1, 1 << 60, len(sky)).astype(np.uint64))
        tree.update(w, sky)
        blk = np.array([[60 + 8 * step, 40, 60]])
        w.put_blocks(blk, np.zeros(1, np.uint32), np.full(1, 4242, np.uint64), level=w.levels)
        tree.update(w, blk, level=w.levels)
        tree.sync()
        fresh = w.build().upload(0)
        for ci, (org, cd) in enumerate(cams):
            cam = rt.normalize(cd)
            for S in (30, 300):
                _frames_equal(rt, tree.cast_frame(org, cam, 480, 270, S), fresh.cast_frame(org, cam, 480, 270, S),
                              "step %d cam %d S=%d" % (step, ci, S))
        a = tree.shade_frame(cams[0][0], rt.normalize(cams[0][1]), 240, 136, 300, sun=rt.sun_dir())
        b = fresh.shade_frame(cams[0][0], rt.normalize(cams[0][1]), 240, 136, 300, sun=rt.sun_dir())
        assert torch_cuda.equal(a, b)


def test_sync_after_rebuild_and_growth(rt, torch_cuda):
    """many edits on a small world: the tree is rebuilt / outgrows its device allocation; sync re-uploads"""
    rng = np.random.default_rng(2)
    w = rt.World(levels=4)
    w.put_block(10, 10, 10, 0, 3)
    tree = w.build().upload(0)
    for _ in range(20):
        pts = rng.integers(0, 256, size=(200, 3))
        w.put_blocks(pts, np.zeros(len(pts), np.uint32), rng.integers(1, 50, len(pts)).astype(np.uint64))
        tree.update(w, pts)
        tree.sync()
    fresh = w.build().upload(0)
    cam = rt.normalize((1.0, -0.3, 0.7))
    _frames_equal(rt, tree.cast_frame((-20.5, 180.0, -10.0), cam, 256, 144, 600), fresh.cast_frame((-20.5, 180.0, -10.0), cam, 256, 144, 600),
                  "growth")


def test_patched_tree_casts_match_oracle(rt, oracle_mod, torch_cuda):
    """svo_tree_update + svo_tree_sync after a putBlock / deleteBlock sequence (levels 6 / 5 / 4) on the
    GPU vs the oracle's reference-layout tree after the same edits (tests/test_edits.py
    _oracle_edit_replay: putBlock tetrahexa_tree.cpp:176-291, deleteBlock :293-359): every cast field
    bit-exact, frames at two poses and budgets; the shading pass over the patched tree equals the
    one over a fresh upload."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_edits import _oracle_edit_replay

    w = rt.World.reference()
    tree = w.build().upload(0)

    def on_edit(pts, lv):
        tree.update(w, pts, level=lv)
        tree.sync()

    _, T, edits = _oracle_edit_replay(oracle_mod, np.random.default_rng(17), w=w, on_edit=on_edit)
    pal = tree.palette()
    pf = np.array([p[0] for p in pal], np.uint32)
    pc = np.array([p[1] for p in pal], np.uint64)
    for org, cd in (((35.0, 50.0, 35.0), (1.0, 0.0, 1.0)), ((4.0, 90.0, 4.0), (1.0, -0.45, 1.0)),
                    ((60.5, 75.25, 20.75), (0.4, -0.5, 1.0))):
        cam = rt.normalize(cd)
        for S in (30, 300):
            g = rt.decode_hits(tree.cast_frame(org, cam, 256, 192, S))
            ref = T.cast_frame(org, cam, 256, 192, S)
            assert ref["rc"] == 0
            assert np.array_equal(g["pos"], ref["pos"]) and np.array_equal(g["steps"], ref["steps"]), (org, S)
            assert np.array_equal(g["hit"], ref["hit"] != 0) and np.array_equal(g["last_pos"], ref["last"]), (org, S)
            mid = np.where(g["hit"], g["material"], 0)
            assert np.array_equal(pf[mid], ref["flags"]) and np.array_equal(pc[mid], ref["color"]), (org, S)
            assert np.array_equal(g["t"], ref["t"].astype(np.float32)), (org, S)
    fresh = w.build().upload(0)
    a = tree.shade_frame((4.0, 90.0, 4.0), rt.normalize((1.0, -0.45, 1.0)), 240, 136, 300, sun=rt.sun_dir())
    b = fresh.shade_frame((4.0, 90.0, 4.0), rt.normalize((1.0, -0.45, 1.0)), 240, 136, 300, sun=rt.sun_dir())
    assert torch_cuda.equal(a, b)


def _pairs_of(c, E, k0, lv, step):
    """the pair table the kernels read, derived from the ceilings (svo_cast.hip ceil_pairs): level j with level
    min(j + step, lv - 1)"""
    offs, o = [], 0
    for j in range(lv):
        rows = E >> (2 * (k0 + j))
        offs.append((o, rows))
        o += rows * rows
    p = np.zeros(len(c), np.uint32)
    for j in range(lv):
        o, rows = offs[j]
        up = min(j + step, lv - 1)
        ou, ru = offs[up]
        sh = 2 * (up - j)
        lvl = c[o:o + rows * rows].reshape(rows, rows).astype(np.uint16).astype(np.uint32)
        par = c[ou:ou + ru * ru].reshape(ru, ru).astype(np.uint16).astype(np.uint32)
        p[o:o + rows * rows] = (lvl | (np.repeat(np.repeat(par, 1 << sh, 0), 1 << sh, 1) << 16)).reshape(-1)
    return p


def _quads_of(c, E, k0, levels):
    """tests' restatement of svo_tree.d_ceilq: per finest block, the ceilings of the blocks of levels 0..3 holding it"""
    rows0 = E >> (2 * k0)
    q = np.zeros((rows0, rows0), np.uint64)
    o = 0
    for j in range(4):
        if j < levels:
            rows = rows0 >> (2 * j)
            lvl = c[o:o + rows * rows].reshape(rows, rows).astype(np.uint16).astype(np.uint64)
            o += rows * rows
            v = np.repeat(np.repeat(lvl, 1 << (2 * j), 0), 1 << (2 * j), 1)
        else:
            v = np.full((rows0, rows0), 0x7FFF, np.uint64)
        q |= v << np.uint64(16 * j)
    return q.reshape(-1)


def test_sync_updates_device_ceilings_incrementally(rt, torch_cuda):
    """svo_tree_sync recomputes only the edited columns' ceilings and uploads their rows into the
    device tables already there.  After every edit + sync the tables in HBM equal a full recomputation over
    the patched tree (svo_tree_ceilings) and the pairs derived from it; a sync with nothing changed is a no-op."""
    import time

    rng = np.random.default_rng(5)
    w = rt.World.reference()
    tree = w.build().upload(0)
    E = 1 << (2 * w.levels)
    lv0, c0, p0 = tree.device_ceilings()
    assert lv0 >= 2
    times = []
    for step in range(6):
        if step % 2 == 0:  # raise columns (a tower), then carve terrain away
            pts = np.stack([rng.integers(0, 400, 30), rng.integers(60, 200, 30), rng.integers(0, 400, 30)], 1)
            w.put_blocks(pts, np.zeros(len(pts), np.uint32), np.full(len(pts), 77, np.uint64))
        else:
            pts = np.stack([rng.integers(0, 200, 60), rng.integers(1, 64, 60), rng.integers(0, 200, 60)], 1)
            for p in pts:
                w.delete_block(*[int(v) for v in p])
        t0 = time.perf_counter()
        tree.update(w, pts)
        tree.sync()
        times.append(time.perf_counter() - t0)
        lv, c, p = tree.device_ceilings()
        full = np.concatenate([x.reshape(-1) for x in tree.ceilings()])
        assert lv == lv0 and np.array_equal(c, full), "step %d: device ceilings differ from a full recomputation" % step
        k0, step_ = rt.ceiling_layout()
        assert np.array_equal(p, _pairs_of(full, E, k0, lv, step_)), "step %d: pair table" % step
        assert np.array_equal(tree.device_ceiling_quads(), _quads_of(full, E, k0, lv)), "step %d: quads" % step
    tree.sync()  # nothing changed: no-op
    assert np.array_equal(tree.device_ceilings()[1], c)
    print("edit + sync of 30-60 blocks: %s ms" % ", ".join("%.2f" % (x * 1e3) for x in times))
