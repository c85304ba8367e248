"""Host side of the product (libsvo_rt.so) on CPU: the C ABI loads and exports every symbol of
include/svo_rt.h, the world / builders / ray generation agree with the oracle, and error paths
return status codes instead of exiting.  No kernel launches here (no GPU in the build container)."""
import ctypes as C
import json
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def test_abi_exports_every_declared_symbol(rt):
    hdr = open(os.path.join(ROOT, "include", "svo_rt.h")).read()
    declared = set(re.findall(r"^\s*(?:const char\*|int|void)\s+(svo_\w+)\(", hdr, re.M))
    assert declared == set(rt.ABI_SYMBOLS)
    L = C.CDLL(rt.LIB_PATH)
    for s in declared:
        assert hasattr(L, s), s
    assert rt.lib().svo_version() == 7


def test_product_noise_matches_reference_golden(rt):
    g = np.load(os.path.join(GOLD, "noise_ref.npz"))
    for seed in np.unique(g["seed"]):
        m = g["seed"] == seed
        got = rt.noise2(int(seed), g["x"][m], g["y"][m])
        assert np.array_equal(got.view(np.uint64), g["value"][m].view(np.uint64)), seed


def test_terrain_heights_match_oracle(rt, oracle_mod):
    assert np.array_equal(rt.terrain_heights(512, 384), oracle_mod.heights(512, 384))


def test_world_matches_oracle_getblock(rt, ref_world, ref_world_oracle):
    # parity domain: everything outside root child 63 ([768,1024)^3)
    rc, f, c = ref_world_oracle.dump_box(0, 0, 0, 256, 112, 256)
    assert rc == 0
    zz, yy, xx = np.meshgrid(np.arange(256), np.arange(112), np.arange(256), indexing="ij")
    pts = np.stack([xx.ravel(), yy.ravel(), zz.ravel()], 1)
    gf, gc, _ = ref_world.get_blocks(pts)
    assert np.array_equal(gf, f.ravel()) and np.array_equal(gc, c.ravel())
    # wrapped and negative coordinates
    for p in [(1034, 5, 10), (-1014, 40, 3), (5, -990, 7), (260, 30, 1300)]:
        assert ref_world.get_block(*p)[:2] == ref_world_oracle.get_block(*p)[:2]


def test_linearised_tree_matches_solid_view(rt, ref_tree, ref_world_oracle):
    pal = ref_tree.palette()
    rc, f, c = ref_world_oracle.dump_box(0, 0, 0, 256, 112, 256)
    zz, yy, xx = np.meshgrid(np.arange(256), np.arange(112), np.arange(256), indexing="ij")
    pts = np.stack([xx.ravel(), yy.ravel(), zz.ravel()], 1)
    ids = ref_tree.get_blocks(pts)
    pf = np.array([p[0] for p in pal], np.uint32)[ids]
    pc = np.array([p[1] for p in pal], np.uint64)[ids]
    solid = (c.ravel() != np.uint64(0xFFFFFFFFFFFFFFFF)) & ((f.ravel() & 0x10) == 0)
    assert np.array_equal(pf[solid], f.ravel()[solid]) and np.array_equal(pc[solid], c.ravel()[solid])
    assert np.all(ids[~solid] == 0)


@pytest.mark.parametrize("view", [0, 1])
def test_terrain_builder_equals_edit_builder(rt, view):
    """the column builder (min/max pyramid classes, svo_noise.h terrain_region_class) emits what the
    edit-tree builder emits from genWorld's putBlocks, in both views (SVO_VIEW_ALL stores the water)"""
    for levels, W, L in ((4, 256, 256), (4, 200, 150), (5, 300, 1024)):
        w = rt.World(levels)
        w.gen_world(W, L)
        a = w.build(view)
        b = rt.Tree.terrain(levels, W, L, view=view)
        assert a.info().view == b.info().view == view
        na, ma = a.export()
        nb, mb = b.export()
        assert a.palette() == b.palette()
        assert np.array_equal(na, nb) and np.array_equal(ma, mb), (levels, W, L)


def test_full_view_stores_liquid(rt, ref_world):
    """SVO_VIEW_ALL (the shading scene) holds every stored block, water included; the solid view
    (castRayFromCam, ray_caster.cpp:82) leaves liquid empty; both agree everywhere else"""
    a, b = ref_world.build(), ref_world.build(rt.VIEW_ALL)
    g = np.stack(np.meshgrid(np.arange(0, 210, 3), np.arange(0, 40), np.arange(0, 210, 3), indexing="ij"), -1).reshape(-1, 3)
    f, c, _ = ref_world.get_blocks(g)
    ida, idb = a.get_blocks(g), b.get_blocks(g)
    liq = (f & rt.LIQUID) != 0
    assert liq.sum() > 1000  # the reference world's lakes
    assert np.all(ida[liq] == 0) and np.all(idb[liq] != 0)
    assert np.array_equal(ida[~liq], idb[~liq])
    pal = b.palette()
    assert all(pal[i][0] == 0x15 for i in np.unique(idb[liq]))  # REFRACTIVE | LIQUID | stored


def test_oracle_sin_is_correctly_rounded(oracle_mod):
    """the liquid wobble's sin (svo_common.h sin_f32 and its oracle restatement): float(sin(double))"""
    xs = np.concatenate([np.linspace(-300, 300, 60001), np.random.default_rng(3).uniform(-9000, 9000, 20000)]).astype(np.float32)
    got = np.array([oracle_mod.sin_f32(float(x)) for x in xs], np.float32)
    assert np.array_equal(got, np.sin(xs.astype(np.float64)).astype(np.float32))
    # beyond the exact reduction range (time is caller-given): defined, bounded, NaN only for non-finite x
    for x in (1e7, -3.3e9, 1e20, -1e30, 3.4e38, -3.4e38):
        assert -1.0 <= oracle_mod.sin_f32(x) <= 1.0, x
    for x in (float("inf"), float("-inf"), float("nan")):
        assert np.isnan(oracle_mod.sin_f32(x))


def test_raygen_bit_exact_with_oracle(rt, oracle_mod):
    for cam, W, H in (([1, 0, 1], 256, 256), ([1, -0.45, 1], 1920, 1080), ([1, -1.2, 0.3], 640, 360), ([0, -1, 0.001], 64, 48)):
        d = rt.normalize(cam)
        assert np.array_equal(d.view(np.uint32), oracle_mod.normalize(cam).view(np.uint32))
        ppx, ppy = rt.proj_plane(W, H)
        assert (ppx, ppy) == oracle_mod.proj_plane(W, H)
        got = rt.pixel_dirs(d, W, H)
        rng = np.random.default_rng(W)
        for _ in range(300):
            px, py = int(rng.integers(0, W)), int(rng.integers(0, H))
            ref = oracle_mod.pixel_dir(d, ppx, ppy, W, H, px, py)
            assert np.array_equal(got[py, px].view(np.uint32), ref.view(np.uint32)), (cam, px, py)


def test_hemisphere_golden_is_consistent():
    g = json.load(open(os.path.join(GOLD, "hemisphere_ref.json")))
    a = np.array(g["generator_stdout"], np.float32)
    b = np.array(g["shader_literals"], np.float32)
    assert a.shape == (20, 3) and np.array_equal(a, b)


def test_put_delete_semantics(rt, oracle_mod):
    w = rt.World(5)
    T = oracle_mod.Tree(5)
    T.L.orc_init_clean_root(T.h)
    rng = np.random.default_rng(3)
    for _ in range(400):
        x, y, z = (int(v) for v in rng.integers(0, 64, 3))
        lvl = int(rng.choice([6, 6, 6, 5, 4]))
        fl = int(rng.integers(0, 32))
        col = int(rng.integers(0, 1 << 40))
        w.put_block(x, y, z, fl, col, 0.0, lvl)
        T.put_block(x, y, z, fl, col, 0.0, lvl)
    rc, f, c = T.dump_box(0, 0, 0, 64, 64, 64)
    zz, yy, xx = np.meshgrid(np.arange(64), np.arange(64), np.arange(64), indexing="ij")
    gf, gc, _ = w.get_blocks(np.stack([xx.ravel(), yy.ravel(), zz.ravel()], 1))
    assert np.array_equal(gf, f.ravel()) and np.array_equal(gc, c.ravel())
    # intended deleteBlock: the region becomes empty, neighbours keep their blocks
    w.put_block(10, 10, 10, 0, 123, 0.0, 6)
    w.put_block(11, 10, 10, 0, 456, 0.0, 6)
    assert w.delete_block(10, 10, 10, 6)[1] == 123
    assert w.get_block(10, 10, 10)[1] == 0xFFFFFFFFFFFFFFFF and w.get_block(11, 10, 10)[1] == 456


def test_error_paths(rt):
    h = C.c_void_p()
    assert rt.lib().svo_world_create(0, C.byref(h)) == -1
    assert rt.lib().svo_world_create(9, C.byref(h)) == -1
    assert b"levels" in rt.lib().svo_last_error()
    w = rt.World(3)
    with pytest.raises(rt.SvoError):
        w.put_block(0, 0, 0, 0, 1, 0.0, 9)
    t = w.build()
    d = rt.Tree.frame_desc([1, 1, 1], [1, 0, 0], 16, 16, 10)
    hits = rt.Hits(None, None, None)
    assert rt.lib().svo_cast_rays(t._h, C.byref(d), C.byref(hits), None) == -1  # NULL outputs
    hits = rt.Hits(16, 16, 16)
    assert rt.lib().svo_cast_rays(t._h, C.byref(d), C.byref(hits), None) == -4  # not uploaded
    with pytest.raises(rt.SvoError):
        rt.Tree.terrain(1, 4, 4)


def test_cast_count_sharding(rt):
    for H in (1080, 1077, 8, 5):
        total = rt.Tree.count(rt.Tree.frame_desc([0, 0, 0], [1, 0, 0], 33, H, 1))
        assert total == 33 * H
        for step in (2, 3, 8):
            parts = [rt.Tree.count(rt.Tree.frame_desc([0, 0, 0], [1, 0, 0], 33, H, 1, tile_row_start=s, tile_row_step=step))
                     for s in range(step)]
            assert sum(parts) == total


def test_cast_blocks_per_footprint(rt):
    """blocks (64-lane wavefronts) per launch: one per 16x4 footprint by default, 8x8 / 32x2 by flag,
    one per 64 explicit rays; every block covers at most 64 rays.  A small launch (below 20480 wavefronts of whole
    footprints: svo_common.h frame_half_rows) adds one wavefront per footprint of its first tile rows (half footprints)
    — as many rows as keep it within 20480 — and none bottom-first"""
    for W, H in ((1920, 1080), (3840, 2160), (33, 17), (8, 8), (100, 60)):
        for step in (1, 2, 3, 8):
            for start in range(step):
                tile_rows = len(range(start, (H + 7) // 8, step))
                for flags, tw in ((0, 16), (rt.CAST_TILE_8X8, 8), (rt.CAST_TILE_32X2, 32), (rt.CAST_BOTTOM_FIRST, 16)):
                    d = rt.Tree.frame_desc([0, 0, 0], [1, 0, 0], W, H, 1, tile_row_start=start, tile_row_step=step, flags=flags)
                    cols = (8 * tw // 64) * ((W + tw - 1) // tw)
                    half = 0 if flags == rt.CAST_BOTTOM_FIRST else max(0, min(tile_rows, 20480 // cols - tile_rows))
                    assert rt.Tree.blocks(d) == (tile_rows + half) * cols, (W, H, step, start, flags)
                    assert rt.Tree.blocks(d) * 64 >= rt.Tree.count(d)
    # a whole 1080p frame keeps whole footprints; its 1/8 shard is all half footprints
    d = rt.Tree.frame_desc([0, 0, 0], [1, 0, 0], 1920, 1080, 1)
    assert rt.Tree.blocks(d) == 135 * 240
    d = rt.Tree.frame_desc([0, 0, 0], [1, 0, 0], 1920, 1080, 1, tile_row_start=0, tile_row_step=8)
    assert rt.Tree.blocks(d) == 2 * 17 * 240
    d = rt.Tree.frame_desc([0, 0, 0], [1, 0, 0], 8, 8, 1)
    d.ray_dirs, d.n_rays = 1, 130  # explicit mode: only the count is read
    assert rt.Tree.blocks(d) == 3


def test_hemisphere_table_matches_reference_generator(rt, oracle_mod):
    g = json.load(open(os.path.join(GOLD, "hemisphere_ref.json")))
    py = np.array(g["generator_stdout"], np.float32)  # printed as (x, pole, y)
    want = np.stack([py[:, 0], py[:, 2], py[:, 1]], 1)
    assert np.array_equal(rt.hemisphere(20).view(np.uint32), want.view(np.uint32))
    # N = 16 (BASELINE config C4): same formula; the reference only ships N = 20 (parity via formula)
    for n in (1, 8, 16, 32, 64):
        assert np.array_equal(rt.hemisphere(n).view(np.uint32), oracle_mod.hemisphere(n).view(np.uint32)), n


def test_heightfield_builders_agree_on_adversarial_heights(rt):
    """column tops 0 (dirt at y = 0 under water), 1..3 (short dirt runs), exactly 20, aligned steps
    and partial footprints: the column builder must equal per-voxel putBlock node for node"""
    rng = np.random.default_rng(17)
    for levels, W, L in ((4, 64, 64), (4, 130, 77), (5, 256, 256)):
        h = rng.integers(0, 40, (W, L)).astype(np.int32)
        h[::7, :] = 0
        h[:, ::5] = 20
        h[10:30, 10:30] = 19
        h[40:48, 0:16] = 3  # a flat aligned plateau: uniform dirt bricks
        w = rt.World(levels)
        w.gen_heightfield(h)
        a, b = w.build(), rt.Tree.heightfield(levels, h)
        na, ma = a.export()
        nb, mb = b.export()
        assert a.palette() == b.palette()
        assert np.array_equal(na, nb) and np.array_equal(ma, mb), (levels, W, L)


@pytest.mark.parametrize("view", [0, 1])
def test_tree_checkpoint_round_trip(rt, ref_world, tmp_path, view):
    """svo_tree_save / svo_tree_load (SURVEY.md §5 checkpoint): the loaded tree is the saved one, array for
    array; an edited (patched, not re-collapsed) tree too"""
    trees = [ref_world.build(view), rt.Tree.terrain(5, 300, 700, view=view)]
    w = rt.World.reference()
    t = w.build(view)
    pts = np.array([[40, 30, 40], [41, 30, 40], [150, 15, 158]], np.int32)
    w.put_blocks(pts, np.zeros(3, np.uint32), np.full(3, 777, np.uint64))
    t.update(w, pts)
    trees.append(t)
    for i, a in enumerate(trees):
        p = str(tmp_path / ("t%d.svo" % i))
        a.save(p)
        b = rt.Tree.load(p)
        na, ma = a.export()
        nb, mb = b.export()
        assert np.array_equal(na, nb) and np.array_equal(ma, mb)
        assert a.palette() == b.palette()
        ia, ib = a.info(), b.info()
        assert (ia.levels, ia.view, ia.n_bricks, list(ia.nodes_per_level)) == (ib.levels, ib.view, ib.n_bricks, list(ib.nodes_per_level))
        assert ib.device == -1  # not uploaded
        g = np.random.default_rng(i).integers(0, 300, size=(5000, 3)).astype(np.int32)
        assert np.array_equal(a.get_blocks(g), b.get_blocks(g))


def test_tree_checkpoint_rejects_damage(rt, ref_tree, tmp_path):
    """a damaged file fails with SVO_EIO (-6) before any of it can reach a kernel"""
    p = tmp_path / "t.svo"
    ref_tree.save(str(p))
    raw = bytearray(p.read_bytes())
    cases = {"truncated": raw[: len(raw) // 2], "flipped": raw[:200] + bytes([raw[200] ^ 0x40]) + raw[201:], "magic": b"XXXX" + raw[4:],
             "empty": b""}
    for name, data in cases.items():
        q = tmp_path / (name + ".svo")
        q.write_bytes(bytes(data))
        with pytest.raises(RuntimeError, match="svo_tree_load"):
            rt.Tree.load(str(q))
    # a consistent checksum over an out-of-range child reference: caught by the validation
    import struct

    hdr = 8 + 4 * 4 + 8 * 3 + 8 * 8
    npal = struct.unpack_from("<I", raw, 8 + 12)[0]
    body = bytearray(raw[:-8])
    off = hdr + npal * 24  # node 0 (the root): mask, ref, info
    struct.pack_into("<I", body, off + 8, 0x7FFFFFF0)
    h = 1469598103934665603
    for b in body:
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    q = tmp_path / "badref.svo"
    q.write_bytes(bytes(body) + struct.pack("<Q", h))
    with pytest.raises(RuntimeError, match="out of range"):
        rt.Tree.load(str(q))
    with pytest.raises(RuntimeError):
        rt.Tree.load(str(tmp_path / "missing.svo"))

    # structural damage under a consistent checksum (every reference in range): node kinds at the
    # wrong depth, and a child reference back to an ancestor's block (a cycle)
    def resealed(edit, name):
        b = bytearray(raw[:-8])
        edit(b)
        h = 1469598103934665603
        for x in b:
            h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
        q = tmp_path / name
        q.write_bytes(bytes(b) + struct.pack("<Q", h))
        return str(q)

    nodes = np.frombuffer(bytes(raw[off:off + 16 * ref_tree.info().n_nodes]), dtype=np.uint32).reshape(-1, 4)
    kinds = nodes[:, 3] & 3
    cnt = np.array([bin(int(m)).count("1") for m in (nodes[:, 0].astype(np.uint64) | (nodes[:, 1].astype(np.uint64) << np.uint64(32)))])
    # a brick whose material run, read as a child block, stays inside the node array (so only the kind check sees it)
    brick = int(np.nonzero((kinds == 1) & (nodes[:, 2] > 0) & (nodes[:, 2].astype(np.int64) + cnt < len(nodes)))[0][0])
    inner = int(np.nonzero(kinds[1:] == 0)[0][0]) + 1  # an interior node below the root

    def set_kind(i, k):
        def f(b):
            info = struct.unpack_from("<I", b, off + 16 * i + 12)[0]
            struct.pack_into("<I", b, off + 16 * i + 12, (info & ~3) | k)
        return f

    def point_back(b):  # an interior node's children = the root's child block
        struct.pack_into("<I", b, off + 16 * inner + 8, int(nodes[0, 2]))

    for name, edit, msg in (("brick_as_interior.svo", set_kind(brick, 0), "interior node at the brick level"),
                            ("interior_as_brick.svo", set_kind(inner, 1), "brick node above the brick level"),
                            ("cycle.svo", point_back, "reached twice")):
        with pytest.raises(RuntimeError, match=msg):
            rt.Tree.load(resealed(edit, name))


@pytest.mark.parametrize("view", [0, 1])
def test_column_ceilings(rt, view):
    """svo_tree_ceilings (what the casts' ceiling moves rely on): per aligned block of 4^k x 4^k columns the highest
    stored row — for a terrain tree, the column tops (water up to row 20 above tops below it in the full view)
    maximised over the block; -1 over columns that hold nothing"""
    W, L = 300, 700
    t = rt.Tree.terrain(5, W, L, view=view)
    H = rt.terrain_heights(W, L).astype(np.int64)
    top = np.full((1024, 1024), -1, np.int64)  # [x, z]
    top[:W, :L] = np.where(H < 20, 20, H) if view == rt.VIEW_ALL else H
    cs = t.ceilings()
    assert len(cs) == 5 - t.ceil_k0  # k = 3, 4 (64- and 256-column blocks) below the 1024-wide world
    for j, c in enumerate(cs):
        B = 4 ** (t.ceil_k0 + j)
        want = top.reshape(1024 // B, B, 1024 // B, B).max(axis=(1, 3))
        assert np.array_equal(c.astype(np.int64), want.T), j


def test_column_ceilings_edited_world(rt, ref_world):
    """the reference world (putBlock / genWorld + the debug blocks: (10,100,10) and (1000,1000,1000)) and an edit:
    each probed block's ceiling equals the highest stored row getBlock finds in its columns"""
    w = rt.World.reference()
    w.put_block(700, 611, 300, 0, 12345, 0.0)  # a floating voxel
    t = w.build(rt.VIEW_ALL)
    c64 = t.ceilings()[3 - t.ceil_k0]  # (the 64-column level)
    for bx, bz in ((0, 0), (15, 15), (10, 4), (3, 3)):
        xs, zs, ys = np.arange(bx * 64, bx * 64 + 64), np.arange(bz * 64, bz * 64 + 64), np.arange(1024)
        best = -1
        for y0 in range(0, 1024, 128):  # (in slabs: 64 x 64 x 128 lookups at a time)
            g = np.stack(np.meshgrid(xs, ys[y0:y0 + 128], zs, indexing="ij"), -1).reshape(-1, 3)
            _, col, _ = w.get_blocks(g)
            stored = col != np.uint64(0xFFFFFFFFFFFFFFFF)
            if stored.any():
                best = max(best, int(g[stored][:, 1].max()))
        assert c64[bz, bx] == best, (bx, bz, c64[bz, bx], best)
