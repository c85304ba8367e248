"""The oracle (oracle/oracle.c, a CPU restatement of the reference) pinned against the golden
vectors the reference itself produced (tests/golden/, see make_golden.py)."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def facts():
    return json.load(open(os.path.join(GOLD, "reference_facts.json")))


def test_noise_matches_reference_bitwise(oracle_mod):
    g = np.load(os.path.join(GOLD, "noise_ref.npz"))
    for seed in np.unique(g["seed"]):
        m = g["seed"] == seed
        got = np.array([oracle_mod.noise2(int(seed), a, b) for a, b in zip(g["x"][m], g["y"][m])])
        assert np.array_equal(got.view(np.uint64), g["value"][m].view(np.uint64)), seed


def test_noise_matches_compiled_reference_live(oracle_mod):
    # the reference's own OpenSimplexNoise.cpp, compiled into oracle/_ref (build container only)
    if not os.path.exists("/root/reference/include/OpenSimplexNoise.cpp"):
        pytest.skip("reference sources not present (GPU box)")
    oracle_mod.build_ref()
    rng = np.random.default_rng(7)
    x, y = rng.uniform(-500, 500, 5000), rng.uniform(-500, 500, 5000)
    ref = oracle_mod.ref_noise_batch(42, x, y)
    got = np.array([oracle_mod.noise2(42, a, b) for a, b in zip(x, y)])
    assert np.array_equal(ref.view(np.uint64), got.view(np.uint64))


def test_test_cpp_known_answer(oracle_mod):
    k = facts()["test_cpp_kat"]
    d = oracle_mod.normalize(k["dir_unnormalized"])
    pos = np.zeros(3, np.int32)
    ax = oracle_mod.C.c_int32()
    oracle_mod.lib().orc_dda_free(oracle_mod.f3(k["origin"]), d, k["steps"], pos, oracle_mod.C.byref(ax))
    assert list(pos) == k["round"] and ax.value == k["last_hit"]


def test_reference_world_structure(ref_world_oracle):
    f = facts()
    T = ref_world_oracle
    assert T.nodes() == f["reference_world"]["nodes"]
    assert T.arrays() == f["reference_world"]["arrays"]
    assert T.root_bitmap() == int(f["reference_world"]["root_bitmap"], 16)
    a, b = f["wrap"]["a"], f["wrap"]["b"]
    assert T.get_block(*a) == T.get_block(*b)
    for p in f["max_depth_exit"]["points"]:
        with pytest.raises(RuntimeError):
            T.get_block(*p)
    lv = f["debug_blocks"]["level5_leaf"]
    for x in range(lv["min"][0], lv["max"][0] + 1):
        for y in range(lv["min"][1], lv["max"][1] + 1):
            for z in range(lv["min"][2], lv["max"][2] + 1):
                assert T.get_block(x, y, z)[0] == lv["flags"]
    rv = f["debug_blocks"]["reflective_voxel"]
    assert T.get_block(*rv["pos"])[0] == rv["flags"]


def test_pick_ray_walks_z(oracle_mod, ref_world_oracle):
    f = facts()["pick_ray_default_camera"]
    d = oracle_mod.normalize(f["dir_unnormalized"])
    r = ref_world_oracle.cast_ray(f["origin"], d, 30)
    assert r.axis == f["walks_axis"] and list(r.pos) == [35, 50, 65] and r.hit == 0


def test_default_camera_frame_statistics(oracle_mod, ref_world_oracle):
    f = facts()["frame_default_camera"]
    d = oracle_mod.normalize([1, 0, 1])
    out = ref_world_oracle.cast_frame([35, 50, 35], d, f["width"], f["height"], f["steps"])
    assert out["rc"] == 0
    hit = out["hit"].mean()
    steps = out["dda_steps"] / (f["width"] * f["height"])
    assert abs(hit - f["hit_fraction"]) < f["tolerance"][0]
    assert abs(steps - f["mean_dda_steps"]) < f["tolerance"][1]


def test_collapse_builder_equals_putblock(oracle_mod):
    A = oracle_mod.Tree.terrain(4, 256, 256)
    B = oracle_mod.Tree.terrain_putblock(4, 256, 256)
    ra, fa, ca = A.dump_box(0, 0, 0, 256, 72, 256)
    rb, fb, cb = B.dump_box(0, 0, 0, 256, 72, 256)
    assert ra == 0 and rb == 0
    assert np.array_equal(fa, fb) and np.array_equal(ca, cb)


@pytest.mark.parametrize("levels", [6, 7])
def test_collapse_builder_equals_putblock_at_config_depths(oracle_mod, levels):
    """The collapse builder behind the C3 (6 levels) and C5 (7 levels) oracle trees against the reference's own
    construction, genWorld's putBlock per voxel (tetrahexa_tree.cpp:176-291, world_gen.cpp:13-42), at those depths: a
    512 x 512-column patch at the world origin, every voxel of its bounding box (and a margin of empty columns past
    it) compared — flags and colour"""
    n = 512
    A = oracle_mod.Tree.terrain(levels, n, n)
    B = oracle_mod.Tree.terrain_putblock(levels, n, n)
    ra, fa, ca = A.dump_box(0, 0, 0, n + 8, 72, n + 8)
    rb, fb, cb = B.dump_box(0, 0, 0, n + 8, 72, n + 8)
    assert ra == 0 and rb == 0
    assert np.array_equal(fa, fb) and np.array_equal(ca, cb)
    assert (fa[:, :, :n] != 0).any() and (fa[:, :, n:] == 0).all() and (fa[n:] == 0).all()  # solid inside, empty past it
    h = oracle_mod.heights(n, n)
    assert int(h.max()) < 72  # the box holds every column's top


def test_terrain_height_range(oracle_mod):
    r = facts()["terrain_4096_height_range"]
    h = oracle_mod.heights(4096, 4096)
    assert h.min() == r["min"] and h.max() == r["max"]


def test_oracle_sky_matches_numpy_restatement(oracle_mod):
    """oracle shading of rays that miss = genSkyBox (low_res.frag:157-168) restated in numpy float32"""
    O = oracle_mod
    t = O.Tree.reference_world()
    sun = O.normalize((2.0, 1.0, 4.0))
    W, H = 16, 9
    cam = O.normalize((0.2, 1.0, 0.1))
    rgba = t.shade_frame((50.0, 200.0, 50.0), cam, W, H, 300, sun)
    f = np.float32
    ppx, ppy = O.proj_plane(W, H)
    np.seterr(over="ignore")  # exp(-x*k) may overflow to inf: the sigmoid is then 0, as in f32 C
    for k in range(W * H):
        d = np.array(O.pixel_dir(cam, ppx, ppy, W, H, k % W, k // W), f)
        dy = d[1] * f(1.4) if d[1] < 0 else d[1]
        haze = (f(0.1) - abs(min(max(dy, f(-0.3)), f(0.3)))) * f(0.8) + f(0.1)
        sig = lambda x, s, kk: f(1.0) / (f(1.0) + np.exp(-x * f(kk), dtype=f)) * f(s)  # noqa: E731 (exp may overflow to inf: sigmoid -> 0)
        modifier = min(max(sig(f(1.0) - haze * f(2.0), 1.0, 2.0), f(0)), f(1))
        e = np.array([d[0] - sun[0], dy - sun[1], d[2] - sun[2]], f)
        b = np.sqrt((e[0] * e[0] + e[1] * e[1]) + e[2] * e[2], dtype=f) * f(50.0)
        sv = sig(f(1.5) - b, 1.0, 1.6)
        h3 = min(max(haze, f(0)), f(1)) * f(3.0)
        want = np.array([(f(0.2) + h3) * modifier + sv, (f(0.4) + h3) * modifier + sv, (f(1.0) + h3) * modifier], f)
        assert np.allclose(rgba[k, :3], want, rtol=0, atol=2e-6), (k, rgba[k], want)
        assert rgba[k, 3] == 0.0


def test_shade_entries_restate_the_primary_model(oracle_mod):
    """orc_shade_entries (the shading pass's §8(d) entries, oracle/bray.py C3_shade) rides along the shading walk with
    the primary model's restart rule: with no shadow rays and no reflecting / refracting block in reach (a 512^2
    terrain without water: liquid mode off, terrain has none of flags 3 / 5) it counts exactly orc_frame_entries,
    and shadow rays only add entries and one root read each."""
    O = oracle_mod
    t = O.Tree.terrain(5, 512, 512)
    org, cam = (4.0, 90.0, 4.0), O.normalize((1.0, -0.45, 1.0))
    sun = O.normalize((2.0, 1.0, 4.0))
    W, H = 160, 90
    e0, _, lk0 = t.shade_entries(org, cam, W, H, 2000, sun, shadow_steps=0)
    assert e0 == t.frame_entries(org, cam, W, H, 2000)
    e1, sh1, lk1 = t.shade_entries(org, cam, W, H, 2000, sun, shadow_steps=75)
    assert sh1 > 0 and e1 >= e0 and lk1 > lk0
