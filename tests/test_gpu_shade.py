"""GPU parity of the shading pass (svo_shade_rays) against the oracle's restatement
(oracle.c §shading: low_res.frag's colour model over castRayFromCam hits, reflections on flags&7==3).

Bar: hit records bit-exact (they are the primary cast); lit / shadowed / highlighted / reflected
colours bit-exact (the same f32 operations in the same order on both sides); sky colours within
2e-6 absolute (genSkyBox's exp and sqrt: device libm vs host libm may differ in the last ulp)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SKY_ATOL = 2e-6

CAMERAS = [
    ((35.0, 50.0, 35.0), (1.0, 0.0, 1.0)),        # reference default (globals.cpp:20-21)
    ((4.0, 90.0, 4.0), (1.0, -0.45, 1.0)),        # C1 pose
    ((150.3, 44.7, 20.9), (-0.6, -0.2, 1.0)),     # fractional origin, negative x
    ((4.5, 103.5, 4.5), (5.5, -3.5, 5.5)),        # looks at the reflective voxel (10,100,10), flags 3
]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def gtree(torch_cuda, ref_tree):
    ref_tree.upload(0)
    return ref_tree


def _check(rgba_gpu, rgba_ref, hit, label):
    g = rgba_gpu.cpu().numpy()
    assert g.shape == rgba_ref.shape, label
    assert np.all(np.isfinite(g)), label
    lit = hit != 0
    assert np.array_equal(g[lit], rgba_ref[lit]), "%s: %d lit pixels differ" % (label, int((g[lit] != rgba_ref[lit]).any(1).sum()))
    d = np.abs(g[~lit] - rgba_ref[~lit])
    assert d.size == 0 or d.max() <= SKY_ATOL, "%s: sky differs by %g" % (label, d.max())


@pytest.mark.parametrize("cam", range(len(CAMERAS)))
def test_shade_reference_world(rt, oracle_mod, gtree, ref_world_oracle, cam):
    O = oracle_mod
    org, cd = CAMERAS[cam]
    cam_dir = rt.normalize(cd)
    W, H, S = 240, 136, 300
    sun = rt.sun_dir()
    rgba, hits = gtree.shade_frame(org, cam_dir, W, H, S, sun=sun, with_hits=True)
    # the primary cast inside the shading pass is the drop-in cast (reflections aside)
    ref = ref_world_oracle.shade_frame(org, cam_dir, W, H, S, sun)
    g = rt.decode_hits(hits)
    _check(rgba, ref, g["hit"], "cam%d" % cam)


def test_shade_reflection_exercised(rt, gtree, ref_world_oracle):
    """camera 3 sees the reflective voxel: the plain cast hits it, the shading pass bounces off it"""
    org, cd = CAMERAS[3]
    cam_dir = rt.normalize(cd)
    out = gtree.cast_frame(org, cam_dir, 240, 136, 300)
    g = rt.decode_hits(out)
    on_mirror = g["hit"] & np.all(g["pos"] == np.array([10, 100, 10]), axis=1)
    assert on_mirror.sum() > 50
    rgba, hits = gtree.shade_frame(org, cam_dir, 240, 136, 300, sun=rt.sun_dir(), with_hits=True)
    h = rt.decode_hits(hits)
    assert not np.any(h["hit"][on_mirror] & np.all(h["pos"][on_mirror] == np.array([10, 100, 10]), axis=1))


def test_shade_look_at_and_budget(rt, gtree, ref_world_oracle):
    """lookingAtBlock highlight (main.cpp:81,89: castRayFromCam(30) from the camera) and small budgets"""
    org, cd = CAMERAS[0]
    cam_dir = rt.normalize(cd)
    (pos, _, _), _ = gtree.cast_ray_from_cam(org, cam_dir, 30)
    for S, shadow in ((300, 75), (40, 75), (300, 3)):
        rgba, hits = gtree.shade_frame(org, cam_dir, 160, 90, S, sun=rt.sun_dir(), look_at=pos, shadow_steps=shadow, with_hits=True)
        ref = ref_world_oracle.shade_frame(org, cam_dir, 160, 90, S, rt.sun_dir(), look_at=pos, shadow_steps=shadow)
        _check(rgba, ref, rt.decode_hits(hits)["hit"], "look S=%d shadow=%d" % (S, shadow))


def test_pick_ray_on_device(rt, gtree, torch_cuda):
    """the per-frame pick ray (main.cpp:81,89) without a host round trip —
    svo_cast_ray_from_cam_async writes the RayResult to device memory on the frame's stream, equal to the
    synchronous svo_cast_ray_from_cam (hits, misses, a hit on the last step, budget 0), and the shading pass reads
    lookingAtBlock from that record: the image equals the one with the host-side look_at, and the highlight shows."""
    torch = torch_cuda
    s = torch.cuda.Stream()
    rec = torch.zeros(64, dtype=torch.int32, device="cuda")
    for org, cd in CAMERAS + [((35.0, 50.0, 35.0), (0.0, -1.0, 0.0)), ((-20.5, 300.0, 7.25), (0.2, 1.0, 0.1))]:
        cam_dir = rt.normalize(cd)
        for steps in (0, 1, 7, 30, 300):
            (pos, last, left), _ = gtree.cast_ray_from_cam(org, cam_dir, steps)
            rec.fill_(-7)
            gtree.cast_ray_from_cam_async(org, cam_dir, steps, rec, stream=s)
            s.synchronize()
            r = rec[:7].cpu().numpy()
            assert tuple(r[:3]) == tuple(pos) and tuple(r[3:6]) == tuple(last) and r[6] == left, (org, cd, steps, r, pos, last, left)
    # a pose whose 30-step pick ray lands on terrain in view (the reference default camera's pick walks +z only, into
    # air: its highlight never shows); the oracle highlights 531 pixels of this frame
    org, cd = (35.0, 50.0, 35.0), (1.0, -1.0, 1.0)
    cam_dir = rt.normalize(cd)
    (pos, _, left), _ = gtree.cast_ray_from_cam(org, cam_dir, 30)
    assert tuple(pos) == (39, 44, 40) and left == 15
    d = gtree.frame_desc(org, cam_dir, 160, 90, 300)
    a = torch.empty((160 * 90, 4), dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    none = torch.empty_like(a)
    with torch.cuda.stream(s):
        gtree.cast_ray_from_cam_async(org, cam_dir, 30, rec, stream=s)
        gtree.shade(d, a, sun=rt.sun_dir(), look_at=rec, stream=s)
        gtree.shade(d, b, sun=rt.sun_dir(), look_at=pos, stream=s)
        gtree.shade(d, none, sun=rt.sun_dir(), stream=s)
    s.synchronize()
    assert torch.equal(a, b)
    assert int((a != none).any(1).sum()) > 100  # the looked-at voxel is in view and highlighted


def test_shade_other_suns(rt, gtree, ref_world_oracle):
    org, cd = CAMERAS[1]
    cam_dir = rt.normalize(cd)
    for sun in ((0.0, 1.0, 0.0), (-1.0, 0.5, -0.2), (0.3, -0.8, 0.5)):
        s = rt.normalize(sun)
        rgba, hits = gtree.shade_frame(org, cam_dir, 160, 90, 300, sun=s, with_hits=True)
        ref = ref_world_oracle.shade_frame(org, cam_dir, 160, 90, 300, s)
        _check(rgba, ref, rt.decode_hits(hits)["hit"], "sun %s" % (sun,))


def test_shade_depth12_sampled(rt, oracle_mod, torch_cuda):
    """C3 terrain at 1080p: sampled pixels against the oracle's terrain tree"""
    O = oracle_mod
    W, H = 1920, 1080
    tree = rt.Tree.terrain(6, 1024, 1024).upload(0)
    org, cam_dir = (4.0, 90.0, 4.0), rt.normalize((1.0, -0.45, 1.0))
    rgba, hits = tree.shade_frame(org, cam_dir, W, H, 16384, sun=rt.sun_dir(), with_hits=True)
    ot = O.Tree.terrain(6, 1024, 1024)
    pix = np.random.default_rng(5).choice(W * H, 4000, replace=False)
    ref = ot.shade_frame(org, cam_dir, W, H, 16384, rt.sun_dir(), pixels=pix)
    # hit records are indexed by pixel row from the bottom: the frame is unsharded, index = py * W + px
    g = rt.decode_hits(hits)
    _check(rgba[torch_cuda.as_tensor(pix, device=rgba.device)], ref, g["hit"][pix], "depth12")


GLASS, MIRROR = 0x4, 0x2


def _glass_edits():
    """glass (flags 4 -> stored 5) in view of both cameras, a mirror behind a glass wall, a 4^3 glass block"""
    pts, flags = [], []
    for x in (60, 61):  # wall across camera 0's view
        for y in range(44, 57):
            for z in range(40, 91):
                pts.append((x, y, z)); flags.append(GLASS)
    for y in range(44, 57):  # mirror behind it
        for z in range(50, 71):
            pts.append((70, y, z)); flags.append(MIRROR)
    for x in range(30, 101):  # slab in camera 1's view, above the terrain
        for z in range(30, 101):
            for y in (62, 63):
                pts.append((x, y, z)); flags.append(GLASS)
    return np.array(pts, np.int32), np.array(flags, np.uint32)


@pytest.fixture(scope="module")
def glass_worlds(rt, oracle_mod, torch_cuda):
    pts, flags = _glass_edits()
    colors = (np.arange(len(pts), dtype=np.uint64) * np.uint64(2654435761)) % np.uint64(1 << 63)
    w = rt.World.reference()
    w.put_blocks(pts, flags, colors)
    w.put_block(100, 72, 100, GLASS, 777, level=w.levels)  # a 4^3 glass block (one uniform node)
    o = oracle_mod.Tree.reference_world()
    for p, f, c in zip(pts, flags, colors):
        o.put_block(int(p[0]), int(p[1]), int(p[2]), int(f), int(c))
    o.put_block(100, 72, 100, GLASS, 777, level=5)
    return w.build().upload(0), o


@pytest.mark.parametrize("cam", [0, 1])
def test_shade_refraction(rt, glass_worlds, cam):
    """refractive solids (flags & 7 == 5): tint 0.95 per block passed, the first one bends the ray"""
    gt, ot = glass_worlds
    org, cd = CAMERAS[cam]
    cam_dir = rt.normalize(cd)
    for S in (300, 40):
        rgba, hits = gt.shade_frame(org, cam_dir, 240, 136, S, sun=rt.sun_dir(), with_hits=True)
        ref = ot.shade_frame(org, cam_dir, 240, 136, S, rt.sun_dir())
        _check(rgba, ref, rt.decode_hits(hits)["hit"], "glass cam%d S=%d" % (cam, S))
        if S != 300:
            continue
        # the bend is exercised: the shading pass ends elsewhere than the plain cast on many rays
        plain = rt.decode_hits(gt.cast_frame(org, cam_dir, 240, 136, S))["pos"]
        moved = np.any(rt.decode_hits(hits)["pos"] != plain, axis=1).sum()
        assert moved > 500, moved


# ---- liquid (low_res.frag:214-229, :325-326): water refracts and tints when the scene holds it --
LAKE_CAMERAS = [
    ((4.0, 90.0, 4.0), (1.0, -0.45, 1.0)),        # C1 pose: the lakes around (150, 20, 158) far ahead
    ((150.5, 40.25, 120.5), (0.1, -0.6, 1.0)),    # looking down into a lake
    ((162.5, 16.5, 128.5), (0.7, 0.15, -0.4)),    # under water (column top 10)
]


@pytest.fixture(scope="module")
def lake_scene(rt, ref_world, torch_cuda):
    return ref_world.build(rt.VIEW_ALL).upload(0)


@pytest.mark.parametrize("cam", range(len(LAKE_CAMERAS)))
@pytest.mark.parametrize("tm", [0.0, 2.75])
def test_shade_liquid_reference_world(rt, gtree, lake_scene, ref_world_oracle, cam, tm):
    """with the SVO_VIEW_ALL scene, water (flags 0x15) tints by (0.94, 0.97, 1.0) per voxel and the
    first refractive voxel bends the ray with the wave wobble of time `tm`; against the oracle's
    liquid mode, the same contract as the glass tests"""
    org, cd = LAKE_CAMERAS[cam]
    cam_dir = rt.normalize(cd)
    W, H, S = 240, 136, 300
    rgba, hits = gtree.shade_frame(org, cam_dir, W, H, S, sun=rt.sun_dir(), with_hits=True, scene=lake_scene, time=tm)
    ref = ref_world_oracle.shade_frame(org, cam_dir, W, H, S, rt.sun_dir(), liquid=True, time=tm)
    _check(rgba, ref, rt.decode_hits(hits)["hit"], "lake cam%d t=%g" % (cam, tm))
    # liquid is exercised: against the shading pass without the scene (water passes unbent)
    dry = gtree.shade_frame(org, cam_dir, W, H, S, sun=rt.sun_dir()).cpu().numpy()
    assert np.any(dry != rgba.cpu().numpy(), axis=1).sum() > 100


def test_shade_liquid_time_moves_the_bend(rt, gtree, lake_scene):
    org, cd = LAKE_CAMERAS[1]
    cam_dir = rt.normalize(cd)
    a = rt.decode_hits(gtree.shade_frame(org, cam_dir, 160, 90, 300, sun=rt.sun_dir(), with_hits=True, scene=lake_scene, time=0.0)[1])
    b = rt.decode_hits(gtree.shade_frame(org, cam_dir, 160, 90, 300, sun=rt.sun_dir(), with_hits=True, scene=lake_scene, time=0.37)[1])
    assert np.any(a["pos"] != b["pos"], axis=1).sum() > 100


def test_shade_liquid_depth12_sampled(rt, oracle_mod, torch_cuda):
    """C3 pose over 1024^2 terrain columns with their lakes: the GPU-built full-view scene, sampled
    pixels against the oracle's terrain tree in liquid mode"""
    W, H = 1920, 1080
    tree = rt.Tree.terrain_gpu(6, 1024, 1024, 0)
    scene = rt.Tree.terrain_gpu(6, 1024, 1024, 0, view=rt.VIEW_ALL)
    org, cam_dir = (4.0, 90.0, 4.0), rt.normalize((1.0, -0.45, 1.0))
    rgba, hits = tree.shade_frame(org, cam_dir, W, H, 16384, sun=rt.sun_dir(), with_hits=True, scene=scene, time=1.25)
    ot = oracle_mod.Tree.terrain(6, 1024, 1024)
    pix = np.random.default_rng(6).choice(W * H, 4000, replace=False)
    ref = ot.shade_frame(org, cam_dir, W, H, 16384, rt.sun_dir(), pixels=pix, liquid=True, time=1.25)
    g = rt.decode_hits(hits)
    _check(rgba[torch_cuda.as_tensor(pix, device=rgba.device)], ref, g["hit"][pix], "depth12 lakes")
    # column-ceiling moves (primary and refracted rays) change nothing: the whole image and its records
    rgba2, hits2 = tree.shade_frame(org, cam_dir, W, H, 16384, sun=rt.sun_dir(), with_hits=True, scene=scene, time=1.25,
                                    flags=rt.CAST_NO_CEILINGS)
    assert torch_cuda.equal(rgba, rgba2)
    for k in hits:
        assert torch_cuda.equal(hits[k], hits2[k]), k


def test_full_view_tree_is_not_castable(rt, lake_scene):
    """castRayFromCam semantics need the solid view: a full-view tree is refused, not silently cast"""
    with pytest.raises(RuntimeError):
        lake_scene.cast_frame((4.0, 90.0, 4.0), rt.normalize((1.0, -0.45, 1.0)), 16, 16, 300)


@pytest.mark.parametrize("cam", range(len(LAKE_CAMERAS)))
def test_shade_escape_is_exact(rt, gtree, lake_scene, cam):
    """without hit records, shading rays moving up above the highest stored voxel row stop early (no
    voxel can be hit any more, and none of the remaining steps wraps in y): the image equals the one
    rendered with hit records (every ray walks its whole budget), bit for bit, at large budgets too"""
    org, cd = LAKE_CAMERAS[cam]
    cam_dir = rt.normalize(cd)
    for S in (300, 5000):
        full, _ = gtree.shade_frame(org, cam_dir, 200, 120, S, sun=rt.sun_dir(), with_hits=True, scene=lake_scene, time=0.5)
        fast = gtree.shade_frame(org, cam_dir, 200, 120, S, sun=rt.sun_dir(), scene=lake_scene, time=0.5)
        assert np.array_equal(full.cpu().numpy(), fast.cpu().numpy()), (cam, S)
        f2, _ = gtree.shade_frame(org, cam_dir, 200, 120, S, sun=rt.sun_dir(), with_hits=True)
        g2 = gtree.shade_frame(org, cam_dir, 200, 120, S, sun=rt.sun_dir())
        assert np.array_equal(f2.cpu().numpy(), g2.cpu().numpy()), (cam, S)


def test_shade_bench_scene_full_frame(rt, depth12, oracle12, torch_cuda):
    """The shaded workload bench.py --shade times, every pixel: the GPU-built 4096^2-column solid and full-view
    (water) trees, the C3 pose, S = 16384, the reference sun; the image without hit records (the bench's form:
    escaping rays stop early) against the oracle's liquid mode over the whole 1080p frame (low_res.frag:139-252,
    319-391), equal to the image rendered with hit records, and the water is exercised (refracted rays travel
    4x further before wrapping than on the 1024^2 scenes above)."""
    torch = torch_cuda
    scene = rt.Tree.terrain_gpu(6, 4096, 4096, 0, view=rt.VIEW_ALL)
    org, cam_dir = (4.0, 90.0, 4.0), rt.normalize((1.0, -0.45, 1.0))
    W, H, S = 1920, 1080, 16384
    img = depth12.shade_frame(org, cam_dir, W, H, S, sun=rt.sun_dir(), scene=scene)
    rgba, hits = depth12.shade_frame(org, cam_dir, W, H, S, sun=rt.sun_dir(), with_hits=True, scene=scene)
    assert torch.equal(img, rgba)  # escape is exact
    ref = oracle12.shade_frame(org, cam_dir, W, H, S, rt.sun_dir(), liquid=True, nthreads=16)
    hit = rt.decode_hits(hits)["hit"]
    _check(img, ref, hit, "bench scene")
    dry = depth12.shade_frame(org, cam_dir, W, H, S, sun=rt.sun_dir())
    wet = int((dry != img).any(1).sum().item())
    assert wet > 100000, wet  # lake pixels: tinted and refracted
    del scene
