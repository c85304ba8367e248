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


def test_shade_liquid_depth14_sampled(rt, oracle_mod, torch_cuda):
    """a 7-level tree (depth 14, the deepest the builders take: the shading kernel's LDS path is sized by the launch's
    depth, path_lds) over 1024^2 terrain columns with lakes: sampled pixels against the oracle, and the image without
    hit records (the no-record instances: escape, no crossing value, the straight trace without segment bounds) equal
    to the one with them"""
    W, H = 960, 540
    tree = rt.Tree.terrain_gpu(7, 1024, 1024, 0)
    scene = rt.Tree.terrain_gpu(7, 1024, 1024, 0, view=rt.VIEW_ALL)
    org, cam_dir = (4.0, 90.0, 4.0), rt.normalize((1.0, -0.45, 1.0))
    rgba, hits = tree.shade_frame(org, cam_dir, W, H, 16384, sun=rt.sun_dir(), with_hits=True, scene=scene, time=0.5)
    ot = oracle_mod.Tree.terrain(7, 1024, 1024)
    pix = np.random.default_rng(14).choice(W * H, 3000, replace=False)
    ref = ot.shade_frame(org, cam_dir, W, H, 16384, rt.sun_dir(), pixels=pix, liquid=True, time=0.5)
    g = rt.decode_hits(hits)
    _check(rgba[torch_cuda.as_tensor(pix, device=rgba.device)], ref, g["hit"][pix], "depth14 lakes")
    rgba2 = tree.shade_frame(org, cam_dir, W, H, 16384, sun=rt.sun_dir(), scene=scene, time=0.5)
    assert torch_cuda.equal(rgba, rgba2)


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


@pytest.mark.parametrize("sun", [None, (2.0, -1.0, 4.0), (-2.0, 1.0, -4.0)])
def test_shadow_octant_equals_sign_flags(rt, gtree, lake_scene, sun):
    """Shadow rays of the reference sun, normalize(2, 1, 4) (globals.cpp:23), run a copy of the trace with that step
    octant compiled in; SVO_CAST_NO_OCTANT gives every shadow (and primary) ray per-wave sign flags instead.  The images
    are identical, for that sun and for suns of other octants (which take the flags either way)."""
    org, cd = LAKE_CAMERAS[1]  # looking down into a lake: lit and shadowed faces
    cam_dir = rt.normalize(cd)
    s = rt.sun_dir() if sun is None else tuple(rt.normalize(sun))
    a = gtree.shade_frame(org, cam_dir, 200, 120, 5000, sun=s, scene=lake_scene, time=0.5)
    b = gtree.shade_frame(org, cam_dir, 200, 120, 5000, sun=s, scene=lake_scene, time=0.5, flags=rt.CAST_NO_OCTANT)
    assert np.array_equal(a.cpu().numpy(), b.cpu().numpy())
    c = gtree.shade_frame(org, cam_dir, 200, 120, 5000, sun=s, scene=lake_scene, time=0.5, shadow_steps=0)
    assert not np.array_equal(a.cpu().numpy(), c.cpu().numpy())  # (the shadow rays darken some pixels: exercised)


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


def test_shadow_rays_use_the_solid_trees_ceilings(rt, torch_cuda):
    """Shadow rays walk the solid tree, so they cross the solid tree's own column-ceiling boxes (trace CEIL 3), not the
    scene's: with the scene one edit behind (a 4^3 block put above the 16-column block's old ceiling, the solid tree
    synced, the scene not), the image equals the one rendered without ceilings (SVO_CAST_NO_CEILINGS: ceilings are an
    exact acceleration), and the new block's shadow shows.  (Round 4 used the scene's table: shadow rays jumped over
    the new block.)"""
    torch = torch_cuda
    w = rt.World.reference()
    t = w.build().upload(0)
    sc = w.build(rt.VIEW_ALL).upload(0)
    org, cam_dir = (50.0, 70.0, 40.0), rt.normalize((20.0, -28.0, 25.0))
    W, H, S = 160, 120, 300
    before = t.shade_frame(org, cam_dir, W, H, S, sun=rt.sun_dir(), scene=sc)
    w.put_block(72, 46, 72, 0, 777, level=5)  # rows 44-47 over columns (72..75, 72..75); the block's ceiling was 43
    t.update(w, np.array([[72, 46, 72]], np.int32), level=5)
    t.sync()  # the scene lags
    a = t.shade_frame(org, cam_dir, W, H, S, sun=rt.sun_dir(), scene=sc)
    b = t.shade_frame(org, cam_dir, W, H, S, sun=rt.sun_dir(), scene=sc, flags=rt.CAST_NO_CEILINGS)
    assert torch.equal(a, b)
    assert int((a != before).any(1).sum()) > 50  # the shadow (the lagging scene does not draw the block itself)


def test_shade_escape_and_look_at(rt, gtree, lake_scene, torch_cuda):
    """An escaped ray (no hit records: it stops once only empty voxels lie ahead) keeps the position where it escaped,
    but low_res.frag:347 compares every ray's END with lookingAtBlock, misses included.  A launch whose look-at voxel
    the scene may not store — a host look-at on an empty voxel, or a device pick record that is not a sure hit —
    lets no ray escape; with a hit pick, escaped rays skip the comparison (they end on empty voxels only).  Each image
    equals the one rendered with hit records (where no ray escapes), and the highlight of a miss's end voxel shows."""
    torch = torch_cuda
    s = torch.cuda.Stream()
    org, cam_dir = (4.0, 90.0, 4.0), rt.normalize((1.0, -0.45, 1.0))
    W, H, S = 200, 120, 300
    sun = rt.sun_dir()
    full, hits = gtree.shade_frame(org, cam_dir, W, H, S, sun=sun, with_hits=True, scene=lake_scene)
    g = rt.decode_hits(hits)
    miss = np.nonzero(~g["hit"])[0]
    assert len(miss) > 100
    # host look-at on the end voxel of a miss (an empty voxel): the reference highlights that pixel
    p = int(miss[len(miss) // 2])
    look = tuple(int(v) for v in g["pos"][p])
    ref, _ = gtree.shade_frame(org, cam_dir, W, H, S, sun=sun, look_at=look, with_hits=True, scene=lake_scene)
    fast = gtree.shade_frame(org, cam_dir, W, H, S, sun=sun, look_at=look, scene=lake_scene)
    assert torch.equal(ref, fast)
    assert bool((ref[p] != full[p]).any())
    # the device record of a pick along a missing pixel's own ray with the frame's budget: a miss (stepsLeft 0) that
    # ends on that pixel's end voxel
    ppx, ppy = rt.proj_plane(W, H)
    rec = torch.zeros(64, dtype=torch.int32, device="cuda")
    desc = gtree.frame_desc(org, cam_dir, W, H, S)
    found = 0
    for p in miss[::max(1, len(miss) // 40)]:
        p = int(p)
        d = rt.pixel_dir(cam_dir, ppx, ppy, W, H, p % W, p // W)
        gtree.cast_ray_from_cam_async(org, d, S, rec, stream=s)
        s.synchronize()
        r = rec[:7].cpu().numpy()
        if tuple(r[:3]) != tuple(g["pos"][p]) or r[6] != 0:
            continue  # (a ray bent by water in the scene ends elsewhere)
        a = torch.empty((W * H, 4), dtype=torch.float32, device="cuda")
        b = torch.empty_like(a)
        out = gtree.alloc_hits(W * H, 0)
        with torch.cuda.stream(s):
            gtree.shade(desc, a, sun=sun, look_at=rec, stream=s, scene=lake_scene)
            gtree.shade(desc, b, sun=sun, look_at=rec, out=out, stream=s, scene=lake_scene)
        s.synchronize()
        assert torch.equal(a, b), p
        assert bool((a[p] != full[p]).any()), p
        found += 1
        if found == 3:
            break
    assert found > 0
    # a sure hit (stepsLeft 15 > 0): rays escape and escaped ones skip the comparison
    org2, cam2 = (35.0, 50.0, 35.0), rt.normalize((1.0, -1.0, 1.0))
    gtree.cast_ray_from_cam_async(org2, cam2, 30, rec, stream=s)
    s.synchronize()
    assert int(rec[6]) == 15
    d2 = gtree.frame_desc(org2, cam2, W, H, S)
    a = torch.empty((W * H, 4), dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    out = gtree.alloc_hits(W * H, 0)
    with torch.cuda.stream(s):
        gtree.shade(d2, a, sun=sun, look_at=rec, stream=s, scene=lake_scene)
        gtree.shade(d2, b, sun=sun, look_at=rec, out=out, stream=s, scene=lake_scene)
    s.synchronize()
    assert torch.equal(a, b)
