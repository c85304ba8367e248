"""GPU parity: the gfx950 cast kernel (through the C ABI) against the oracle's restatement of
castRayFromCam (src/ray_caster.cpp:54-87) on the same inputs.

Bar: bit-exact voxel position, lastPos, stepsLeft, hit flag and block (flags, colour); hit.t
within 1e-5 relative (north_star) — the kernel actually reproduces it bit-exactly, which is also
checked.  Parity domain: outside root child 63 of the reference world."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

T_RTOL = 1e-5  # north_star tolerance on hit.t


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


def compare(rt, tree, gpu_out, ref, label):
    g = rt.decode_hits(gpu_out)
    pal = tree.palette()
    pf = np.array([p[0] for p in pal], np.uint32)
    pc = np.array([p[1] for p in pal], np.uint64)
    n = len(ref["hit"])
    assert len(g["hit"]) == n, label
    bad = np.nonzero((g["pos"] != ref["pos"]).any(1))[0]
    assert len(bad) == 0, "%s: pos differs at %d rays, first %s gpu=%s ref=%s" % (label, len(bad), bad[:5], g["pos"][bad[:3]], ref["pos"][bad[:3]])
    assert np.array_equal(g["hit"], ref["hit"] != 0), label
    assert np.array_equal(g["steps"], ref["steps"]), label
    assert np.array_equal(g["last_pos"], ref["last"]), label
    mid = np.where(g["hit"], g["material"], 0)
    assert np.array_equal(pf[mid], ref["flags"]) and np.array_equal(pc[mid], ref["color"]), label
    with np.errstate(over="ignore"):  # (crossing values beyond the f32 range are inf on both sides)
        rt_ = ref["t"].astype(np.float32)
    gt = g["t"]
    fin = np.isfinite(rt_)
    assert np.array_equal(np.isnan(gt), np.isnan(rt_)), label
    assert np.all(np.abs(gt[fin] - rt_[fin]) <= T_RTOL * np.maximum(1.0, np.abs(rt_[fin]))), label
    assert np.array_equal(gt[fin], rt_[fin]), label + " (t not bit-exact)"


CAMERAS = [
    ((35.0, 50.0, 35.0), (1.0, 0.0, 1.0)),      # reference default (globals.cpp:20-21)
    ((4.0, 90.0, 4.0), (1.0, -0.45, 1.0)),      # SURVEY.md C1 pose
    ((100.0, 120.0, 100.0), (1.0, -1.2, 0.3)),
    ((150.3, 44.7, 20.9), (-0.6, -0.2, 1.0)),   # fractional origin, negative x
    ((60.5, 70.5, 40.5), (1.0, -0.5, 0.6)),     # half-integral origins: the linear (no-segment) instance
    ((-20.5, 55.5, 130.5), (0.7, -0.3, 1.0)),   # (negative x: trunc != floor, deltaPos starts at 1.5a / -0.5a)
]


@pytest.mark.parametrize("cam", range(len(CAMERAS)))
@pytest.mark.parametrize("steps", [30, 300])
def test_reference_world_frames(rt, oracle_mod, gtree, ref_world_oracle, cam, steps):
    org, d = CAMERAS[cam]
    dn = rt.normalize(d)
    W = H = 256
    ref = ref_world_oracle.cast_frame(org, dn, W, H, steps)
    assert ref["rc"] == 0
    for flags in (0, rt.CAST_ITERATIVE, rt.CAST_BOTTOM_FIRST, rt.CAST_TILE_8X8, rt.CAST_TILE_32X2, rt.CAST_WIDE_ADDR, rt.CAST_NO_CEILINGS, rt.CAST_SEGMENTS, rt.CAST_NO_OCTANT, rt.CAST_SEGMENTS | rt.CAST_ITERATIVE):
        out = gtree.cast_frame(org, dn, W, H, steps, flags=flags)
        compare(rt, gtree, out, ref, "cam%d S=%d flags=%d" % (cam, steps, flags))


def test_reference_world_1080p(rt, gtree, ref_world_oracle):
    org, d = CAMERAS[0]
    dn = rt.normalize(d)
    out = gtree.cast_frame(org, dn, 1920, 1080, 300)
    ref = ref_world_oracle.cast_frame(org, dn, 1920, 1080, 300, nthreads=16)
    compare(rt, gtree, out, ref, "1080p")
    g = rt.decode_hits(out)
    assert abs(g["hit"].mean() - 0.469) < 5e-4  # SURVEY.md §6 (reference probe)


def _explicit(rt, torch, tree, T, origins, dirs, steps, flags=0):
    dirs = np.ascontiguousarray(dirs, np.float32)
    origins = np.ascontiguousarray(origins, np.float32)
    gd = torch.from_numpy(dirs).cuda()
    go = torch.from_numpy(origins).cuda()
    out = tree.cast_rays(gd, go, steps=steps, flags=flags)
    ref = {k: [] for k in ("pos", "last", "steps", "hit", "flags", "color", "t")}
    for o, d in zip(origins, dirs):
        r = T.cast_ray(o, d, steps)
        assert r.err == 0
        ref["pos"].append(list(r.pos))
        ref["last"].append(list(r.last))
        ref["steps"].append(r.steps)
        ref["hit"].append(r.hit)
        ref["flags"].append(r.flags)
        ref["color"].append(r.color)
        ref["t"].append(r.t)
    dt = {"flags": np.uint32, "color": np.uint64, "t": np.float64}
    ref = {k: np.array(v, dtype=dt.get(k, np.int64)) for k, v in ref.items()}
    return out, ref


def test_edge_case_rays(rt, oracle_mod, torch_cuda, gtree, ref_world_oracle):
    hs = rt.terrain_heights(200, 200)
    lake = np.argwhere(hs < 17)[0]
    n = rt.normalize
    cases = [
        ((35, 50, 35), n([1, 0, 1]), 30),           # the reference pick ray: NaN deltaPos, walks z
        ((35, 50, 35), n([1, 0, 1]), 300),
        ((50.5, 60, 50.5), (0.0, -1.0, 0.0), 300),  # exact zero components
        ((50.0, 60, 50.0), (0.0, -1.0, 0.0), 300),  # integral origin + zero dir: NaN on x and z
        ((50.5, 60, 50.5), (-0.0, -1.0, -0.0), 300),  # negative zeros: step +1, delta -inf
        ((-3.5, 40.25, -2.75), n([1, -0.3, 1]), 300),  # trunc != floor
        ((-0.5, 45.0, 120.5), n([-1, -0.2, 0.1]), 300),
        ((1020.5, 35.5, 50.5), n([1, -0.05, 0.01]), 300),  # wraps past 1024
        ((30.5, 40.5, 1022.5), n([0.02, -0.1, 1]), 300),
        ((lake[0] + 0.5, 40.5, lake[1] + 0.5), (0.0, -1.0, 0.0), 300),  # water pass-through
        ((21.5, 30.0, 201.5), (0.0, -1.0, 0.0), 300),  # level-5 leaf, flags 5
        ((10.5, 110.0, 10.5), (0.0, -1.0, 0.0), 300),  # reflective voxel (10,100,10), flags 3
        ((10.5, 110.0, 10.5), (0.0, -1.0, 0.0), 10),   # hit on the last step: steps = 0
        ((10.5, 110.0, 10.5), (0.0, -1.0, 0.0), 9),    # one short: miss
        ((10.5, 110.0, 10.5), (0.0, -1.0, 0.0), 0),    # no step at all
        ((10.5, 110.0, 10.5), (0.0, 0.0, 0.0), 50),    # zero direction: all NaN, walks z
        ((12.25, 70.5, 80.75), (float("nan"), -1.0, 0.0), 50),
        ((99.9, 33.3, 66.6), n([1e-30, -1, 1e-30]), 300),
        ((5.5, 200.0, 5.5), n([0.3, -1, 0.2]), 300),
    ]
    origins = np.array([c[0] for c in cases], np.float32)
    dirs = np.array([c[1] for c in cases], np.float32)
    for steps in sorted(set(c[2] for c in cases)):
        sel = [i for i, c in enumerate(cases) if c[2] == steps]
        for flags in (0, rt.CAST_ITERATIVE, rt.CAST_WIDE_ADDR):
            out, ref = _explicit(rt, torch_cuda, gtree, ref_world_oracle, origins[sel], dirs[sel], steps, flags)
            compare(rt, gtree, out, ref, "edge S=%d flags=%d" % (steps, flags))


def test_tiny_direction_rays(rt, torch_cuda, gtree, ref_world_oracle):
    """Unnormalised directions with tiny components (absDelta up to ~1e37): crossing values far above
    the f32 range.  castRayFromCam's double DDA walks them like the unit directions they scale; the
    kernel's closed-form crossings estimate counts in f32, so rays whose every absDelta is >= 2^100
    take the stepping path (span_ok), the others cross boxes as usual."""
    n = rt.normalize
    base = [((5.5, 200.0, 5.5), n([0.3, -1, 0.2])), ((40.0, 90.0, 40.0), n([1, -0.45, 1])),
            ((120.25, 70.5, 30.75), n([-0.6, -0.5, 0.4])), ((60.0, 61.0, 60.0), n([0.01, -1, 0.02]))]
    origins, dirs = [], []
    for o, d in base:
        # (8e-38: every absDelta above 2^100 and every box exit event beyond the f32 range; the 0.01
        # component becomes subnormal there, an infinite absDelta)
        for scale in (1.0, 3e-20, 1.7e-30, 1e-34, 8e-38):
            origins.append(o)
            dirs.append([np.float32(c * scale) for c in d])
    origins = np.array(origins, np.float32)
    dirs = np.array(dirs, np.float32)
    for steps in (300, 3000):
        for flags in (0, rt.CAST_ITERATIVE):
            out, ref = _explicit(rt, torch_cuda, gtree, ref_world_oracle, origins, dirs, steps, flags)
            compare(rt, gtree, out, ref, "tiny dirs S=%d flags=%d" % (steps, flags))
            assert ref["hit"].sum() >= len(base) * 3  # they reach the terrain


def test_huge_origin_rays_terminate(rt, torch_cuda, gtree):
    """Origins beyond the int range (castRayFromCam's `(int)` of them is undefined behaviour, so there is
    no reference result): the launch must end, and the closed-form path must agree with voxel stepping
    (both start from the same clamped cell)."""
    rng = np.random.default_rng(5)
    vals = [1e10, -3e9, 2147483648.0, -2147483904.0, 1.5e30, -3.4e38, 1073741824.0, 1073741760.5]
    org = np.array([[rng.choice(vals), rng.uniform(0, 120), rng.uniform(0, 200)] for _ in range(64)], np.float32)
    org[::2] = org[::2][:, [1, 0, 2]]
    org[::3] = org[::3][:, [2, 1, 0]]
    d = rng.normal(size=(64, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    gd, go = torch_cuda.from_numpy(d).cuda(), torch_cuda.from_numpy(org).cuda()
    for steps in (300, 5000):
        a = rt.decode_hits(gtree.cast_rays(gd, go, steps=steps))
        b = rt.decode_hits(gtree.cast_rays(gd, go, steps=steps, flags=rt.CAST_ITERATIVE))
        for k in ("pos", "hit", "steps", "last_pos"):
            assert np.array_equal(a[k], b[k]), (steps, k)


def _segment_hits_box(o, d, tmax, lo, hi):
    """slab test of segments o + t d, t in [0, tmax], against the box [lo, hi] (conservative)"""
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d.astype(np.float64)
        t1 = (lo - 1.0 - o) * inv
        t2 = (hi + 1.0 - o) * inv
    tn = np.where(np.isnan(t1), -np.inf, np.minimum(t1, t2))
    tf = np.where(np.isnan(t2), np.inf, np.maximum(t1, t2))
    inside = (o >= lo - 1.0) & (o <= hi + 1.0)
    tn = np.where(d == 0, np.where(inside, -np.inf, np.inf), tn)
    tf = np.where(d == 0, np.where(inside, np.inf, -np.inf), tf)
    enter = np.maximum(tn.max(1), 0.0)
    leave = np.minimum(tf.min(1), tmax)
    return enter <= leave


def test_random_rays(rt, torch_cuda, gtree, ref_world_oracle):
    rng = np.random.default_rng(11)
    n = 4000
    org = np.stack([rng.uniform(-50, 250, n), rng.uniform(0, 120, n), rng.uniform(-50, 250, n)], 1).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[::7, 1] = 0.0  # plenty of exact zero components
    d[::11, 0] = 0.0
    # parity domain: drop rays whose first 300 DDA steps (ray parameter t <= 301, as the L1 norm of
    # a unit direction is >= 1) can reach root child 63 = [768,1024)^3 after wrapping, i.e. the
    # octant box [-256, 0)^3 for these origins
    keep = ~_segment_hits_box(org, d, 301.0, np.full(3, -256.0), np.zeros(3))
    org, d = org[keep], d[keep]
    for flags in (0, rt.CAST_ITERATIVE):
        out, ref = _explicit(rt, torch_cuda, gtree, ref_world_oracle, org, d, 300, flags)
        compare(rt, gtree, out, ref, "random flags=%d" % flags)


def test_cast_ray_from_cam_dropin(rt, gtree, ref_world_oracle):
    for (org, d) in CAMERAS:
        dn = rt.normalize(d)
        for steps in (0, 1, 30, 300):
            (pos, last, st), blk = gtree.cast_ray_from_cam(org, dn, steps)
            r = ref_world_oracle.cast_ray(org, dn, steps)
            assert pos == tuple(r.pos) and last == tuple(r.last) and st == r.steps
            assert blk[:2] == (r.flags, r.color)


def test_tile_row_sharding_reassembles(rt, torch_cuda, gtree):
    org, d = CAMERAS[1]
    dn = rt.normalize(d)
    W, H = 320, 200  # 25 tile rows
    full = rt.decode_hits(gtree.cast_frame(org, dn, W, H, 300))
    for G in (2, 3, 4):
        rows = np.zeros((H, W), bool)
        for r in range(G):
            part = rt.decode_hits(gtree.cast_frame(org, dn, W, H, 300, tile_row_start=r, tile_row_step=G))
            tr = list(range(r, (H + 7) // 8, G))
            py = np.concatenate([np.arange(t * 8, min(H, t * 8 + 8)) for t in tr])
            idx = (py[:, None] * W + np.arange(W)[None, :]).ravel()
            for k in ("pos", "steps", "material", "t"):
                assert np.array_equal(part[k], full[k][idx]), (G, r, k)
            rows[py] = True
        assert rows.all()


def test_wavefront_footprints_ragged_frames(rt, gtree):
    """8x8 / 32x2 wavefront footprints (scheduling only) write the same records as the default 16x4,
    on frame sizes that are not multiples of the footprint, whole and sharded."""
    org, d = CAMERAS[2]
    dn = rt.normalize(d)
    for W, H in ((100, 60), (33, 17), (8, 8)):
        for start, step in ((0, 1), (1, 3)):
            if start >= (H + 7) // 8:
                continue  # an empty shard
            base = rt.decode_hits(gtree.cast_frame(org, dn, W, H, 300, tile_row_start=start, tile_row_step=step))
            for flags in (rt.CAST_TILE_8X8, rt.CAST_TILE_32X2, rt.CAST_BOTTOM_FIRST, rt.CAST_BOTTOM_FIRST | rt.CAST_TILE_8X8):
                got = rt.decode_hits(gtree.cast_frame(org, dn, W, H, 300, tile_row_start=start, tile_row_step=step, flags=flags))
                for k in base:
                    assert np.array_equal(got[k], base[k]), (W, H, start, step, flags, k)


def test_multi_frame_launch(rt, torch_cuda, gtree):
    """Several frames (camera positions) in one launch, whole and sharded: frame f's records equal
    a single-frame cast of it; the AO counts and the shading pass follow the same layout."""
    _, d = CAMERAS[1]
    dn = rt.normalize(d)
    origins = [(4.0, 90.0, 4.0), (68.0, 90.0, 68.0), (-30.5, 70.25, 12.75), (150.3, 44.7, 20.9)]
    W, H = 72, 44
    for start, step in ((0, 1), (1, 3)):
        desc = rt.Tree.frame_desc(origins[0], dn, W, H, 300, tile_row_start=start, tile_row_step=step, frame_origins=origins,
                                  ao_samples=16, ao_steps=5)
        n = rt.Tree.count(desc)
        out = rt.Tree.alloc_hits(n, 0, ao=True)
        gtree.cast(desc, out)
        torch_cuda.cuda.synchronize()
        multi = rt.decode_hits(out)
        per = n // len(origins)
        for f, org in enumerate(origins):
            one = rt.decode_hits(gtree.cast_frame(org, dn, W, H, 300, tile_row_start=start, tile_row_step=step, ao_samples=16))
            for k in one:
                assert np.array_equal(multi[k][f * per:(f + 1) * per], one[k]), (start, step, f, k)


def test_wire_formats(rt, torch_cuda, gtree):
    """svo_hits_pack / svo_hits_unpack / svo_cast_wire (the exchange formats of the tile-row gather) against
    the numpy restatements in tests/wire_ref.py, and unpack(pack(records)) == records: 8-B compact records
    for frames from integral / half-integral camera positions (the receiver rebuilds each pixel's ray for
    the position and t), 12-B records for other origins and explicit rays; hits and misses (budget 30),
    several frames, axis-aligned camera directions (exact zero components: NaN / infinite deltaPos)."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import wire_ref

    torch = torch_cuda
    cases = [([(35.0, 50.0, 35.0), (-3.5, 40.25, -2.75), (1020.5, 35.5, 50.5)], (1.0, 0.0, 1.0), 12),
             ([(35.0, 50.0, 35.0), (-3.5, 40.5, -2.0), (1020.5, 35.5, 50.5)], (1.0, 0.0, 1.0), 8),
             ([(4.0, 90.0, 4.0), (60.5, 70.5, 40.5)], (1.0, -0.45, 1.0), 8),
             ([(50.5, 60.0, 50.5)], (0.0, -1.0, 0.0), 8), ([(100.0, 80.0, 20.0)], (-0.3, -0.4, 1.0), 8)]
    kinds = set()
    for origins, cam, wb in cases:
        dn = rt.normalize(cam)
        for steps in (30, 300):
            desc = rt.Tree.frame_desc(origins[0], dn, 64, 40, steps, frame_origins=origins if len(origins) > 1 else None)
            assert gtree.wire_bytes(desc) == wb, (origins, wb)
            n = rt.Tree.count(desc)
            out = rt.Tree.alloc_hits(n, 0)
            gtree.cast(desc, out)
            wire = torch.zeros((n, wb), dtype=torch.uint8, device="cuda")
            gtree.pack_hits(desc, out, wire)
            fused = torch.zeros((n, wb), dtype=torch.uint8, device="cuda")
            gtree.cast_wire(desc, fused)
            back = rt.Tree.alloc_hits(n, 0)
            gtree.unpack_hits(desc, wire, back)
            torch.cuda.synchronize()
            assert torch.equal(fused, wire), (origins, steps)  # the cast kernel's own wire records == pack(cast)
            per = n // len(origins)
            o = np.repeat(np.asarray(origins, np.float32), per, 0)
            cells = np.trunc(o).astype(np.int32)
            ps, t, info = out["pos_steps"].cpu().numpy(), out["t"].cpu().numpy(), out["info"].cpu().numpy().view(np.uint32)
            w = wire.cpu().numpy()
            if wb == 12:
                assert np.array_equal(w, wire_ref.pack(ps, t, info, cells)), steps
            else:
                assert np.array_equal(w, wire_ref.pack_compact(ps, info, cells)), steps
                dirs = np.tile(rt.pixel_dirs(dn, 64, 40).reshape(-1, 3), (len(origins), 1))
                ps2, t2, info2 = wire_ref.unpack_compact(w, o, dirs, steps)
                assert np.array_equal(ps2, ps) and np.array_equal(info2, info) and np.array_equal(t2.view(np.uint32), t.view(np.uint32))
            for k in ("pos_steps", "t", "info"):
                assert np.array_equal(back[k].cpu().numpy().view(np.uint32), out[k].cpu().numpy().view(np.uint32)), (origins, steps, k)
            g = rt.decode_hits(out)
            kinds.add((steps, bool(g["hit"].any()), bool((~g["hit"]).any())))
    assert (30, True, True) in kinds  # hits and misses in one frame at the small budget
    rng = np.random.default_rng(3)
    org = np.stack([rng.uniform(-50, 250, 500), rng.uniform(0, 120, 500), rng.uniform(-50, 250, 500)], 1).astype(np.float32)
    dr = rng.normal(size=(500, 3)).astype(np.float32)
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    go, gd = torch.from_numpy(org).cuda(), torch.from_numpy(dr).cuda()
    out = gtree.cast_rays(gd, go, steps=300)
    desc = rt.CastDesc()
    desc.ray_dirs, desc.ray_origins, desc.n_rays, desc.steps = gd.data_ptr(), go.data_ptr(), 500, 300
    assert gtree.wire_bytes(desc) == 12
    wire = torch.zeros((500, 12), dtype=torch.uint8, device="cuda")
    gtree.pack_hits(desc, out, wire)
    back = rt.Tree.alloc_hits(500, 0)
    gtree.unpack_hits(desc, wire, back)
    torch.cuda.synchronize()
    for k in ("pos_steps", "t", "info"):
        assert np.array_equal(back[k].cpu().numpy(), out[k].cpu().numpy()), k


@pytest.mark.parametrize("N", [2, 3])
def test_wire_scatter_shards(rt, torch_cuda, gtree, N):
    """The display side of the N > 1 exchange on one GPU: every rank's shard (tile rows r, r + N, ... of two
    frames, a height that is not a multiple of 8) cast straight to wire records (svo_cast_wire) and decoded
    into its pixels of the whole frames (svo_wire_scatter, the exchange's decode): the union equals one
    unsharded cast of each frame, in both wire formats, AO counts alongside."""
    torch = torch_cuda
    cam = rt.normalize((1.0, -0.45, 1.0))
    W, H = 50, 37
    for origins in ([(4.0, 90.0, 4.0), (60.5, 70.5, 40.5)], [(4.25, 90.0, 4.0), (60.5, 70.5, 40.5)]):
        frames = rt.Tree.alloc_hits(2 * W * H, 0, ao=True)
        for k in frames:
            frames[k].fill_(-1 if frames[k].dtype != torch.uint8 else 255)
        for r in range(N):
            d = rt.Tree.frame_desc(origins[0], cam, W, H, 300, tile_row_start=r, tile_row_step=N, frame_origins=origins, ao_samples=16)
            n = rt.Tree.count(d)
            wb = gtree.wire_bytes(d)
            assert wb == (8 if origins[0][0] == 4.0 else 12)
            wire = torch.zeros((n, wb), dtype=torch.uint8, device="cuda")
            ao = torch.zeros(n, dtype=torch.uint8, device="cuda")
            gtree.cast_wire(d, wire, ao)
            gtree.wire_scatter(d, wire, frames, ao=ao)
        torch.cuda.synchronize()
        for f, org in enumerate(origins):
            one = gtree.cast_frame(org, cam, W, H, 300, ao_samples=16)
            for k in ("pos_steps", "t", "info", "ao"):
                got = frames[k][f * W * H:(f + 1) * W * H]
                assert torch.equal(got, one[k]), (N, origins, f, k)


def test_dense_grid_c1(rt, oracle_mod, torch_cuda, ref_world_oracle):
    """Config C1: the reference world's [0,256)^3 as a dense grid (coordinates & 255) on the CPU
    oracle vs the same voxels in a 4-level tree on the GPU."""
    D = oracle_mod.Dense(ref_world_oracle, 256)
    rc, f, c = ref_world_oracle.dump_box(0, 0, 0, 256, 256, 256)
    nz = np.argwhere(c != np.uint64(0xFFFFFFFFFFFFFFFF))
    w = rt.World(4)
    pts = nz[:, ::-1]  # (z,y,x) -> (x,y,z)
    w.put_blocks(pts, f[c != np.uint64(0xFFFFFFFFFFFFFFFF)] & ~np.uint32(1), c[c != np.uint64(0xFFFFFFFFFFFFFFFF)])
    t = w.build().upload(0)
    dn = rt.normalize([1, 0, 1])
    out = rt.decode_hits(t.cast_frame((35, 50, 35), dn, 256, 256, 300))
    ref = D.cast_frame((35, 50, 35), dn, 256, 256, 300)
    assert np.array_equal(out["pos"], ref["pos"]) and np.array_equal(out["steps"], ref["steps"])
    assert np.array_equal(out["hit"], ref["hit"] != 0)
    pal = t.palette()
    pc = np.array([p[1] for p in pal], np.uint64)
    assert np.array_equal(pc[np.where(out["hit"], out["material"], 0)], ref["color"])


def test_depth12_full_frame_parity(rt, depth12, oracle12):
    """C3: depth-12 terrain (4096^2 columns, 6 levels), the C1 pose, S = 16384; every pixel of the
    1080p frame against the oracle's reference-format tree, every field (the frame bench.py times)."""
    dn = rt.normalize([1, -0.45, 1])
    W, H = 1920, 1080
    out = depth12.cast_frame((4, 90, 4), dn, W, H, 16384)
    ref = oracle12.cast_frame((4, 90, 4), dn, W, H, 16384, nthreads=16)
    assert ref["rc"] == 0
    compare(rt, depth12, out, ref, "C3 full frame")
    assert (ref["hit"] != 0).mean() > 0.99  # every ray points down and lands on terrain
    # no launch over the tree so far ended a ray on the progress guard (such a ray would carry stepsLeft -1)
    assert depth12.guard_trips() == 0
    assert (rt.decode_hits(out)["steps"] >= 0).all()


@pytest.mark.parametrize("org", [(4.5, 90.5, 4.5), (-3.5, 80.5, -2.5), (2000.5, 70.0, 1000.5)])
def test_depth12_half_integral_camera(rt, depth12, oracle12, org):
    """Half-integral camera positions take the linear (no-segment) instance, like integral ones
    (need_seg: every ray from such an origin is linear, dda_axis starts at a, 0, a/2, 3a/2 or -a/2):
    the whole 1080p frame (a quarter-resolution one for the off-centre poses) against the oracle, every
    field, and equal to the segment instance (SVO_CAST_SEGMENTS) and to voxel stepping."""
    dn = rt.normalize([1, -0.45, 1] if org[0] < 1000 else [-0.3, -0.2, 1])
    W, H = (1920, 1080) if org[0] == 4.5 else (480, 270)
    out = depth12.cast_frame(org, dn, W, H, 16384)
    ref = oracle12.cast_frame(org, dn, W, H, 16384, nthreads=16)
    assert ref["rc"] == 0
    compare(rt, depth12, out, ref, "half-integral %s" % (org,))
    a = rt.decode_hits(out)
    for flags in (rt.CAST_SEGMENTS, rt.CAST_ITERATIVE, rt.CAST_NO_OCTANT, rt.CAST_NO_CEILINGS):
        b = rt.decode_hits(depth12.cast_frame(org, dn, W, H, 16384, flags=flags))
        for k in a:
            assert np.array_equal(a[k], b[k]), (org, flags, k)


@pytest.mark.parametrize("pose,steps", [(((4, 90, 4), (1, -0.45, 1)), 200), (((4, 90, 4), (1, 0.3, 1)), 37),
                                        (((4, 90, 4), (1, 0.3, 1)), 3000), (((2000.5, 70.25, 1000.75), (-0.3, 0.2, 1)), 777)])
def test_depth12_budget_ends_in_air(rt, depth12, oracle12, pose, steps):
    """Budgets that end in empty space, far from any voxel: those lanes leave the traversal loop
    and take their last DDA steps after it (svo_cast.hip, trace); sampled pixels against the oracle,
    every output field, also for a fractional origin (rays that are not exact walk empty bricks)."""
    org, d = pose
    T = oracle12
    dn = rt.normalize(list(d))
    W, H = 480, 270
    out = rt.decode_hits(depth12.cast_frame(org, dn, W, H, steps))
    pix = np.unique(np.random.default_rng(steps).integers(0, W * H, 3000))
    ref = T.cast_frame(org, dn, W, H, steps, pixels=pix, nthreads=16)
    assert ref["rc"] == 0
    sub = {k: v[pix] for k, v in out.items()}
    assert np.array_equal(sub["pos"], ref["pos"]) and np.array_equal(sub["steps"], ref["steps"])
    assert np.array_equal(sub["hit"], ref["hit"] != 0) and np.array_equal(sub["last_pos"], ref["last"])
    assert np.array_equal(sub["t"], ref["t"].astype(np.float32))
    assert (~sub["hit"]).mean() > 0.2  # most of these rays end their budget in the air


@pytest.mark.parametrize("org", [(4.37, 90.61, 4.23), (-7.3, 88.125, 1000.01)])
def test_depth12_fractional_camera(rt, depth12, oracle12, org):
    """C3 from non-integral camera positions, S = 16384: the rays are not linear (their crossings
    round once per binade), so the kernel crosses empty regions in exact segments (svo_cast.hip,
    seg_cap).  Sampled pixels (top and bottom rows, the horizon band) against the oracle; the whole
    frame identical to the voxel-by-voxel path; still O(1) crossings (not voxel stepping)."""
    T = oracle12
    dn = rt.normalize([1, -0.45, 1])
    W, H = 1920, 1080
    out = rt.decode_hits(depth12.cast_frame(org, dn, W, H, 16384))
    rng = np.random.default_rng(int(abs(org[0]) * 100))
    pix = np.unique(np.concatenate([rng.integers(0, W * H, 4000), np.arange(W * 539, W * 540), np.arange(0, W, 3), np.arange(W * (H - 1), W * H, 3)]))
    ref = T.cast_frame(org, dn, W, H, 16384, pixels=pix, nthreads=16)
    assert ref["rc"] == 0
    sub = {k: v[pix] for k, v in out.items()}
    assert np.array_equal(sub["pos"], ref["pos"]) and np.array_equal(sub["steps"], ref["steps"])
    assert np.array_equal(sub["hit"], ref["hit"] != 0) and np.array_equal(sub["last_pos"], ref["last"])
    assert np.array_equal(sub["t"], ref["t"].astype(np.float32))
    for flags in (rt.CAST_ITERATIVE, rt.CAST_NO_OCTANT, rt.CAST_NO_CEILINGS):
        o2 = rt.decode_hits(depth12.cast_frame(org, dn, W, H, 16384, flags=flags))
        for k in out:
            assert np.array_equal(out[k], o2[k]), (k, flags)
    st = depth12.cast_stats(org, dn, W, H, 16384)
    assert st["skips"] > 5.0 and st["lookups"] < 3.0 * st["skips"], st  # empty space crossed in O(1) moves


def test_depth12_full_frame_properties(rt, depth12):
    """Size-independent properties at the full bench size: determinism, every hit voxel is solid
    in the tree and its predecessor is not, steps accounting."""
    dn = rt.normalize([1, -0.45, 1])
    a = rt.decode_hits(depth12.cast_frame((4, 90, 4), dn, 1920, 1080, 16384))
    b = rt.decode_hits(depth12.cast_frame((4, 90, 4), dn, 1920, 1080, 16384))
    c = rt.decode_hits(depth12.cast_frame((4, 90, 4), dn, 1920, 1080, 16384, flags=rt.CAST_ITERATIVE))
    e = rt.decode_hits(depth12.cast_frame((4, 90, 4), dn, 1920, 1080, 16384, flags=rt.CAST_WIDE_ADDR))
    f = rt.decode_hits(depth12.cast_frame((4, 90, 4), dn, 1920, 1080, 16384, flags=rt.CAST_NO_OCTANT))
    nc = rt.decode_hits(depth12.cast_frame((4, 90, 4), dn, 1920, 1080, 16384, flags=rt.CAST_NO_CEILINGS))
    for k in a:
        assert np.array_equal(a[k], nc[k]), k
        assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(a[k], c[k]), k
        assert np.array_equal(a[k], e[k]), k
        assert np.array_equal(a[k], f[k]), k
    rng = np.random.default_rng(9)
    idx = rng.integers(0, len(a["hit"]), 20000)
    ids = depth12.get_blocks(a["pos"][idx])
    assert np.array_equal(ids != 0, a["hit"][idx])
    assert np.array_equal(np.where(a["hit"][idx], a["material"][idx], 0), ids)
    assert np.all(depth12.get_blocks(a["last_pos"][idx][a["hit"][idx]]) == 0)
    # L1 distance from trunc(origin) to pos == steps used (one axis step per DDA step)
    used = 16384 - a["steps"]
    l1 = np.abs(a["pos"] - np.array([4, 90, 4])).sum(1)
    assert np.array_equal(l1[a["hit"]], used[a["hit"]])


@pytest.mark.parametrize("octant", range(8))
def test_octant_frames(rt, gtree, ref_world_oracle, octant):
    """Frames whose rays all step with one sign octant run an instance with the signs compiled in
    (svo_cast.hip: frame_dirs); every octant, integral and fractional origins, against the oracle and
    against the per-wave sign flags (SVO_CAST_NO_OCTANT)."""
    sx, sy, sz = [(-1.0 if (octant >> k) & 1 else 1.0) for k in range(3)]
    dn = rt.normalize([sx * 1.0, sy * 0.45, sz * 0.8])
    W, H = 96, 64
    for org in ((128.0, 60.0, 128.0), (131.3, 58.7, 125.45)):
        ref = ref_world_oracle.cast_frame(org, dn, W, H, 300, ppx=0.6, ppy=0.4)
        for flags in (0, rt.CAST_NO_OCTANT):
            out = gtree.cast_frame(org, dn, W, H, 300, ppx=0.6, ppy=0.4, flags=flags)
            compare(rt, gtree, out, ref, "octant %d org %s flags %d" % (octant, org, flags))


def test_ao_fractional_origin(rt, gtree, ref_world_oracle):
    """AO (C4) from a non-integral camera: the AO instance with segment-exact primaries (and its
    sign-octant form) against the oracle's AO counts."""
    org, dn = (40.25, 70.5, 33.75), rt.normalize([1.0, -0.5, 0.7])
    ao, hit = ref_world_oracle.cast_frame_ao(org, dn, 128, 96, 300, 16, 5)
    for flags in (0, rt.CAST_NO_OCTANT):
        out = rt.decode_hits(gtree.cast_frame(org, dn, 128, 96, 300, ao_samples=16, ao_steps=5, flags=flags))
        assert np.array_equal(out["hit"], hit != 0)
        assert np.array_equal(out["ao"], ao), flags


@pytest.mark.parametrize("n_ao", [16, 20])
def test_ao_reference_world(rt, gtree, ref_world_oracle, n_ao):
    """A8 / C4: hemisphere AO counts (per pixel, rays that hit within 5 steps) against the oracle,
    through the per-face voxel plan (default) and by tracing every AO ray (CAST_AO_TRACE)."""
    for org, d in CAMERAS[:3]:
        dn = rt.normalize(d)
        ao, hit = ref_world_oracle.cast_frame_ao(org, dn, 128, 128, 300, n_ao, 5)
        for flags in (0, rt.CAST_AO_TRACE):
            out = rt.decode_hits(gtree.cast_frame(org, dn, 128, 128, 300, ao_samples=n_ao, ao_steps=5, flags=flags))
            assert np.array_equal(out["hit"], hit != 0)
            assert np.array_equal(out["ao"], ao), (org, n_ao, flags)
            assert out["ao"].max() <= n_ao


def test_ao_upper_level_solids(rt, oracle_mod, torch_cuda):
    """AO on hits inside SOLID regions above the brick level (16^3 blocks put at level 4, floating
    in the camera's view): the AO primaries' split lookup leaves the region's parent shift for the
    plan (lookup: PSH); counts against the oracle for the plan, its octant-free form and traced rays."""
    corners = [(64, 48, 64), (112, 48, 96), (80, 64, 80), (96, 32, 48), (48, 64, 112)]
    w = rt.World.reference()
    o = oracle_mod.Tree.reference_world()
    for i, (x, y, z) in enumerate(corners):
        w.put_block(x, y, z, 0, 1000 + i, level=4)
        assert o.put_block(x, y, z, 0, 1000 + i, 0.0, 4) == 0
    gt = w.build().upload(0)
    for org, d in CAMERAS[:2]:
        dn = rt.normalize(d)
        ao, hit = o.cast_frame_ao(org, dn, 128, 96, 300, 16, 5)
        for flags in (0, rt.CAST_NO_OCTANT, rt.CAST_AO_TRACE):
            out = rt.decode_hits(gt.cast_frame(org, dn, 128, 96, 300, ao_samples=16, ao_steps=5, flags=flags))
            assert np.array_equal(out["hit"], hit != 0)
            assert np.array_equal(out["ao"], ao), (org, flags)
        # the blocks are hit (their faces, not only bricks around them)
        pos = out["pos"][out["hit"]]
        inb = np.zeros(len(pos), bool)
        for c in corners:
            inb |= np.all((pos >= np.array(c)) & (pos < np.array(c) + 16), axis=1)
        assert inb.sum() > 200, (org, inb.sum())


@pytest.mark.parametrize("n_ao,ao_steps", [(1, 5), (16, 0), (16, 1), (20, 12), (64, 3), (7, 40)])
def test_ao_plan_budgets(rt, gtree, ref_world_oracle, n_ao, ao_steps):
    """The AO plan over sample counts and budgets (1 .. 64 samples, 0 .. 40 steps) against the oracle."""
    # the C1 pose, and one whose hits lie at negative (wrapped) coordinates: those AO rays do not
    # start at lastPos (trunc of -x.5) and are traced instead of planned
    for org, d in (CAMERAS[1], ((-30.5, 60.0, -10.5), (-1.0, -0.6, -0.4))):
        dn = rt.normalize(d)
        ao, hit = ref_world_oracle.cast_frame_ao(org, dn, 96, 64, 300, n_ao, ao_steps)
        out = rt.decode_hits(gtree.cast_frame(org, dn, 96, 64, 300, ao_samples=n_ao, ao_steps=ao_steps))
        assert np.array_equal(out["hit"], hit != 0)
        assert np.array_equal(out["ao"], ao), (org, n_ao, ao_steps)


@pytest.mark.parametrize("n_ao", [16, 20])
def test_ao_depth12_full_frame(rt, depth12, oracle12, n_ao):
    """C4: the C3 frame + 16 (and 20) hemisphere AO rays of 5 steps per hit; every pixel's AO count and hit
    flag against the oracle, and the per-face plan equal to tracing every AO ray (CAST_AO_TRACE)."""
    dn = rt.normalize([1, -0.45, 1])
    out = rt.decode_hits(depth12.cast_frame((4, 90, 4), dn, 1920, 1080, 16384, ao_samples=n_ao, ao_steps=5))
    ao, hit = oracle12.cast_frame_ao((4, 90, 4), dn, 1920, 1080, 16384, n_ao, 5, nthreads=16)
    assert np.array_equal(out["hit"], hit != 0)
    bad = np.nonzero(out["ao"] != ao)[0]
    assert len(bad) == 0, "AO differs at %d pixels, first %s: gpu %s oracle %s" % (len(bad), bad[:5], out["ao"][bad[:5]], ao[bad[:5]])
    tr = rt.decode_hits(depth12.cast_frame((4, 90, 4), dn, 1920, 1080, 16384, ao_samples=n_ao, ao_steps=5, flags=rt.CAST_AO_TRACE))
    assert np.array_equal(out["ao"], tr["ao"])  # plan == traced AO rays over the whole frame
    assert out["ao"].mean() > 0.5  # terrain occludes part of the hemisphere


def test_depth14_4k_sampled_parity(rt, oracle_mod, torch_cuda):
    """C5: depth-14 (16384^2 columns, 7 levels), 3840x2160 from the C1 pose; sampled pixels against the
    oracle's 7-level reference-format tree over the first 4096^2 columns (every ray of this pose lands
    within ~2,600 voxels; the full reference-format tree would exceed its 2^32-byte pools)."""
    t = rt.Tree.terrain_gpu(7, 16384, 16384, 0)  # the tree bench.py --config c5 times
    T = oracle_mod.Tree.terrain(7, 4096, 4096, nthreads=16)
    dn = rt.normalize([1, -0.45, 1])
    W, H = 3840, 2160
    out = rt.decode_hits(t.cast_frame((4, 90, 4), dn, W, H, 16384))
    pix = np.unique(np.concatenate([np.random.default_rng(14).integers(0, W * H, 40000), np.arange(0, W, 2), np.arange(W * 1079, W * 1081)]))
    ref = T.cast_frame((4, 90, 4), dn, W, H, 16384, pixels=pix, nthreads=16)
    assert ref["rc"] == 0
    assert np.array_equal(out["pos"][pix], ref["pos"]) and np.array_equal(out["steps"][pix], ref["steps"])
    assert np.array_equal(out["hit"][pix], ref["hit"] != 0)
    assert np.array_equal(out["last_pos"][pix], ref["last"])
    # the block at pos: palette flags and colour (ray_caster.cpp:83) against the oracle's getBlock
    pal = t.palette()
    pf = np.array([p[0] for p in pal], np.uint32)
    pc = np.array([p[1] for p in pal], np.uint64)
    mid = np.where(out["hit"][pix], out["material"][pix], 0)
    assert np.array_equal(pf[mid], ref["flags"]) and np.array_equal(pc[mid], ref["color"])
    assert np.array_equal(out["t"][pix], ref["t"].astype(np.float32))
    assert np.abs(out["pos"][:, [0, 2]]).max() < 4096  # the premise of the 4096^2 oracle
    del t


def test_exchange_single_rank_python(rt, gtree, torch_cuda):
    """svo_exchange_frames through the Python binding (rt.Exchange) on a one-rank RCCL communicator: the
    frames it unpacks equal the cast records (ragged frame, several frames per launch, AO counts)"""
    torch = torch_cuda
    x = rt.Exchange(1, 0, rt.Exchange.unique_id(), 0)
    cam = rt.normalize((1.0, -0.45, 1.0))
    try:
        for nf, W, H, ao in ((1, 100, 37, 0), (3, 64, 48, 16)):
            origins = [(4.0 + 8.5 * f, 90.0, 4.0 + 3.25 * f) for f in range(nf)]
            d = rt.Tree.frame_desc(origins[0], cam, W, H, 300, frame_origins=origins if nf > 1 else None, ao_samples=ao)
            n = rt.Tree.count(d)
            assert n == nf * W * H
            mine = rt.Tree.alloc_hits(n, 0, ao=ao > 0)
            gtree.cast(d, mine)
            out = rt.Tree.alloc_hits(n, 0, ao=ao > 0)
            x.frames(gtree, d, mine, out)
            torch.cuda.synchronize()
            for k in mine:
                assert torch.equal(out[k], mine[k]), (nf, k)
            # the fused path: the cast writes wire records, the exchange decodes them
            wire = torch.zeros((n, gtree.wire_bytes(d)), dtype=torch.uint8, device="cuda")
            wao = torch.zeros(n, dtype=torch.uint8, device="cuda") if ao else None
            gtree.cast_wire(d, wire, wao)
            out2 = rt.Tree.alloc_hits(n, 0, ao=ao > 0)
            x.wire(gtree, d, wire, out2, ao=wao)
            torch.cuda.synchronize()
            for k in mine:
                assert torch.equal(out2[k], mine[k]), (nf, k, "wire")
    finally:
        x.close()


def test_pick_ray_repeated(rt, gtree):
    """the per-frame pick ray (main.cpp:81: castRayFromCam(30) every frame, svo_cast_ray_from_cam) uses the
    tree's own result record: repeated picks agree, and one costs well under a millisecond"""
    import time

    cam = rt.normalize((1.0, 0.0, 1.0))
    first = gtree.cast_ray_from_cam((35.0, 50.0, 35.0), cam, 30)
    t0 = time.perf_counter()
    for _ in range(200):
        assert gtree.cast_ray_from_cam((35.0, 50.0, 35.0), cam, 30) == first
    dt = (time.perf_counter() - t0) / 200
    print("pick ray: %.1f us per call" % (dt * 1e6))
    assert dt < 1e-3
