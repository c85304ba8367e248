"""Frame schedules (include/svo_rt.h SVO_CAST_NO_SCHEDULE, svo_tree_schedule): a shaded frame of more than
SVO_SCHED_MIN_BLOCKS blocks is dispatched longest block first by the durations the last frame of the same geometry
measured on the same stream.  Only the order of the blocks changes: every scheduled frame must be bit-identical to
the same frame in the default order — across repeated frames, a turning camera, a geometry change and two
streams — and the stored order must be a permutation sorted by its durations.  Primary casts keep no schedule."""
import numpy as np
import pytest

import raytracing_test_amd as rt

pytestmark = pytest.mark.gpu

W, H, S = 1920, 1080, 16384
ORG = (4.0, 90.0, 4.0)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def worlds(torch_cuda):
    solid = rt.Tree.terrain_gpu(6, 4096, 4096, 0)
    scene = rt.Tree.terrain_gpu(6, 4096, 4096, 0, view=rt.VIEW_ALL)
    return solid, scene


def _shade(worlds, cam, w=W, h=H, flags=0, stream=None):
    solid, scene = worlds
    return solid.shade_frame(ORG, rt.normalize(cam), w, h, S, flags=flags, stream=stream, scene=scene).cpu().numpy().view(np.uint32)


def _check_schedule(order, cost, label):
    assert len(cost) == len(order) * rt.SCHED_GROUP, label
    cost = cost.reshape(-1, rt.SCHED_GROUP).max(axis=1)  # a group's duration: its longest block's
    n = len(order)
    assert np.array_equal(np.sort(order), np.arange(n, dtype=np.uint32)), label + ": order is not a permutation"
    # the sort's 256 logarithmic buckets (k_sched_order's sched_key: f32 exponent and 3 mantissa bits), longest first
    k = np.minimum((cost.astype(np.float32).view(np.uint32) >> 20).astype(np.int64) - 127 * 8, 255)
    key = np.where(cost == 0, 255, 255 - k)
    assert np.all(np.diff(key[order]) >= 0), label + ": not longest first"
    assert np.all(np.diff(cost[order][::max(1, n // 64)].astype(np.int64)) <= cost.max() // 7), label
    assert cost.max() > 0, label


def test_shaded_frames_identical_under_schedule(worlds, torch_cuda):
    solid, _ = worlds
    s = torch_cuda.cuda.Stream()
    cams = [(1.0, -0.45, 1.0), (1.0, -0.43, 1.02), (0.97, -0.47, 1.0)]  # a camera turning frame to frame
    for i, cam in enumerate(cams):
        ref = _shade(worlds, cam, flags=rt.CAST_NO_SCHEDULE, stream=s)
        for rep in range(3):  # (a camera 1-2 deg from the last: default order, then sorted, then scheduled)
            assert np.array_equal(_shade(worlds, cam, stream=s), ref), "camera %d frame %d" % (i, rep)
    order, cost = solid.schedule(rt.SCHED_SHADE, stream=s)
    assert order is not None and len(order) * rt.SCHED_GROUP == solid.blocks(solid.frame_desc(ORG, rt.normalize(cams[0]), W, H, S))
    _check_schedule(order, cost, "shading")
    # a new geometry starts over in the default order, then schedules
    ref = _shade(worlds, cams[0], 1280, 720, flags=rt.CAST_NO_SCHEDULE, stream=s)
    for rep in range(3):
        assert np.array_equal(_shade(worlds, cams[0], 1280, 720, stream=s), ref), "720p frame %d" % rep
    order, cost = solid.schedule(rt.SCHED_SHADE, stream=s)
    # (720p, 14400 wavefronts of whole footprints: a small launch, its first tile rows in half footprints — svo_cast_blocks)
    assert len(order) * rt.SCHED_GROUP == solid.blocks(solid.frame_desc(ORG, rt.normalize(cams[0]), 1280, 720, S)) > 1280 * 720 // 64
    _check_schedule(order, cost, "shading 720p")


def test_small_frames_and_primary_casts_keep_no_schedule(worlds, torch_cuda):
    solid, _ = worlds
    s = torch_cuda.cuda.Stream()
    ref = _shade(worlds, (1.0, -0.45, 1.0), 256, 256, flags=rt.CAST_NO_SCHEDULE, stream=s)
    assert np.array_equal(_shade(worlds, (1.0, -0.45, 1.0), 256, 256, stream=s), ref)
    assert 256 * 256 // 64 <= rt.SCHED_MIN_BLOCKS
    assert solid.schedule(rt.SCHED_SHADE, stream=s) == (None, None)
    # 1040 x 800: 20410 blocks (100 tile rows of 130 footprints, 57 of them in half footprints), not a multiple of the
    # schedule's groups
    nb = solid.blocks(solid.frame_desc(ORG, rt.normalize((1.0, -0.45, 1.0)), 1040, 800, S))
    assert nb > rt.SCHED_MIN_BLOCKS and nb % rt.SCHED_GROUP != 0
    ref = _shade(worlds, (1.0, -0.45, 1.0), 1040, 800, flags=rt.CAST_NO_SCHEDULE, stream=s)
    for rep in range(2):
        assert np.array_equal(_shade(worlds, (1.0, -0.45, 1.0), 1040, 800, stream=s), ref)
    assert solid.schedule(rt.SCHED_SHADE, stream=s) == (None, None)
    for ao in (0, 16):
        solid.cast_frame(ORG, rt.normalize((1.0, -0.45, 1.0)), W, H, S, stream=s, ao_samples=ao)
    assert solid.schedule(rt.SCHED_PRIMARY, stream=s) == (None, None)
    assert solid.schedule(rt.SCHED_AO, stream=s) == (None, None)


def test_two_streams_keep_separate_schedules(worlds, torch_cuda):
    """two shaded frames in flight on two streams: each stream's schedule is its own"""
    solid, scene = worlds
    torch = torch_cuda
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    ref = _shade(worlds, (1.0, -0.45, 1.0), flags=rt.CAST_NO_SCHEDULE)
    d = solid.frame_desc(ORG, rt.normalize((1.0, -0.45, 1.0)), W, H, S)
    n = solid.count(d)
    outs = [torch.empty((n, 4), dtype=torch.float32, device="cuda") for _ in range(4)]
    for rep in range(3):
        solid.shade(d, outs[0], stream=sa, scene=scene)
        solid.shade(d, outs[1], stream=sb, scene=scene)
        solid.shade(d, outs[2], stream=sa, scene=scene)
        solid.shade(d, outs[3], stream=sb, scene=scene)
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        assert np.array_equal(o.cpu().numpy().view(np.uint32), ref), "stream frame %d" % i
    for st in (sa, sb):
        order, cost = solid.schedule(rt.SCHED_SHADE, stream=st)
        _check_schedule(order, cost, "stream")


def test_schedule_gated_on_camera_motion(worlds, torch_cuda):
    """a frame whose camera turned more than 0.5 deg (or moved more than a voxel) since the last one runs the default
    order and leaves no sorted order behind; the next frame near it sorts again"""
    solid, _ = worlds
    s = torch_cuda.cuda.Stream()
    a, b = (1.0, -0.45, 1.0), (1.0, -0.45, 0.8)  # ~6 deg apart
    ref_a = _shade(worlds, a, flags=rt.CAST_NO_SCHEDULE, stream=s)
    ref_b = _shade(worlds, b, flags=rt.CAST_NO_SCHEDULE, stream=s)
    for rep in range(3):
        assert np.array_equal(_shade(worlds, a, stream=s), ref_a), "still %d" % rep
    assert solid.schedule(rt.SCHED_SHADE, stream=s)[0] is not None
    assert np.array_equal(_shade(worlds, b, stream=s), ref_b), "after the turn"
    assert solid.schedule(rt.SCHED_SHADE, stream=s) == (None, None)  # (the turned frame was not sorted)
    assert np.array_equal(_shade(worlds, b, stream=s), ref_b), "settled"
    order, cost = solid.schedule(rt.SCHED_SHADE, stream=s)
    _check_schedule(order, cost, "settled")
