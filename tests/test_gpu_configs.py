"""GPU parity on BASELINE.json's configs as worded: config 2 is a "depth-8 SVO from world_gen.cpp
OpenSimplex terrain, 1080p primary rays".  Depth 8 = 256^3 voxels = a 4-level 64-ary tree.
Two such trees, full 1080p frames at the reference budget (S = 300), every field against the oracle:

* the reference's own construction at that depth: a clean root + genWorld's putBlock per voxel over its
  200 x 200 columns (src/world_gen.cpp:13-42, src/voxel_data/tetrahexa_tree.cpp:176-291), built by the
  product's editable world (svo_world) and by the oracle (orc_gen_world);
* genWorld's column formula over the full 256^2 footprint (wraps seamlessly at 256), built on the GPU
  (svo_build_terrain_gpu) and by the oracle's collapse builder.

Poses: the C1 / C3 pose, the reference's default camera (globals.cpp:20-21), half-integral and
fractional origins (the linear and segment instances)."""
import pytest

from test_gpu_parity import compare

pytestmark = pytest.mark.gpu

POSES = [
    ((4.0, 90.0, 4.0), (1.0, -0.45, 1.0)),
    ((35.0, 50.0, 35.0), (1.0, 0.0, 1.0)),
    ((100.5, 70.5, 20.5), (-0.3, -0.4, 1.0)),
    ((-30.5, 60.5, -10.5), (1.0, -0.5, 0.8)),
    ((150.3, 44.7, 20.9), (-0.6, -0.2, 1.0)),
]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def d8_worldgen(rt, torch_cuda):
    w = rt.World(4)
    w.gen_world(200, 200)
    return w.build().upload(0)


@pytest.fixture(scope="module")
def d8_worldgen_oracle(oracle_mod):
    return oracle_mod.Tree.terrain_putblock(4, 200, 200)


@pytest.mark.parametrize("pose", range(len(POSES)))
def test_depth8_worldgen_1080p(rt, d8_worldgen, d8_worldgen_oracle, pose):
    org, d = POSES[pose]
    dn = rt.normalize(d)
    out = d8_worldgen.cast_frame(org, dn, 1920, 1080, 300)
    ref = d8_worldgen_oracle.cast_frame(org, dn, 1920, 1080, 300, nthreads=16)
    assert ref["rc"] == 0
    compare(rt, d8_worldgen, out, ref, "depth-8 genWorld pose %d" % pose)
    assert 0.05 < (ref["hit"] != 0).mean()


def test_depth8_terrain_gpu_1080p(rt, oracle_mod, torch_cuda):
    t = rt.Tree.terrain_gpu(4, 256, 256, 0)
    T = oracle_mod.Tree.terrain(4, 256, 256, nthreads=16)
    for pose in (0, 2, 4):
        org, d = POSES[pose]
        dn = rt.normalize(d)
        out = t.cast_frame(org, dn, 1920, 1080, 300)
        ref = T.cast_frame(org, dn, 1920, 1080, 300, nthreads=16)
        assert ref["rc"] == 0
        compare(rt, t, out, ref, "depth-8 terrain pose %d" % pose)
