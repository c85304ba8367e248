import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O

    O.build()
    return O


@pytest.fixture(scope="session")
def rt():
    import raytracing_test_amd as rt
    from raytracing_test_amd import build

    build.build()
    return rt


@pytest.fixture(scope="session")
def ref_world_oracle(oracle_mod):
    return oracle_mod.Tree.reference_world()


@pytest.fixture(scope="session")
def ref_world(rt):
    return rt.World.reference()


@pytest.fixture(scope="session")
def ref_tree(ref_world):
    return ref_world.build()


@pytest.fixture(scope="session")
def depth12(rt):
    # the tree bench.py times: noise + build on the GPU (svo_build_terrain_gpu), so the
    # C3 / C4 / shaded parity tests pin the on-device builder to the oracle as well
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return rt.Tree.terrain_gpu(6, 4096, 4096, 0)


@pytest.fixture(scope="session")
def oracle12(oracle_mod):
    # the oracle's reference-format (collapsed) depth-12 tree, built once for the C3 / C4 / shaded tests
    return oracle_mod.Tree.terrain(6, 4096, 4096, nthreads=16)
