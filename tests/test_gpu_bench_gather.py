"""bench.py's N > 1 gather on one GPU: two gloo ranks (one process each, sharing the card) cast their tile rows of
the step's frames, exchange the wire records through torch.distributed (TorchExchange) and verify every displayed
frame against a one-GPU cast (--verify -> gather_verified).  Weak mode sends frame f to rank f, so the all-to-all
splits fall inside a rank's packed records: the compact 8-B format (integral camera, C3) and the 12-B one (the
fractional C3 camera) both.  (Round 3 sized the rows at 12 B for 8-B records, and weak-mode frames did not verify.)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(port, *extra):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "2",
           "--warmup", "1", "--verify", "--no-cpu-baseline"] + list(extra)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert line, p.stdout[-2000:]
    return json.loads(line[-1])


@pytest.mark.parametrize("config,port", [("c3", 29611), ("c3f", 29612)])
def test_weak_gather_verified(config, port):
    d = _run(port, "--config", config)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["gather_verified"] is True, d


def test_strong_two_frames_verified():
    d = _run(29613, "--frames", "2")
    assert d["scaling"] == "strong"
    assert d["gather_verified"] is True, d


def test_strong_frames_in_flight_verified():
    """--inflight 2: consecutive steps' casts alternate between two streams (two frames in flight per rank), each
    buffer set's exchange ordered after its own cast — every displayed frame still verifies"""
    d = _run(29614, "--frames", "1", "--inflight", "2", "--steps", "4")
    assert d["scaling"] == "strong" and d["config"]["frames_in_flight"] == 2
    assert d["gather_verified"] is True, d


def test_launcher_free_two_ranks_verified():
    """`python bench.py --gpus 2` with no launcher: bench.py starts the two ranks itself (before any GPU call),
    and the line reports the communicator's size"""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1",
           "--verify", "--no-cpu-baseline"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0's line only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["gather_verified"] is True, d


STANDIN = os.path.join(ROOT, "tests", "standin", "_build", "librccl_standin.so")


@pytest.mark.parametrize("n,extra", [
    (2, ()),                               # weak C3: frame f -> rank f, one all-to-all group per step
    (3, ()),
    (2, ("--frames", "1")),                # strong: one frame over N ranks, gathered to rank 0
    (3, ("--frames", "1")),
    (2, ("--ao", "16")),                   # C4's AO counts travel beside the records
    (3, ("--frames", "1", "--ao", "16")),
])
def test_capi_exchange_on_one_gpu(n, extra, tmp_path):
    """The C-ABI exchange's N > 1 code — svo_cast_wire + svo_exchange_wire, its ncclGroupStart / ncclSend / ncclRecv /
    ncclGroupEnd pairing and the display-side decode of every received shard — with N ranks on one GPU: libsvo_rt
    loads the test-only host-staged stand-in (SVO_RCCL_LIB, tests/standin/rccl_standin.cpp) in place of RCCL,
    which cannot form a communicator of two ranks on one device.  bench.py verifies every displayed frame against a
    one-GPU cast by default at N > 1."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert os.path.exists(STANDIN), "the stand-in is not built (raytracing_test_amd/build.py build_rccl_standin)"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(SVO_RCCL_LIB=STANDIN, SVO_RCCL_STANDIN="1", SVO_STANDIN_DIR=str(tmp_path), SVO_STANDIN_TIMEOUT_S="60")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dist-backend", "gloo", "--exchange", "capi",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline"] + list(extra)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == n  # svo_exchange_info of the communicator the step ran over
    assert d["config"]["exchange"].startswith("svo_cast_wire + svo_exchange_wire") and "stand-in" in d["config"]["exchange"], d
    assert d["scaling"] == ("strong" if "--frames" in extra else "weak")
    assert d["transport"] == "standin", d  # (never to be read as RCCL multi-GPU evidence)
    ranks = d["per_rank"]["ranks"]  # every rank's own cast / exchange / decode cost (a slow rank can be named)
    assert [r["rank"] for r in ranks] == list(range(n))
    assert all(r["cast_ms"] > 0 and r["exchange_ms"] is not None and r["exchange_ms"] > 0 and r["decode_shard_ms"] > 0 for r in ranks), ranks
    assert d["gather_verified"] is True, d
    assert [x for x in os.listdir(tmp_path) if x.startswith("svo_rccl_standin_")] == []  # every message was received


def test_stalled_receive_ends_the_run(tmp_path):
    """A receive that never completes (the stand-in's test hook withholds rank 1's third send, a timed step's) must not
    hang the job: the stuck ranks' watchdogs fire within their bound (here at least 10 s: SVO_WATCHDOG_MIN_S, factor 1
    over the warm-up's time per step), name the step and phase on stderr, and the run exits with WATCHDOG_RC (124)
    instead of waiting for the stand-in's own 600-s receive timeout"""
    import time

    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert os.path.exists(STANDIN), "the stand-in is not built (raytracing_test_amd/build.py build_rccl_standin)"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(SVO_RCCL_LIB=STANDIN, SVO_RCCL_STANDIN="1", SVO_STANDIN_DIR=str(tmp_path), SVO_STANDIN_TIMEOUT_S="600",
               SVO_STANDIN_WITHHOLD="1:2", SVO_WATCHDOG_MIN_S="10", SVO_WATCHDOG_FACTOR="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--exchange", "capi",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    t0 = time.monotonic()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=200, cwd=ROOT, env=env)
    took = time.monotonic() - t0
    assert p.returncode == 124, (p.returncode, p.stderr[-3000:])
    assert "TEST HOOK withholds" in p.stderr
    assert "rank 0 of 2: WATCHDOG: the timed region" in p.stderr, p.stderr[-3000:]
    assert "stuck in phase: step 2: exchange" in p.stderr, p.stderr[-3000:]  # rank 0 waits for rank 1's step-2 message
    assert "GPU events of the last steps" in p.stderr
    assert took < 150, took
