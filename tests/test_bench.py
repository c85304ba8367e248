"""bench.py's host logic on CPU: the CPU-baseline thread rule and its report, the roofline object (the
§8(d) model next to the committed counters, `bound` from the counters), and the torch exchange's
all-to-all splits for any frames / ranks (each sender's split to a rank equals that rank's split from
it).  No kernel launches."""
import argparse
import importlib.util
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _args(**kw):
    a = dict(config="c3", ao=0, shade=False)
    a.update(kw)
    return argparse.Namespace(**a)


def test_cpu_info_reports_cores_and_model(bench, monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    ci = bench.cpu_info()
    for k in ("nproc", "affinity_cpus", "cgroup_quota_cpus", "cpu_model", "threads", "threads_rule"):
        assert k in ci
    assert ci["threads"] == min(3, ci["affinity_cpus"]) and "OMP_NUM_THREADS" in ci["threads_rule"]
    monkeypatch.delenv("OMP_NUM_THREADS")
    ci = bench.cpu_info()
    assert 1 <= ci["threads"] <= ci["affinity_cpus"] and ci["nproc"] >= ci["affinity_cpus"]


def test_run_keys(bench):
    assert bench.run_key(_args()) == "c3"
    assert bench.run_key(_args(ao=16)) == "c3_ao16"
    assert bench.run_key(_args(config="c5")) == "c5"
    assert bench.run_key(_args(shade=True)) == "c3_shade"


def test_roofline_model_and_counters(bench):
    cfg = bench.CONFIGS["c3"]
    bray = json.load(open(os.path.join(ROOT, "profiles", "bray.json")))
    pmc = json.load(open(os.path.join(ROOT, "profiles", "pmc_c3.json")))
    sha = pmc["lib_sha256"]  # the counters' build: used as if this run loaded it
    r = bench.roofline(_args(), cfg, 2073600, 0.23e-3, 1, sha)
    b = bray["C3"]["bytes_per_ray"]
    assert abs(r["bytes_per_ray"] - b) < 0.01
    assert abs(r["achieved"] - b * 2073600 / 0.23e-3 / 1e9) < 0.01
    assert abs(r["frac"] - r["achieved"] / 8000.0) < 1e-4
    assert r["traffic"] == round(pmc["hbm_bytes_per_launch"])  # the same rays per launch: unscaled
    assert r["counters_build"] == sha and "measured on this build" in r["counters"]
    assert r["bound"] == "hbm" and "wait to issue" in r["limiter"]  # (the contract's roofline; the SQ counters name the limiter)
    # C4: the primary bytes + the AO plan's node loads (not the traced-AO model, which is reported beside it)
    r4 = bench.roofline(_args(ao=16), cfg, 2073600, 0.31e-3, 1, sha)
    kb = bray["C4_ao16_kernel"]["ao_node_loads_per_ray"]
    assert abs(r4["bytes_per_ray"] - (b + 16 * kb + 1)) < 0.01 and r4["bytes_per_ray"] > r["bytes_per_ray"]
    assert abs(r4["bytes_per_ray_traced_ao_model"] - bray["C4_ao16"]["bytes_per_ray"]) < 0.01
    # a fraction above 1 is never published
    rf = bench.roofline(_args(), cfg, 2073600, 0.05e-3, 1, sha)
    assert rf["frac"] is None and "withheld" in rf["note"]
    rs = bench.roofline(_args(shade=True), cfg, 2073600, 1.3e-3, 1, sha)
    # the shading pass: priced by its own §8(d) entries (oracle/bray.py C3_shade)
    sb = bray["C3_shade"]
    assert abs(rs["bytes_per_ray"] - sb["bytes_per_ray"]) < 0.01 and "shading pass" in rs["bytes_model"]
    assert abs(rs["frac"] - sb["bytes_per_ray"] * 2073600 / 1.3e-3 / 1e9 / 8000.0) < 1e-4
    # counters measured at N = 1 scale per ray to another launch size (a rank's shard)
    rh = bench.roofline(_args(), cfg, 2073600 // 2, 0.12e-3, 2, sha)
    assert rh["traffic"] == round(pmc["hbm_bytes_per_launch"] / 2)
    # counters of another build are not used: marked stale, no traffic
    rx = bench.roofline(_args(), cfg, 2073600, 0.23e-3, 1, "0" * 64)
    assert rx["traffic"] is None and rx["counters"].startswith("stale") and "limiter" not in rx


def test_committed_counters_name_their_build():
    """every committed PMC summary records the libsvo_rt.so it was measured on (tools/pmc_summary.py)"""
    import glob

    for f in glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")):
        d = json.load(open(f))
        assert len(d.get("lib_sha256") or "") == 64, f


@pytest.mark.parametrize("world,nframes", [(1, 1), (2, 1), (2, 2), (3, 2), (3, 5), (4, 4), (8, 8), (8, 1)])
def test_torch_exchange_splits_pair_up(bench, world, nframes):
    from raytracing_test_amd import shard

    W, H = 64, 37
    counts = [shard.shard_count(W, H, r, world) for r in range(world)]
    send, recv = {}, {}
    for rank in range(world):
        x = bench.TorchExchange.__new__(bench.TorchExchange)
        x.world, x.rank, x.counts, x.n_mine, x.nframes = world, rank, counts, counts[rank], nframes
        x.mine = list(range(rank, nframes, world))
        send[rank], recv[rank] = x._splits(1)
        # the regrouped send buffer: frames grouped by destination rank (frames r, r + N, ...), each once
        import torch

        x.torch = torch
        buf = torch.arange(counts[rank] * nframes)
        got = x._order_send(buf).numpy()
        want = np.concatenate([np.arange(f * counts[rank], (f + 1) * counts[rank]) for r in range(world) for f in range(r, nframes, world)])
        assert np.array_equal(got, want)
        assert sum(send[rank]) == counts[rank] * nframes
        assert sum(recv[rank]) == len(x.mine) * W * H
    for s in range(world):
        for r in range(world):
            assert send[s][r] == recv[r][s], (s, r)


# ---- the launcher-free N-rank start (`python bench.py --gpus N` with no WORLD_SIZE) ----
_CHILD = r'''
import os, sys, time
r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["MASTER_PORT"]) > 0
mode = sys.argv[1]
if mode == "ok":
    if r == 0:
        print('{"n": %d, "args": "%s"}' % (n, " ".join(sys.argv[1:])), flush=True)
    sys.exit(0)
if mode == "fail":  # rank 1 fails at once, the others would wait forever (a barrier that never completes)
    if r == 1:
        sys.exit(3)
    time.sleep(600)
'''


def test_launch_ranks_starts_n_children(bench, tmp_path, capfd):
    child = tmp_path / "child.py"
    child.write_text(_CHILD)
    assert bench.launch_ranks(3, ["ok", "--x"], script=str(child)) == 0
    out = capfd.readouterr().out.strip().splitlines()
    assert out == ['{"n": 3, "args": "ok --x"}']  # rank 0's line only


def test_launch_ranks_failure_ends_the_job(bench, tmp_path):
    import time

    child = tmp_path / "child.py"
    child.write_text(_CHILD)
    t0 = time.monotonic()
    assert bench.launch_ranks(3, ["fail"], grace_s=1.0, script=str(child)) == 3  # the failing rank's status
    assert time.monotonic() - t0 < 30  # the waiting ranks were terminated, not waited for


def test_world_size_must_match_gpus(monkeypatch):
    import subprocess
    import sys

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True, text=True, env=env,
                       timeout=120)
    assert p.returncode == 2 and "differs from --gpus" in p.stderr


def test_product_build_is_a_noop_when_up_to_date(monkeypatch, tmp_path):
    """build() compiles nothing when libsvo_rt.so carries the stamp of the current sources, even without its objects
    (gpurun snapshots leave *.o behind: the GPU box must time the library the PMC passes measured) and whatever the
    files' mtimes say (tests/test_build_stamp.py: a changed source does rebuild)"""
    from raytracing_test_amd import build as b

    b.build()  # (up to date, or brought up to date here)
    calls = []
    monkeypatch.setattr(b, "_run", lambda cmd: calls.append(cmd))
    monkeypatch.setattr(b, "BUILD", str(tmp_path / "no_objects"))  # as on the box: no objects at all
    assert b.build() == b.OUT and calls == []
    src = os.path.join(os.path.dirname(b.__file__), "csrc", "svo_exchange.hip")
    st = os.stat(b.OUT)
    real = os.path.getmtime
    monkeypatch.setattr(os.path, "getmtime", lambda p: st.st_mtime + 10 if p == src else (real(p) if os.path.exists(p) else 0.0))
    assert b.build() == b.OUT and calls == []  # newer, unchanged: no rebuild


_WATCHDOG_CHILD = r'''
import importlib.util, sys, time
spec = importlib.util.spec_from_file_location("bench", sys.argv[1])
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
wd = bench.Watchdog(1, 2)
wd.diag = lambda: "step 7: cast done, exchange PENDING"
wd.phase = "step 7: exchange (svo_exchange_wire)"
wd.arm(0.5, "the timed region (3 steps)")
time.sleep(60)  # a receive that never returns
'''


def test_watchdog_names_the_stuck_phase_and_exits(tmp_path):
    """The per-rank watchdog (bench.Watchdog, N > 1): past its deadline the rank reports the step, phase and GPU event
    state, dumps every thread's traceback and exits with WATCHDOG_RC, well before the stuck call would return"""
    import subprocess
    import sys
    import time

    child = tmp_path / "wd.py"
    child.write_text(_WATCHDOG_CHILD)
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, str(child), os.path.join(ROOT, "bench.py")], capture_output=True, text=True, timeout=60)
    assert p.returncode == 124, p.stderr
    assert time.monotonic() - t0 < 30
    assert "rank 1 of 2: WATCHDOG: the timed region (3 steps) did not finish within 0.5 s" in p.stderr
    assert "stuck in phase: step 7: exchange (svo_exchange_wire)" in p.stderr
    assert "GPU events of the last steps: step 7: cast done, exchange PENDING" in p.stderr
    assert "most recent call first" in p.stderr  # faulthandler's dump of the threads


def test_watchdog_bound_from_the_warmup(bench, monkeypatch):
    monkeypatch.delenv("SVO_WATCHDOG_MIN_S", raising=False)
    monkeypatch.delenv("SVO_WATCHDOG_FACTOR", raising=False)
    assert bench.watchdog_bound(0.5, 5, 100) == pytest.approx(204.0)  # 0.1 s per warm-up step x (100 + 2) x 20
    assert bench.watchdog_bound(0.01, 1, 10) == 60.0  # at least a minute
    monkeypatch.setenv("SVO_WATCHDOG_MIN_S", "10")
    monkeypatch.setenv("SVO_WATCHDOG_FACTOR", "1")
    assert bench.watchdog_bound(2.0, 1, 3) == 10.0
