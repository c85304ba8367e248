"""The test-only RCCL stand-in (tests/standin/rccl_standin.cpp), which lets libsvo_rt's N > 1 exchange run
with several ranks on one GPU (SVO_RCCL_LIB), checked here without a GPU in its host-only mode: N processes
form a communicator and run the exchange's own pattern — one group per step of sends of every frame shard
to its display rank and receives of every shard of the frames displayed here (svo_exchange.hip
exchange_wire), ragged sizes, empty shards skipped, several steps in a row — and every payload arrives
intact at the right place.  NCCL's rules hold: sends and receives between a pair match in issue order, a
size mismatch is an error (ncclInvalidUsage) rather than a truncation, and a receive with no sender fails
with ncclSystemError after the timeout instead of hanging."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = textwrap.dedent(r'''
    import ctypes, os, sys, time
    lib = ctypes.CDLL(os.environ["STANDIN"])
    class Uid(ctypes.Structure):
        _fields_ = [("internal", ctypes.c_char * 128)]
    N, me, mode, idfile = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    uid = Uid()
    if me == 0:
        assert lib.ncclGetUniqueId(ctypes.byref(uid)) == 0
        open(idfile + ".tmp", "wb").write(bytes(uid.internal))
        os.rename(idfile + ".tmp", idfile)
    else:
        while not os.path.exists(idfile):
            time.sleep(0.01)
        ctypes.memmove(ctypes.byref(uid), open(idfile, "rb").read(), 128)
    if mode == "late" and me == N - 1:
        time.sleep(2.0)  # joins after the others have finished and left
    comm = ctypes.c_void_p()
    rc = lib.ncclCommInitRank(ctypes.byref(comm), N, uid, me)
    assert rc == 0, rc
    n, r = ctypes.c_int(), ctypes.c_int()
    assert lib.ncclCommCount(comm, ctypes.byref(n)) == 0 and n.value == N
    assert lib.ncclCommUserRank(comm, ctypes.byref(r)) == 0 and r.value == me
    U8 = 1  # ncclUint8 (ncclInt8 = 0)

    def payload(step, frame, src, nbytes):
        return bytes(((step * 131 + frame * 17 + src * 7 + i) & 255) for i in range(nbytes))

    if mode == "exchange":
        # exchange_wire's pattern: frame f -> rank f % N; shard of rank r holds cnt[r] records (ragged, some empty)
        nf = 2 * N + 1
        cnt = [(r * 37 + 11) % 53 for r in range(N)]
        cnt[N - 1] = 0  # an empty shard: no send, no receive
        for step in range(3):
            sends = [ctypes.create_string_buffer(payload(step, f, me, cnt[me]), max(1, cnt[me])) for f in range(nf)]
            mine = [f for f in range(nf) if f % N == me]
            recvs = {(f, s): ctypes.create_string_buffer(max(1, cnt[s])) for f in mine for s in range(N) if s != me and cnt[s]}
            assert lib.ncclGroupStart() == 0
            for f in range(nf):
                if f % N != me and cnt[me]:
                    assert lib.ncclSend(sends[f], ctypes.c_size_t(cnt[me]), U8, f % N, comm, None) == 0
            for f in mine:
                for s in range(N):
                    if s != me and cnt[s]:
                        assert lib.ncclRecv(recvs[(f, s)], ctypes.c_size_t(cnt[s]), U8, s, comm, None) == 0
            rc = lib.ncclGroupEnd()
            assert rc == 0, (rc, lib.ncclGetErrorString(rc))
            for (f, s), b in recvs.items():
                assert b.raw[:cnt[s]] == payload(step, f, s, cnt[s]), (step, f, s)
        print("ok exchange", me)
    elif mode == "mismatch":
        if me == 0:
            buf = ctypes.create_string_buffer(b"x" * 10, 10)
            assert lib.ncclSend(buf, ctypes.c_size_t(10), U8, 1, comm, None) == 0
        else:
            buf = ctypes.create_string_buffer(8)
            rc = lib.ncclRecv(buf, ctypes.c_size_t(8), U8, 0, comm, None)
            assert rc == 5, rc  # ncclInvalidUsage
        print("ok mismatch", me)
    elif mode == "late":
        print("ok late", me)
    elif mode == "timeout":
        if me == 1:
            buf = ctypes.create_string_buffer(8)
            t0 = time.time()
            rc = lib.ncclRecv(buf, ctypes.c_size_t(8), U8, 0, comm, None)
            assert rc == 2 and time.time() - t0 < 30, rc  # ncclSystemError after SVO_STANDIN_TIMEOUT_S
        print("ok timeout", me)
    assert lib.ncclCommDestroy(comm) == 0
''')


@pytest.fixture(scope="module")
def standin():
    from raytracing_test_amd import build as b

    return b.build_rccl_standin()


def _ranks(standin, tmp_path, n, mode, timeout_s="120"):
    env = dict(os.environ, STANDIN=standin, SVO_STANDIN_HOST_ONLY="1", SVO_STANDIN_DIR=str(tmp_path),
               SVO_STANDIN_TIMEOUT_S=timeout_s)
    idf = str(tmp_path / "uid")
    procs = [subprocess.Popen([sys.executable, "-c", RANK_SCRIPT, str(n), str(r), mode, idf], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(n)]
    outs = [p.communicate(timeout=90) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    return outs


@pytest.mark.parametrize("n", [2, 3, 4])
def test_standin_exchange_pattern(standin, tmp_path, n):
    outs = _ranks(standin, tmp_path, n, "exchange")
    assert all("ok exchange" in o for o, _ in outs)
    # the communicator's directory is gone: no message left undelivered
    assert [p for p in os.listdir(tmp_path) if p.startswith("svo_rccl_standin_")] == []


def test_standin_size_mismatch_is_an_error(standin, tmp_path):
    _ranks(standin, tmp_path, 2, "mismatch")


def test_standin_receive_times_out(standin, tmp_path):
    _ranks(standin, tmp_path, 2, "timeout", timeout_s="1")


def test_standin_rank_joining_after_the_others_left(standin, tmp_path):
    """ranks with nothing to exchange may finish and destroy their communicator before a slow rank has passed
    ncclCommInitRank's barrier (seen under a loaded CPU suite): their announcements stay until the last rank is out"""
    outs = _ranks(standin, tmp_path, 3, "late")
    assert all("ok late" in o for o, _ in outs)
    assert [p for p in os.listdir(tmp_path) if p.startswith("svo_rccl_standin_")] == []


_OPT_IN = r'''
import sys
sys.path.insert(0, sys.argv[1])
import raytracing_test_amd as rt
try:
    uid = rt.Exchange.unique_id()
    print("UID", uid[:17].decode("ascii", "replace"))
except rt.SvoError as e:
    print("ERR", e)
'''


@pytest.mark.parametrize("opt_in", [False, True])
def test_standin_needs_both_variables(tmp_path, opt_in):
    """libsvo_rt loads another RCCL implementation only when SVO_RCCL_LIB names it AND SVO_RCCL_STANDIN=1 (ADVICE r05:
    a stray SVO_RCCL_LIB must not turn a measurement into a stand-in run): with the variable alone the exchange's first
    call fails with a message naming the missing opt-in; with both, the stand-in answers (its unique ids carry its
    magic prefix).  Host only: no GPU call is made."""
    from raytracing_test_amd import build as b

    standin = b.build_rccl_standin()
    script = tmp_path / "opt.py"
    script.write_text(_OPT_IN)
    env = {k: v for k, v in os.environ.items() if k not in ("SVO_RCCL_LIB", "SVO_RCCL_STANDIN")}
    env["SVO_RCCL_LIB"] = standin
    env["SVO_STANDIN_HOST_ONLY"] = "1"
    if opt_in:
        env["SVO_RCCL_STANDIN"] = "1"
    p = subprocess.run([sys.executable, str(script), ROOT], capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    if opt_in:
        assert "UID svo-rccl-standin:" in p.stdout, p.stdout
    else:
        assert "ERR" in p.stdout and "SVO_RCCL_STANDIN=1" in p.stdout, p.stdout
