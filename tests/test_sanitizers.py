"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (+ LeakSanitizer), SURVEY.md §5: the
product's host half (raytracing_test_amd/csrc/svo_world.cpp: edits, every builder in both views, patching,
lookups, checkpoint) and the oracle (oracle/oracle.c: casts, AO, shading, deleteBlock), each driven by a
small program in tests/sanitize/ and built with gcc here.  GPU sanitizers are not available on the pool;
these run on the CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-ffp-contract=off", "-pthread"]


def _run(cmd, **kw):
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, **kw)
    assert p.returncode == 0, (" ".join(cmd), p.stdout[-2000:], p.stderr[-4000:])
    return p.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_library_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_sanitize")
    _run(["g++", "-std=c++17"] + SAN + ["-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "sanitize", "host_sanitize.cpp"),
                                       os.path.join(ROOT, "raytracing_test_amd", "csrc", "svo_world.cpp"), "-o", exe])
    out = _run([exe, str(tmp_path / "t.svo")], env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert "host sanitize ok" in out


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_oracle_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_sanitize")
    _run(["gcc", "-std=c11"] + SAN + [os.path.join(ROOT, "tests", "sanitize", "oracle_sanitize.c"), os.path.join(ROOT, "oracle", "oracle.c"),
                                     "-lm", "-o", exe])
    out = _run([exe], env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert "oracle sanitize ok" in out
