"""The shipped library is tied to the committed sources (raytracing_test_amd/build.py: sources_sha256, the stamp that
build() embeds and svo_build_id() returns).  CPU only: nothing here launches a kernel."""
import os
import shutil
import subprocess

import pytest

from raytracing_test_amd import build as B

ROOT = B.ROOT


def _git(*args):
    return subprocess.run(["git", "-C", ROOT] + list(args), capture_output=True)


def test_stamped_files_cover_every_header():
    files = B.stamped_files()
    csrc = os.path.join(ROOT, "raytracing_test_amd", "csrc")
    for name in os.listdir(csrc):
        if name.endswith((".h", ".hip", ".cpp")):
            assert "raytracing_test_amd/csrc/" + name in files, name
    assert "include/svo_rt.h" in files


def test_sources_sha256_matches_head():
    """The stamp recomputed from HEAD's blobs equals the one from the files here whenever they are HEAD's"""
    if _git("rev-parse", "HEAD").returncode != 0:
        pytest.skip("not a git checkout")
    files = B.stamped_files()
    if _git("diff", "--quiet", "HEAD", "--", *files).returncode != 0:
        pytest.skip("stamped sources differ from HEAD (uncommitted edits)")

    def head(rel):
        r = _git("show", "HEAD:" + rel)
        assert r.returncode == 0, rel
        return r.stdout

    assert B.sources_sha256(read=head) == B.sources_sha256()


def test_built_library_carries_current_stamp():
    if not os.path.exists(B.OUT):
        pytest.skip("library not built")
    assert B.read_stamp(B.OUT) == B.sources_sha256(), "libsvo_rt.so is stale: run __graft_entry__.build()"
    assert not B.needs_build()


def test_rebuild_decision_follows_contents_not_mtimes(tmp_path):
    root = str(tmp_path)
    for rel in B.stamped_files():
        os.makedirs(os.path.join(root, os.path.dirname(rel)), exist_ok=True)
        shutil.copy(os.path.join(ROOT, rel), os.path.join(root, rel))
    fake = os.path.join(root, "lib.so")
    with open(fake, "wb") as f:
        f.write(b"\x7fELF..." + B.STAMP_TAG + B.sources_sha256(root).encode() + b"\0rest")
    assert not B.needs_build(fake, root)
    src = os.path.join(root, "raytracing_test_amd", "csrc", "svo_cast.hip")
    st = os.stat(src)
    os.utime(src, (st.st_atime + 3600, st.st_mtime + 3600))  # touched, unchanged: newer than the library
    assert not B.needs_build(fake, root)
    with open(os.path.join(root, "raytracing_test_amd", "csrc", "svo_wire.h"), "a") as f:
        f.write("\n// changed\n")  # a header the kernels include
    assert B.needs_build(fake, root)
    assert B.needs_build(fake, root, defines=("X=1",)) and B.read_stamp(os.path.join(root, "missing.so")) is None
