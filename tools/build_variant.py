"""Build libsvo_rt.so from another git revision (or the working tree with -D defines and / or patches)
into variants/ for A/B timing:
    python tools/build_variant.py <name> [--rev REV] [--patch tools/variants/X.patch ...] [-D NAME=VAL ...]
The product source carries no experiment switches: A/B losers are rebuilt from the revision that had
them (--rev), diagnostics (tools/variants/*.patch) from a patched copy of the sources."""
import argparse
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--rev", default=None)
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--patch", action="append", default=[], help="a unified diff against the source tree (tools/variants/*.patch)")
    ap.add_argument("--flag", action="append", default=[], help="extra hipcc flags, space-separated (e.g. '-mllvm -amdgpu-sched-strategy=max-ilp')")
    a = ap.parse_args()
    src_root = ROOT
    tmp = None
    if a.rev or a.patch:
        tmp = tempfile.mkdtemp()
        if a.rev:
            subprocess.check_call("git -C %s archive %s raytracing_test_amd include | tar -x -C %s" % (ROOT, a.rev, tmp), shell=True)
        else:
            for d in ("raytracing_test_amd", "include"):
                shutil.copytree(os.path.join(ROOT, d), os.path.join(tmp, d), ignore=shutil.ignore_patterns("_build", "*.so", "__pycache__"))
        for pf in a.patch:
            subprocess.check_call(["git", "apply", "--unsafe-paths", "--directory=.", os.path.abspath(pf)], cwd=tmp)
        src_root = tmp
    sys.path.insert(0, os.path.join(src_root, "raytracing_test_amd"))
    import build  # noqa

    out = os.path.join(ROOT, "variants", "libsvo_%s.so" % a.name)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    build.build(force=True, out=out, build_dir=os.path.join(ROOT, "variants", "b_" + a.name), defines=a.D,
                **({"flags": [f for x in a.flag for f in x.split()]} if a.flag else {}))  # (older revisions: no flags)
    if tmp:
        shutil.rmtree(tmp)
    print(out)


if __name__ == "__main__":
    main()
