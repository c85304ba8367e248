"""Build libsvo_rt.so in-tree for gfx950 (hipcc for the kernels, g++ for the host builder).

Flags that matter for parity: -ffp-contract=off everywhere (no FMA contraction of the FP64 DDA,
the noise or the float ray generation), no fast-math.
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libsvo_rt.so")
BUILD = os.path.join(HERE, "_build")
ARCH = os.environ.get("SVO_OFFLOAD_ARCH", "gfx950")

HOST_SRCS = ["svo_world.cpp"]
HIP_SRCS = ["svo_cast.hip", "svo_build.hip", "svo_exchange.hip"]
HEADERS = ["svo_common.h", "svo_noise.h", "svo_internal.h", "svo_hip.h"]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build(force=False, verbose=False, out=None, build_dir=None, defines=(), flags=()):
    """out / build_dir / defines / flags: alternate variants for A/B timing (the default is the product)"""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    OUT_ = out or OUT
    BUILD_ = build_dir or BUILD
    os.makedirs(BUILD_, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(HERE, "..", "include", "svo_rt.h")]
    objs = []
    for s in HOST_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD_, s + ".o")
        if force or _newer(obj, [src] + hdrs):
            _run(["g++", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-pthread", "-Wall"] +
                 ["-D" + d for d in defines] + ["-c", src, "-o", obj])
        objs.append(obj)
    for s in HIP_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(BUILD_, s + ".o")
        if force or _newer(obj, [src] + hdrs):
            _run([hipcc, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
                  "-Wall"] + ["-D" + d for d in defines] + list(flags) + ["-c", src, "-o", obj])
        objs.append(obj)
    if force or _newer(OUT_, objs):
        _run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", OUT_] + objs + ["-pthread", "-ldl"])
    return OUT_


def build_bridge_test(force=False):
    """The drop-in shim (bridge/svo_bridge.cpp) + its C++ test program (tests/bridge/bridge_test.cpp),
    linked against libsvo_rt.so without Python: tests/bridge/_build/bridge_test."""
    root = os.path.dirname(HERE)
    out_dir = os.path.join(root, "tests", "bridge", "_build")
    out = os.path.join(out_dir, "bridge_test")
    srcs = [os.path.join(root, "bridge", "svo_bridge.cpp"), os.path.join(root, "tests", "bridge", "bridge_test.cpp")]
    deps = srcs + [os.path.join(root, "bridge", "svo_bridge.hpp"), os.path.join(root, "tests", "bridge", "svo_bridge_types.hpp"),
                   os.path.join(root, "include", "svo_rt.h"), OUT]
    if not force and not _newer(out, deps):
        return out
    os.makedirs(out_dir, exist_ok=True)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    _run(["g++", "-O2", "-std=c++17", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(rocm, "include"),
          "-I" + os.path.join(root, "include"), "-I" + os.path.join(root, "bridge"), "-I" + os.path.join(root, "tests", "bridge")] + srcs +
         ["-L" + HERE, "-lsvo_rt", "-L" + os.path.join(rocm, "lib"), "-lamdhip64", "-Wl,-rpath,$ORIGIN/../../../raytracing_test_amd",
          "-Wl,-rpath," + os.path.join(rocm, "lib"), "-o", out])
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_bridge_test(force="--force" in sys.argv)
