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
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(HERE, "..", "include", "svo_rt.h")]
    # the product library newer than every source and header is up to date, whether or not its objects travelled with
    # it (gpurun snapshots leave *.o behind: without this the GPU box's first test rebuilt the library there, and the
    # timed build was no longer the one the PMC passes had measured — bench.py's counters_build / timed_build)
    if not force and out is None and not defines and not flags and os.path.exists(OUT_) and \
            not _newer(OUT_, [os.path.join(CSRC, s) for s in HOST_SRCS + HIP_SRCS] + hdrs):
        return OUT_
    os.makedirs(BUILD_, exist_ok=True)
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


def _bridge_cxx(root, rocm, incs):
    return ["g++", "-O2", "-std=c++17", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(rocm, "include"),
            "-I" + os.path.join(root, "include")] + ["-I" + i for i in incs]


def build_bridge_test(force=False):
    """The drop-in shim (bridge/svo_bridge.cpp) + its two C++ test programs, linked against libsvo_rt.so
    without Python: tests/bridge/_build/bridge_test (the application's call sequence, edits, the exchange)
    and tests/bridge/_build/main_shape (a main.cpp-shaped TU that includes the replacement
    voxel_allocator.hpp, bridge/reference/voxel_data/; its object is kept for the nm check of
    tests/test_bridge_link.py).  Returns the bridge_test path."""
    root = os.path.dirname(HERE)
    out_dir = os.path.join(root, "tests", "bridge", "_build")
    os.makedirs(out_dir, exist_ok=True)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    # tests/bridge first: its svo_bridge_types.hpp (the GLM-free mirror), not bridge/reference's
    incs = [os.path.join(root, "tests", "bridge"), os.path.join(root, "bridge"), os.path.join(root, "bridge", "reference")]
    hdrs = [os.path.join(root, "bridge", "svo_bridge.hpp"), os.path.join(root, "tests", "bridge", "svo_bridge_types.hpp"),
            os.path.join(root, "bridge", "reference", "voxel_data", "voxel_allocator.hpp"), os.path.join(root, "include", "svo_rt.h")]
    link = ["-L" + HERE, "-lsvo_rt", "-L" + os.path.join(rocm, "lib"), "-lamdhip64", "-Wl,-rpath,$ORIGIN/../../../raytracing_test_amd",
            "-Wl,-rpath," + os.path.join(rocm, "lib")]
    objs = {}
    for name, src in (("svo_bridge", os.path.join(root, "bridge", "svo_bridge.cpp")),
                      ("bridge_test", os.path.join(root, "tests", "bridge", "bridge_test.cpp")),
                      ("main_shape", os.path.join(root, "tests", "bridge", "main_shape.cpp"))):
        obj = os.path.join(out_dir, name + ".o")
        if force or _newer(obj, [src] + hdrs):
            _run(_bridge_cxx(root, rocm, incs) + ["-c", src, "-o", obj])
        objs[name] = obj
    for prog in ("bridge_test", "main_shape"):
        out = os.path.join(out_dir, prog)
        if force or _newer(out, [objs["svo_bridge"], objs[prog], OUT]):
            # no voxel_allocator.cpp / tetrahexa_tree.cpp / ray_caster.cpp / world_gen.cpp: the shim and libsvo_rt only
            _run(["g++", objs[prog], objs["svo_bridge"]] + link + ["-o", out])
    return os.path.join(out_dir, "bridge_test")


STANDIN = os.path.join(os.path.dirname(HERE), "tests", "standin", "_build", "librccl_standin.so")


def build_rccl_standin(force=False):
    """TEST-ONLY: tests/standin/rccl_standin.cpp -> tests/standin/_build/librccl_standin.so, the host-staged
    stand-in for librccl.so.1 that libsvo_rt loads when SVO_RCCL_LIB names it (several ranks of the exchange on
    one GPU).  Host code only; -Bsymbolic so its entry points never bind to an RCCL already in the process."""
    src = os.path.join(os.path.dirname(HERE), "tests", "standin", "rccl_standin.cpp")
    if not force and not _newer(STANDIN, [src]):
        return STANDIN
    os.makedirs(os.path.dirname(STANDIN), exist_ok=True)
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    _run([hipcc, "--offload-arch=" + ARCH, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-fvisibility=hidden",
          "-Wl,-Bsymbolic", src, "-o", STANDIN])
    return STANDIN


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_bridge_test(force="--force" in sys.argv)
    build_rccl_standin(force="--force" in sys.argv)
