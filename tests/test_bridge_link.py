"""The drop-in links against a main.cpp-shaped translation unit ("main.cpp / input.cpp
link unchanged").  The reference's src/voxel_data/voxel_allocator.hpp defines updateSsboData() and
initVoxelDataAllocator() inline with GL bodies (voxel_allocator.hpp:38-91) that read arrayBlocks /
nodeBlocks, defined only in voxel_allocator.cpp (:6,22), which the integration drops; main.cpp:183,212
call them.  INTEGRATION.md step 2 swaps that header for bridge/reference/voxel_data/voxel_allocator.hpp.
These checks need no GPU: the object of tests/bridge/main_shape.cpp (which includes the replacement
header by main.cpp's own include name) must leave both functions as undefined references, bound at link
time to the shim's definitions; the program must link with no voxel_allocator.cpp."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "bridge", "_build")
HDR = os.path.join(ROOT, "bridge", "reference", "voxel_data", "voxel_allocator.hpp")
SYMS = ("_Z14updateSsboDatav", "_Z22initVoxelDataAllocatorv")


@pytest.fixture(scope="module")
def built():
    from raytracing_test_amd import build as b

    if not os.path.exists(b.OUT):
        b.build()
    b.build_bridge_test()
    return BUILD


def _nm(path):
    out = subprocess.run(["nm", path], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1]: ln.split()[-2] for ln in out.splitlines() if ln.split()}


def test_replacement_header_declares_only(built):
    """the replacement holds declarations only: no GL / Windows / GLM include, no function body"""
    src = open(HDR).read()
    code = "\n".join(ln for ln in src.splitlines() if not ln.lstrip().startswith("//"))
    assert "#include" not in code
    assert "{" not in code
    for name in ("void initVoxelDataAllocator();", "void updateSsboData();"):
        assert name in code


def test_main_shape_references_the_shim(built):
    """main_shape.o (main.cpp's include of voxel_allocator.hpp) refers to both functions (type U), the
    shim's object defines them (type T): nothing inline from the header reaches main's TU"""
    main = _nm(os.path.join(built, "main_shape.o"))
    shim = _nm(os.path.join(built, "svo_bridge.o"))
    for s in SYMS:
        assert main.get(s) == "U", (s, main.get(s))
        assert shim.get(s) == "T", (s, shim.get(s))
    # nor does main's TU pull in the reference allocator's pools
    assert not any("arrayBlocks" in k or "nodeBlocks" in k for k in main)


def test_main_shape_links_without_voxel_allocator(built):
    """the linked program resolves both calls inside itself (the shim's definitions) and depends on no
    reference allocator symbol"""
    prog = os.path.join(built, "main_shape")
    assert os.path.exists(prog)
    syms = _nm(prog)
    for s in SYMS:
        assert syms.get(s) == "T", (s, syms.get(s))
    assert not any(k.endswith(("arrayBlocks", "nodeBlocks")) for k in syms)


def test_gl_present_helper_compiles_and_links(built, tmp_path):
    """bridge/svo_present_gl.cpp (svoPresentShaded: svoRenderShaded into a HIP-registered GL pixel buffer, a texture
    upload and a blit — what replaces render()'s glDrawArrays, main.cpp:105-107) compiles against the system GL
    headers and hip_gl_interop.h, and a main.cpp-shaped program links with it, the shim and libsvo_rt, every GL entry
    point from libGL and every HIP one from libamdhip64 (no GL context here: nothing is run)"""
    gl = [d for d in ("/usr/lib/x86_64-linux-gnu", "/usr/lib64", "/usr/lib") if os.path.exists(os.path.join(d, "libGL.so"))]
    if not os.path.exists("/usr/include/GL/glext.h") or not gl:
        pytest.skip("no GL headers / libGL in this image")
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    obj = str(tmp_path / "svo_present_gl.o")
    inc = ["-I" + os.path.join(rocm, "include"), "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "tests", "bridge"),
           "-I" + os.path.join(ROOT, "bridge"), "-I" + os.path.join(ROOT, "bridge", "reference")]
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__"] + inc +
                   ["-c", os.path.join(ROOT, "bridge", "svo_present_gl.cpp"), "-o", obj], check=True)
    syms = _nm(obj)
    assert syms.get("_Z16svoPresentShadediifP12ihipStream_t") == "T"
    for s in ("hipGraphicsGLRegisterBuffer", "hipGraphicsMapResources", "hipGraphicsResourceGetMappedPointer",
              "hipGraphicsUnmapResources", "glTexSubImage2D", "glBlitFramebuffer", "_Z15svoRenderShadediiPfP12ihipStream_tf"):
        assert syms.get(s) == "U", s
    prog = str(tmp_path / "main_shape_gl")
    from raytracing_test_amd import build as b
    subprocess.run(["g++", os.path.join(built, "main_shape.o"), os.path.join(built, "svo_bridge.o"), obj, "-L" + b.HERE, "-lsvo_rt",
                    "-L" + os.path.join(rocm, "lib"), "-lamdhip64", "-L" + gl[0], "-lGL", "-o", prog], check=True)
    assert _nm(prog).get("_Z16svoPresentShadediifP12ihipStream_t") == "T"
