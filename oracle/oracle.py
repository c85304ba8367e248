"""ORACLE — test infrastructure only (ctypes wrapper over oracle/_build/liboracle.so).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker /
timed CPU baseline.  The product (raytracing_test_amd/) never imports this module.
See oracle/oracle.c for the reference file:line each function restates.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
def _cpu_tag():
    # -march=native objects are only valid on the CPU model they were built on (build container vs GPU box)
    import hashlib
    import platform

    model = platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name") or line.startswith("flags"):
                model += line
    except OSError:
        pass
    return hashlib.sha1(model.encode()).hexdigest()[:10]


LIB_NATIVE = os.path.join(HERE, "_build", "liboracle_native_%s.so" % _cpu_tag())
REF_NOISE = os.path.join(HERE, "_ref", "libref_noise.so")

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C")
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C")


class RayRes(C.Structure):
    _fields_ = [
        ("pos", C.c_int32 * 3),
        ("last", C.c_int32 * 3),
        ("steps", C.c_int32),
        ("hit", C.c_int32),
        ("axis", C.c_int32),
        ("flags", C.c_uint32),
        ("color", C.c_uint64),
        ("meta", C.c_float),
        ("t", C.c_double),
        ("err", C.c_int32),
        ("n_dda", C.c_uint32),
    ]


def build(native=False):
    if native:
        if not os.path.exists(LIB_NATIVE) or os.path.getmtime(LIB_NATIVE) < os.path.getmtime(os.path.join(HERE, "oracle.c")):
            os.makedirs(os.path.join(HERE, "_build"), exist_ok=True)
            subprocess.check_call(["gcc", "-O3", "-std=c11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-pthread",
                                   "-march=native", "-shared", "-o", LIB_NATIVE, os.path.join(HERE, "oracle.c"), "-lm"])
        return
    subprocess.check_call(["make", "-s", "-C", HERE, "_build/liboracle.so"])


LIB_O0 = os.path.join(HERE, "_build", "liboracle_O0.so")


def lib_O0():
    """the same restatement at -O0 (the reference's own build flags, build.bat:4: `g++ -g`), for the CPU
    baseline's -O0 figure; trees built by lib() are used through it unchanged (same source, same layout)"""
    if not os.path.exists(LIB_O0) or os.path.getmtime(LIB_O0) < os.path.getmtime(os.path.join(HERE, "oracle.c")):
        os.makedirs(os.path.join(HERE, "_build"), exist_ok=True)
        subprocess.check_call(["gcc", "-O0", "-std=c11", "-fPIC", "-ffp-contract=off", "-pthread", "-shared", "-o", LIB_O0,
                               os.path.join(HERE, "oracle.c"), "-lm"])
    if LIB_O0 not in _libs:
        L = C.CDLL(LIB_O0)
        L.orc_cast_frame.argtypes = lib().orc_cast_frame.argtypes
        _libs[LIB_O0] = L
    return _libs[LIB_O0]


def build_ref():
    subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


_libs = {}


def lib(native=False):
    path = LIB_NATIVE if native else LIB
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        build(native)
    L = C.CDLL(path)
    vp = C.c_void_p
    L.orc_tree_new.restype = vp
    L.orc_tree_new.argtypes = [C.c_int]
    L.orc_tree_free.argtypes = [vp]
    L.orc_tree_error.argtypes = [vp]
    for n in ("orc_tree_nodes", "orc_tree_arrays", "orc_root_bitmap"):
        getattr(L, n).restype = C.c_uint64
        getattr(L, n).argtypes = [vp]
    L.orc_root_children.restype = C.c_uint32
    L.orc_root_children.argtypes = [vp]
    L.orc_root_flags.restype = C.c_uint32
    L.orc_root_flags.argtypes = [vp]
    L.orc_get_block.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_float)]
    L.orc_put_block.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_uint64, C.c_float, C.c_int]
    L.orc_delete_block.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_float)]
    L.orc_init_tetra_hexa_tree.argtypes = [vp]
    L.orc_init_clean_root.argtypes = [vp]
    L.orc_noise2.restype = C.c_double
    L.orc_noise2.argtypes = [C.c_int64, C.c_double, C.c_double]
    L.orc_noise_perm.argtypes = [C.c_int64, np.ctypeslib.ndpointer(np.int16, flags="C")]
    L.orc_rgb.restype = C.c_uint64
    L.orc_rgb.argtypes = [C.c_int, C.c_int, C.c_int]
    L.orc_heights.argtypes = [C.c_int, C.c_int, _i32p, C.c_int]
    L.orc_gen_world.argtypes = [vp, C.c_int, C.c_int]
    L.orc_build_terrain_collapsed.argtypes = [vp, _i32p, C.c_int, C.c_int]
    L.orc_normalize.argtypes = [_f32p, _f32p]
    L.orc_pixel_dir.argtypes = [_f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, _f32p]
    L.orc_proj_plane.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    L.orc_cast_ray.argtypes = [vp, _f32p, _f32p, C.c_int, C.POINTER(RayRes)]
    L.orc_dda_free.argtypes = [_f32p, _f32p, C.c_int, _i32p, C.POINTER(C.c_int32)]
    L.orc_cast_frame.argtypes = [vp, _f32p, _f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, vp, C.c_int64, C.c_int,
                                 vp, vp, vp, vp, vp, vp, vp, vp, C.POINTER(C.c_uint64)]
    L.orc_dense_from_tree.restype = vp
    L.orc_dense_from_tree.argtypes = [vp, C.c_int]
    L.orc_dense_free.argtypes = [vp]
    L.orc_cast_frame_dense.argtypes = [vp, _f32p, _f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int,
                                       vp, vp, vp, vp, C.POINTER(C.c_uint64)]
    L.orc_frame_entries.restype = C.c_uint64
    L.orc_frame_entries.argtypes = [vp, _f32p, _f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, vp, C.c_int64, C.c_int]
    L.orc_frame_entries_ao.restype = C.c_uint64
    L.orc_frame_entries_ao.argtypes = [vp, _f32p, _f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int64,
                                       C.c_int]
    L.orc_digest_box.restype = C.c_uint64
    L.orc_digest_box.argtypes = [vp] + [C.c_int] * 6
    L.orc_dump_box.argtypes = [vp] + [C.c_int] * 6 + [_u32p, _u64p]
    L.orc_hemisphere.argtypes = [C.c_int, _f32p]
    L.orc_cast_frame_ao.argtypes = [vp, _f32p, _f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int64,
                                    C.c_int, vp, vp]
    L.orc_shade_frame.argtypes = [vp, _f32p, _f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, _f32p, vp, C.c_int, vp, C.c_int64,
                                  C.c_int, vp, C.c_int, C.c_float]
    L.orc_shade_entries.argtypes = [vp, _f32p, _f32p, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, _f32p, C.c_int, vp, C.c_int64,
                                    C.c_int, C.c_int, C.c_float, vp]
    L.orc_sin_f32.restype = C.c_float
    L.orc_sin_f32.argtypes = [C.c_float]
    _libs[path] = L
    return L


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def f3(v):
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32).reshape(3))


def normalize(v):
    o = np.zeros(3, np.float32)
    lib().orc_normalize(f3(v), o)
    return o


def proj_plane(W, H):
    a, b = C.c_float(), C.c_float()
    lib().orc_proj_plane(W, H, C.byref(a), C.byref(b))
    return a.value, b.value


def pixel_dir(cam, ppx, ppy, W, H, px, py):
    o = np.zeros(3, np.float32)
    lib().orc_pixel_dir(f3(cam), ppx, ppy, W, H, px, py, o)
    return o


def hemisphere(n):
    out = np.zeros(3 * n, np.float32)
    lib().orc_hemisphere(n, out)
    return out.reshape(n, 3)


def sin_f32(x):
    return lib().orc_sin_f32(x)


def noise2(seed, x, y):
    return lib().orc_noise2(seed, x, y)


def heights(W, L, nthreads=8):
    out = np.zeros(W * L, np.int32)
    lib().orc_heights(W, L, out, nthreads)
    return out.reshape(W, L)


class Tree:
    """A reference-layout tree (16 B nodes + 256 B child arrays)."""

    def __init__(self, levels=5, native=False):
        self.L = lib(native)
        self.levels = levels
        self.h = self.L.orc_tree_new(levels)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_tree_free(self.h)
            self.h = None

    @classmethod
    def reference_world(cls, width=200, length=200, native=False):
        """initTetraHexaTree() + genWorld() at maxDepth 6 (the reference application's world)."""
        t = cls(5, native)
        t.L.orc_init_tetra_hexa_tree(t.h)
        t.L.orc_gen_world(t.h, width, length)
        return t

    @classmethod
    def terrain(cls, levels, width, length, native=False, nthreads=8):
        """genWorld's column formula on width x length, built with uniform-region collapse."""
        t = cls(levels, native)
        hg = np.ascontiguousarray(heights(width, length, nthreads).reshape(-1))
        rc = t.L.orc_build_terrain_collapsed(t.h, hg, width, length)
        if rc:
            raise ValueError("terrain out of range for levels=%d (rc=%d)" % (levels, rc))
        return t

    @classmethod
    def heightfield(cls, levels, hts, native=False):
        """The same collapse builder from given column tops, hts shape (width, length)."""
        t = cls(levels, native)
        hg = np.ascontiguousarray(np.asarray(hts, np.int32).reshape(-1))
        rc = t.L.orc_build_terrain_collapsed(t.h, hg, hts.shape[0], hts.shape[1])
        if rc:
            raise ValueError("heights out of range for levels=%d (rc=%d)" % (levels, rc))
        return t

    @classmethod
    def terrain_putblock(cls, levels, width, length, native=False):
        """Clean root + genWorld via per-voxel putBlock (no debug blocks)."""
        t = cls(levels, native)
        t.L.orc_init_clean_root(t.h)
        t.L.orc_gen_world(t.h, width, length)
        return t

    def put_block(self, x, y, z, flags, color, meta=0.0, level=6):
        return self.L.orc_put_block(self.h, x, y, z, flags, color, meta, level)

    def delete_block(self, x, y, z, level=6, ref_shift=False):
        """deleteBlock (tetrahexa_tree.cpp:293-359); ref_shift reproduces its int `1 << index` bitmap
        update (x86 semantics), else the intended bit clear.  Returns (rc, (flags, color, meta))."""
        f, c, m = C.c_uint32(), C.c_uint64(), C.c_float()
        rc = self.L.orc_delete_block(self.h, x, y, z, level, 1 if ref_shift else 0, C.byref(f), C.byref(c), C.byref(m))
        return rc, (f.value, c.value, m.value)

    def get_block(self, x, y, z):
        f, c, m = C.c_uint32(), C.c_uint64(), C.c_float()
        rc = self.L.orc_get_block(self.h, x, y, z, C.byref(f), C.byref(c), C.byref(m))
        if rc:
            raise RuntimeError("getBlock hit max depth at (%d,%d,%d)" % (x, y, z))
        return f.value, c.value, m.value

    def nodes(self):
        return self.L.orc_tree_nodes(self.h)

    def arrays(self):
        return self.L.orc_tree_arrays(self.h)

    def root_bitmap(self):
        return self.L.orc_root_bitmap(self.h)

    def digest_box(self, x0, y0, z0, nx, ny, nz):
        return self.L.orc_digest_box(self.h, x0, y0, z0, nx, ny, nz)

    def dump_box(self, x0, y0, z0, nx, ny, nz):
        n = nx * ny * nz
        f = np.zeros(n, np.uint32)
        c = np.zeros(n, np.uint64)
        rc = self.L.orc_dump_box(self.h, x0, y0, z0, nx, ny, nz, f, c)
        return rc, f.reshape(nz, ny, nx), c.reshape(nz, ny, nx)

    def cast_ray(self, org, d, steps):
        r = RayRes()
        self.L.orc_cast_ray(self.h, f3(org), f3(d), steps, C.byref(r))
        return r

    def cast_frame(self, org, cam, W, H, steps, ppx=None, ppy=None, pixels=None, nthreads=8, L=None):
        """castRayFromCam semantics for every pixel ray (or a subset); returns a dict of arrays.
        L: another build of the same restatement (lib_O0()) to run it with"""
        if ppx is None:
            ppx, ppy = proj_plane(W, H)
        n = W * H if pixels is None else len(pixels)
        pix = None if pixels is None else np.ascontiguousarray(pixels, dtype=np.int64)
        out = dict(
            pos=np.zeros((n, 3), np.int32),
            last=np.zeros((n, 3), np.int32),
            steps=np.zeros(n, np.int32),
            hit=np.zeros(n, np.int32),
            t=np.zeros(n, np.float64),
            color=np.zeros(n, np.uint64),
            flags=np.zeros(n, np.uint32),
            axis=np.zeros(n, np.int32),
        )
        dda = C.c_uint64()
        rc = (L or self.L).orc_cast_frame(self.h, f3(org), f3(cam), ppx, ppy, W, H, steps, _ptr(pix), n, nthreads,
                                   _ptr(out["pos"]), _ptr(out["last"]), _ptr(out["steps"]), _ptr(out["hit"]), _ptr(out["t"]),
                                   _ptr(out["color"]), _ptr(out["flags"]), _ptr(out["axis"]), C.byref(dda))
        out["rc"] = rc
        out["dda_steps"] = dda.value
        return out

    def cast_frame_ao(self, org, cam, W, H, steps, n_ao, ao_steps=5, ppx=None, ppy=None, pixels=None, nthreads=8):
        """primary rays + hemisphere AO: per-pixel count of AO rays that hit (see oracle.c A8)"""
        if ppx is None:
            ppx, ppy = proj_plane(W, H)
        n = W * H if pixels is None else len(pixels)
        pix = None if pixels is None else np.ascontiguousarray(pixels, dtype=np.int64)
        ao = np.zeros(n, np.uint8)
        hit = np.zeros(n, np.int32)
        self.L.orc_cast_frame_ao(self.h, f3(org), f3(cam), ppx, ppy, W, H, steps, n_ao, ao_steps, _ptr(pix), n, nthreads, _ptr(ao),
                                 _ptr(hit))
        return ao, hit

    def shade_frame(self, org, cam, W, H, steps, sun, look_at=None, shadow_steps=75, ppx=None, ppy=None, pixels=None, nthreads=8,
                    liquid=False, time=0.0):
        """shaded frame (svo_shade_rays contract, oracle.c §shading): (n, 4) float32 rgba in pixel order;
        liquid: water refracts and tints as in low_res.frag (the product's SVO_VIEW_ALL scene)"""
        if ppx is None:
            ppx, ppy = proj_plane(W, H)
        n = W * H if pixels is None else len(pixels)
        pix = None if pixels is None else np.ascontiguousarray(pixels, dtype=np.int64)
        look = None if look_at is None else np.ascontiguousarray(look_at, dtype=np.int32)
        rgba = np.zeros((n, 4), np.float32)
        self.L.orc_shade_frame(self.h, f3(org), f3(cam), ppx, ppy, W, H, steps, f3(sun), _ptr(look), shadow_steps, _ptr(pix), n, nthreads,
                               _ptr(rgba), 1 if liquid else 0, time)
        return rgba

    def frame_entries(self, org, cam, W, H, steps, ppx=None, ppy=None, pixels=None, nthreads=8):
        if ppx is None:
            ppx, ppy = proj_plane(W, H)
        n = W * H if pixels is None else len(pixels)
        pix = None if pixels is None else np.ascontiguousarray(pixels, dtype=np.int64)
        return self.L.orc_frame_entries(self.h, f3(org), f3(cam), ppx, ppy, W, H, steps, _ptr(pix), n, nthreads)

    def frame_entries_ao(self, org, cam, W, H, steps, n_ao, ao_steps=5, ppx=None, ppy=None, pixels=None, nthreads=8):
        """node entries of the hits' AO rays (restart model continued from each primary's final lookup)"""
        if ppx is None:
            ppx, ppy = proj_plane(W, H)
        n = W * H if pixels is None else len(pixels)
        pix = None if pixels is None else np.ascontiguousarray(pixels, dtype=np.int64)
        return self.L.orc_frame_entries_ao(self.h, f3(org), f3(cam), ppx, ppy, W, H, steps, n_ao, ao_steps, _ptr(pix), n, nthreads)

    def shade_entries(self, org, cam, W, H, steps, sun, shadow_steps=75, ppx=None, ppy=None, pixels=None, nthreads=8, liquid=False,
                      time=0.0):
        """§8(d) node entries of the shading pass (oracle.c orc_shade_entries): (entries, shadow rays, DDA lookups)
        summed over the frame's pixels (or a subset)"""
        if ppx is None:
            ppx, ppy = proj_plane(W, H)
        n = W * H if pixels is None else len(pixels)
        pix = None if pixels is None else np.ascontiguousarray(pixels, dtype=np.int64)
        out = np.zeros(3, np.uint64)
        self.L.orc_shade_entries(self.h, f3(org), f3(cam), ppx, ppy, W, H, steps, f3(sun), shadow_steps, _ptr(pix), n, nthreads,
                                 1 if liquid else 0, time, _ptr(out))
        return int(out[0]), int(out[1]), int(out[2])


class Dense:
    """Config C1: a dense u8 material grid materialised from a tree's [0,n)^3 via getBlock."""

    def __init__(self, tree, n=256):
        self.L = tree.L
        self.h = self.L.orc_dense_from_tree(tree.h, n)
        self.n = n

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_dense_free(self.h)
            self.h = None

    def cast_frame(self, org, cam, W, H, steps, nthreads=8):
        ppx, ppy = proj_plane(W, H)
        n = W * H
        pos = np.zeros((n, 3), np.int32)
        stp = np.zeros(n, np.int32)
        hit = np.zeros(n, np.int32)
        col = np.zeros(n, np.uint64)
        dda = C.c_uint64()
        self.L.orc_cast_frame_dense(self.h, f3(org), f3(cam), ppx, ppy, W, H, steps, nthreads, _ptr(pos), _ptr(stp), _ptr(hit),
                                    _ptr(col), C.byref(dda))
        return dict(pos=pos, steps=stp, hit=hit, color=col, dda_steps=dda.value)


def ref_noise_batch(seed, x, y):
    """The reference's own OpenSimplex (compiled into oracle/_ref); None when unavailable."""
    if not os.path.exists(REF_NOISE):
        return None
    L = C.CDLL(REF_NOISE)
    L.ref_noise2_batch.argtypes = [C.c_int64, _f64p, _f64p, _f64p, C.c_long]
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    out = np.zeros(len(x), np.float64)
    L.ref_noise2_batch(seed, x, y, out, len(x))
    return out
