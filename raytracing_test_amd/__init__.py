"""raytracing_test_amd — MI355X-native sparse-voxel-tree primary raycaster.

Python host mirror of the C ABI in include/svo_rt.h (libsvo_rt.so, built in-tree by
raytracing_test_amd/build.py).  Names follow the reference (reedthorngag/raytracing_test):

    World.init_tetra_hexa_tree()   initTetraHexaTree()        src/voxel_data/tetrahexa_tree.cpp:13
    World.put_block(...)           putBlock(Pos, Block, int)   src/voxel_data/tetrahexa_tree.cpp:176
    World.get_block(...)           getBlock(Pos)               src/voxel_data/tetrahexa_tree.cpp:113
    World.delete_block(...)        deleteBlock(Pos, int)       src/voxel_data/tetrahexa_tree.cpp:293
    World.gen_world(w, l)          genWorld()                  src/world_gen.cpp:13
    Tree.upload(device)            updateSsboData()            src/voxel_data/voxel_allocator.hpp:38
    Tree.cast_ray_from_cam(...)    RAY_CASTER::castRayFromCam  src/ray_caster.cpp:54
    Tree.cast_frame(...)           the low_res.frag per-pixel traversal, as one HIP launch

There is no CPU fallback: every cast runs the gfx950 kernel, and importing this package without
the built library raises.  torch is used only for device buffers and streams.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SVO_LIB") or os.path.join(_HERE, "libsvo_rt.so")

SVO_OK = 0
HIT_BIT = 1 << 31
AXIS_SHIFT = 16
NEG_BIT = 1 << 18
MAT_MASK = 0xFFFF

# Block flags (src/globals.hpp:68-74)
NONE, REFLECTIVE, REFRACTIVE, LUMINESCENT, LIQUID = 0x0, 0x2, 0x4, 0x8, 0x10
CAST_ITERATIVE = 1  # svo_cast_desc.flags: voxel-by-voxel stepping (A/B reference path)
CAST_STATS = 2  # svo_cast_desc.flags: accumulate traversal counters into desc.stats
CAST_BOTTOM_FIRST = 4  # scheduling: bottom tile rows first (default is top first)
CAST_TIMELINE = 32  # per-block start/end stamps only
CAST_AO_TRACE = 128  # AO: trace every AO ray instead of the per-face voxel plan (A/B reference)
CAST_TILE_8X8 = 256  # scheduling: one wavefront per 8x8 tile (default: 16x4 pixels of its 8-pixel tile row)
CAST_TILE_32X2 = 512  # scheduling: one wavefront per 32x2 pixels of its 8-pixel tile row
CAST_WIDE_ADDR = 2048  # 64-bit node addresses even for trees below 2^28 nodes (results identical)
CAST_SEGMENTS = 4096  # force the kernel instance with segment-exact crossings (results identical)
CAST_NO_OCTANT = 16384  # per-wave step-sign flags instead of the launch's compiled-in sign octant (results identical)
CAST_NO_CEILINGS = 32768  # walk the tree instead of crossing column-ceiling boxes (results identical)
CAST_NO_SCHEDULE = 65536  # keep the default dispatch order instead of the last frame's longest-first schedule (results identical)
SCHED_MIN_BLOCKS = 4096  # frames of more blocks are scheduled (SVO_SCHED_MIN_BLOCKS)
SCHED_PRIMARY, SCHED_AO, SCHED_SHADE = 0, 1, 2  # Tree.schedule kinds
SCHED_GROUP = 4  # the schedule orders groups of this many consecutive blocks (SVO_SCHED_GROUP)
STAT_NAMES = ("rays", "lookups", "node_loads", "skips", "skip_budget_out", "brick_steps", "plain_steps", "lane_work",
              "wave_max_work_x64", "skips_4", "skips_16", "skips_64", "skips_256plus", "bricks",
              "wave_iters", "wave_brick_steps",
              "no_progress", "root_starts", "cache_empty", "wave_skips", "wave_descents",
              "path_starts", "ao_node_loads", "ceil_moves", "iters_above_top", "bends", "tints", "tint_iters")  # wave_*: per wave (64 rays)
STATS_HEADER = 32  # u64 counters before the per-block stamps (SVO_STATS_HEADER)
MAX_FRAMES = 16  # SVO_MAX_FRAMES: frames in one launch
WIRE_BYTES = 12  # SVO_WIRE_BYTES: the larger wire record (12 B general, 8 B compact: Tree.wire_bytes(desc))
CEIL_K0 = 2  # SVO_CEIL_K0 of include/svo_rt.h (the finest column-ceiling blocks are 4^k0 columns wide); the loaded library's: ceiling_layout()
VIEW_SOLID, VIEW_ALL = 0, 1  # SVO_VIEW_*: castRayFromCam's blocks / every stored block (the shading scene)


class SvoError(RuntimeError):
    pass


class Block(C.Structure):
    """Block (src/globals.hpp:76-80)."""

    _fields_ = [("flags", C.c_uint32), ("color", C.c_uint64), ("metadata", C.c_float)]

    def astuple(self):
        return (self.flags, self.color, self.metadata)

    def __repr__(self):
        return "Block(flags=%#x, color=%#x, metadata=%g)" % self.astuple()


class RayResult(C.Structure):
    """RayResult (src/ray_caster.hpp:6-10)."""

    _fields_ = [("pos", C.c_int32 * 3), ("last_pos", C.c_int32 * 3), ("steps", C.c_int32)]


class TreeInfo(C.Structure):
    _fields_ = [
        ("levels", C.c_int32),
        ("n_materials", C.c_uint32),
        ("n_nodes", C.c_uint64),
        ("n_mat_bytes", C.c_uint64),
        ("n_bricks", C.c_uint64),
        ("nodes_per_level", C.c_uint64 * 8),
        ("device_bytes", C.c_uint64),
        ("device", C.c_int32),
        ("view", C.c_int32),
    ]


class CastDesc(C.Structure):
    _fields_ = [
        ("origin", C.c_float * 3),
        ("cam_dir", C.c_float * 3),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("ppx", C.c_float),
        ("ppy", C.c_float),
        ("tile_row_start", C.c_int32),
        ("tile_row_step", C.c_int32),
        ("ray_dirs", C.c_void_p),
        ("ray_origins", C.c_void_p),
        ("n_rays", C.c_int32),
        ("steps", C.c_int32),
        ("flags", C.c_int32),
        ("ao_samples", C.c_int32),
        ("ao_steps", C.c_int32),
        ("stats", C.c_void_p),
        ("n_frames", C.c_int32),
        ("frame_origins", C.c_void_p),
    ]


class Hits(C.Structure):
    _fields_ = [("pos_steps", C.c_void_p), ("t", C.c_void_p), ("info", C.c_void_p), ("ao", C.c_void_p)]


class ShadeDesc(C.Structure):
    _fields_ = [("sun_dir", C.c_float * 3), ("look_at", C.c_int32 * 3), ("look_at_valid", C.c_int32), ("shadow_steps", C.c_int32),
                ("scene", C.c_void_p), ("time", C.c_float), ("look_at_dev", C.c_void_p)]


# globals.cpp:23: sun = normalize(vec3(2, 1, 4))
SUN_DIR = None  # filled lazily by sun_dir() (svo_normalize, bit-identical to the device)


_lib = None

# every symbol include/svo_rt.h declares (tests check the library exports all of them)
ABI_SYMBOLS = (
    "svo_last_error", "svo_version", "svo_world_create", "svo_world_destroy", "svo_init_tetra_hexa_tree",
    "svo_put_block", "svo_get_block", "svo_delete_block", "svo_gen_world", "svo_world_node_count", "svo_build",
    "svo_build_terrain", "svo_tree_get_info", "svo_tree_palette", "svo_tree_get_block", "svo_tree_export",
    "svo_upload", "svo_tree_destroy", "svo_cast_count", "svo_cast_blocks", "svo_cast_rays", "svo_cast_ray_from_cam", "svo_sync",
    "svo_proj_plane", "svo_normalize", "svo_pixel_dir", "svo_pixel_dirs", "svo_get_blocks", "svo_put_blocks",
    "svo_tree_get_blocks", "svo_noise2", "svo_terrain_heights", "svo_hemisphere", "svo_gen_heightfield",
    "svo_build_heightfield", "svo_shade_rays", "svo_tree_update", "svo_tree_sync",
    "svo_build_terrain_gpu", "svo_build_heightfield_gpu", "svo_hits_pack", "svo_hits_unpack", "svo_tree_node_indices",
    "svo_nccl_unique_id", "svo_exchange_create", "svo_exchange_wrap", "svo_exchange_destroy", "svo_exchange_info",
    "svo_exchange_frames", "svo_build_view", "svo_build_terrain_view", "svo_build_terrain_gpu_view",
    "svo_tree_save", "svo_tree_load", "svo_wire_bytes", "svo_cast_wire", "svo_wire_scatter", "svo_exchange_wire", "svo_tree_ceilings",
    "svo_tree_guard_trips", "svo_ceiling_layout", "svo_tree_device_ceilings", "svo_tree_device_ceiling_quads", "svo_tree_schedule", "svo_cast_ray_from_cam_async",
    "svo_build_id",
)


_lib_sha = None


def lib_sha256():
    """sha256 of the libsvo_rt.so this process loads (LIB_PATH): the build a measurement belongs to (bench.py puts it on
    its line; tools/pmc_summary.py records it with the PMC counters, and bench.py uses committed counters only when
    they were measured on the same build)."""
    global _lib_sha
    if _lib_sha is None:
        import hashlib

        with open(LIB_PATH, "rb") as f:
            _lib_sha = hashlib.sha256(f.read()).hexdigest()
    return _lib_sha


def build_id():
    """The sources_sha256 stamped into the loaded library (svo_build_id; None for a build that predates the stamp)"""
    L = lib()
    if not hasattr(L, "svo_build_id"):
        return None
    L.svo_build_id.restype = C.c_char_p
    return L.svo_build_id().decode()


def ceiling_layout():
    """(k0, pair_step) of the loaded library (svo_ceiling_layout): the finest column-ceiling blocks are 4^k0 columns wide,
    and the pair table pairs level j with level j + pair_step"""
    k0, st = C.c_int32(), C.c_int32()
    _check(lib().svo_ceiling_layout(C.byref(k0), C.byref(st)), "svo_ceiling_layout")
    return k0.value, st.value


def lib():
    """Load libsvo_rt.so (raises if it has not been built: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libsvo_rt.so not built: run `python -m raytracing_test_amd.build` (or __graft_entry__.build())")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 / libhsa-runtime64.so.1.  If
    # torch is importable it must be loaded first, so that libsvo_rt.so binds to that runtime instead
    # of pulling /opt/rocm's copy next to it (two runtimes on one KFD: "no ROCm-capable device").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, i32, f32 = C.c_void_p, C.c_int32, C.c_float
    f3 = C.POINTER(C.c_float)
    L.svo_last_error.restype = C.c_char_p
    L.svo_world_create.argtypes = [i32, C.POINTER(vp)]
    L.svo_world_destroy.argtypes = [vp]
    L.svo_world_destroy.restype = None
    L.svo_init_tetra_hexa_tree.argtypes = [vp]
    L.svo_put_block.argtypes = [vp, i32, i32, i32, C.POINTER(Block), i32]
    L.svo_get_block.argtypes = [vp, i32, i32, i32, C.POINTER(Block)]
    L.svo_delete_block.argtypes = [vp, i32, i32, i32, i32, C.POINTER(Block)]
    L.svo_gen_world.argtypes = [vp, i32, i32]
    L.svo_world_node_count.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.svo_build.argtypes = [vp, C.POINTER(vp)]
    # (entry points newer than SVO_RT_VERSION 3 are bound only when present, so that A/B timing against
    # library builds of earlier revisions (tools/build_variant.py) loads them through this module)
    for name, at in (("svo_build_view", [vp, i32, C.POINTER(vp)]), ("svo_build_terrain_view", [i32, i32, i32, i32, i32, C.POINTER(vp)]),
                     ("svo_build_terrain_gpu_view", [i32, i32, i32, i32, i32, C.POINTER(vp)]),
                     ("svo_tree_save", [vp, C.c_char_p]), ("svo_tree_load", [C.c_char_p, C.POINTER(vp)]),
                     ("svo_wire_bytes", [vp, C.POINTER(CastDesc), C.POINTER(i32)]), ("svo_cast_wire", [vp, C.POINTER(CastDesc), vp, vp, vp]),
                     ("svo_wire_scatter", [vp, C.POINTER(CastDesc), vp, vp, C.POINTER(Hits), vp]),
                     ("svo_exchange_wire", [vp, vp, C.POINTER(CastDesc), vp, vp, C.POINTER(Hits), vp]),
                     ("svo_tree_ceilings", [vp, vp, C.c_int64, C.POINTER(i32), C.POINTER(C.c_int64)]),
                     ("svo_tree_guard_trips", [vp, C.POINTER(C.c_uint64), i32]),
                     ("svo_tree_device_ceilings", [vp, vp, vp, C.c_int64, C.POINTER(i32), C.POINTER(C.c_int64)]),
                     ("svo_tree_device_ceiling_quads", [vp, vp, C.c_int64, C.POINTER(C.c_int64)]),
                     ("svo_tree_schedule", [vp, vp, C.c_int32, vp, vp, C.c_int64, C.POINTER(C.c_int64)]),
                     ("svo_cast_ray_from_cam_async", [vp, f3, f3, i32, vp, vp])):
        if hasattr(L, name):
            getattr(L, name).argtypes = at
    L.svo_build_terrain.argtypes = [i32, i32, i32, i32, C.POINTER(vp)]
    L.svo_tree_get_info.argtypes = [vp, C.POINTER(TreeInfo)]
    L.svo_tree_palette.argtypes = [vp, C.c_uint32, C.POINTER(Block)]
    L.svo_tree_get_block.argtypes = [vp, i32, i32, i32, C.POINTER(Block), C.POINTER(C.c_uint32)]
    L.svo_tree_export.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64]
    L.svo_upload.argtypes = [vp, i32]
    L.svo_tree_update.argtypes = [vp, vp, vp, C.c_int64, i32]
    L.svo_tree_sync.argtypes = [vp]
    L.svo_tree_destroy.argtypes = [vp]
    L.svo_tree_destroy.restype = None
    L.svo_cast_count.argtypes = [C.POINTER(CastDesc), C.POINTER(C.c_int64)]
    L.svo_cast_blocks.argtypes = [C.POINTER(CastDesc), C.POINTER(C.c_int64)]
    L.svo_hits_pack.argtypes = [vp, C.POINTER(CastDesc), C.POINTER(Hits), vp, vp]
    L.svo_hits_unpack.argtypes = [vp, C.POINTER(CastDesc), vp, C.POINTER(Hits), vp]
    L.svo_cast_rays.argtypes = [vp, C.POINTER(CastDesc), C.POINTER(Hits), vp]
    L.svo_shade_rays.argtypes = [vp, C.POINTER(CastDesc), C.POINTER(ShadeDesc), vp, C.POINTER(Hits), vp]
    L.svo_cast_ray_from_cam.argtypes = [vp, f3, f3, i32, C.POINTER(RayResult), C.POINTER(Block)]
    L.svo_sync.argtypes = [vp]
    L.svo_proj_plane.argtypes = [i32, i32, C.POINTER(f32), C.POINTER(f32)]
    L.svo_normalize.argtypes = [f3, f3]
    L.svo_pixel_dir.argtypes = [f3, f32, f32, i32, i32, i32, i32, f3]
    L.svo_pixel_dirs.argtypes = [f3, f32, f32, i32, i32, vp]
    L.svo_get_blocks.argtypes = [vp, vp, C.c_int64, vp]
    L.svo_put_blocks.argtypes = [vp, vp, vp, C.c_int64, i32]
    L.svo_tree_get_blocks.argtypes = [vp, vp, C.c_int64, vp]
    L.svo_tree_node_indices.argtypes = [vp, vp, C.c_int64, vp]
    L.svo_noise2.argtypes = [C.c_int64, vp, vp, C.c_int64, vp]
    L.svo_terrain_heights.argtypes = [i32, i32, i32, vp]
    L.svo_hemisphere.argtypes = [i32, vp]
    L.svo_gen_heightfield.argtypes = [vp, i32, i32, vp]
    L.svo_build_heightfield.argtypes = [i32, i32, i32, vp, i32, C.POINTER(vp)]
    L.svo_build_terrain_gpu.argtypes = [i32, i32, i32, i32, C.POINTER(vp)]
    L.svo_build_heightfield_gpu.argtypes = [i32, i32, i32, vp, i32, C.POINTER(vp)]
    L.svo_nccl_unique_id.argtypes = [vp]
    L.svo_exchange_create.argtypes = [i32, i32, vp, i32, C.POINTER(vp)]
    L.svo_exchange_wrap.argtypes = [vp, i32, C.POINTER(vp)]
    L.svo_exchange_destroy.argtypes = [vp]
    L.svo_exchange_destroy.restype = None
    L.svo_exchange_info.argtypes = [vp, C.POINTER(i32), C.POINTER(i32)]
    L.svo_exchange_frames.argtypes = [vp, vp, C.POINTER(CastDesc), C.POINTER(Hits), C.POINTER(Hits), vp]
    _lib = L
    return L


def _check(rc, what):
    if rc != SVO_OK:
        msg = lib().svo_last_error()
        raise SvoError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))


def _f3(v):
    a = (C.c_float * 3)(*[float(x) for x in v])
    return a


def proj_plane(width, height):
    """projPlaneSize uniform of src/main.cpp:94."""
    a, b = C.c_float(), C.c_float()
    _check(lib().svo_proj_plane(width, height, C.byref(a), C.byref(b)), "svo_proj_plane")
    return a.value, b.value


def normalize(v):
    """glm::normalize in float (the camera direction of src/main.cpp:195)."""
    o = (C.c_float * 3)()
    _check(lib().svo_normalize(_f3(v), o), "svo_normalize")
    return np.array(list(o), np.float32)


def pixel_dir(cam_dir, ppx, ppy, width, height, px, py):
    o = (C.c_float * 3)()
    _check(lib().svo_pixel_dir(_f3(cam_dir), ppx, ppy, width, height, px, py, o), "svo_pixel_dir")
    return np.array(list(o), np.float32)


def pixel_dirs(cam_dir, width, height, ppx=None, ppy=None):
    """Every pixel's primary-ray direction, shape (height, width, 3), rows from the bottom."""
    if ppx is None:
        ppx, ppy = proj_plane(width, height)
    out = np.zeros((height, width, 3), np.float32)
    _check(lib().svo_pixel_dirs(_f3(cam_dir), ppx, ppy, width, height, out.ctypes.data_as(C.c_void_p)), "svo_pixel_dirs")
    return out


def hemisphere(n):
    """gen_hemisphare_distrib.py's sample table for n points, (n, 3) float32 as (x, y, pole)"""
    out = np.zeros((n, 3), np.float32)
    _check(lib().svo_hemisphere(n, out.ctypes.data_as(C.c_void_p)), "svo_hemisphere")
    return out


def noise2(seed, x, y):
    """OpenSimplex 2D (include/OpenSimplexNoise.cpp:77-208) at arrays of points."""
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    out = np.zeros(len(x), np.float64)
    _check(lib().svo_noise2(int(seed), x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p), len(x),
                            out.ctypes.data_as(C.c_void_p)), "svo_noise2")
    return out


def terrain_heights(width, length, nthreads=0):
    """genWorld's column tops (world_gen.cpp:22), shape (width, length)."""
    out = np.zeros((width, length), np.int32)
    _check(lib().svo_terrain_heights(width, length, nthreads, out.ctypes.data_as(C.c_void_p)), "svo_terrain_heights")
    return out


def _xyz(points):
    return np.ascontiguousarray(np.asarray(points, dtype=np.int32).reshape(-1, 3))


class World:
    """Host-side editable 64-ary voxel tree (the reference's global `root` + pools)."""

    def __init__(self, levels=5):
        self.levels = levels
        h = C.c_void_p()
        _check(lib().svo_world_create(levels, C.byref(h)), "svo_world_create")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.svo_world_destroy(self._h)
            self._h = None

    @classmethod
    def reference(cls, width=200, length=200):
        """initTetraHexaTree() + genWorld(): the reference application's world (1024^3)."""
        w = cls(5)
        w.init_tetra_hexa_tree()
        w.gen_world(width, length)
        return w

    def init_tetra_hexa_tree(self):
        _check(lib().svo_init_tetra_hexa_tree(self._h), "svo_init_tetra_hexa_tree")

    def put_block(self, x, y, z, flags, color, metadata=0.0, level=None):
        b = Block(flags, color, metadata)
        lv = self.levels + 1 if level is None else level
        _check(lib().svo_put_block(self._h, x, y, z, C.byref(b), lv), "svo_put_block")

    def get_block(self, x, y, z):
        b = Block()
        _check(lib().svo_get_block(self._h, x, y, z, C.byref(b)), "svo_get_block")
        return b.astuple()

    def delete_block(self, x, y, z, level=None):
        b = Block()
        lv = self.levels + 1 if level is None else level
        _check(lib().svo_delete_block(self._h, x, y, z, lv, C.byref(b)), "svo_delete_block")
        return b.astuple()

    def get_blocks(self, points):
        """Batched getBlock: returns (flags u32, color u64, metadata f32) arrays."""
        p = _xyz(points)
        out = (Block * len(p))()
        _check(lib().svo_get_blocks(self._h, p.ctypes.data_as(C.c_void_p), len(p), C.cast(out, C.c_void_p)), "svo_get_blocks")
        a = np.frombuffer(out, dtype=np.dtype([("flags", "<u4"), ("pad", "<u4"), ("color", "<u8"), ("metadata", "<f4"), ("pad2", "<u4")]))
        return a["flags"].copy(), a["color"].copy(), a["metadata"].copy()

    def put_blocks(self, points, flags, colors, metadata=None, level=None):
        p = _xyz(points)
        n = len(p)
        arr = (Block * n)()
        a = np.frombuffer(arr, dtype=np.dtype([("flags", "<u4"), ("pad", "<u4"), ("color", "<u8"), ("metadata", "<f4"), ("pad2", "<u4")]))
        a["flags"] = flags
        a["color"] = colors
        a["metadata"] = 0.0 if metadata is None else metadata
        lv = self.levels + 1 if level is None else level
        _check(lib().svo_put_blocks(self._h, p.ctypes.data_as(C.c_void_p), C.cast(arr, C.c_void_p), n, lv), "svo_put_blocks")

    def gen_world(self, width=200, length=200):
        _check(lib().svo_gen_world(self._h, width, length), "svo_gen_world")

    def gen_heightfield(self, heights):
        """genWorld's column puts from given column tops, heights shape (width, length)"""
        h = np.ascontiguousarray(heights, np.int32)
        _check(lib().svo_gen_heightfield(self._h, h.shape[0], h.shape[1], h.ctypes.data_as(C.c_void_p)), "svo_gen_heightfield")

    def node_count(self):
        n = C.c_uint64()
        _check(lib().svo_world_node_count(self._h, C.byref(n)), "svo_world_node_count")
        return n.value

    def build(self, view=VIEW_SOLID):
        """the linearised tree of this world: VIEW_SOLID for casts, VIEW_ALL (liquid stored) as a shading scene"""
        h = C.c_void_p()
        if view == VIEW_SOLID:
            _check(lib().svo_build(self._h, C.byref(h)), "svo_build")
        else:
            _check(lib().svo_build_view(self._h, view, C.byref(h)), "svo_build_view")
        return Tree(h)


def _torch():
    import torch  # plumbing only: device buffers and streams

    return torch


class Tree:
    """Breadth-first linearised tree: host image + HBM copy after upload()."""

    def __init__(self, handle):
        self._h = handle
        self._scratch = {}

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.svo_tree_destroy(self._h)
            self._h = None

    @classmethod
    def terrain(cls, levels, width, length, nthreads=0, view=VIEW_SOLID):
        """genWorld's column formula over width x length columns, built without per-voxel putBlock."""
        h = C.c_void_p()
        if view == VIEW_SOLID:
            _check(lib().svo_build_terrain(levels, width, length, nthreads, C.byref(h)), "svo_build_terrain")
        else:
            _check(lib().svo_build_terrain_view(levels, width, length, nthreads, view, C.byref(h)), "svo_build_terrain_view")
        return cls(h)

    @classmethod
    def heightfield(cls, levels, heights, nthreads=0):
        """the terrain builder on given column tops, heights shape (width, length)"""
        h = np.ascontiguousarray(heights, np.int32)
        t = C.c_void_p()
        _check(lib().svo_build_heightfield(levels, h.shape[0], h.shape[1], h.ctypes.data_as(C.c_void_p), nthreads, C.byref(t)),
               "svo_build_heightfield")
        return cls(t)

    @classmethod
    def terrain_gpu(cls, levels, width, length, device=0, view=VIEW_SOLID):
        """svo_build_terrain on the GPU (noise + build in HBM): the tree comes back uploaded to `device`."""
        h = C.c_void_p()
        if view == VIEW_SOLID:
            _check(lib().svo_build_terrain_gpu(levels, width, length, device, C.byref(h)), "svo_build_terrain_gpu")
        else:
            _check(lib().svo_build_terrain_gpu_view(levels, width, length, device, view, C.byref(h)), "svo_build_terrain_gpu_view")
        return cls(h)

    @classmethod
    def heightfield_gpu(cls, levels, heights, device=0):
        h = np.ascontiguousarray(heights, np.int32)
        t = C.c_void_p()
        _check(lib().svo_build_heightfield_gpu(levels, h.shape[0], h.shape[1], h.ctypes.data_as(C.c_void_p), device, C.byref(t)),
               "svo_build_heightfield_gpu")
        return cls(t)

    def save(self, path):
        """checkpoint the linearised tree to a file (svo_tree_save)"""
        _check(lib().svo_tree_save(self._h, os.fsencode(path)), "svo_tree_save")

    @classmethod
    def load(cls, path):
        """a tree read back from svo_tree_save's file (validated; not uploaded)"""
        h = C.c_void_p()
        _check(lib().svo_tree_load(os.fsencode(path), C.byref(h)), "svo_tree_load")
        return cls(h)

    def info(self):
        i = TreeInfo()
        _check(lib().svo_tree_get_info(self._h, C.byref(i)), "svo_tree_get_info")
        return i

    def palette(self):
        out = []
        for k in range(self.info().n_materials):
            b = Block()
            _check(lib().svo_tree_palette(self._h, k, C.byref(b)), "svo_tree_palette")
            out.append(b.astuple())
        return out

    def get_block(self, x, y, z):
        b, m = Block(), C.c_uint32()
        _check(lib().svo_tree_get_block(self._h, x, y, z, C.byref(b), C.byref(m)), "svo_tree_get_block")
        return b.astuple(), m.value

    def get_blocks(self, points):
        """Batched lookup in the linearised tree: palette ids (0 = empty, LIQUID counts as empty)."""
        p = _xyz(points)
        ids = np.zeros(len(p), np.uint32)
        _check(lib().svo_tree_get_blocks(self._h, p.ctypes.data_as(C.c_void_p), len(p), ids.ctypes.data_as(C.c_void_p)),
               "svo_tree_get_blocks")
        return ids

    def node_indices(self, points):
        """Index of the deepest node a lookup of each voxel reads (diagnostics: svo_tree_node_indices)."""
        p = _xyz(points)
        out = np.zeros(len(p), np.uint64)
        _check(lib().svo_tree_node_indices(self._h, p.ctypes.data_as(C.c_void_p), len(p), out.ctypes.data_as(C.c_void_p)),
               "svo_tree_node_indices")
        return out

    def update(self, world, points, level=None):
        """Incremental edits: patch this tree after world.put_block / delete_block at `level` on
        `points` (svo_tree_update); then sync() to update the device copy."""
        p = _xyz(points)
        lv = self.info().levels + 1 if level is None else level
        _check(lib().svo_tree_update(self._h, world._h, p.ctypes.data_as(C.c_void_p), len(p), lv), "svo_tree_update")
        return self

    def sync(self):
        """Upload what update() changed (svo_tree_sync)."""
        _check(lib().svo_tree_sync(self._h), "svo_tree_sync")
        return self

    def export(self):
        i = self.info()
        nodes = np.zeros(i.n_nodes * 2, np.uint64)
        mats = np.zeros(max(1, i.n_mat_bytes // 2), np.uint16)
        _check(lib().svo_tree_export(self._h, nodes.ctypes.data_as(C.c_void_p), nodes.nbytes,
                                     mats.ctypes.data_as(C.c_void_p), mats.nbytes), "svo_tree_export")
        return nodes.reshape(-1, 2), mats[: i.n_mat_bytes // 2]

    def upload(self, device=0):
        _check(lib().svo_upload(self._h, device), "svo_upload")
        return self

    # ------------------------------------------------------------------------------ casting --
    @staticmethod
    def frame_desc(origin, cam_dir, width, height, steps, ppx=None, ppy=None, tile_row_start=0, tile_row_step=1, flags=0,
                   ao_samples=0, ao_steps=5, frame_origins=None):
        """frame_origins: several frames (camera positions) in one launch; records of frame f
        follow those of frame f-1 (origin is then ignored)"""
        if ppx is None:
            ppx, ppy = proj_plane(width, height)
        d = CastDesc()
        if frame_origins is not None and len(frame_origins) > 0:
            fo = np.ascontiguousarray(np.asarray(frame_origins, np.float32).reshape(-1, 3))
            d._frame_origins = fo  # keep the host array alive with the desc
            d.n_frames = len(fo)
            d.frame_origins = fo.ctypes.data
            origin = fo[0]
        d.origin[:] = [float(x) for x in origin]
        d.cam_dir[:] = [float(x) for x in cam_dir]
        d.width, d.height, d.ppx, d.ppy = width, height, ppx, ppy
        d.tile_row_start, d.tile_row_step = tile_row_start, tile_row_step
        d.steps = steps
        d.flags = flags
        d.ao_samples = ao_samples
        d.ao_steps = ao_steps
        return d

    @staticmethod
    def count(desc):
        n = C.c_int64()
        _check(lib().svo_cast_count(C.byref(desc), C.byref(n)), "svo_cast_count")
        return n.value

    @staticmethod
    def blocks(desc):
        """blocks (64-lane wavefronts) a cast of desc launches: the stats buffer holds 2 stamps each"""
        n = C.c_int64()
        _check(lib().svo_cast_blocks(C.byref(desc), C.byref(n)), "svo_cast_blocks")
        return n.value

    @staticmethod
    def alloc_hits(n, device, ao=False):
        torch = _torch()
        dev = torch.device("cuda", device)
        out = dict(
            pos_steps=torch.empty((n, 4), dtype=torch.int32, device=dev),
            t=torch.empty(n, dtype=torch.float32, device=dev),
            info=torch.empty(n, dtype=torch.int32, device=dev),
        )
        if ao:
            out["ao"] = torch.empty(n, dtype=torch.uint8, device=dev)
        return out

    def ceilings(self):
        """the column ceilings (svo_tree_ceilings): a list of (E / 4^k) x (E / 4^k) int16 arrays [z][x], k = CEIL_K0, CEIL_K0 + 1, ..."""
        lv, n = C.c_int32(), C.c_int64()
        _check(lib().svo_tree_ceilings(self._h, None, 0, C.byref(lv), C.byref(n)), "svo_tree_ceilings")
        out = np.zeros(n.value, np.int16)
        _check(lib().svo_tree_ceilings(self._h, out.ctypes.data_as(C.c_void_p), n.value, C.byref(lv), C.byref(n)), "svo_tree_ceilings")
        E = 1 << (2 * self.info().levels)
        k0 = ceiling_layout()[0]  # the finest level's blocks are 4^SVO_CEIL_K0 columns wide
        assert sum((E >> (2 * (k0 + j))) ** 2 for j in range(lv.value)) == n.value
        self.ceil_k0 = k0
        res, off = [], 0
        for j in range(lv.value):
            rows = E >> (2 * (k0 + j))
            res.append(out[off:off + rows * rows].reshape(rows, rows))
            off += rows * rows
        return res

    def wire_bytes(self, desc):
        """bytes per wire record of desc's records: 8 (compact: frames from integral / half-integral camera
        positions) or 12 (include/svo_rt.h)"""
        b = C.c_int32()
        _check(lib().svo_wire_bytes(self._h, C.byref(desc), C.byref(b)), "svo_wire_bytes")
        return b.value

    def cast_wire(self, desc, wire, ao=None, stream=None):
        """svo_cast_wire: cast desc's rays straight into wire records (uint8 device tensor of count x
        wire_bytes), AO counts into `ao` (uint8 device tensor) when desc.ao_samples > 0"""
        s = getattr(stream, "cuda_stream", stream)
        _check(lib().svo_cast_wire(self._h, C.byref(desc), C.c_void_p(wire.data_ptr()), C.c_void_p(ao.data_ptr()) if ao is not None else None,
                                   C.c_void_p(s) if s else None), "svo_cast_wire")

    def wire_scatter(self, desc, wire, frames, ao=None, stream=None):
        """svo_wire_scatter: the shard desc's wire records into whole frames (desc.n_frames x W x H records,
        pixel order); only the shard's pixels are written"""
        s = getattr(stream, "cuda_stream", stream)
        _check(lib().svo_wire_scatter(self._h, C.byref(desc), C.c_void_p(wire.data_ptr()), C.c_void_p(ao.data_ptr()) if ao is not None else None,
                                      C.byref(_hits(frames)), C.c_void_p(s) if s else None), "svo_wire_scatter")

    def pack_hits(self, desc, out, wire, stream=None):
        """hit records (device) -> the wire records of include/svo_rt.h in `wire` (uint8 tensor, wire_bytes(desc) per record)"""
        h = Hits(out["pos_steps"].data_ptr(), out["t"].data_ptr(), out["info"].data_ptr(), None)
        s = getattr(stream, "cuda_stream", stream)
        _check(lib().svo_hits_pack(self._h, C.byref(desc), C.byref(h), C.c_void_p(wire.data_ptr()), C.c_void_p(s) if s else None),
               "svo_hits_pack")

    def unpack_hits(self, desc, wire, out, stream=None):
        """wire records -> hit records (device), record order"""
        h = Hits(out["pos_steps"].data_ptr(), out["t"].data_ptr(), out["info"].data_ptr(), None)
        s = getattr(stream, "cuda_stream", stream)
        _check(lib().svo_hits_unpack(self._h, C.byref(desc), C.c_void_p(wire.data_ptr()), C.byref(h), C.c_void_p(s) if s else None),
               "svo_hits_unpack")

    def cast(self, desc, out, stream=None):
        """Launch the cast kernel asynchronously on `stream` (a torch.cuda.Stream or raw handle)."""
        ao = out.get("ao")
        h = Hits(out["pos_steps"].data_ptr(), out["t"].data_ptr(), out["info"].data_ptr(), ao.data_ptr() if ao is not None else None)
        s = getattr(stream, "cuda_stream", stream)
        _check(lib().svo_cast_rays(self._h, C.byref(desc), C.byref(h), C.c_void_p(s) if s else None), "svo_cast_rays")

    def cast_frame(self, origin, cam_dir, width, height, steps, ppx=None, ppy=None, tile_row_start=0, tile_row_step=1,
                   out=None, stream=None, sync=True, flags=0, ao_samples=0, ao_steps=5):
        d = self.frame_desc(origin, cam_dir, width, height, steps, ppx, ppy, tile_row_start, tile_row_step, flags, ao_samples,
                            ao_steps)
        n = self.count(d)
        if out is None:
            out = self.alloc_hits(n, self.info().device, ao=ao_samples > 0)
        self.cast(d, out, stream)
        if sync:
            _check(lib().svo_sync(C.c_void_p(getattr(stream, "cuda_stream", stream)) if stream else None), "svo_sync")
        return out

    def cast_stats(self, origin, cam_dir, width, height, steps, flags=0):
        """Traversal counters of one frame (SVO_CAST_STATS), per ray: {STAT_NAMES[k]: value}."""
        torch = _torch()
        d = self.frame_desc(origin, cam_dir, width, height, steps, None, None, 0, 1, flags | CAST_STATS, 0, 5)
        n = self.count(d)
        dev = self.info().device
        st = torch.zeros(STATS_HEADER + 2 * self.blocks(d) + n, dtype=torch.int64, device=torch.device("cuda", dev))
        d.stats = st.data_ptr()
        out = self.alloc_hits(n, dev)
        self.cast(d, out)
        _check(lib().svo_sync(None), "svo_sync")
        v = st[:len(STAT_NAMES)].cpu().numpy().astype(np.float64)
        return {k: v[i] / max(1.0, v[0]) for i, k in enumerate(STAT_NAMES)}

    def device_ceilings(self):
        """(levels, int16 ceilings, uint32 pairs) of the tables in HBM (svo_tree_device_ceilings)"""
        lv, n = C.c_int32(), C.c_int64()
        _check(lib().svo_tree_device_ceilings(self._h, None, None, 0, C.byref(lv), C.byref(n)), "svo_tree_device_ceilings")
        c = np.zeros(n.value, np.int16)
        p = np.zeros(n.value, np.uint32)
        _check(lib().svo_tree_device_ceilings(self._h, c.ctypes.data_as(C.c_void_p), p.ctypes.data_as(C.c_void_p), n.value, C.byref(lv),
                                              C.byref(n)), "svo_tree_device_ceilings")
        return lv.value, c, p

    def device_ceiling_quads(self):
        """uint64 quads of the finest ceiling blocks in HBM: the ceilings of levels 0..3 holding each (svo_tree_device_ceiling_quads)"""
        n = C.c_int64()
        _check(lib().svo_tree_device_ceiling_quads(self._h, None, 0, C.byref(n)), "svo_tree_device_ceiling_quads")
        q = np.zeros(n.value, np.uint64)
        _check(lib().svo_tree_device_ceiling_quads(self._h, q.ctypes.data_as(C.c_void_p), n.value, C.byref(n)),
               "svo_tree_device_ceiling_quads")
        return q

    def schedule(self, kind=0, stream=None):
        """(order, cost) of the frame schedule of (stream, kind: SCHED_PRIMARY / SCHED_AO / SCHED_SHADE) (svo_tree_schedule):
        the next frame's dispatch order of groups of SCHED_GROUP blocks (slot group -> frame group) and the last frame's
        block durations (100 MHz ticks);
        (None, None) before a scheduled frame"""
        s = getattr(stream, "cuda_stream", stream)
        n = C.c_int64()
        _check(lib().svo_tree_schedule(self._h, C.c_void_p(s) if s else None, kind, None, None, 0, C.byref(n)), "svo_tree_schedule")
        if n.value == 0:
            return None, None
        o, c = np.zeros(n.value // SCHED_GROUP, np.uint32), np.zeros(n.value, np.uint32)
        _check(lib().svo_tree_schedule(self._h, C.c_void_p(s) if s else None, kind, o.ctypes.data_as(C.c_void_p), c.ctypes.data_as(C.c_void_p),
                                       n.value, C.byref(n)), "svo_tree_schedule")
        return o, c

    def guard_trips(self, reset=False):
        """Rays of launches over this tree that ended on the progress guard (svo_tree_guard_trips): 0 unless a
        crossing count is wrong; such rays carry stepsLeft -1."""
        v = C.c_uint64()
        _check(lib().svo_tree_guard_trips(self._h, C.byref(v), 1 if reset else 0), "svo_tree_guard_trips")
        return v.value

    def shade_stats(self, origin, cam_dir, width, height, steps, scene=None, flags=0, shadow_steps=75, ray_work=False):
        """Traversal counters of one shaded frame (SVO_CAST_STATS in the shading pass; the shadow rays' work is not
        counted), per pixel: {STAT_NAMES[k]: value}; with ray_work, also the per-pixel packed work words (int64)."""
        torch = _torch()
        d = self.frame_desc(origin, cam_dir, width, height, steps, None, None, 0, 1, flags | CAST_STATS, 0, 5)
        n = self.count(d)
        dev = self.info().device
        st = torch.zeros(STATS_HEADER + 2 * self.blocks(d) + n, dtype=torch.int64, device=torch.device("cuda", dev))
        d.stats = st.data_ptr()
        rgba = torch.empty((n, 4), dtype=torch.float32, device=torch.device("cuda", dev))
        self.shade(d, rgba, shadow_steps=shadow_steps, scene=scene)
        _check(lib().svo_sync(None), "svo_sync")
        v = st[:len(STAT_NAMES)].cpu().numpy().astype(np.float64)
        res = {k: v[i] / max(1.0, v[0]) for i, k in enumerate(STAT_NAMES)}
        if ray_work:
            res["ray_work"] = st[STATS_HEADER + 2 * self.blocks(d):].cpu().numpy()
        return res

    def cast_rays(self, dirs, origins=None, steps=300, origin=(0.0, 0.0, 0.0), out=None, stream=None, sync=True, flags=0):
        """Explicit rays: dirs / origins are (n, 3) float32 device tensors."""
        d = CastDesc()
        d.origin[:] = [float(x) for x in origin]
        d.ray_dirs = dirs.data_ptr()
        d.ray_origins = origins.data_ptr() if origins is not None else None
        d.n_rays = dirs.shape[0]
        d.steps = steps
        d.flags = flags
        if out is None:
            out = self.alloc_hits(d.n_rays, self.info().device)
        self.cast(d, out, stream)
        if sync:
            _check(lib().svo_sync(C.c_void_p(getattr(stream, "cuda_stream", stream)) if stream else None), "svo_sync")
        return out

    def shade(self, desc, rgba, sun=None, look_at=None, shadow_steps=75, out=None, stream=None, scene=None, time=0.0):
        """Launch the shading pass (svo_shade_rays) for `desc`: rgba is a (n, 4) float32 device tensor.
        scene: a VIEW_ALL Tree of the same world (liquid refracts and tints); time: the wobble's deltaTime.
        look_at: a voxel (x, y, z), or a device int32 tensor holding a svo_ray_result (cast_ray_from_cam_async
        on the same stream) whose pos the kernel reads."""
        sd = ShadeDesc()
        sd.scene = scene._h if scene is not None else None
        sd.time = time
        sd.sun_dir[:] = [float(x) for x in (sun if sun is not None else sun_dir())]
        if look_at is not None and hasattr(look_at, "data_ptr"):
            sd.look_at_dev = look_at.data_ptr()
        elif look_at is not None:
            sd.look_at[:] = [int(x) for x in look_at]
            sd.look_at_valid = 1
        sd.shadow_steps = shadow_steps
        h = None
        if out is not None:
            h = Hits(out["pos_steps"].data_ptr(), out["t"].data_ptr(), out["info"].data_ptr(), None)
        s = getattr(stream, "cuda_stream", stream)
        _check(lib().svo_shade_rays(self._h, C.byref(desc), C.byref(sd), C.c_void_p(rgba.data_ptr()), C.byref(h) if h else None,
                                    C.c_void_p(s) if s else None), "svo_shade_rays")

    def shade_frame(self, origin, cam_dir, width, height, steps=300, sun=None, look_at=None, shadow_steps=75, ppx=None, ppy=None,
                    tile_row_start=0, tile_row_step=1, with_hits=False, stream=None, sync=True, flags=0, scene=None, time=0.0):
        """One shaded frame: (n, 4) float32 rgba in hit-record order (and the hit records with with_hits)."""
        torch = _torch()
        d = self.frame_desc(origin, cam_dir, width, height, steps, ppx, ppy, tile_row_start, tile_row_step, flags, 0, 5)
        n = self.count(d)
        dev = self.info().device
        rgba = torch.empty((n, 4), dtype=torch.float32, device=torch.device("cuda", dev))
        out = self.alloc_hits(n, dev) if with_hits else None
        self.shade(d, rgba, sun, look_at, shadow_steps, out, stream, scene=scene, time=time)
        if sync:
            _check(lib().svo_sync(C.c_void_p(getattr(stream, "cuda_stream", stream)) if stream else None), "svo_sync")
        return (rgba, out) if with_hits else rgba

    def cast_ray_from_cam_async(self, pos, cam_dir, steps, out, stream=None):
        """svo_cast_ray_from_cam_async: the pick ray's RayResult (pos, last_pos, steps) written to `out` (an int32 device
        tensor of >= 7 elements, 16-byte aligned) on `stream`, without a host round trip."""
        s = getattr(stream, "cuda_stream", stream)
        _check(lib().svo_cast_ray_from_cam_async(self._h, _f3(pos), _f3(cam_dir), steps, C.c_void_p(out.data_ptr()),
                                                 C.c_void_p(s) if s else None), "svo_cast_ray_from_cam_async")

    def cast_ray_from_cam(self, pos, cam_dir, steps):
        """RAY_CASTER::castRayFromCam(steps) with the camera passed in: (RayResult, Block)."""
        r, b = RayResult(), Block()
        _check(lib().svo_cast_ray_from_cam(self._h, _f3(pos), _f3(cam_dir), steps, C.byref(r), C.byref(b)),
               "svo_cast_ray_from_cam")
        return (tuple(r.pos), tuple(r.last_pos), r.steps), b.astuple()


def _hits(out):
    if out is None:
        return None
    ao = out.get("ao")
    return Hits(out["pos_steps"].data_ptr(), out["t"].data_ptr(), out["info"].data_ptr(), ao.data_ptr() if ao is not None else None)


NCCL_UNIQUE_ID_BYTES = 128


class Exchange:
    """Multi-GPU frame exchange over RCCL (svo_exchange_*): every frame's tile-row shards gathered to
    the rank that displays it (frame f -> rank f % nranks)."""

    @staticmethod
    def unique_id():
        b = (C.c_uint8 * NCCL_UNIQUE_ID_BYTES)()
        _check(lib().svo_nccl_unique_id(b), "svo_nccl_unique_id")
        return bytes(b)

    def __init__(self, nranks, rank, uid, device):
        h = C.c_void_p()
        buf = (C.c_uint8 * NCCL_UNIQUE_ID_BYTES).from_buffer_copy(bytes(uid))
        _check(lib().svo_exchange_create(nranks, rank, buf, device, C.byref(h)), "svo_exchange_create")
        self._h = h
        self.rank, self.nranks = rank, nranks

    def __del__(self):
        self.close()

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.svo_exchange_destroy(self._h)
            self._h = None

    def info(self):
        """(rank, nranks) of the exchange's RCCL communicator (svo_exchange_info)."""
        r, n = C.c_int32(), C.c_int32()
        _check(lib().svo_exchange_info(self._h, C.byref(r), C.byref(n)), "svo_exchange_info")
        return r.value, n.value

    def frames(self, tree, desc, mine, frames_out, stream=None):
        """One step's exchange of `mine` (this rank's shard of desc's frames) into frames_out (the
        whole frames this rank displays), asynchronous on `stream`."""
        s = getattr(stream, "cuda_stream", stream)
        fo = _hits(frames_out)
        _check(lib().svo_exchange_frames(self._h, tree._h, C.byref(desc), C.byref(_hits(mine)), C.byref(fo) if fo else None,
                                         C.c_void_p(s) if s else None), "svo_exchange_frames")

    def wire(self, tree, desc, wire, frames_out, ao=None, stream=None):
        """One step's exchange from wire records this rank cast itself (Tree.cast_wire of desc into `wire`):
        svo_exchange_wire, asynchronous on `stream`."""
        s = getattr(stream, "cuda_stream", stream)
        fo = _hits(frames_out)
        _check(lib().svo_exchange_wire(self._h, tree._h, C.byref(desc), C.c_void_p(wire.data_ptr()),
                                       C.c_void_p(ao.data_ptr()) if ao is not None else None, C.byref(fo) if fo else None,
                                       C.c_void_p(s) if s else None), "svo_exchange_wire")


def sun_dir():
    """The reference's sun direction, normalize(2, 1, 4) (globals.cpp:23), as the library computes it."""
    global SUN_DIR
    if SUN_DIR is None:
        SUN_DIR = tuple(normalize((2.0, 1.0, 4.0)))
    return SUN_DIR


def decode_hits(out):
    """Device hit buffers -> numpy dict (pos, last_pos, steps, hit, axis, material, t)."""
    ps = out["pos_steps"].cpu().numpy()
    info = out["info"].cpu().numpy().view(np.uint32)
    t = out["t"].cpu().numpy()
    axis = (info >> AXIS_SHIFT) & 3
    neg = (info & NEG_BIT) != 0
    pos = ps[:, :3].copy()
    last = pos.copy()
    for a in range(3):
        sel = axis == a
        last[sel, a] -= np.where(neg[sel], -1, 1)
    res = dict(pos=pos, last_pos=last, steps=ps[:, 3].copy(), hit=(info & HIT_BIT) != 0, axis=axis.astype(np.int32),
               material=(info & MAT_MASK).astype(np.int32), t=t)
    if out.get("ao") is not None:
        res["ao"] = out["ao"].cpu().numpy()
    return res
