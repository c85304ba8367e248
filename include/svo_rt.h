/*
 * svo_rt.h — C ABI of the MI355X-native sparse-voxel-tree primary raycaster (libsvo_rt.so).
 *
 * Drop-in boundary for reedthorngag/raytracing_test's hot path (paths relative to the reference):
 *   - src/ray_caster.hpp:6-14          RayResult / RAY_CASTER::castRayFromCam(int steps)
 *   - src/voxel_data/tetrahexa_tree.hpp:12-22  initTetraHexaTree / putBlock / getBlock / deleteBlock
 *   - src/world_gen.hpp:3              genWorld()
 *   - src/voxel_data/voxel_allocator.hpp:38-91  updateSsboData / initVoxelDataAllocator (device upload)
 *   - src/shaders/low_res.frag:256-333,446-531  the per-pixel DDA + tree traversal, replaced by
 *                                      svo_cast_rays() (a hand-written gfx950 HIP kernel)
 *
 * Conventions: every function returns an int status (SVO_OK = 0, negative on error) and never
 * exits; svo_last_error() gives the message of the calling thread's last failure.  Pointers marked
 * "device" are HBM pointers on the tree's device (e.g. a torch tensor's data_ptr()); a hip_stream
 * argument is a hipStream_t (NULL = the null stream).  The tree is read-only during a cast.
 */
#ifndef SVO_RT_H
#define SVO_RT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SVO_RT_VERSION 7  /* 2: svo_cast_desc.n_frames / frame_origins, wire records; 3: svo_exchange_*, 64-bit node addressing;
                             4: tree views (liquid stored for the shading pass), svo_shade_desc.scene / time;
                             6: svo_tree_save / svo_tree_load (5, a cost-ordered dispatch, was measured slower
                             and removed); 7: 8-B compact wire records, svo_wire_bytes / svo_cast_wire /
                             svo_wire_scatter / svo_exchange_wire */

enum {
    SVO_OK = 0,
    SVO_EINVAL = -1,  /* bad argument */
    SVO_ENOMEM = -2,  /* host or device allocation failed */
    SVO_EDEVICE = -3, /* HIP runtime error / no GPU */
    SVO_ESTATE = -4,  /* object not in the required state (e.g. tree not uploaded) */
    SVO_ERANGE = -5,  /* value outside what the structure supports */
    SVO_EIO = -6      /* file I/O failed, or the file is not a valid tree (svo_tree_load) */
};

/* Block (src/globals.hpp:76-80): leaf flags (bit 0 set for a stored voxel; REFLECTIVE 0x2,
   REFRACTIVE 0x4, LUMINESCENT 0x8, LIQUID 0x10), 3 x 21-bit packed colour (src/types.hpp:6-9),
   metadata.  The empty block is {0, ~0ull, 0}. */
typedef struct {
    uint32_t flags;
    uint64_t color;
    float metadata;
} svo_block;

/* RayResult (src/ray_caster.hpp:6-10) */
typedef struct {
    int32_t pos[3];
    int32_t last_pos[3];
    int32_t steps;
} svo_ray_result;

typedef struct svo_world svo_world; /* host-side editable 64-ary voxel tree */
typedef struct svo_tree svo_tree;   /* breadth-first linearised tree (host image + HBM copy) */

const char* svo_last_error(void);
int svo_version(void);
/* sha256 of the sources, headers and compile flags this library was built from (raytracing_test_amd/build.py
   sources_sha256; 64 hex digits): ties a measurement to the committed files */
const char* svo_build_id(void);

/* ---------------------------------------------------------------- world (host, editable) ---- */
/* levels = descending tree levels; extent = 4^levels voxels per axis (reference: 5 -> 1024^3,
   maxDepth 6 at src/voxel_data/tetrahexa_tree.hpp:6).  1 <= levels <= 7. */
int svo_world_create(int32_t levels, svo_world** out);
void svo_world_destroy(svo_world* w);
/* initTetraHexaTree (tetrahexa_tree.cpp:13-41): root + the reference's 8 debug blocks.  The
   reference's aliased root child array is NOT reproduced: the block at
   (1000,1000,1000) exists here, while the reference cannot reach it. */
int svo_init_tetra_hexa_tree(svo_world* w);
/* putBlock (tetrahexa_tree.cpp:176-291): level levels+1 = one voxel (reference: 6), levels = a
   4^3 block (reference: 5), ... 1 = the whole world.  Stored flags = 1 | b.flags. */
int svo_put_block(svo_world* w, int32_t x, int32_t y, int32_t z, const svo_block* b, int32_t level);
/* getBlock (tetrahexa_tree.cpp:113-157); coordinates wrap modulo the extent */
int svo_get_block(const svo_world* w, int32_t x, int32_t y, int32_t z, svo_block* out);
/* deleteBlock (tetrahexa_tree.cpp:293-359) with its intended meaning: clears the level-`level`
   region containing (x,y,z) (level as putBlock's) and returns the block found there. */
int svo_delete_block(svo_world* w, int32_t x, int32_t y, int32_t z, int32_t level, svo_block* removed);
/* genWorld (world_gen.cpp:13-42) over width x length columns (reference: 200 x 200) */
int svo_gen_world(svo_world* w, int32_t width, int32_t length);
/* genWorld's column puts (world_gen.cpp:24-39) from caller-given tops heights[x*length + z] */
int svo_gen_heightfield(svo_world* w, int32_t width, int32_t length, const int32_t* heights);
/* number of putBlock-visible tree nodes (diagnostics) */
int svo_world_node_count(const svo_world* w, uint64_t* nodes);
/* batched getBlock over n positions (xyz = 3 x int32 each) — the traverseTree batch lookup of
   tetrahexa_tree.cpp:43-111, made usable */
int svo_get_blocks(const svo_world* w, const int32_t* xyz, int64_t n, svo_block* out);
/* batched putBlock of n blocks, all at `level`, applied in order */
int svo_put_blocks(svo_world* w, const int32_t* xyz, const svo_block* blocks, int64_t n, int32_t level);
/* OpenSimplex 2D (include/OpenSimplexNoise.cpp:77-208) for n points, and genWorld's column tops
   (world_gen.cpp:22) for x in [0,width), z in [0,length): out[x*length + z] */
int svo_noise2(int64_t seed, const double* x, const double* y, int64_t n, double* out);
int svo_terrain_heights(int32_t width, int32_t length, int32_t nthreads, int32_t* out);

/* ------------------------------------------------------------ tree (BFS, HBM-resident) ------ */
typedef struct {
    int32_t levels;
    uint32_t n_materials;         /* palette entries including id 0 (empty) */
    uint64_t n_nodes;             /* 16 B nodes */
    uint64_t n_mat_bytes;         /* per-voxel material bytes of mixed-material bricks */
    uint64_t n_bricks;            /* 4^3 brick nodes */
    uint64_t nodes_per_level[8];  /* nodes at depth 0..levels-1 */
    uint64_t device_bytes;        /* HBM footprint after svo_upload (0 before) */
    int32_t device;               /* -1 before svo_upload */
    int32_t view;                 /* SVO_VIEW_SOLID / SVO_VIEW_ALL */
} svo_tree_info;

/* Tree views.  SVO_VIEW_SOLID (every cast): the blocks castRayFromCam hits (ray_caster.cpp:82) —
   empty and LIQUID blocks are empty.  SVO_VIEW_ALL (the scene of the shading pass,
   svo_shade_desc.scene): every stored block, liquid included, as low_res.frag's getBlock sees it. */
#define SVO_VIEW_SOLID 0
#define SVO_VIEW_ALL 1

/* Linearise a world: collapse uniform regions, drop non-solid (empty / LIQUID) voxels, emit the
   breadth-first node array + material bytes + palette. */
int svo_build(const svo_world* w, svo_tree** out);
/* the same for a view (svo_build = SVO_VIEW_SOLID); edits (svo_tree_update) keep the tree's view */
int svo_build_view(const svo_world* w, int32_t view, svo_tree** out);
/* Build the same tree straight from genWorld's column formula over width x length columns
   (no per-voxel putBlock: depth-12 / depth-14 terrain); nthreads host threads (0 = all). */
int svo_build_terrain(int32_t levels, int32_t width, int32_t length, int32_t nthreads, svo_tree** out);
int svo_build_terrain_view(int32_t levels, int32_t width, int32_t length, int32_t nthreads, int32_t view, svo_tree** out);
/* the same builder from caller-given column tops heights[x*length + z] (0 <= h <= extent-2) */
int svo_build_heightfield(int32_t levels, int32_t width, int32_t length, const int32_t* heights, int32_t nthreads,
                          svo_tree** out);
/* The same two builders on the GPU: noise per column, min/max pyramid and a
   level-synchronous breadth-first build in HBM (one wavefront per region, ballots + scans).  The
   node / material arrays equal svo_build_terrain's byte for byte; the tree comes back already
   uploaded to `device` (plus its host image). */
int svo_build_terrain_gpu(int32_t levels, int32_t width, int32_t length, int32_t device, svo_tree** out);
int svo_build_terrain_gpu_view(int32_t levels, int32_t width, int32_t length, int32_t device, int32_t view, svo_tree** out);
int svo_build_heightfield_gpu(int32_t levels, int32_t width, int32_t length, const int32_t* heights, int32_t device, svo_tree** out);
int svo_tree_get_info(const svo_tree* t, svo_tree_info* out);
/* palette entry `id` (id 0 = empty block) */
int svo_tree_palette(const svo_tree* t, uint32_t id, svo_block* out);
/* host-side lookup in the linearised tree; returns the solid-view block (empty for LIQUID) */
int svo_tree_get_block(const svo_tree* t, int32_t x, int32_t y, int32_t z, svo_block* out, uint32_t* material_id);
/* batched host lookup: palette ids (0 = empty) of n positions */
int svo_tree_get_blocks(const svo_tree* t, const int32_t* xyz, int64_t n, uint32_t* material_ids);
/* diagnostics: index of the deepest node a lookup of each voxel reads (the brick / SOLID node holding
   it, or the interior node whose child slot for it is empty) */
int svo_tree_node_indices(const svo_tree* t, const int32_t* xyz, int64_t n, uint64_t* node_index);
/* copy the host image out (for tests / serialisation); byte sizes from svo_tree_get_info */
int svo_tree_export(const svo_tree* t, void* nodes, uint64_t nodes_bytes, void* mats, uint64_t mats_bytes);
/* updateSsboData analogue: (re)upload the image to HBM of `device` (with room for edit blocks) */
int svo_upload(svo_tree* t, int32_t device);
/* Incremental edits: after putBlock / deleteBlock at `level` on the n positions
   xyz of `w` (the world `t` was built from), patch `t` in place: each edited region's subtree is
   re-linearised from `w` and its parent's child block rewritten at the end of the array (only
   that parent's 16-B record changes in place).  The content equals a fresh svo_build of `w`; the
   layout is not re-collapsed, and the tree is rebuilt from `w` when superseded blocks exceed half
   of it.  Host only; svo_tree_sync brings the device copy up to date. */
int svo_tree_update(svo_tree* t, const svo_world* w, const int32_t* xyz, int64_t n, int32_t level);
/* upload what svo_tree_update changed: the appended tail and the rewritten records (or everything
   after a rebuild / when the device allocation is outgrown).  Synchronises the device first (device
   memory is rewritten in place): call it between frames, as updateSsboData is (main.cpp:212). */
int svo_tree_sync(svo_tree* t);
void svo_tree_destroy(svo_tree* t);
/* The column ceilings the casts use (SVO_CAST_NO_CEILINGS): for k = SVO_CEIL_K0 .. min(levels - 1, SVO_CEIL_K0 + 3)
   (blocks of 16, 64, 256 and 1024 columns), per aligned block of 4^k x 4^k columns, the highest stored voxel row of
   the tree in those columns (-1: none), row-major [z][x], level after level (finest first; level j's blocks are
   4^(SVO_CEIL_K0 + j) columns wide).  out may be NULL (count only); levels = number of levels, n = elements. */
#define SVO_CEIL_K0 2
int svo_tree_ceilings(const svo_tree* t, int16_t* out, int64_t cap, int32_t* levels, int64_t* n);
/* The pairs the casts read: level j's block ceiling with that of the level min(j + SVO_CEIL_PAIR_STEP, levels - 1)
   block holding it (primary casts and shadow rays check levels 0 and SVO_CEIL_PAIR_STEP of the table) */
#define SVO_CEIL_PAIR_STEP 1
/* the ceiling layout this library was built with: SVO_CEIL_K0 and SVO_CEIL_PAIR_STEP (either may be NULL) */
int svo_ceiling_layout(int32_t* k0, int32_t* pair_step);
/* The column-ceiling tables in HBM as the casts read them (inspection / tests): the int16 ceilings in
   svo_tree_ceilings' layout and their uint32 pairs (low: the block's ceiling, high: the ceiling of the level
   j + SVO_CEIL_PAIR_STEP block holding it, the coarsest level there is).  levels = 0 when the tree has none.
   Either buffer may be NULL. */
int svo_tree_device_ceilings(const svo_tree* t, int16_t* ceil, uint32_t* pairs, int64_t cap, int32_t* levels, int64_t* n);
/* The per-level quads in HBM (the shading pass's walk over every ceiling level): for every block of the finest
   level (4^SVO_CEIL_K0 columns, row-major [z][x]), the ceilings of the blocks of levels 0..3 holding it, int16 each,
   level j in bits 16j..16j+15 (a level the tree lacks: 0x7FFF).  quads may be NULL (count only); n = elements. */
int svo_tree_device_ceiling_quads(const svo_tree* t, uint64_t* quads, int64_t cap, int64_t* n);
/* The frame schedule of (hip_stream, kind: 2 shading; 0 / 1, primary and AO casts, keep none) over t (inspection /
   tests; SVO_CAST_NO_SCHEDULE): the dispatch order of the next frames of that geometry, by groups of SVO_SCHED_GROUP
   consecutive blocks (order[slot group] = frame group; n / SVO_SCHED_GROUP entries) and the block durations of the frame
   it was sorted from (100 MHz ticks, n entries); n = blocks (0: no schedule yet).  Either buffer may be NULL;
   synchronises hip_stream. */
int svo_tree_schedule(const svo_tree* t, void* hip_stream, int32_t kind, uint32_t* order, uint32_t* cost, int64_t cap, int64_t* n);
/* Checkpoint (the reference regenerates its world at every start, main.cpp:190): write the
   linearised tree (levels, view, palette, nodes, material runs; a checksum) to `path`, and read it back
   as a new tree (not uploaded).  Loading validates every child / material reference against the array
   sizes, so a damaged file fails with SVO_EIO instead of reaching a kernel. */
int svo_tree_save(const svo_tree* t, const char* path);
int svo_tree_load(const char* path, svo_tree** out);

/* ---------------------------------------------------------------------------- casting ------- */
/* Hit record per ray (caller-owned device buffers, 24 B / ray):
     pos_steps[4*i .. 4*i+3] = {x, y, z, stepsLeft}   (RayResult.pos / .steps)
     t[i]                    = deltaPos[axis] before its last increment (entry distance of pos)
     info[i]                 = bit 31 hit | bits 16-17 last axis (3 = no step) | bit 18 step < 0
                               on that axis | bits 0-15 material id (0 = none)
   RayResult.lastPos = pos - (axis step).  Frame rays: index = row * width + px, rows counted
   from the bottom (gl_FragCoord), restricted to the tile rows of this shard.
   Hemisphere AO (light_scattering.frag:133-236): for a hit, ao_samples rays
   start at the centre of lastPos, directions = svo_hemisphere's table with its pole (component 2)
   turned to the hit face's normal by a signed axis permutation (pole -> normal axis, components
   0/1 -> the next two axes cyclically), each cast with castRayFromCam semantics and ao_steps
   steps; ao[i] = number of them that hit. */
typedef struct {
    int32_t* pos_steps;
    float* t;
    uint32_t* info;
    uint8_t* ao;       /* per ray: AO rays that hit (0..ao_samples); required when ao_samples > 0 */
} svo_hits;

typedef struct {
    /* frame mode (ray_dirs == NULL): one primary ray per pixel, low_res.frag:264-288 */
    float origin[3];   /* cameraPos (also the origin of explicit rays when ray_origins == NULL) */
    float cam_dir[3];  /* normalised cameraDir */
    int32_t width, height;
    float ppx, ppy;    /* projPlaneSize uniform (main.cpp:94); see svo_proj_plane */
    int32_t tile_row_start, tile_row_step; /* shard: 8-pixel tile rows start, start+step, ... */
    /* explicit mode: n_rays rays, device float3 arrays */
    const float* ray_dirs;
    const float* ray_origins; /* optional */
    int32_t n_rays;
    int32_t steps;     /* DDA step budget per ray (castRayFromCam's `steps`) */
    int32_t flags;     /* SVO_CAST_* bits, 0 = default */
    int32_t ao_samples; /* hemisphere AO rays per primary hit (0 = off, <= 64; reference: 20) */
    int32_t ao_steps;   /* DDA budget of each AO ray (reference: 5, light_scattering.frag:231) */
    uint64_t* stats;   /* optional device u64[SVO_STATS_HEADER] accumulating per-launch counters when
                          flags & SVO_CAST_STATS: rays, lookups, node loads, cell skips,
                          skips that ran out of budget, brick voxel steps, plain voxel steps,
                          lane work units, wave-max work units x 64, crossings by box cell
                          size (4 slots), brick visits, wave-level loop iterations,
                          wave-level brick voxel steps, loop iterations that took no DDA
                          step and were ended by the progress guard (0 unless a count is wrong),
                          lookups started at
                          the root, lookups answered by the cached parent, wave-level
                          crossings, wave-level descent levels, lookups restarted from the
                          per-lane path, node loads of the AO plan's brick lookups;
                          then 2 stamps per block (svo_cast_blocks);
                          then, with SVO_CAST_STATS in frame mode, one word per
                          output pixel: lookups | brick steps << 32
                          (SVO_CAST_STATS or SVO_CAST_TIMELINE) */
    /* frame mode, several frames in one launch (the multi-GPU step: one launch per rank covers its
       tile rows of every frame): n_frames <= SVO_MAX_FRAMES (0 or 1: one frame at `origin`);
       frame_origins = host array of n_frames camera positions (origin is then ignored).  Records
       of frame f follow those of frame f-1: svo_cast_count / svo_cast_blocks count all frames. */
    int32_t n_frames;
    const float* frame_origins;
} svo_cast_desc;

#define SVO_MAX_FRAMES 16

/* svo_cast_desc.flags: take every DDA step one at a time (disables the exact closed-form crossing
   of empty regions; results are identical — for testing and A/B timing) */
#define SVO_CAST_ITERATIVE 1
/* svo_cast_desc.flags: accumulate traversal counters into svo_cast_desc.stats (diagnostics) */
#define SVO_CAST_STATS 2
/* svo_cast_desc.flags, scheduling (results identical): frames are dispatched top tile row first
   (longest rays first); this bit restores bottom-first order */
#define SVO_CAST_BOTTOM_FIRST 4
/* svo_cast_desc.flags: write per-block start/end stamps (100 MHz) to stats[SVO_STATS_HEADER + 2*block] only;
   stats must hold SVO_STATS_HEADER + 2 * svo_cast_blocks() [+ pixels with SVO_CAST_STATS] words */
#define SVO_STATS_HEADER 32
#define SVO_CAST_TIMELINE 32
/* (bits 16 and 1024 were round-2 dispatch experiments, XCD-contiguous bands and horizon-first row order:
   measured slower or equal, removed) */
/* svo_cast_desc.flags, AO (results identical): trace every AO ray through the tree instead of the
   per-face voxel plan (A/B reference path) */
#define SVO_CAST_AO_TRACE 128
/* svo_cast_desc.flags, scheduling (results identical): in frame mode each wavefront (one block)
   covers 16x4 pixels of its 8-pixel tile row; these bits select 8x8 or 32x2 instead.  A small launch (a
   strong-scaling shard: whole footprints would make fewer than 20480 wavefronts) casts its first-dispatched tile rows
   by half footprints, 32 pixels per wavefront; svo_cast_blocks counts those wavefronts too */
#define SVO_CAST_TILE_8X8 256
#define SVO_CAST_TILE_32X2 512
/* svo_cast_desc.flags (results identical): read nodes through 64-bit addresses even when the tree is
   small enough for 32-bit buffer offsets (trees of more than 2^28 nodes always use them) */
#define SVO_CAST_WIDE_ADDR 2048
/* svo_cast_desc.flags (results identical): the kernel instance picks itself by the origins — from
   integral or half-integral origins every ray's crossings are exact linear sums; other rays cross
   empty regions in exact segments.  SEGMENTS forces the segment-capable instance for any origin */
#define SVO_CAST_SEGMENTS 4096
/* svo_cast_desc.flags (results identical): frames whose rays all step with the same signs run an
   instance with those signs compiled in; this bit keeps the per-wave sign flags instead */
#define SVO_CAST_NO_OCTANT 16384
/* svo_cast_desc.flags (results identical): rays above the highest stored row of the column block they are in
   (primary casts: 16- and 64-column blocks; the shading pass: 64 and 256) cross the empty box above that row in
   one move, without a tree lookup (column ceilings, svo_tree_ceilings, computed at upload / sync); this bit walks
   the tree instead */
#define SVO_CAST_NO_CEILINGS 32768
/* svo_cast_desc.flags, scheduling (results identical): shaded frames (svo_shade_rays) of more than
   SVO_SCHED_MIN_BLOCKS blocks are dispatched longest block first, by the block durations a recent frame of the same
   geometry measured on the same stream (frame-to-frame coherence; a small sort kernel after every 4th frame orders the
   next ones, used while the camera stays within 0.5 deg / 1 voxel of the frame sorted); the first frame of a geometry
   runs in the default order.  This bit keeps the default order (and leaves the
   schedule untouched).  Primary casts always run in the default order (their longest waves are its first) */
#define SVO_CAST_NO_SCHEDULE 65536
#define SVO_SCHED_MIN_BLOCKS 4096
#define SVO_SCHED_GROUP 4 /* the schedule orders groups of this many consecutive blocks (frames of a multiple of it) */

/* number of rays a desc produces on this shard (= records written) */
int svo_cast_count(const svo_cast_desc* d, int64_t* n);
/* number of blocks (64-lane wavefronts) a cast of this desc launches */
int svo_cast_blocks(const svo_cast_desc* d, int64_t* n);
/* asynchronous on hip_stream */
int svo_cast_rays(const svo_tree* t, const svo_cast_desc* d, const svo_hits* out, void* hip_stream);
/* RAY_CASTER::castRayFromCam with explicit camera (synchronous, one ray on the GPU) */
int svo_cast_ray_from_cam(const svo_tree* t, const float pos[3], const float dir[3], int32_t steps, svo_ray_result* out,
                          svo_block* block);
/* Launches over t whose rays ended on the traversal's progress guard (an iteration that took no DDA step:
   only a wrong crossing count can cause it).  Such a ray's record has stepsLeft = -1 and no hit; the count
   should be 0 (shading launches count on t, the tree their shadow rays walk).  reset != 0 zeroes the counter.
   Synchronous: waits for the whole device (launches on any stream), then reads device memory. */
int svo_tree_guard_trips(const svo_tree* t, uint64_t* trips, int32_t reset);
/* the same pick ray, stream-ordered and without a host round trip: the result (svo_ray_result, 28 B) is
   written to d_result, device memory aligned to 16 bytes, on hip_stream (two small launches) — for the
   per-frame lookingAtBlock ray (main.cpp:81,89; svo_shade_desc.look_at_dev).  The block is not returned. */
int svo_cast_ray_from_cam_async(const svo_tree* t, const float pos[3], const float dir[3], int32_t steps, svo_ray_result* d_result,
                                void* hip_stream);
int svo_sync(void* hip_stream);

/* Wire formats of hit records for the exchange between GPUs (the tile-row gather):
   12 B (any desc)  int16 dx, dy, dz   pos - trunc(origin of the ray's frame, or of the explicit ray)
                    uint16 info16      hit << 15 | axis << 13 | (step < 0) << 12 | material id (12 bits)
                    float t
   8 B (compact)    u64: n_x | n_y << 15 | n_z << 30 | hit << 45 | axis << 46 | material id << 48, n_k = the DDA
                    steps the ray took on axis k.  Used for frame descs whose every camera position is integral
                    or half-integral: the receiver regenerates each pixel's ray and recovers the step signs,
                    the position, the steps left and t exactly (every crossing sum from such origins is exact).
   stepsLeft is not sent: every DDA step moves one axis by one voxel, so a hit leaves
   steps - |dx| - |dy| - |dz| and a miss 0.  Both need steps <= 32767 and at most 4096 palette entries
   (SVO_ERANGE otherwise).  svo_wire_bytes gives a desc's record size (8 or 12).  d describes the
   records (svo_cast_count of them, the frames / origins and tile rows they were cast from); wire and
   hits are device buffers; asynchronous. */
#define SVO_WIRE_BYTES 12 /* the larger of the two */
int svo_wire_bytes(const svo_tree* t, const svo_cast_desc* d, int32_t* bytes);
int svo_hits_pack(const svo_tree* t, const svo_cast_desc* d, const svo_hits* hits, void* wire, void* hip_stream);
int svo_hits_unpack(const svo_tree* t, const svo_cast_desc* d, const void* wire, const svo_hits* hits, void* hip_stream);
/* svo_cast_rays writing the wire record of each ray (svo_wire_bytes(d) bytes, record order) instead of its hit
   record — the cast and the pack in one pass; ao: the AO counts as svo_hits.ao (when d->ao_samples > 0) */
int svo_cast_wire(const svo_tree* t, const svo_cast_desc* d, void* wire, uint8_t* ao, void* hip_stream);
/* decode the wire records of the shard d describes (tile rows tile_row_start, +tile_row_step, ... of its
   n_frames frames) into whole frames: frames holds n_frames x width x height records in pixel order (the
   layout of an unsharded svo_cast_rays); only this shard's pixels are written.  ao: AO counts in record
   order (or NULL) */
int svo_wire_scatter(const svo_tree* t, const svo_cast_desc* d, const void* wire, const uint8_t* ao, const svo_hits* frames,
                     void* hip_stream);

/* ------------------------------------------------------------- multi-GPU frame exchange ----- */
/* frames sharded by interleaved 8-pixel tile rows (svo_cast_desc.tile_row_start = rank,
   tile_row_step = nranks), each frame's shards gathered over RCCL to the rank that displays it.  RCCL
   is bound at run time (librccl.so.1; the instance already in the process, e.g. torch's, if any). */
typedef struct svo_exchange svo_exchange;
#define SVO_NCCL_UNIQUE_ID_BYTES 128
/* ncclGetUniqueId: call on one rank and hand the bytes to every rank */
int svo_nccl_unique_id(void* out);
/* a communicator of nranks ranks (ncclCommInitRank; every rank calls it), this rank's GPU `device` */
int svo_exchange_create(int32_t nranks, int32_t rank, const void* unique_id, int32_t device, svo_exchange** out);
/* an exchange over a communicator the caller owns (an ncclComm_t of the same RCCL instance) */
int svo_exchange_wrap(void* nccl_comm, int32_t device, svo_exchange** out);
void svo_exchange_destroy(svo_exchange* x);
int svo_exchange_info(const svo_exchange* x, int32_t* rank, int32_t* nranks);
/* One step's exchange.  d: this rank's shard of n_frames frames (as cast into `mine`, records of frame f
   after those of frame f-1); frame f is displayed by rank f % nranks.  Packs `mine` into wire records
   (svo_hits_pack; AO counts alongside when d->ao_samples > 0), sends every frame's shard to its
   display rank and receives the shards of the frames this rank displays — one RCCL group of
   point-to-point transfers: a gather for one frame, an all-to-all for nranks frames — then unpacks them
   into frames_out: the whole frames (width x height records each, the layout of an unsharded
   svo_cast_rays) of frames rank, rank + nranks, ... in that order (unused on ranks that display none).
   This rank's own shards of its frames never travel.  Returns SVO_EINVAL when t lives on another device.
   Asynchronous on hip_stream; `mine` must not be overwritten before the stream passes this call. */
int svo_exchange_frames(svo_exchange* x, const svo_tree* t, const svo_cast_desc* d, const svo_hits* mine, const svo_hits* frames_out,
                        void* hip_stream);
/* the same exchange from wire records this rank cast itself (svo_cast_wire of d into `wire`, with `ao` when
   d->ao_samples > 0): no pack pass; the records of the frames this rank displays are decoded from `wire`
   in place (they never travel).  `wire` and `ao` must not be overwritten before the stream passes this call. */
int svo_exchange_wire(svo_exchange* x, const svo_tree* t, const svo_cast_desc* d, const void* wire, const uint8_t* ao,
                      const svo_hits* frames_out, void* hip_stream);

/* ---------------------------------------------------------------------------- shading ------- */
/* Shading pass: low_res.frag's colour model over castRayFromCam hits, one float4
   (r, g, b, 0) per ray in the order of the hit records:
     miss            -> genSkyBox (low_res.frag:157-168) of the final direction x finalColorMod
     hit             -> colour x calcLightIntensity (:242-252) x finalColorMod; unless reflected, 0.3 x
                        colour x finalColorMod when the face turns away from the sun or a shadow ray
                        (castRayFromCam semantics from the centre of lastPos towards sun_dir,
                        shadow_steps steps, liquid passes) hits (:361-391)
     look_at voxel   -> colour x 2 + 0.3 (:340-343)
   A block with flags & 7 == 3 reflects the ray while budget remains (:170-189, :319-331):
   the last crossing on the hit axis is undone, that axis's step and direction flip, the DDA
   continues; finalColorMod *= 0.94 per reflection.  A refractive block (flags & 7 == 5) while
   budget remains is passed with finalColorMod *= (0.94, 0.97, 1.0) for liquid, 0.95 otherwise
   (:214); the first one bends the ray (refractRay :196-240, n 1.0 -> 1.1, normal = hit axis x step,
   for liquid plus the shader's wobble sin((time + exact.x * 0.2 - exact.z * 0.1) * 10) * 0.2 on x
   and renormalised, :225-229; the shader's origin-based exact position) and deltaPos restarts from
   the current cell.  Liquid is seen only through a scene tree of SVO_VIEW_ALL (built from the same
   world or terrain as t); without one (scene == NULL) liquid passes unbent, as in castRayFromCam.
   Single precision in the shader's operation order; sin through double precision, rounded once. */
typedef struct {
    float sun_dir[3];      /* normalised sunDir (globals.cpp:23: normalize(2,1,4)) */
    int32_t look_at[3];    /* lookingAtBlock (main.cpp:81,89) */
    int32_t look_at_valid; /* 0: no highlight */
    int32_t shadow_steps;  /* 75 (low_res.frag:382) */
    const svo_tree* scene; /* SVO_VIEW_ALL tree the primary / reflected / refracted ray walks (NULL: t);
                              shadow rays walk t (liquid passes) */
    float time;            /* deltaTime uniform of the liquid wobble (low_res.frag:226) */
    const svo_ray_result* look_at_dev; /* device record (NULL: use look_at / look_at_valid): lookingAtBlock is its
                              pos, read by the kernel — e.g. written by svo_cast_ray_from_cam_async on the same
                              stream, so a frame needs no host round trip (main.cpp:81,89) */
} svo_shade_desc;

/* asynchronous on hip_stream; rgba: device float4 per ray; hits: optional hit records (may be NULL) */
int svo_shade_rays(const svo_tree* t, const svo_cast_desc* d, const svo_shade_desc* s, float* rgba, const svo_hits* hits,
                   void* hip_stream);

/* host helpers shared bit-for-bit with the device code */
int svo_proj_plane(int32_t width, int32_t height, float* ppx, float* ppy);
int svo_normalize(const float v[3], float out[3]);
int svo_pixel_dir(const float cam_dir[3], float ppx, float ppy, int32_t width, int32_t height, int32_t px, int32_t py,
                  float out[3]);
/* every pixel's direction, out[3 * (py * width + px) + a] */
int svo_pixel_dirs(const float cam_dir[3], float ppx, float ppy, int32_t width, int32_t height, float* out);
/* gen_hemisphare_distrib.py's table for n points (x, y, pole) as float: phi = acos(1-(i+.5)*.85/n),
   theta = pi*(1+sqrt 5)*(i+.5) */
int svo_hemisphere(int32_t n, float* out);

#ifdef __cplusplus
}
#endif
#endif /* SVO_RT_H */
