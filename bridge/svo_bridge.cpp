// svo_bridge.cpp — drop-in shim: the reference's free functions over libsvo_rt's C ABI, so that
// reedthorngag/raytracing_test's main.cpp / input.cpp link unchanged with src/ray_caster.cpp,
// src/voxel_data/tetrahexa_tree.cpp, src/voxel_data/voxel_allocator.cpp and src/world_gen.cpp removed
// from build.bat.  State is global, as in the reference (the global `root`,
// tetrahexa_tree.hpp:10; the camera globals, globals.hpp:63-64); errors end the program as the
// reference's own exit(1) paths do (tetrahexa_tree.cpp:154-155).
#include "svo_bridge.hpp"

#include <stdio.h>
#include <stdlib.h>

namespace {
svo_world* g_world = nullptr;
svo_tree* g_tree = nullptr;   // solid view: castRayFromCam, primary frames, shadow rays
svo_tree* g_scene = nullptr;  // full view (water stored): what the shaded frame's rays walk (low_res.frag)
bool g_rebuild = true;  // the world changed without a tree to patch (genWorld, edits before the first upload)
svo_ray_result* g_look = nullptr;  // device record of the frame's lookingAtBlock pick ray (svoRenderShaded)
int g_device = 0;  // the GPU the trees live on (initVoxelDataAllocator: SVO_DEVICE, default 0)

void check(int rc, const char* what) {
    if (rc) {
        fprintf(stderr, "svo_bridge: %s failed (%d): %s\n", what, rc, svo_last_error());
        exit(1);
    }
}

// putBlock / deleteBlock mark the edited region; the linear tree is patched in place (svo_tree_update)
// and the next updateSsboData uploads what changed, as the reference's modified-block flags do
// (voxel_allocator.hpp:38-78)
void edited(const Pos& p, int level) {
    if (!g_tree) {
        g_rebuild = true;
        return;
    }
    const int32_t xyz[3] = {p.x, p.y, p.z};
    check(svo_tree_update(g_tree, g_world, xyz, 1, level), "svo_tree_update");
    check(svo_tree_update(g_scene, g_world, xyz, 1, level), "svo_tree_update");
}

void drop_trees() {
    if (g_tree) svo_tree_destroy(g_tree);
    if (g_scene) svo_tree_destroy(g_scene);
    g_tree = g_scene = nullptr;
}

void camera(float o[3], float d[3]) {
    o[0] = cameraPos.x;
    o[1] = cameraPos.y;
    o[2] = cameraPos.z;
    d[0] = cameraDir.x;
    d[1] = cameraDir.y;
    d[2] = cameraDir.z;
}
}  // namespace

// tetrahexa_tree.cpp:13-41 (maxDepth 6 = 5 levels, tetrahexa_tree.hpp:6)
void initTetraHexaTree() {
    drop_trees();
    if (g_world) svo_world_destroy(g_world);
    check(svo_world_create(maxDepth - 1, &g_world), "svo_world_create");
    check(svo_init_tetra_hexa_tree(g_world), "svo_init_tetra_hexa_tree");
    g_rebuild = true;
}

// world_gen.cpp:13-42 (200 x 200 columns)
void genWorld() {
    check(svo_gen_world(g_world, 200, 200), "svo_gen_world");
    drop_trees();
    g_rebuild = true;
}

// tetrahexa_tree.cpp:176-291
void putBlock(Pos pos, Block block, int targetDepth) {
    const svo_block b{block.flags, block.color, block.metadata};
    check(svo_put_block(g_world, pos.x, pos.y, pos.z, &b, targetDepth), "svo_put_block");
    edited(pos, targetDepth);
}

// tetrahexa_tree.cpp:113-157
Block getBlock(Pos pos) {
    svo_block b;
    check(svo_get_block(g_world, pos.x, pos.y, pos.z, &b), "svo_get_block");
    return Block{b.flags, b.color, b.metadata};
}

// tetrahexa_tree.cpp:293-359.  The reference removes the node at depth `level` (5: a voxel, 4: a 4^3
// block — one level finer than putBlock's meaning); its only caller's level 6 (input.cpp:146) removes
// the voxel as well (a split into 64 copies, of which getBlock reads the dropped one).  Its bitmap
// update `1 << index` (:352) is an int shift that flips the wrong bits for child slots >= 31; the
// intended clear is done here (tests/test_edits.py pins both).
Block deleteBlock(Pos pos, int level) {
    const int lv = level >= maxDepth ? maxDepth : level + 1;  // svo_delete_block takes putBlock's level
    svo_block b;
    check(svo_delete_block(g_world, pos.x, pos.y, pos.z, lv, &b), "svo_delete_block");
    edited(pos, lv);
    return Block{b.flags, b.color, b.metadata};
}

// tetrahexa_tree.cpp:43-111 (declared, its call commented out at :37): a batched getBlock
void traverseTree(Pos* pos, int count) {
    for (int i = 0; i < count; i++) (void)getBlock(pos[i]);
}

// voxel_allocator.hpp:80-91, called once after initTetraHexaTree (main.cpp:183).  The reference creates its two
// SSBOs here (bindings 2 and 3); the GPU side of the shim is the device the trees will live on: SVO_DEVICE
// (default 0), checked to exist.  Nothing is uploaded yet: the world is empty until genWorld, and the first
// updateSsboData (main.cpp:212) builds and uploads it
void initVoxelDataAllocator() {
    const char* e = getenv("SVO_DEVICE");
    const int dev = e && *e ? atoi(e) : 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || dev < 0 || dev >= n) {
        fprintf(stderr, "svo_bridge: initVoxelDataAllocator: device %d not available (%d visible)\n", dev, n);
        exit(1);
    }
    if (dev != g_device) {
        if (g_tree) g_rebuild = true;  // (a re-init onto another device re-uploads)
        if (g_look) {  // the look-at record lives on the old device: freed there, allocated again on the new one
            check(hipSetDevice(g_device) == hipSuccess ? 0 : SVO_EDEVICE, "hipSetDevice");
            check(hipFree(g_look) == hipSuccess ? 0 : SVO_EDEVICE, "hipFree (look-at record)");
            g_look = nullptr;
        }
    }
    check(hipSetDevice(dev) == hipSuccess ? 0 : SVO_EDEVICE, "hipSetDevice");
    g_device = dev;
}

// voxel_allocator.hpp:38-78, called every frame (main.cpp:212): the first call (and any call after
// genWorld) builds and uploads the tree; later calls upload only what edits changed
void updateSsboData() {
    if (g_rebuild || !g_tree) {
        drop_trees();
        check(svo_build(g_world, &g_tree), "svo_build");
        check(svo_upload(g_tree, g_device), "svo_upload");
        check(svo_build_view(g_world, SVO_VIEW_ALL, &g_scene), "svo_build_view");
        check(svo_upload(g_scene, g_device), "svo_upload");
        g_rebuild = false;
        return;
    }
    check(svo_tree_sync(g_tree), "svo_tree_sync");
    check(svo_tree_sync(g_scene), "svo_tree_sync");
}

svo_tree* svoTree() { return g_tree; }
svo_tree* svoScene() { return g_scene; }

namespace RAY_CASTER {
// ray_caster.cpp:54-87 on the GPU (one ray, synchronous)
RayResult castRayFromCam(int steps) {
    if (!g_tree) updateSsboData();
    float o[3], d[3];
    camera(o, d);
    svo_ray_result r;
    check(svo_cast_ray_from_cam(g_tree, o, d, steps, &r, nullptr), "svo_cast_ray_from_cam");
    return RayResult{SVO_BRIDGE_IVEC3(r.pos[0], r.pos[1], r.pos[2]), SVO_BRIDGE_IVEC3(r.last_pos[0], r.last_pos[1], r.last_pos[2]), r.steps};
}
}  // namespace RAY_CASTER

static svo_cast_desc frame_desc(int32_t width, int32_t height, int32_t steps) {
    svo_cast_desc d{};
    camera(d.origin, d.cam_dir);
    d.width = width;
    d.height = height;
    d.tile_row_start = 0;
    d.tile_row_step = 1;
    d.steps = steps;
    check(svo_proj_plane(width, height, &d.ppx, &d.ppy), "svo_proj_plane");  // main.cpp:94
    return d;
}

void svoCastPrimaryRays(int32_t width, int32_t height, int32_t steps, int32_t* pos_steps, float* t, uint32_t* info, hipStream_t stream) {
    if (!g_tree) updateSsboData();
    const svo_cast_desc d = frame_desc(width, height, steps);
    const svo_hits h{pos_steps, t, info, nullptr};
    check(svo_cast_rays(g_tree, &d, &h, stream), "svo_cast_rays");
}

void svoRenderShaded(int32_t width, int32_t height, float* rgba, hipStream_t stream, float time) {
    if (!g_tree) updateSsboData();
    const svo_cast_desc d = frame_desc(width, height, 300);  // low_res.frag:310
    // main.cpp:81, castRayFromCam(30) for the lookingAtBlock uniform (:89), cast on the frame's stream into a
    // device record the shading kernel reads: the frame loop never waits for the host
    if (!g_look) check(hipMalloc(reinterpret_cast<void**>(&g_look), 256) == hipSuccess ? 0 : SVO_ENOMEM, "hipMalloc (look-at record)");
    float o[3], dir[3];
    camera(o, dir);
    check(svo_cast_ray_from_cam_async(g_tree, o, dir, 30, g_look, stream), "svo_cast_ray_from_cam_async");
    svo_shade_desc sd{};
    sd.sun_dir[0] = sun.x;
    sd.sun_dir[1] = sun.y;
    sd.sun_dir[2] = sun.z;
    sd.look_at_dev = g_look;
    sd.shadow_steps = 75;  // low_res.frag:382
    sd.scene = g_scene;    // water refracts and tints (low_res.frag:214-229)
    sd.time = time;        // the deltaTime uniform
    check(svo_shade_rays(g_tree, &d, &sd, rgba, nullptr, stream), "svo_shade_rays");
}
