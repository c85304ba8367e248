// main_shape.cpp — a translation unit shaped like the reference's src/main.cpp, linked the way
// INTEGRATION.md tells a maintainer to link the real one: against the shim (bridge/svo_bridge.cpp) and
// libsvo_rt, with src/ray_caster.cpp, src/voxel_data/tetrahexa_tree.cpp, src/voxel_data/voxel_allocator.cpp
// and src/world_gen.cpp absent.  It includes the replacement header the maintainer copies over
// src/voxel_data/voxel_allocator.hpp — the very file, bridge/reference/voxel_data/voxel_allocator.hpp,
// found on the include path as main.cpp:12 names it — so the program links only if that header leaves
// updateSsboData / initVoxelDataAllocator to the shim (the original's inline GL bodies,
// voxel_allocator.hpp:38-91, read arrayBlocks / nodeBlocks, which are defined nowhere once
// voxel_allocator.cpp is gone).  tests/test_bridge_link.py checks with nm that both are undefined
// references of this object; tests/test_gpu_bridge.py runs it.
//
// The call sequence is main.cpp's: initTetraHexaTree (:182), initVoxelDataAllocator (:183), genWorld
// (:190), cameraDir = normalize(cameraDir) (:195), then per frame updateSsboData (:212) and render()
// (:214) — castRayFromCam(30) for lookingAtBlock (:81, :89) and the frame (:107; here svoRenderShaded /
// svoCastPrimaryRays) — and the mouse callbacks of input.cpp:141-159 between frames.  Writes one JSON
// object to argv[1].
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>

#include <vector>

#include "svo_bridge_types.hpp"            // globals.hpp / tetrahexa_tree.hpp / ray_caster.hpp / world_gen.hpp (main.cpp:7-13)
#include "voxel_data/voxel_allocator.hpp"  // main.cpp:12 -> the replacement header
#include "svo_bridge.hpp"                  // svoRenderShaded / svoCastPrimaryRays / svoTree (the draw's replacement)

vec3 cameraPos{35.0f, 50.0f, 35.0f};  // globals.cpp:20-21 position; direction chosen to look down at the terrain
vec3 cameraDir{1.0f, -1.0f, 1.0f};
vec3 sun;

// globals.cpp:36-62 hotbar[2]: REFLECTIVE, RGB_TO_U64(255,0,0) (types.hpp:8-9: 255 -> 2^21 - 1 in bits 42-62), 0.94
static const Block kHotbar2{0x2u, 2097151ull << 42, 0.94f};

static FILE* g_out;

static void print_ray(const char* key, const RayResult& r) {
    fprintf(g_out, "\"%s\": [%d, %d, %d, %d, %d, %d, %d],\n", key, r.pos.x, r.pos.y, r.pos.z, r.lastPos.x, r.lastPos.y, r.lastPos.z,
            r.steps);
}

// input.cpp:141-151 (left button released): delete what the pick ray hits
static void left_click() {
    const RayResult result = RAY_CASTER::castRayFromCam(30);
    if (result.steps) deleteBlock(Pos{result.pos.x, result.pos.y, result.pos.z}, 6);
}

// input.cpp:154-159 (right button released): put the selected hotbar block at the pick ray's last position
static void right_click() {
    const RayResult r = RAY_CASTER::castRayFromCam(30);
    putBlock(Pos{r.lastPos.x, r.lastPos.y, r.lastPos.z}, kHotbar2, 6);
}

int main(int argc, char** argv) {
    if (argc < 2 || !(g_out = fopen(argv[1], "w"))) return 4;
    const float s[3] = {2.0f, 1.0f, 4.0f};  // globals.cpp:23
    float sn[3];
    svo_normalize(s, sn);
    sun = vec3{sn[0], sn[1], sn[2]};

    initTetraHexaTree();       // main.cpp:182
    initVoxelDataAllocator();  // main.cpp:183
    genWorld();                // main.cpp:190
    {
        const float c[3] = {cameraDir.x, cameraDir.y, cameraDir.z};  // main.cpp:195
        float n[3];
        svo_normalize(c, n);
        cameraDir = vec3{n[0], n[1], n[2]};
    }
    fprintf(g_out, "{\n");
    const int W = 64, H = 48, N = W * H;
    float* rgba = nullptr;
    int32_t* dps = nullptr;
    float* dt = nullptr;
    uint32_t* di = nullptr;
    if (hipMalloc(&rgba, (size_t)N * 16) != hipSuccess || hipMalloc(&dps, (size_t)N * 16) != hipSuccess ||
        hipMalloc(&dt, (size_t)N * 4) != hipSuccess || hipMalloc(&di, (size_t)N * 4) != hipSuccess)
        return 2;
    int finite = 1;
    for (int frame = 0; frame < 4; frame++) {  // main.cpp:208-227
        updateSsboData();                      // main.cpp:212
        if (frame == 0) fprintf(g_out, "\"tree_after_first_update\": %d,\n", svoTree() != nullptr ? 1 : 0);
        // render(): the lookingAtBlock pick (main.cpp:81) and the frame (main.cpp:107)
        char key[32];
        snprintf(key, sizeof key, "pick_%d", frame);
        print_ray(key, RAY_CASTER::castRayFromCam(30));
        svoRenderShaded(W, H, rgba, nullptr, 0.25f * frame);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        std::vector<float> img((size_t)N * 4);
        if (hipMemcpy(img.data(), rgba, img.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
        for (float v : img) finite &= isfinite(v) ? 1 : 0;
        // doInputUpdates / the mouse callbacks between frames (main.cpp:218-219)
        if (frame == 0) left_click();
        if (frame == 1) right_click();
        if (frame == 2) left_click();
    }
    // the last frame's primary rays (S = 300, low_res.frag:310) for the whole-frame comparison
    svoCastPrimaryRays(W, H, 300, dps, dt, di, nullptr);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<int32_t> hps((size_t)N * 4);
    if (hipMemcpy(hps.data(), dps, hps.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    fprintf(g_out, "\"shade_finite\": %d,\n\"frame\": [", finite);
    for (int i = 0; i < N; i++) fprintf(g_out, "%d,%d,%d,%d%s", hps[4 * i], hps[4 * i + 1], hps[4 * i + 2], hps[4 * i + 3], i + 1 < N ? "," : "");
    fprintf(g_out, "]\n}\n");
    fclose(g_out);
    (void)hipFree(rgba);
    (void)hipFree(dps);
    (void)hipFree(dt);
    (void)hipFree(di);
    return 0;
}
