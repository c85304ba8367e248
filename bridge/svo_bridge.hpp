// svo_bridge.hpp — what the drop-in shim (svo_bridge.cpp) adds to reedthorngag/raytracing_test beside
// the reference's own declarations, which it defines over libsvo_rt (include/svo_rt.h):
//   RAY_CASTER::castRayFromCam(int)              src/ray_caster.hpp:14
//   initTetraHexaTree / putBlock / getBlock /
//   deleteBlock / traverseTree                   src/voxel_data/tetrahexa_tree.hpp:12-22
//   genWorld()                                   src/world_gen.hpp:3
//   initVoxelDataAllocator() / updateSsboData()  src/voxel_data/voxel_allocator.hpp:38-91 (inline GL
//                                                bodies in the original: the reference build swaps that
//                                                header for bridge/reference/voxel_data/voxel_allocator.hpp,
//                                                which only declares them)
// The reference types (Pos, Block, RayResult, glm::vec3 cameraPos / cameraDir) come from
// svo_bridge_types.hpp: bridge/reference/ (the reference's headers) in the reference build; the C++
// test program (tests/bridge/) brings its own.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "svo_bridge_types.hpp"
#include "svo_rt.h"

void initVoxelDataAllocator();
void updateSsboData();

// render() without GL (replaces glDrawArrays of the low_res program, src/main.cpp:105-107): one
// castRayFromCam-semantics primary ray per pixel of the camera's width x height frame into caller-owned
// device buffers (24 B per pixel, include/svo_rt.h svo_hits), asynchronously on `stream`
void svoCastPrimaryRays(int32_t width, int32_t height, int32_t steps, int32_t* pos_steps, float* t, uint32_t* info, hipStream_t stream);
// the same frame shaded (low_res.frag's colour model, svo_shade_rays, water refracting through the
// full-view scene the shim keeps beside the solid tree): one float4 per pixel; time = deltaTime.  The
// lookingAtBlock pick ray runs on `stream` too (svo_cast_ray_from_cam_async): no host round trip per frame
void svoRenderShaded(int32_t width, int32_t height, float* rgba, hipStream_t stream, float time = 0.0f);
// the tree the shim keeps in HBM (for direct use of the C ABI, e.g. svo_exchange_frames)
svo_tree* svoTree();
// the full-view scene tree svoRenderShaded's rays walk
svo_tree* svoScene();
// svoRenderShaded's image on screen (bridge/svo_present_gl.cpp, needs the application's GL context): rendered into a
// HIP-registered GL pixel buffer, uploaded to a texture and blitted to the default framebuffer — the replacement of
// render()'s glUseProgram(lowResProgram) / glDrawArrays (src/main.cpp:73,105-107)
void svoPresentShaded(int32_t width, int32_t height, float time = 0.0f, hipStream_t stream = nullptr);
// frees its GL objects and the HIP registration (before the GL context goes)
void svoPresentRelease();
