// voxel_allocator.hpp — the replacement for reedthorngag/raytracing_test's
// src/voxel_data/voxel_allocator.hpp in a build that links libsvo_rt through the drop-in shim
// (bridge/svo_bridge.cpp).  Copy this file over src/voxel_data/voxel_allocator.hpp (INTEGRATION.md,
// step 2): main.cpp:12 includes it with quotes, so the compiler finds the file beside main.cpp before
// any -I path, and the original's inline GL bodies of updateSsboData() / initVoxelDataAllocator()
// (voxel_allocator.hpp:38-91) would otherwise be compiled into main.cpp in place of the shim's.
//
// What the original declared and who still needs it once src/voxel_data/tetrahexa_tree.cpp and
// voxel_allocator.cpp leave the build:
//   updateSsboData()            voxel_allocator.hpp:38-78, called each frame at main.cpp:212 -> declared
//                               here, defined by the shim (incremental upload of edited regions)
//   initVoxelDataAllocator()    voxel_allocator.hpp:80-91, called once at main.cpp:183 -> declared here,
//                               defined by the shim (device selection; the first upload is lazy)
//   the 4 MiB block pools, free lists, allocNode / allocArray / convertToPtr / freeNode
//                               (voxel_allocator.hpp:12-36,93-137, voxel_allocator.cpp:5-96): used only
//                               by tetrahexa_tree.cpp; libsvo_rt owns the voxel data (svo_world /
//                               svo_tree), so they are not declared here and nothing can reach the
//                               undefined arrayBlocks / nodeBlocks (voxel_allocator.cpp:6,22).
// The header is self-contained (no GL, Windows or GLM headers) so that tests/bridge/ compiles the very
// same file into its main.cpp-shaped program.
#pragma once

void initVoxelDataAllocator();
void updateSsboData();
