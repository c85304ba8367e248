// svo_bridge_types.hpp for the C++ test program (tests/bridge/bridge_test.cpp): the names and member
// layout of the reference's declarations the shim defines or reads (src/ray_caster.hpp:6-14,
// src/voxel_data/types.hpp:7-27, src/globals.hpp:63-80, src/voxel_data/tetrahexa_tree.hpp:6-22,
// src/world_gen.hpp:3), written here so the shim compiles and runs without GLM / GL.
#pragma once
#include <stdint.h>

struct vec3 {
    float x, y, z;
};
struct ivec3 {
    int x, y, z;
};
struct Pos {
    int x, y, z;
};
struct Block {
    uint32_t flags;
    uint64_t color;
    float metadata;
};
struct RayResult {
    ivec3 pos;
    ivec3 lastPos;
    int steps;
};
const int maxDepth = 6;
extern vec3 cameraPos, cameraDir, sun;

namespace RAY_CASTER {
RayResult castRayFromCam(int steps);
}
void initTetraHexaTree();
void traverseTree(Pos* pos, int count);
void putBlock(Pos pos, Block block, int targetDepth);
Block getBlock(Pos pos);
Block deleteBlock(Pos pos, int level);
void genWorld();
#define SVO_BRIDGE_IVEC3(x, y, z) ivec3{(x), (y), (z)}
