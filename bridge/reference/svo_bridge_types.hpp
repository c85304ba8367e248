// svo_bridge_types.hpp for the reference build (-I bridge/reference -I src): the reference's own types
// and globals.  Not compiled in this repository (the reference needs GLM / GLFW / GLEW).
#pragma once
#include "globals.hpp"                   // glm::vec3 cameraPos, cameraDir, sun; Block; properties
#include "ray_caster.hpp"                // RayResult, RAY_CASTER::castRayFromCam
#include "voxel_data/tetrahexa_tree.hpp" // Pos, initTetraHexaTree, putBlock, getBlock, deleteBlock
#include "world_gen.hpp"                 // genWorld
#define SVO_BRIDGE_IVEC3(x, y, z) glm::ivec3((x), (y), (z))
