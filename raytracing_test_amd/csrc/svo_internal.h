// svo_internal.h — host-side object layouts shared by svo_world.cpp (builders, C++ host) and
// svo_cast.hip (device upload + kernels).  Not part of the public ABI (include/svo_rt.h).
#pragma once

#include <stdint.h>

#include <array>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/svo_rt.h"
#include "svo_common.h"

namespace svo {

struct Material {
    uint32_t flags;
    uint64_t color;
    float meta;
};

inline bool material_solid(const Material& m) {
    // castRayFromCam's hit test (ray_caster.cpp:82)
    return m.color != ~0ull && (m.flags & 0x10u) == 0;
}

// stored by a tree of `view` (SVO_VIEW_SOLID: what castRayFromCam hits; SVO_VIEW_ALL: every block)
inline bool material_in_view(const Material& m, int32_t view) { return view ? m.color != ~0ull : material_solid(m); }

void set_error(const std::string& msg);

// RGB_TO_U64 (src/types.hpp:6-9)
inline uint64_t rgb_to_u64(int r, int g, int b) {
    auto cs = [](int c) -> uint64_t {
        return (uint64_t)((double)(float)c / 255.0 * (double)((1 << 21) - 1)) & ((1u << 21) - 1);
    };
    return (cs(r) << 42) | (cs(g) << 21) | cs(b);
}

}  // namespace svo

// Linearised tree: host image + optional HBM copy
struct svo_tree {
    int32_t levels = 0;
    int32_t view = 0;                     // SVO_VIEW_SOLID / SVO_VIEW_ALL
    std::vector<svo::Node> nodes;
    std::vector<uint16_t> mats;           // per-voxel material ids of mixed-material bricks
    std::vector<svo::Material> palette;   // id 0 = empty block {0, ~0, 0}
    uint64_t nodes_per_level[8] = {0};
    uint64_t n_bricks = 0;
    // device side (svo_cast.hip)
    int32_t device = -1;
    void* d_nodes = nullptr;
    void* d_mats = nullptr;
    void* d_pick = nullptr;   // device side buffer (kSideBytes): the pick ray's record, the guard-trip counter (offsets below)
    void* d_pal = nullptr;    // palette for shading: u64 colour[n] then u32 flags[n]
    // hemisphere AO plan (svo_cast.hip, built on first use for (ao_samples, ao_steps))
    mutable void* d_ao_plan = nullptr;
    mutable int32_t ao_plan_n = 0, ao_plan_steps = -1;
    mutable std::mutex pick_mu;  // one pick ray at a time per tree (d_pick)
    uint64_t device_bytes = 0;
    // incremental edits (svo_tree_update in svo_world.cpp, svo_tree_sync in svo_cast.hip): changed
    // node blocks are appended; superseded ones are garbage until the next full rebuild
    uint64_t garbage_nodes = 0, garbage_mats = 0;
    uint64_t synced_nodes = 0, synced_mats = 0;  // prefix of nodes / mats already in HBM
    std::vector<uint32_t> dirty_nodes;           // rewritten in place below synced_nodes
    bool palette_dirty = false, full_upload = false;
    uint64_t dev_node_cap = 0, dev_mat_cap = 0, dev_pal_n = 0;  // device allocations (elements)
    // highest voxel row holding a stored voxel (tree_top_y; -1: empty tree), cached until an edit
    mutable int32_t top_y = -1;
    mutable bool top_valid = false;
    mutable std::mutex top_mu;  // (casts from several threads compute it once)
    int32_t dev_top_y = -1;     // tree_top_y of the image in HBM (set by upload / adopt / sync; -1: none)
    // column ceilings of the image in HBM (tree_ceilings, uploaded with it): d_ceil holds, for each
    // level j < ceil_levels, the highest stored voxel row (int16, -1: none) of every aligned block of
    // 4^(kCeilK0 + j) x 4^(kCeilK0 + j) columns, row-major [z][x], starting at element ceil_off[j]
    void* d_ceil = nullptr;
    int32_t ceil_levels = 0;
    int64_t ceil_off[4] = {0, 0, 0, 0};
    // the same ceilings paired for one-load reads: for every block of level j, its ceiling (low 16 bits) and that of
    // its level-(j+1) block (high 16 bits; the last level repeats its own), uint32 at element ceilp_off[j] of d_ceilp
    void* d_ceilp = nullptr;
    int64_t ceilp_off[4] = {0, 0, 0, 0};
    // every level at once for the finest level's blocks (the shading pass's max-mipmap walk): for each level-0 block, the
    // ceilings of the blocks of levels 0..3 holding it, int16 each (level j in bits 16j .. 16j+15; a level the tree lacks:
    // 0x7FFF, which no row is above), uint64 row-major [z][x] in d_ceilq
    void* d_ceilq = nullptr;
    std::vector<uint64_t> ceilq_host;
    int64_t ceil_dev_n = 0;            // elements of the d_ceil / d_ceilp allocations
    std::vector<int16_t> ceil_host;    // the host copies of d_ceil / d_ceilp (svo_tree_sync updates them in place)
    std::vector<uint32_t> ceilp_host;
    // column rectangles {x0, z0, x1, z1} (wrapped, half-open) whose ceilings svo_tree_update's edits may have changed
    std::vector<std::array<int64_t, 4>> ceil_dirty;
    // frame schedules (svo_cast.hip sched_attach): per (stream, launch kind) the block durations of the last frame of one
    // geometry and the dispatch order sorted from them (longest first) for the next; d_buf = u32 order[blocks], u32
    // cost[blocks]
    struct Sched {
        void* stream;
        int32_t kind;
        int64_t sig[7];
        int64_t blocks;
        void* d_buf;
        uint64_t last_use;
        bool primed;  // order holds a sorted schedule (else: the frame runs in the natural order and writes costs)
        int32_t since;  // scheduled frames since the last sort (a sort every kSchedEvery frames)
        float cam[6];  // the camera (origin of the launch's first frame, direction) of the frame whose durations it holds
        float last_cam[6];  // the camera of the last frame on this schedule
    };
    mutable std::vector<Sched> scheds;
    mutable std::mutex sched_mu;
    mutable uint64_t sched_clock = 0;
};

namespace svo {
// the tree's device side buffer (svo_tree.d_pick): byte offsets
constexpr size_t kSidePick = 0;     // svo_cast_ray_from_cam's result record (64 B)
constexpr size_t kSideGuard = 256;  // u32: progress-guard trips of every launch over the tree (svo_tree_guard_trips)
constexpr size_t kSideBytes = 4096;
int32_t tree_top_y(const svo_tree* t);  // svo_world.cpp
// Column ceilings (svo_world.cpp): per aligned block of 4^k x 4^k columns, k = kCeilK0 .. levels - 1 (at
// most kCeilMax levels), the highest stored voxel row in those columns (-1: none) — every voxel above it
// in the block is empty, whatever the tree holds (overhangs included).  Level j's blocks are row-major
// [z][x] at out[off[j] ..]; returns the number of levels.
constexpr int32_t kCeilK0 = SVO_CEIL_K0, kCeilMax = 4;  // 16-, 64-, 256- and 1024-column blocks
constexpr int32_t kCeilPairStep = SVO_CEIL_PAIR_STEP;    // the pair table: level j with level j + kCeilPairStep
int32_t tree_ceilings(const svo_tree* t, std::vector<int16_t>& out, int64_t off[kCeilMax]);
// levels 1 .. nlev-1 re-derived over the blocks holding columns [x0, x1) x [z0, z1)
void ceilings_coarsen(const svo_tree* t, std::vector<int16_t>& out, const int64_t off[kCeilMax], int32_t nlev, int64_t x0, int64_t z0,
                      int64_t x1, int64_t z1);
// every level over the columns [x0, x1) x [z0, z1) recomputed from the tree (an edit's region: svo_tree_sync)
void ceilings_update_rect(const svo_tree* t, std::vector<int16_t>& out, const int64_t off[kCeilMax], int32_t nlev, int64_t x0, int64_t z0,
                          int64_t x1, int64_t z1);
void tree_release_device(svo_tree* t);  // svo_cast.hip
// take over device arrays built on `device` (node_cap / mat_cap elements allocated, the host image
// already equal to their first nodes.size() / mats.size() elements): svo_cast.hip
int adopt_device(svo_tree* t, int32_t device, void* d_nodes, uint64_t node_cap, void* d_mats, uint64_t mat_cap);
}
