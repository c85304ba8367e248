// svo_world.cpp — host side of libsvo_rt: the editable 64-ary voxel world (the reference's
// putBlock / getBlock / deleteBlock / genWorld API), and the two builders that emit the
// breadth-first linearised tree the gfx950 kernel walks:
//   * svo_build          — from an edited world (reference world: initTetraHexaTree + genWorld)
//   * svo_build_terrain  — straight from genWorld's column formula, level-synchronous and
//                          multi-threaded, for depth-12 / depth-14 terrain that the reference's
//                          one-leaf-per-voxel layout cannot hold.
// Both emit the same canonical form (tests check they agree node for node), defined in
// svo_common.h.  Reference paths are relative to the reedthorngag/raytracing_test snapshot.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <system_error>
#include <deque>
#include <functional>
#include <unordered_map>
#include <map>
#include <memory>
#include <thread>
#include <vector>

#include "../../include/svo_rt.h"
#include "svo_internal.h"
#include "svo_noise.h"

using namespace svo;

static thread_local std::string g_err;
void svo::set_error(const std::string& msg) { g_err = msg; }

extern "C" const char* svo_last_error(void) { return g_err.c_str(); }
extern "C" int svo_version(void) { return SVO_RT_VERSION; }

#define SVO_FAIL(code, msg)     \
    do {                        \
        svo::set_error(msg);    \
        return (code);          \
    } while (0)

static void parallel_for(int64_t n, int nthreads, const std::function<void(int64_t, int64_t)>& fn) {
    // default: the machine's threads, at most 16 (a GPU box exposes many more cores than its share)
    if (nthreads <= 0) nthreads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    nthreads = (int)std::min<int64_t>(nthreads, std::max<int64_t>(1, n / 64));
    if (nthreads <= 1 || n < 2) {
        fn(0, n);
        return;
    }
    std::vector<std::thread> th;
    std::atomic<int64_t> next(0);
    const int64_t chunk = std::max<int64_t>(1, n / (nthreads * 8));
    for (int i = 0; i < nthreads; i++)
        th.emplace_back([&] {
            for (;;) {
                int64_t b = next.fetch_add(chunk);
                if (b >= n) break;
                fn(b, std::min(n, b + chunk));
            }
        });
    for (auto& t : th) t.join();
}

// ================================================================================================
// Palette
// ================================================================================================
namespace {
struct Palette {
    std::vector<Material> m;
    std::map<std::tuple<uint32_t, uint64_t, uint32_t>, uint16_t> index;
    Palette() { m.push_back(Material{0, ~0ull, 0.0f}); }
    int intern(const Material& x) {
        uint32_t mb;
        memcpy(&mb, &x.meta, 4);
        auto key = std::make_tuple(x.flags, x.color, mb);
        auto it = index.find(key);
        if (it != index.end()) return it->second;
        if (m.size() >= 0xFFFFu) return -1;
        uint16_t id = (uint16_t)m.size();
        m.push_back(x);
        index[key] = id;
        return id;
    }
};
}  // namespace

// ================================================================================================
// Editable world: a 64-ary pointer tree with the reference's semantics (tetrahexa_tree.cpp), minus
// its root-array aliasing.  Node 0 is the root; a child id of 0 means "absent" (bitmap bit clear).
// Leaves may sit at any depth (putBlock level < levels+1 stores a uniform region).
// ================================================================================================
struct svo_world {
    int32_t levels;
    Palette pal;
    struct ENode {
        uint32_t kids;  // branch: index of its 64-slot child block
        uint16_t mat;   // leaf: palette id
        uint8_t leaf;
    };
    std::vector<ENode> nodes;
    std::vector<uint32_t> kid_blocks;  // 64 ids per block
    std::vector<uint32_t> free_nodes, free_blocks;
    uint64_t live_nodes = 0;

    uint32_t new_block() {
        uint32_t b;
        if (!free_blocks.empty()) {
            b = free_blocks.back();
            free_blocks.pop_back();
        } else {
            b = (uint32_t)(kid_blocks.size() / 64);
            kid_blocks.resize(kid_blocks.size() + 64);
        }
        std::fill(kid_blocks.begin() + (size_t)b * 64, kid_blocks.begin() + (size_t)b * 64 + 64, 0u);
        return b;
    }
    uint32_t new_node(uint8_t leaf, uint16_t mat) {
        uint32_t n;
        if (!free_nodes.empty()) {
            n = free_nodes.back();
            free_nodes.pop_back();
        } else {
            n = (uint32_t)nodes.size();
            nodes.push_back(ENode{0, 0, 0});
        }
        nodes[n].leaf = leaf;
        nodes[n].mat = mat;
        nodes[n].kids = leaf ? 0 : new_block();
        live_nodes++;
        return n;
    }
    uint32_t* kids(uint32_t n) { return &kid_blocks[(size_t)nodes[n].kids * 64]; }
    const uint32_t* kids(uint32_t n) const { return &kid_blocks[(size_t)nodes[n].kids * 64]; }
    // deleteChildren (tetrahexa_tree.cpp:159-173)
    void drop_children(uint32_t n) {
        if (nodes[n].leaf) return;
        uint32_t b = nodes[n].kids;
        for (int i = 0; i < 64; i++) {
            uint32_t c = kid_blocks[(size_t)b * 64 + i];
            if (c) {
                drop_children(c);
                free_nodes.push_back(c);
                live_nodes--;
            }
        }
        free_blocks.push_back(b);
    }
    void make_leaf(uint32_t n, uint16_t mat) {
        drop_children(n);
        nodes[n].leaf = 1;
        nodes[n].mat = mat;
        nodes[n].kids = 0;
    }
    // split a leaf into 64 copies of itself (tetrahexa_tree.cpp:221-247)
    void split(uint32_t n) {
        uint16_t m = nodes[n].mat;
        uint32_t b = new_block();
        for (int i = 0; i < 64; i++) {
            uint32_t c = new_node(1, m);
            kid_blocks[(size_t)b * 64 + i] = c;
        }
        nodes[n].leaf = 0;
        nodes[n].kids = b;
    }
    uint32_t wrapmask() const { return (1u << (2 * levels)) - 1u; }
};

extern "C" int svo_world_create(int32_t levels, svo_world** out) {
    if (!out) SVO_FAIL(SVO_EINVAL, "svo_world_create: out is NULL");
    if (levels < 1 || levels > 7) SVO_FAIL(SVO_EINVAL, "svo_world_create: levels must be in [1, 7]");
    svo_world* w = new (std::nothrow) svo_world();
    if (!w) SVO_FAIL(SVO_ENOMEM, "svo_world_create: out of memory");
    w->levels = levels;
    w->new_node(0, 0);  // root: an empty branch (tetrahexa_tree.cpp:15-18)
    *out = w;
    return SVO_OK;
}

extern "C" void svo_world_destroy(svo_world* w) { delete w; }

extern "C" int svo_world_node_count(const svo_world* w, uint64_t* n) {
    if (!w || !n) SVO_FAIL(SVO_EINVAL, "svo_world_node_count: NULL argument");
    *n = w->live_nodes;
    return SVO_OK;
}

static int put_block_id(svo_world* w, int32_t x, int32_t y, int32_t z, uint16_t mat, int32_t level) {
    const int target = level - 1;  // putBlock: `level--` (tetrahexa_tree.cpp:178)
    const uint32_t mk = w->wrapmask();
    const uint32_t wx = (uint32_t)x & mk, wy = (uint32_t)y & mk, wz = (uint32_t)z & mk;
    uint32_t n = 0;
    for (int depth = 0;; depth++) {
        if (depth == target) {
            w->make_leaf(n, mat);
            return SVO_OK;
        }
        if (w->nodes[n].leaf) w->split(n);
        const uint32_t slot = child_slot(wx, wy, wz, (uint32_t)(2 * (w->levels - 1 - depth)));
        uint32_t c = w->kids(n)[slot];
        if (!c) {
            if (depth + 1 == target) {
                c = w->new_node(1, mat);
                w->kids(n)[slot] = c;
                return SVO_OK;
            }
            c = w->new_node(0, 0);
            w->kids(n)[slot] = c;
        }
        n = c;
    }
}

extern "C" int svo_put_block(svo_world* w, int32_t x, int32_t y, int32_t z, const svo_block* b, int32_t level) {
    if (!w || !b) SVO_FAIL(SVO_EINVAL, "svo_put_block: NULL argument");
    if (level < 1 || level > w->levels + 1) SVO_FAIL(SVO_EINVAL, "svo_put_block: level out of range");
    int id = w->pal.intern(Material{1u | b->flags, b->color, b->metadata});
    if (id < 0) SVO_FAIL(SVO_ERANGE, "svo_put_block: more than 65534 distinct blocks");
    return put_block_id(w, x, y, z, (uint16_t)id, level);
}

extern "C" int svo_get_block(const svo_world* w, int32_t x, int32_t y, int32_t z, svo_block* out) {
    if (!w || !out) SVO_FAIL(SVO_EINVAL, "svo_get_block: NULL argument");
    const uint32_t mk = w->wrapmask();
    const uint32_t wx = (uint32_t)x & mk, wy = (uint32_t)y & mk, wz = (uint32_t)z & mk;
    uint32_t n = 0;
    for (int depth = 0; depth <= w->levels; depth++) {
        if (w->nodes[n].leaf) {
            const Material& m = w->pal.m[w->nodes[n].mat];
            *out = svo_block{m.flags, m.color, m.meta};
            return SVO_OK;
        }
        if (depth == w->levels) break;
        uint32_t c = w->kids(n)[child_slot(wx, wy, wz, (uint32_t)(2 * (w->levels - 1 - depth)))];
        if (!c) {
            *out = svo_block{0, ~0ull, 0.0f};
            return SVO_OK;
        }
        n = c;
    }
    SVO_FAIL(SVO_ESTATE, "svo_get_block: branch at voxel depth (corrupt world)");
}

extern "C" int svo_delete_block(svo_world* w, int32_t x, int32_t y, int32_t z, int32_t level, svo_block* removed) {
    if (!w) SVO_FAIL(SVO_EINVAL, "svo_delete_block: NULL world");
    if (level < 1 || level > w->levels + 1) SVO_FAIL(SVO_EINVAL, "svo_delete_block: level out of range");
    const int target = level - 1;
    const uint32_t mk = w->wrapmask();
    const uint32_t wx = (uint32_t)x & mk, wy = (uint32_t)y & mk, wz = (uint32_t)z & mk;
    svo_block found{0, ~0ull, 0.0f};
    if (target == 0) {
        if (w->nodes[0].leaf) {
            const Material& m = w->pal.m[w->nodes[0].mat];
            found = svo_block{m.flags, m.color, m.meta};
        }
        w->drop_children(0);
        w->nodes[0].leaf = 0;
        w->nodes[0].kids = w->new_block();
        if (removed) *removed = found;
        return SVO_OK;
    }
    uint32_t n = 0;
    for (int depth = 0;; depth++) {
        if (w->nodes[n].leaf) w->split(n);
        const uint32_t slot = child_slot(wx, wy, wz, (uint32_t)(2 * (w->levels - 1 - depth)));
        uint32_t c = w->kids(n)[slot];
        if (!c) break;  // already empty
        if (depth + 1 == target) {
            if (w->nodes[c].leaf) {
                const Material& m = w->pal.m[w->nodes[c].mat];
                found = svo_block{m.flags, m.color, m.meta};
            }
            w->drop_children(c);
            w->free_nodes.push_back(c);
            w->live_nodes--;
            w->kids(n)[slot] = 0;
            break;
        }
        n = c;
    }
    if (removed) *removed = found;
    return SVO_OK;
}

// initTetraHexaTree's debug blocks (tetrahexa_tree.cpp:20-27)
extern "C" int svo_init_tetra_hexa_tree(svo_world* w) {
    if (!w) SVO_FAIL(SVO_EINVAL, "svo_init_tetra_hexa_tree: NULL world");
    struct P {
        int x, y, z;
        uint32_t f;
        int level;
    } puts[8] = {{1000, 1000, 1000, 1, 5}, {10, 100, 10, 2, 6}, {100, 10, 100, 3, 6}, {20, 10, 200, 4, 5},
                 {1, 10, 10, 5, 6},        {2, 10, 10, 6, 6},    {3, 10, 10, 7, 6},    {4, 10, 10, 8, 6}};
    // the reference's levels are for maxDepth 6; rescale so "6" stays one voxel
    for (auto& p : puts) {
        svo_block b{p.f, 0ull, 0.0f};
        int lv = p.level + (w->levels - 5);
        if (lv < 1) lv = 1;
        int rc = svo_put_block(w, p.x, p.y, p.z, &b, lv);
        if (rc) return rc;
    }
    return SVO_OK;
}

namespace {
struct TerrainIds {
    uint16_t water, grass, dirt, stone;
};
}  // namespace

// genWorld's column puts (world_gen.cpp:24-39) for one column with top y
static void gen_column(svo_world* w, int32_t x, int32_t z, int32_t y);

// genWorld (world_gen.cpp:13-42) over width x length columns
extern "C" int svo_gen_world(svo_world* w, int32_t width, int32_t length) {
    if (!w || width < 0 || length < 0) SVO_FAIL(SVO_EINVAL, "svo_gen_world: bad argument");
    Simplex2 n42, n64, n100;
    simplex2_seed(n42, 42);
    simplex2_seed(n64, 64);
    simplex2_seed(n100, 100);
    for (int32_t x = 0; x < width; x++)
        for (int32_t z = 0; z < length; z++) gen_column(w, x, z, terrain_height(n42.perm, n64.perm, n100.perm, x, z));
    return SVO_OK;
}

// the same puts from caller-given column tops heights[x*length + z]
extern "C" int svo_gen_heightfield(svo_world* w, int32_t width, int32_t length, const int32_t* heights) {
    if (!w || width < 0 || length < 0 || (!heights && (int64_t)width * length > 0)) SVO_FAIL(SVO_EINVAL, "svo_gen_heightfield: bad argument");
    for (int32_t x = 0; x < width; x++)
        for (int32_t z = 0; z < length; z++) gen_column(w, x, z, heights[(size_t)x * length + z]);
    return SVO_OK;
}

static void gen_column(svo_world* w, int32_t x, int32_t z, int32_t y) {
    const uint64_t green = rgb_to_u64(0, 150, 10), brown = rgb_to_u64(45, 18, 0), grey = rgb_to_u64(33, 33, 33);
    const int32_t voxel = w->levels + 1;
    auto id = [&](uint32_t f, uint64_t c) { return (uint16_t)w->pal.intern(Material{1u | f, c, 0.0f}); };
    if (y < 20) {
        const uint16_t water = id(0x4u | 0x10u, green);
        for (int32_t i = 20; i > y; i--) put_block_id(w, x, i, z, water, voxel);
        put_block_id(w, x, y, z, id(0, brown), voxel);
    } else {
        put_block_id(w, x, y, z, id(0, green), voxel);
    }
    y--;
    for (int i = 3; y > 0 && i; i--, y--) put_block_id(w, x, y, z, id(0, brown), voxel);
    for (; y > 0; y--) put_block_id(w, x, y, z, id(0, grey), voxel);
}

// ================================================================================================
// Canonical linearisation.  Region classes in the solid view (non-solid blocks count as empty):
//   EMPTY, SOLID(material), MIXED.  A MIXED region at depth levels-1 becomes a BRICK, deeper up an
//   INTERIOR node whose non-EMPTY children follow in breadth-first order.
// ================================================================================================
static constexpr uint32_t C_EMPTY = 0u;
static constexpr uint32_t C_MIXED = 0xFFFFFFFFu;  // otherwise SOLID with material = class

struct BrickOut {
    uint64_t mask;
    uint32_t info;
};

// fold 64 voxel classes (EMPTY or SOLID ids) into brick mask + material run
static BrickOut make_brick(const uint32_t* vox, std::vector<uint16_t>* mats_out) {
    uint64_t mask = 0;
    uint32_t first = C_EMPTY;
    bool uniform = true;
    for (int v = 0; v < 64; v++) {
        if (vox[v] == C_EMPTY) continue;
        mask |= 1ull << v;
        if (first == C_EMPTY) first = vox[v];
        else if (vox[v] != first) uniform = false;
    }
    if (uniform) return BrickOut{mask, K_BRICK | K_UNIFORM | (first << 16)};
    if (mats_out)
        for (int v = 0; v < 64; v++)
            if (vox[v] != C_EMPTY) mats_out->push_back((uint16_t)vox[v]);
    return BrickOut{mask, K_BRICK};
}

static uint32_t fold_classes(const uint32_t* c) {
    uint32_t f = c[0];
    if (f == C_MIXED) return C_MIXED;
    for (int i = 1; i < 64; i++)
        if (c[i] != f) return C_MIXED;
    return f;  // all EMPTY or all SOLID(m)
}

static void finish_tree_stats(svo_tree* t) {
    (void)t;
}

extern "C" int svo_build(const svo_world* w, svo_tree** out) { return svo_build_view(w, SVO_VIEW_SOLID, out); }

extern "C" int svo_build_view(const svo_world* w, int32_t view, svo_tree** out) {
    if (!w || !out) SVO_FAIL(SVO_EINVAL, "svo_build: NULL argument");
    if (view != SVO_VIEW_SOLID && view != SVO_VIEW_ALL) SVO_FAIL(SVO_EINVAL, "svo_build_view: unknown view");
    const int L = w->levels;
    std::vector<uint8_t> solid(w->pal.m.size());
    for (size_t i = 0; i < solid.size(); i++) solid[i] = material_in_view(w->pal.m[i], view);
    // post-order classes of every live edit node
    std::vector<uint32_t> cls(w->nodes.size(), C_EMPTY);
    std::function<uint32_t(uint32_t, int)> classify = [&](uint32_t n, int depth) -> uint32_t {
        const auto& e = w->nodes[n];
        uint32_t c;
        if (e.leaf) {
            c = solid[e.mat] ? (uint32_t)e.mat : C_EMPTY;
        } else {
            uint32_t kc[64];
            const uint32_t* k = w->kids(n);
            for (int i = 0; i < 64; i++) kc[i] = k[i] ? classify(k[i], depth + 1) : C_EMPTY;
            c = fold_classes(kc);
        }
        cls[n] = c;
        return c;
    };
    classify(0, 0);

    svo_tree* t = new (std::nothrow) svo_tree();
    if (!t) SVO_FAIL(SVO_ENOMEM, "svo_build: out of memory");
    t->levels = L;
    t->view = view;
    t->palette = w->pal.m;
    // level-synchronous emission; `cur` = edit ids of this depth's nodes (in node order)
    std::vector<uint32_t> cur{0};
    t->nodes.push_back(Node{0, 0, K_INTERIOR});
    uint64_t level_base = 0;
    for (int d = 0; d < L && !cur.empty(); d++) {
        t->nodes_per_level[d] = cur.size();
        std::vector<uint32_t> next;
        uint64_t next_base = level_base + cur.size();
        for (size_t i = 0; i < cur.size(); i++) {
            uint32_t e = cur[i];
            Node& nd = t->nodes[level_base + i];
            uint32_t c = cls[e];
            if (c == C_EMPTY) {  // only the root can be an empty node
                nd = Node{0, 0, K_INTERIOR};
                continue;
            }
            if (c != C_MIXED) {
                nd = Node{~0ull, 0, K_SOLID | (c << 16)};
                continue;
            }
            const uint32_t* k = w->kids(e);
            if (d == L - 1) {
                uint32_t vox[64];
                for (int v = 0; v < 64; v++) vox[v] = k[v] ? cls[k[v]] : C_EMPTY;
                uint32_t ref = (uint32_t)t->mats.size();
                BrickOut b = make_brick(vox, &t->mats);
                t->nodes[level_base + i] = Node{b.mask, (b.info & K_UNIFORM) ? 0u : ref, b.info};
                t->n_bricks++;
                continue;
            }
            uint64_t mask = 0;
            for (int s = 0; s < 64; s++)
                if (k[s] && cls[k[s]] != C_EMPTY) {
                    mask |= 1ull << s;
                    next.push_back(k[s]);
                }
            t->nodes[level_base + i] = Node{mask, (uint32_t)(next_base + (next.size() - __builtin_popcountll(mask))), K_INTERIOR};
        }
        t->nodes.resize(next_base + next.size(), Node{0, 0, 0});
        level_base = next_base;
        cur.swap(next);
    }
    if (t->nodes.size() > 0xFFFFFFFFull || t->mats.size() > 0xFFFFFFFFull) {
        delete t;
        SVO_FAIL(SVO_ERANGE, "svo_build: tree exceeds 2^32 nodes");
    }
    finish_tree_stats(t);
    *out = t;
    return SVO_OK;
}

// ================================================================================================
// Incremental edits (putBlock / deleteBlock + updateSsboData,
// voxel_allocator.hpp:38-78).  After world edits, the linearised tree is patched instead of
// rebuilt: for each edited region, the deepest interior node A above it whose subtree still holds
// the old content is found; the edited child of A is re-linearised from the world (its subtree
// appended breadth-first), and A's child block is rewritten at the end of the array with the new
// child record (siblings are copied: their own subtrees stay where they are).  Only A's record is
// changed in place.  Results are the tree's *content*, not its canonical layout: regions that
// become uniform are not re-collapsed (traversal is unaffected); when superseded blocks exceed
// half the array, the tree is rebuilt from the world.  svo_tree_sync uploads the appended tail
// and the rewritten records.
// ================================================================================================
namespace {
struct Emitter {
    svo_tree* t;
    const svo_world* w;
    std::vector<uint8_t> solid;
    std::unordered_map<uint32_t, uint32_t> cls;  // classes of the world nodes visited

    uint32_t classify(uint32_t n) {
        auto it = cls.find(n);
        if (it != cls.end()) return it->second;
        const auto& e = w->nodes[n];
        uint32_t c;
        if (e.leaf) {
            c = solid[e.mat] ? (uint32_t)e.mat : C_EMPTY;
        } else {
            uint32_t kc[64];
            const uint32_t* k = w->kids(n);
            for (int i = 0; i < 64; i++) kc[i] = k[i] ? classify(k[i]) : C_EMPTY;
            c = fold_classes(kc);
        }
        cls[n] = c;
        return c;
    }

    // record of world node e at depth d; its descendants are appended breadth-first.  The record
    // is written to *root_rec (index -1) or t->nodes[idx].
    Node emit(uint32_t e, int d) {
        const int L = t->levels;
        struct Item {
            uint32_t e;
            int d;
            int64_t idx;
        };
        std::deque<Item> q;
        q.push_back({e, d, -1});
        Node root_rec{0, 0, K_INTERIOR};
        while (!q.empty()) {
            const Item it = q.front();
            q.pop_front();
            const uint32_t c = classify(it.e);
            Node rec{0, 0, K_INTERIOR};
            if (c == C_MIXED) {
                const uint32_t* k = w->kids(it.e);
                if (it.d == L - 1) {
                    uint32_t vox[64];
                    for (int v = 0; v < 64; v++) vox[v] = k[v] ? classify(k[v]) : C_EMPTY;
                    const uint32_t ref = (uint32_t)t->mats.size();
                    BrickOut b = make_brick(vox, &t->mats);
                    rec = Node{b.mask, (b.info & K_UNIFORM) ? 0u : ref, b.info};
                } else {
                    uint64_t mask = 0;
                    for (int sl = 0; sl < 64; sl++)
                        if (k[sl] && classify(k[sl]) != C_EMPTY) mask |= 1ull << sl;
                    const uint64_t base = t->nodes.size();
                    t->nodes.resize(base + __builtin_popcountll(mask), Node{0, 0, 0});
                    int64_t j = (int64_t)base;
                    for (int sl = 0; sl < 64; sl++)
                        if ((mask >> sl) & 1ull) q.push_back({k[sl], it.d + 1, j++});
                    rec = Node{mask, (uint32_t)base, K_INTERIOR};
                }
            } else if (c != C_EMPTY) {
                rec = Node{~0ull, 0, K_SOLID | (c << 16)};
            }
            if (it.idx < 0) root_rec = rec;
            else t->nodes[(size_t)it.idx] = rec;
        }
        return root_rec;
    }
};

// class of the world region of depth `d` holding (x, y, z): its node, or a uniform class when a
// leaf above covers it / nothing is stored there
struct WorldRegion {
    bool has_node;
    uint32_t node;
    uint32_t cls;
};
WorldRegion world_region(const svo_world* w, const std::vector<uint8_t>& solid, uint32_t x, uint32_t y, uint32_t z, int d) {
    uint32_t n = 0;
    for (int depth = 0;; depth++) {
        const auto& e = w->nodes[n];
        if (e.leaf) return {false, 0, solid[e.mat] ? (uint32_t)e.mat : C_EMPTY};
        if (depth == d) return {true, n, 0};
        const uint32_t c = w->kids(n)[child_slot(x, y, z, (uint32_t)(2 * (w->levels - 1 - depth)))];
        if (!c) return {false, 0, C_EMPTY};
        n = c;
    }
}
}  // namespace

extern "C" int svo_tree_update(svo_tree* t, const svo_world* w, const int32_t* xyz, int64_t n, int32_t level) {
    if (!t || !w || (!xyz && n > 0)) SVO_FAIL(SVO_EINVAL, "svo_tree_update: NULL argument");
    if (t->levels != w->levels) SVO_FAIL(SVO_EINVAL, "svo_tree_update: tree and world differ in levels");
    if (level < 1 || level > w->levels + 1) SVO_FAIL(SVO_EINVAL, "svo_tree_update: level out of range");
    const int L = t->levels;
    const int de = level - 1;  // depth of the edited region (putBlock's `level--`)
    if (w->pal.m.size() != t->palette.size()) {
        t->palette = w->pal.m;  // the world's palette only grows: ids stay valid
        t->palette_dirty = true;
    }
    t->top_valid = false;
    Emitter em{t, w, std::vector<uint8_t>(w->pal.m.size()), {}};
    for (size_t i = 0; i < em.solid.size(); i++) em.solid[i] = material_in_view(w->pal.m[i], t->view);
    const uint32_t mk = (1u << (2 * L)) - 1u;
    bool rebuild = de == 0 || node_kind(t->nodes[0].info) != K_INTERIOR;
    for (int64_t i = 0; i < n && !rebuild; i++) {
        const uint32_t x = (uint32_t)xyz[3 * i] & mk, y = (uint32_t)xyz[3 * i + 1] & mk, z = (uint32_t)xyz[3 * i + 2] & mk;
        // A: the deepest interior node above the edited region whose child on the path is interior
        uint32_t a = 0;
        int da = 0;
        while (da < de - 1) {
            const Node& A = t->nodes[a];
            const uint32_t sl = child_slot(x, y, z, (uint32_t)(2 * (L - 1 - da)));
            if (!((A.mask >> sl) & 1ull)) break;
            const uint32_t ci = A.ref + (uint32_t)__builtin_popcountll(A.mask & ((1ull << sl) - 1ull));
            if (node_kind(t->nodes[ci].info) != K_INTERIOR) break;
            a = ci;
            da++;
        }
        // the child of A on the path, re-linearised from the world
        const uint32_t s = child_slot(x, y, z, (uint32_t)(2 * (L - 1 - da)));
        {  // its columns: the only ones whose ceilings can change (svo_tree_sync)
            const int64_t cs = (int64_t)1 << (2 * (L - 1 - da)), cx = (int64_t)(x & ~(uint32_t)(cs - 1)), cz = (int64_t)(z & ~(uint32_t)(cs - 1));
            t->ceil_dirty.push_back({cx, cz, cx + cs, cz + cs});
        }
        const WorldRegion r = world_region(w, em.solid, x, y, z, da + 1);
        Node rec{0, 0, K_INTERIOR};
        bool empty;
        if (r.has_node) {
            empty = em.classify(r.node) == C_EMPTY;
            if (!empty) rec = em.emit(r.node, da + 1);
        } else {
            empty = r.cls == C_EMPTY;
            if (!empty) rec = Node{~0ull, 0, K_SOLID | (r.cls << 16)};
        }
        // A's child block, rewritten at the end of the array
        const Node A = t->nodes[a];
        const uint64_t m_old = A.mask, m_new = empty ? (m_old & ~(1ull << s)) : (m_old | (1ull << s));
        const uint64_t base = t->nodes.size();
        t->nodes.resize(base + __builtin_popcountll(m_new));
        uint64_t j = base;
        for (uint32_t sl = 0; sl < 64; sl++) {
            if (!((m_new >> sl) & 1ull)) continue;
            t->nodes[j++] = sl == s ? rec : t->nodes[A.ref + (uint32_t)__builtin_popcountll(m_old & ((1ull << sl) - 1ull))];
        }
        t->garbage_nodes += (uint64_t)__builtin_popcountll(m_old);
        t->nodes[a] = Node{m_new, (uint32_t)base, K_INTERIOR};
        if (a < t->synced_nodes) t->dirty_nodes.push_back(a);
        em.cls.clear();  // the next edit may change classes on its own path
        if (t->nodes.size() > 0xFFFFFFFFull) rebuild = true;
    }
    if (rebuild || t->garbage_nodes * 2 > t->nodes.size()) {
        svo_tree* f = nullptr;
        int rc = svo_build_view(w, t->view, &f);
        if (rc) return rc;
        t->nodes.swap(f->nodes);
        t->mats.swap(f->mats);
        t->palette.swap(f->palette);
        for (int i = 0; i < 8; i++) t->nodes_per_level[i] = f->nodes_per_level[i];
        t->n_bricks = f->n_bricks;
        t->garbage_nodes = t->garbage_mats = 0;
        t->dirty_nodes.clear();
        t->full_upload = t->palette_dirty = true;
        delete f;
    }
    return SVO_OK;
}

// ================================================================================================
// Terrain builder: genWorld's columns -> canonical tree without a per-voxel edit tree.
// Heights are generated in parallel; a min/max pyramid over aligned 4^k column footprints
// classifies every region in O(1) (see classify_region); the tree is emitted depth by depth with a
// count pass + prefix sum + write pass, all multi-threaded.
// ================================================================================================
namespace {
struct Pyramid {
    int32_t W, L;           // columns
    std::vector<int32_t> dimx, dimz;
    std::vector<std::vector<int16_t>> hmin, hmax;  // level k: ceil(W/4^k) x ceil(L/4^k), [cx*dz + cz]
};

struct TerrainCtx {
    int32_t levels, E, W, L;
    const int16_t* h;  // [x*L + z]
    Pyramid pyr;
    uint32_t id_of[5];  // terrain material -> palette id (0 for non-stored)
    int32_t view;       // SVO_VIEW_SOLID / SVO_VIEW_ALL
};

inline uint32_t solid_class(const TerrainCtx& T, int32_t h, int32_t y) {
    return T.id_of[terrain_material(h, y)];
}

// class of the aligned region [x0,x0+s) x [y0,y0+s) x [z0,z0+s), s = 4^k >= 4 (svo_noise.h
// terrain_region_class over the pyramid's min / max tops of its footprint)
uint32_t classify_region(const TerrainCtx& T, int32_t x0, int32_t y0, int32_t z0, int32_t s, int k) {
    const int32_t y1 = y0 + s - 1;
    if (x0 >= T.W || z0 >= T.L) return C_EMPTY;  // no columns here
    const bool partial = (x0 + s > T.W) || (z0 + s > T.L);
    const int32_t cx = x0 >> (2 * k), cz = z0 >> (2 * k);
    const size_t ci = (size_t)cx * T.pyr.dimz[k] + cz;
    const int32_t hmin = T.pyr.hmin[k][ci], hmax = T.pyr.hmax[k][ci];
    if (terrain_region_empty(T.view, hmax, y0, y1)) return C_EMPTY;
    if (partial) return C_MIXED;
    return terrain_region_class(T.id_of, T.view, hmin, hmax, y0, y1, C_EMPTY, C_MIXED);
}

void brick_voxels(const TerrainCtx& T, int32_t x0, int32_t y0, int32_t z0, uint32_t vox[64]) {
    for (int lz = 0; lz < 4; lz++)
        for (int lx = 0; lx < 4; lx++) {
            const int32_t x = x0 + lx, z = z0 + lz;
            const bool have = x < T.W && z < T.L;
            const int32_t h = have ? T.h[(size_t)x * T.L + z] : 0;
            for (int ly = 0; ly < 4; ly++) vox[(lz << 4) | (ly << 2) | lx] = have ? solid_class(T, h, y0 + ly) : C_EMPTY;
        }
}

struct Region {
    int32_t x0, y0, z0;
};
}  // namespace

static int build_from_heights(int32_t levels, int32_t width, int32_t length, int32_t nthreads, int32_t view, std::vector<int16_t>& hg,
                              svo_tree** out);

extern "C" int svo_build_terrain(int32_t levels, int32_t width, int32_t length, int32_t nthreads, svo_tree** out) {
    return svo_build_terrain_view(levels, width, length, nthreads, SVO_VIEW_SOLID, out);
}

extern "C" int svo_build_terrain_view(int32_t levels, int32_t width, int32_t length, int32_t nthreads, int32_t view, svo_tree** out) {
    if (!out) SVO_FAIL(SVO_EINVAL, "svo_build_terrain: out is NULL");
    if (view != SVO_VIEW_SOLID && view != SVO_VIEW_ALL) SVO_FAIL(SVO_EINVAL, "svo_build_terrain_view: unknown view");
    if (levels < 2 || levels > 7) SVO_FAIL(SVO_EINVAL, "svo_build_terrain: levels must be in [2, 7]");
    const int32_t E = 1 << (2 * levels);
    if (width < 1 || length < 1 || width > E || length > E) SVO_FAIL(SVO_EINVAL, "svo_build_terrain: columns must fit the extent");
    // heights (world_gen.cpp:22), parallel over x
    std::vector<int16_t> hg((size_t)width * length);
    Simplex2 n42, n64, n100;
    simplex2_seed(n42, 42);
    simplex2_seed(n64, 64);
    simplex2_seed(n100, 100);
    std::atomic<int> bad(0);
    parallel_for(width, nthreads, [&](int64_t b, int64_t e) {
        for (int64_t x = b; x < e; x++)
            for (int32_t z = 0; z < length; z++) {
                int32_t h = terrain_height(n42.perm, n64.perm, n100.perm, (int32_t)x, z);
                if (h < 0 || h > 32767) bad = 1;
                hg[(size_t)x * length + z] = (int16_t)h;
            }
    });
    if (bad) SVO_FAIL(SVO_ERANGE, "svo_build_terrain: a column top falls outside [0, 32767]");
    return build_from_heights(levels, width, length, nthreads, view, hg, out);
}

extern "C" int svo_build_heightfield(int32_t levels, int32_t width, int32_t length, const int32_t* heights, int32_t nthreads,
                                     svo_tree** out) {
    if (!out || !heights) SVO_FAIL(SVO_EINVAL, "svo_build_heightfield: NULL argument");
    if (levels < 2 || levels > 7) SVO_FAIL(SVO_EINVAL, "svo_build_heightfield: levels must be in [2, 7]");
    const int32_t E = 1 << (2 * levels);
    if (width < 1 || length < 1 || width > E || length > E) SVO_FAIL(SVO_EINVAL, "svo_build_heightfield: columns must fit the extent");
    std::vector<int16_t> hg((size_t)width * length);
    for (size_t i = 0; i < hg.size(); i++) {
        if (heights[i] < 0 || heights[i] > 32767) SVO_FAIL(SVO_ERANGE, "svo_build_heightfield: heights must be in [0, extent-2]");
        hg[i] = (int16_t)heights[i];
    }
    return build_from_heights(levels, width, length, nthreads, SVO_VIEW_SOLID, hg, out);
}

static int build_from_heights(int32_t levels, int32_t width, int32_t length, int32_t nthreads, int32_t view, std::vector<int16_t>& hg,
                              svo_tree** out) {
    const int32_t E = 1 << (2 * levels);
    for (size_t i = 0; i < hg.size(); i++)
        if (hg[i] + 1 >= E || 21 >= E)
            SVO_FAIL(SVO_ERANGE, "svo_build_terrain: a column top falls outside [0, extent-2] (wrap not supported here; use svo_gen_world)");
    TerrainCtx T;
    T.levels = levels;
    T.E = E;
    T.W = width;
    T.L = length;
    T.h = hg.data();
    T.view = view;
    // ---- min/max pyramid over aligned 4^k footprints
    T.pyr.W = width;
    T.pyr.L = length;
    T.pyr.dimx.push_back(width);
    T.pyr.dimz.push_back(length);
    T.pyr.hmin.push_back(hg);
    T.pyr.hmax.push_back(hg);
    for (int k = 1; k <= levels; k++) {
        const int32_t px = T.pyr.dimx[k - 1], pz = T.pyr.dimz[k - 1];
        const int32_t dx = (px + 3) / 4, dz = (pz + 3) / 4;
        std::vector<int16_t> mn((size_t)dx * dz), mx((size_t)dx * dz);
        const auto& pmn = T.pyr.hmin[k - 1];
        const auto& pmx = T.pyr.hmax[k - 1];
        parallel_for(dx, nthreads, [&](int64_t b, int64_t e) {
            for (int64_t cx = b; cx < e; cx++)
                for (int32_t cz = 0; cz < dz; cz++) {
                    int16_t a = 32767, c = -32768;
                    for (int i = 0; i < 4; i++)
                        for (int j = 0; j < 4; j++) {
                            const int64_t sx = cx * 4 + i, sz = (int64_t)cz * 4 + j;
                            if (sx >= px || sz >= pz) continue;
                            a = std::min(a, pmn[(size_t)sx * pz + sz]);
                            c = std::max(c, pmx[(size_t)sx * pz + sz]);
                        }
                    mn[(size_t)cx * dz + cz] = a;
                    mx[(size_t)cx * dz + cz] = c;
                }
        });
        T.pyr.dimx.push_back(dx);
        T.pyr.dimz.push_back(dz);
        T.pyr.hmin.push_back(std::move(mn));
        T.pyr.hmax.push_back(std::move(mx));
    }
    svo_tree* t = new (std::nothrow) svo_tree();
    if (!t) SVO_FAIL(SVO_ENOMEM, "svo_build_terrain: out of memory");
    t->levels = levels;
    t->view = view;
    // palette: the blocks genWorld stores (stored flags = 1 | Block.flags)
    t->palette.push_back(Material{0, ~0ull, 0.0f});
    t->palette.push_back(Material{1u, rgb_to_u64(0, 150, 10), 0.0f});  // 1 grass
    t->palette.push_back(Material{1u, rgb_to_u64(45, 18, 0), 0.0f});   // 2 dirt
    t->palette.push_back(Material{1u, rgb_to_u64(33, 33, 33), 0.0f});  // 3 stone
    t->palette.push_back(Material{1u | 0x14u, rgb_to_u64(0, 150, 10), 0.0f});  // 4 water (LIQUID)
    T.id_of[TM_AIR] = C_EMPTY;
    T.id_of[TM_WATER] = view ? 4u : C_EMPTY;
    T.id_of[TM_GRASS] = 1;
    T.id_of[TM_DIRT] = 2;
    T.id_of[TM_STONE] = 3;

    // root
    const uint32_t rc = classify_region(T, 0, 0, 0, E, levels);
    if (rc == C_EMPTY) {
        t->nodes.push_back(Node{0, 0, K_INTERIOR});
        t->nodes_per_level[0] = 1;
        *out = t;
        return SVO_OK;
    }
    if (rc != C_MIXED) {
        t->nodes.push_back(Node{~0ull, 0, K_SOLID | (rc << 16)});
        t->nodes_per_level[0] = 1;
        *out = t;
        return SVO_OK;
    }
    std::vector<Region> cur{{0, 0, 0}};
    std::vector<uint64_t> cur_node{0};  // node index of each MIXED region
    t->nodes.push_back(Node{0, 0, K_INTERIOR});
    t->nodes_per_level[0] = 1;
    uint64_t level_end = 1;  // nodes emitted so far = start of the next depth
    for (int d = 0; d < levels && !cur.empty(); d++) {
        const int32_t s = 1 << (2 * (levels - d));  // region size at depth d
        const int32_t cs = s >> 2;
        const int64_t nr = (int64_t)cur.size();
        if (d == levels - 1) {
            // bricks: two passes for the material run offsets
            std::vector<uint32_t> nmat(nr);
            std::vector<BrickOut> bo(nr);
            parallel_for(nr, nthreads, [&](int64_t b, int64_t e) {
                uint32_t vox[64];
                for (int64_t i = b; i < e; i++) {
                    brick_voxels(T, cur[i].x0, cur[i].y0, cur[i].z0, vox);
                    bo[i] = make_brick(vox, nullptr);
                    nmat[i] = (bo[i].info & K_UNIFORM) ? 0u : (uint32_t)__builtin_popcountll(bo[i].mask);
                }
            });
            std::vector<uint64_t> moff(nr + 1, 0);
            for (int64_t i = 0; i < nr; i++) moff[i + 1] = moff[i] + nmat[i];
            t->mats.resize(moff[nr]);
            parallel_for(nr, nthreads, [&](int64_t b, int64_t e) {
                uint32_t vox[64];
                for (int64_t i = b; i < e; i++) {
                    uint32_t ref = 0;
                    if (nmat[i]) {
                        brick_voxels(T, cur[i].x0, cur[i].y0, cur[i].z0, vox);
                        uint64_t o = moff[i];
                        for (int v = 0; v < 64; v++)
                            if (vox[v] != C_EMPTY) t->mats[o++] = (uint16_t)vox[v];
                        ref = (uint32_t)moff[i];
                    }
                    t->nodes[cur_node[i]] = Node{bo[i].mask, ref, bo[i].info};
                }
            });
            t->n_bricks = (uint64_t)nr;
            break;
        }
        // pass 1: per region, count non-empty and mixed children
        std::vector<uint32_t> nkid(nr), nmix(nr);
        parallel_for(nr, nthreads, [&](int64_t b, int64_t e) {
            for (int64_t i = b; i < e; i++) {
                uint32_t a = 0, m = 0;
                for (int sl = 0; sl < 64; sl++) {
                    uint32_t c = classify_region(T, cur[i].x0 + (sl & 3) * cs, cur[i].y0 + ((sl >> 2) & 3) * cs,
                                                 cur[i].z0 + ((sl >> 4) & 3) * cs, cs, levels - d - 1);
                    a += c != C_EMPTY;
                    m += c == C_MIXED;
                }
                nkid[i] = a;
                nmix[i] = m;
            }
        });
        std::vector<uint64_t> koff(nr + 1, 0), moff(nr + 1, 0);
        for (int64_t i = 0; i < nr; i++) {
            koff[i + 1] = koff[i] + nkid[i];
            moff[i + 1] = moff[i] + nmix[i];
        }
        const uint64_t base = level_end;
        t->nodes.resize(base + koff[nr]);
        t->nodes_per_level[d + 1] = koff[nr];
        std::vector<Region> next(moff[nr]);
        std::vector<uint64_t> next_node(moff[nr]);
        // pass 2: write this depth's INTERIOR nodes and the next depth's SOLID children
        parallel_for(nr, nthreads, [&](int64_t b, int64_t e) {
            for (int64_t i = b; i < e; i++) {
                uint64_t mask = 0, kpos = base + koff[i], mpos = moff[i];
                for (int sl = 0; sl < 64; sl++) {
                    const int32_t x = cur[i].x0 + (sl & 3) * cs, y = cur[i].y0 + ((sl >> 2) & 3) * cs,
                                  z = cur[i].z0 + ((sl >> 4) & 3) * cs;
                    uint32_t c = classify_region(T, x, y, z, cs, levels - d - 1);
                    if (c == C_EMPTY) continue;
                    mask |= 1ull << sl;
                    if (c == C_MIXED) {
                        next[mpos] = Region{x, y, z};
                        next_node[mpos] = kpos;
                        mpos++;
                    } else {
                        t->nodes[kpos] = Node{~0ull, 0, K_SOLID | (c << 16)};
                    }
                    kpos++;
                }
                t->nodes[cur_node[i]] = Node{mask, (uint32_t)(base + koff[i]), K_INTERIOR};
            }
        });
        level_end = base + koff[nr];
        cur.swap(next);
        cur_node.swap(next_node);
    }
    if (t->nodes.size() > 0xFFFFFFFFull) {
        delete t;
        SVO_FAIL(SVO_ERANGE, "svo_build_terrain: tree exceeds 2^32 nodes");
    }
    *out = t;
    return SVO_OK;
}

// ================================================================================================
// Tree queries
// ================================================================================================
extern "C" int svo_tree_get_info(const svo_tree* t, svo_tree_info* o) {
    if (!t || !o) SVO_FAIL(SVO_EINVAL, "svo_tree_get_info: NULL argument");
    memset(o, 0, sizeof(*o));
    o->levels = t->levels;
    o->n_materials = (uint32_t)t->palette.size();
    o->n_nodes = t->nodes.size();
    o->n_mat_bytes = t->mats.size() * sizeof(uint16_t);
    o->n_bricks = t->n_bricks;
    for (int i = 0; i < 8; i++) o->nodes_per_level[i] = t->nodes_per_level[i];
    o->device_bytes = t->device_bytes;
    o->device = t->device;
    o->view = t->view;
    return SVO_OK;
}

extern "C" int svo_tree_palette(const svo_tree* t, uint32_t id, svo_block* out) {
    if (!t || !out) SVO_FAIL(SVO_EINVAL, "svo_tree_palette: NULL argument");
    if (id >= t->palette.size()) SVO_FAIL(SVO_ERANGE, "svo_tree_palette: id out of range");
    const Material& m = t->palette[id];
    *out = svo_block{m.flags, m.color, m.meta};
    return SVO_OK;
}

extern "C" int svo_tree_get_block(const svo_tree* t, int32_t x, int32_t y, int32_t z, svo_block* out, uint32_t* mid) {
    if (!t || !out) SVO_FAIL(SVO_EINVAL, "svo_tree_get_block: NULL argument");
    const uint32_t mk = (1u << (2 * t->levels)) - 1u;
    const uint32_t wx = (uint32_t)x & mk, wy = (uint32_t)y & mk, wz = (uint32_t)z & mk;
    uint32_t ni = 0, mat = 0;
    for (int d = 0; d < t->levels; d++) {
        const Node& n = t->nodes[ni];
        const uint32_t kind = node_kind(n.info);
        if (kind == K_SOLID) {
            mat = node_material(n.info);
            break;
        }
        if (kind == K_BRICK) {
            const uint32_t v = child_slot(wx, wy, wz, 0);
            if ((n.mask >> v) & 1ull)
                mat = (n.info & K_UNIFORM) ? node_material(n.info) : t->mats[n.ref + __builtin_popcountll(n.mask & ((1ull << v) - 1ull))];
            break;
        }
        const uint32_t sl = child_slot(wx, wy, wz, (uint32_t)(2 * (t->levels - 1 - d)));
        if (!((n.mask >> sl) & 1ull)) break;
        ni = n.ref + (uint32_t)__builtin_popcountll(n.mask & ((1ull << sl) - 1ull));
    }
    const Material& m = t->palette[mat];
    *out = svo_block{m.flags, m.color, m.meta};
    if (mid) *mid = mat;
    return SVO_OK;
}

// Highest y of any stored voxel (wrapped coordinates), by a descent that visits child slots from the
// top y-row down and prunes regions that cannot beat the best found so far; cached on the tree.
namespace {
int32_t top_y_of(const svo_tree* t, uint32_t ni, int32_t y0, int depth, int32_t best) {
    const Node& n = t->nodes[ni];
    const int32_t size = 1 << (2 * (t->levels - depth));
    if (y0 + size - 1 <= best) return best;
    const uint32_t kind = node_kind(n.info);
    if (kind == K_SOLID) return y0 + size - 1;
    if (kind == K_BRICK) {
        for (int ly = 3; ly >= 0; ly--)
            if (n.mask & (0x000F000F000F000Full << (4 * ly))) return std::max(best, y0 + ly);
        return best;
    }
    const int32_t cs = size >> 2;
    for (int sy = 3; sy >= 0; sy--) {
        if (y0 + (sy + 1) * cs - 1 <= best) break;
        for (int sz = 0; sz < 4; sz++)
            for (int sx = 0; sx < 4; sx++) {
                const uint32_t sl = (uint32_t)((sz << 4) | (sy << 2) | sx);
                if (!((n.mask >> sl) & 1ull)) continue;
                const uint32_t ci = n.ref + (uint32_t)__builtin_popcountll(n.mask & ((1ull << sl) - 1ull));
                best = top_y_of(t, ci, y0 + sy * cs, depth + 1, best);
            }
    }
    return best;
}
}  // namespace

int32_t svo::tree_top_y(const svo_tree* t) {
    std::lock_guard<std::mutex> lock(t->top_mu);
    if (!t->top_valid) {
        t->top_y = t->nodes.empty() ? -1 : top_y_of(t, 0, 0, 0, -1);
        t->top_valid = true;
    }
    return t->top_y;
}

// Column ceilings: one walk over the tree fills the finest level (blocks of 4^kCeilK0 columns) with
// the highest stored row over each block, then coarser levels take maxima of 4 x 4 blocks.
namespace {
struct CeilWalk {
    const svo_tree* t;
    int32_t bsh;   // log2 of the finest block's width
    int64_t rows;  // finest blocks per row
    int16_t* top;
    void put(int64_t bx, int64_t bz, int32_t y) {
        int16_t& c = top[bz * rows + bx];
        if (y > c) c = (int16_t)y;
    }
    // region of node ni: [x0, x0 + size) x [y0, ..) x [z0, ..)
    void walk(uint32_t ni, int32_t x0, int32_t y0, int32_t z0, int depth) {
        const Node& n = t->nodes[ni];
        const int32_t size = 1 << (2 * (t->levels - depth));
        const uint32_t kind = node_kind(n.info);
        if (kind == K_SOLID) {
            const int64_t nb = std::max<int64_t>(1, (int64_t)size >> bsh);
            for (int64_t bz = 0; bz < nb; bz++)
                for (int64_t bx = 0; bx < nb; bx++) put(((int64_t)x0 >> bsh) + bx, ((int64_t)z0 >> bsh) + bz, y0 + size - 1);
            return;
        }
        if (kind == K_BRICK) {
            for (int ly = 3; ly >= 0; ly--)
                if (n.mask & (0x000F000F000F000Full << (4 * ly))) {
                    put((int64_t)x0 >> bsh, (int64_t)z0 >> bsh, y0 + ly);
                    break;
                }
            return;
        }
        const int32_t cs = size >> 2;
        uint64_t m = n.mask;
        uint32_t ci = n.ref;
        while (m) {
            const uint32_t sl = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            walk(ci++, x0 + (int32_t)(sl & 3u) * cs, y0 + (int32_t)((sl >> 2) & 3u) * cs, z0 + (int32_t)(sl >> 4) * cs, depth + 1);
        }
    }
};
}  // namespace

int32_t svo::tree_ceilings(const svo_tree* t, std::vector<int16_t>& out, int64_t off[kCeilMax]) {
    out.clear();
    const int32_t nlev = std::min<int32_t>(kCeilMax, t->levels - kCeilK0);
    if (nlev <= 0 || t->nodes.empty()) return 0;
    int64_t total = 0;
    for (int32_t j = 0; j < nlev; j++) {
        const int64_t rows = (int64_t)1 << (2 * (t->levels - kCeilK0 - j));
        off[j] = total;
        total += rows * rows;
    }
    out.assign((size_t)total, (int16_t)-1);
    CeilWalk cw{t, 2 * kCeilK0, (int64_t)1 << (2 * (t->levels - kCeilK0)), out.data()};
    const Node& root = t->nodes[0];
    if (node_kind(root.info) != K_INTERIOR) {
        cw.walk(0, 0, 0, 0, 0);
    } else {
        // the root's children by column (x, z slot): each thread walks the four children over one
        // quarter x quarter of the columns, so the blocks it writes are its own
        const int32_t cs = 1 << (2 * (t->levels - 1));
        auto quadrant = [&, cs](uint32_t xz) {
            CeilWalk w = cw;
            for (uint32_t y = 0; y < 4; y++) {
                const uint32_t sl = ((xz >> 2) << 4) | (y << 2) | (xz & 3u);
                if (!((root.mask >> sl) & 1ull)) continue;
                const uint32_t ci = root.ref + (uint32_t)__builtin_popcountll(root.mask & ((1ull << sl) - 1ull));
                w.walk(ci, (int32_t)(xz & 3u) * cs, (int32_t)y * cs, (int32_t)(xz >> 2) * cs, 1);
            }
        };
        std::vector<std::thread> th;
        uint32_t started = 0;
        try {
            for (; started < 16; started++) th.emplace_back(quadrant, started);
        } catch (const std::system_error&) {
            // (no more threads: the quadrants not started are walked here)
        }
        for (uint32_t xz = started; xz < 16; xz++) quadrant(xz);
        for (auto& x : th) x.join();
    }
    ceilings_coarsen(t, out, off, nlev, 0, 0, (int64_t)1 << (2 * t->levels), (int64_t)1 << (2 * t->levels));
    return nlev;
}

// levels 1 .. nlev-1 as 4 x 4 maxima of the finer level, over the blocks that hold columns [x0, x1) x [z0, z1)
void svo::ceilings_coarsen(const svo_tree* t, std::vector<int16_t>& out, const int64_t off[kCeilMax], int32_t nlev, int64_t x0, int64_t z0,
                           int64_t x1, int64_t z1) {
    for (int32_t j = 1; j < nlev; j++) {
        const int32_t bsh = 2 * (kCeilK0 + j);
        const int64_t rows = (int64_t)1 << (2 * (t->levels - kCeilK0 - j)), fine = rows * 4;
        const int16_t* f = out.data() + off[j - 1];
        int16_t* c = out.data() + off[j];
        for (int64_t bz = z0 >> bsh; bz < std::min(rows, ((z1 - 1) >> bsh) + 1); bz++)
            for (int64_t bx = x0 >> bsh; bx < std::min(rows, ((x1 - 1) >> bsh) + 1); bx++) {
                int16_t v = -1;
                for (int64_t dz = 0; dz < 4; dz++)
                    for (int64_t dx = 0; dx < 4; dx++) v = std::max(v, f[(bz * 4 + dz) * fine + bx * 4 + dx]);
                c[bz * rows + bx] = v;
            }
    }
}

// The finest level over the columns [x0, x1) x [z0, z1) (aligned to the finest blocks) recomputed from the tree: the
// blocks are cleared, then a walk that enters only the nodes whose columns meet the rectangle raises them again.
namespace {
struct CeilRectWalk {
    CeilWalk cw;
    int64_t x0, z0, x1, z1;
    void walk(uint32_t ni, int64_t nx, int32_t ny, int64_t nz, int depth) {
        const svo_tree* t = cw.t;
        const Node& n = t->nodes[ni];
        const int64_t size = (int64_t)1 << (2 * (t->levels - depth));
        const uint32_t kind = node_kind(n.info);
        if (kind == K_SOLID) {
            const int32_t bsh = cw.bsh;
            const int64_t ax = std::max(nx, x0), bx = std::min(nx + size, x1), az = std::max(nz, z0), bz = std::min(nz + size, z1);
            for (int64_t z = az >> bsh; z <= (bz - 1) >> bsh; z++)
                for (int64_t x = ax >> bsh; x <= (bx - 1) >> bsh; x++) cw.put(x, z, ny + (int32_t)size - 1);
            return;
        }
        if (kind == K_BRICK) {
            cw.walk(ni, (int32_t)nx, ny, (int32_t)nz, depth);
            return;
        }
        const int64_t cs = size >> 2;
        uint64_t m = n.mask;
        uint32_t ci = n.ref;
        while (m) {
            const uint32_t sl = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            const int64_t cx = nx + (int64_t)(sl & 3u) * cs, cz = nz + (int64_t)(sl >> 4) * cs;
            const uint32_t c = ci++;
            if (cx >= x1 || cx + cs <= x0 || cz >= z1 || cz + cs <= z0) continue;
            walk(c, cx, ny + (int32_t)((sl >> 2) & 3u) * (int32_t)cs, cz, depth + 1);
        }
    }
};
}  // namespace

void svo::ceilings_update_rect(const svo_tree* t, std::vector<int16_t>& out, const int64_t off[kCeilMax], int32_t nlev, int64_t x0,
                               int64_t z0, int64_t x1, int64_t z1) {
    if (nlev <= 0 || t->nodes.empty()) return;
    const int32_t bsh = 2 * kCeilK0;
    const int64_t rows = (int64_t)1 << (2 * (t->levels - kCeilK0));
    x0 = (x0 >> bsh) << bsh;
    z0 = (z0 >> bsh) << bsh;
    x1 = (((x1 - 1) >> bsh) + 1) << bsh;
    z1 = (((z1 - 1) >> bsh) + 1) << bsh;
    for (int64_t bz = z0 >> bsh; bz < z1 >> bsh; bz++)
        for (int64_t bx = x0 >> bsh; bx < x1 >> bsh; bx++) out[off[0] + bz * rows + bx] = -1;
    CeilRectWalk w{CeilWalk{t, bsh, rows, out.data() + off[0]}, x0, z0, x1, z1};
    w.walk(0, 0, 0, 0, 0);
    ceilings_coarsen(t, out, off, nlev, x0, z0, x1, z1);
}

extern "C" int svo_tree_ceilings(const svo_tree* t, int16_t* out, int64_t cap, int32_t* levels, int64_t* n) {
    if (!t || !levels || !n) SVO_FAIL(SVO_EINVAL, "svo_tree_ceilings: NULL argument");
    std::vector<int16_t> c;
    int64_t off[kCeilMax] = {0, 0, 0, 0};
    *levels = tree_ceilings(t, c, off);
    *n = (int64_t)c.size();
    if (out) {
        if (cap < *n) SVO_FAIL(SVO_ERANGE, "svo_tree_ceilings: buffer too small");
        if (!c.empty()) memcpy(out, c.data(), c.size() * sizeof(int16_t));
    }
    return SVO_OK;
}

extern "C" int svo_tree_node_indices(const svo_tree* t, const int32_t* xyz, int64_t n, uint64_t* idx) {
    if (!t || ((!xyz || !idx) && n > 0)) SVO_FAIL(SVO_EINVAL, "svo_tree_node_indices: NULL argument");
    const uint32_t mk = (1u << (2 * t->levels)) - 1u;
    for (int64_t i = 0; i < n; i++) {
        const uint32_t wx = (uint32_t)xyz[3 * i] & mk, wy = (uint32_t)xyz[3 * i + 1] & mk, wz = (uint32_t)xyz[3 * i + 2] & mk;
        uint32_t ni = 0;
        for (int d = 0; d < t->levels; d++) {
            const Node& nd = t->nodes[ni];
            if (node_kind(nd.info) != K_INTERIOR) break;
            const uint32_t sl = child_slot(wx, wy, wz, (uint32_t)(2 * (t->levels - 1 - d)));
            if (!((nd.mask >> sl) & 1ull)) break;
            ni = nd.ref + (uint32_t)__builtin_popcountll(nd.mask & ((1ull << sl) - 1ull));
        }
        idx[i] = ni;
    }
    return SVO_OK;
}

extern "C" int svo_tree_export(const svo_tree* t, void* nodes, uint64_t nb, void* mats, uint64_t mb) {
    if (!t) SVO_FAIL(SVO_EINVAL, "svo_tree_export: NULL tree");
    if (nodes) {
        if (nb < t->nodes.size() * sizeof(Node)) SVO_FAIL(SVO_ERANGE, "svo_tree_export: node buffer too small");
        memcpy(nodes, t->nodes.data(), t->nodes.size() * sizeof(Node));
    }
    if (mats) {
        if (mb < t->mats.size() * sizeof(uint16_t)) SVO_FAIL(SVO_ERANGE, "svo_tree_export: material buffer too small");
        memcpy(mats, t->mats.data(), t->mats.size() * sizeof(uint16_t));
    }
    return SVO_OK;
}

// ================================================================================================
// Checkpoint: svo_tree_save / svo_tree_load
//   header  "SVOTREE1" | u32 format 1 | i32 levels | i32 view | u32 n_palette | u64 n_nodes | u64 n_mats |
//           u64 n_bricks | u64 nodes_per_level[8]
//   palette n_palette x {u32 flags, u32 0, u64 color, f32 meta, u32 0}
//   nodes   n_nodes x 16 B, mats n_mats x 2 B, then u64 FNV-1a of everything before it
// ================================================================================================
namespace {
struct Fnv {
    uint64_t h = 1469598103934665603ull;
    void add(const void* p, size_t n) {
        const uint8_t* b = static_cast<const uint8_t*>(p);
        for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
    }
};
struct FileOut {
    FILE* f;
    Fnv sum;
    bool ok = true;
    void put(const void* p, size_t n) {
        if (n && fwrite(p, 1, n, f) != n) ok = false;
        sum.add(p, n);
    }
};
struct FileIn {
    FILE* f;
    Fnv sum;
    bool get(void* p, size_t n) {
        if (n && fread(p, 1, n, f) != n) return false;
        sum.add(p, n);
        return true;
    }
};
const char kMagic[8] = {'S', 'V', 'O', 'T', 'R', 'E', 'E', '1'};
}  // namespace

extern "C" int svo_tree_save(const svo_tree* t, const char* path) {
    if (!t || !path) SVO_FAIL(SVO_EINVAL, "svo_tree_save: NULL argument");
    FileOut o{fopen(path, "wb")};
    if (!o.f) SVO_FAIL(SVO_EIO, std::string("svo_tree_save: cannot open ") + path);
    const uint32_t fmt = 1, npal = (uint32_t)t->palette.size();
    const uint64_t nn = t->nodes.size(), nm = t->mats.size(), nb = t->n_bricks;
    o.put(kMagic, 8);
    o.put(&fmt, 4);
    o.put(&t->levels, 4);
    o.put(&t->view, 4);
    o.put(&npal, 4);
    o.put(&nn, 8);
    o.put(&nm, 8);
    o.put(&nb, 8);
    o.put(t->nodes_per_level, sizeof(t->nodes_per_level));
    for (const Material& m : t->palette) {
        const uint32_t z = 0;
        o.put(&m.flags, 4);
        o.put(&z, 4);
        o.put(&m.color, 8);
        o.put(&m.meta, 4);
        o.put(&z, 4);
    }
    o.put(t->nodes.data(), nn * sizeof(Node));
    o.put(t->mats.data(), nm * sizeof(uint16_t));
    const uint64_t h = o.sum.h;
    o.put(&h, 8);
    const bool closed = fclose(o.f) == 0;
    if (!o.ok || !closed) SVO_FAIL(SVO_EIO, std::string("svo_tree_save: write failed: ") + path);
    return SVO_OK;
}

extern "C" int svo_tree_load(const char* path, svo_tree** out) {
    if (!path || !out) SVO_FAIL(SVO_EINVAL, "svo_tree_load: NULL argument");
    *out = nullptr;
    FileIn in{fopen(path, "rb")};
    if (!in.f) SVO_FAIL(SVO_EIO, std::string("svo_tree_load: cannot open ") + path);
    struct Closer {
        FILE* f;
        ~Closer() { fclose(f); }
    } closer{in.f};
    char magic[8];
    uint32_t fmt = 0, npal = 0;
    int32_t levels = 0, view = 0;
    uint64_t nn = 0, nm = 0, nb = 0, per[8];
    if (!in.get(magic, 8) || memcmp(magic, kMagic, 8) != 0) SVO_FAIL(SVO_EIO, "svo_tree_load: not a tree file");
    if (!in.get(&fmt, 4) || fmt != 1) SVO_FAIL(SVO_EIO, "svo_tree_load: unknown format");
    if (!in.get(&levels, 4) || !in.get(&view, 4) || !in.get(&npal, 4) || !in.get(&nn, 8) || !in.get(&nm, 8) || !in.get(&nb, 8) ||
        !in.get(per, sizeof(per)))
        SVO_FAIL(SVO_EIO, "svo_tree_load: truncated header");
    if (levels < 1 || levels > 7 || (view != SVO_VIEW_SOLID && view != SVO_VIEW_ALL) || npal < 1 || npal > 0xFFFFu || nn < 1 ||
        nn > 0xFFFFFFFFull || nm > 0xFFFFFFFFull)
        SVO_FAIL(SVO_EIO, "svo_tree_load: header out of range");
    std::unique_ptr<svo_tree> t(new (std::nothrow) svo_tree());
    if (!t) SVO_FAIL(SVO_ENOMEM, "svo_tree_load: out of memory");
    t->levels = levels;
    t->view = view;
    t->n_bricks = nb;
    memcpy(t->nodes_per_level, per, sizeof(per));
    t->palette.resize(npal);
    for (Material& m : t->palette) {
        uint32_t z0, z1;
        if (!in.get(&m.flags, 4) || !in.get(&z0, 4) || !in.get(&m.color, 8) || !in.get(&m.meta, 4) || !in.get(&z1, 4))
            SVO_FAIL(SVO_EIO, "svo_tree_load: truncated palette");
    }
    try {
        t->nodes.resize(nn);
        t->mats.resize(nm);
    } catch (...) {
        SVO_FAIL(SVO_ENOMEM, "svo_tree_load: out of memory");
    }
    if (!in.get(t->nodes.data(), nn * sizeof(Node)) || !in.get(t->mats.data(), nm * sizeof(uint16_t)))
        SVO_FAIL(SVO_EIO, "svo_tree_load: truncated arrays");
    const uint64_t want = in.sum.h;
    uint64_t h = 0;
    if (fread(&h, 1, 8, in.f) != 8 || h != want) SVO_FAIL(SVO_EIO, "svo_tree_load: checksum mismatch");
    // every reference inside the arrays: what the kernels will follow
    for (uint64_t i = 0; i < nn; i++) {
        const Node& n = t->nodes[i];
        const uint32_t kind = node_kind(n.info);
        const uint64_t cnt = (uint64_t)__builtin_popcountll(n.mask);
        if (kind == K_INTERIOR) {
            if (cnt && ((uint64_t)n.ref + cnt > nn || n.ref == 0)) SVO_FAIL(SVO_EIO, "svo_tree_load: child reference out of range");
        } else if (kind == K_BRICK) {
            if (n.info & K_UNIFORM) {
                if (node_material(n.info) >= npal) SVO_FAIL(SVO_EIO, "svo_tree_load: material out of range");
            } else if ((uint64_t)n.ref + cnt > nm) {
                SVO_FAIL(SVO_EIO, "svo_tree_load: material run out of range");
            }
        } else if (kind == K_SOLID) {
            if (node_material(n.info) >= npal) SVO_FAIL(SVO_EIO, "svo_tree_load: material out of range");
        } else {
            SVO_FAIL(SVO_EIO, "svo_tree_load: unknown node kind");
        }
    }
    for (uint64_t i = 0; i < nm; i++)
        if (t->mats[i] >= npal) SVO_FAIL(SVO_EIO, "svo_tree_load: material out of range");
    // the structure the kernels assume, walked down from the root with the depth: INTERIOR nodes only
    // above the brick level, BRICK nodes only at it (levels - 1), SOLID anywhere, and every node reached
    // at most once (no cycles, no shared subtrees).  Blocks superseded by edits (svo_tree_update) are
    // unreachable and are not visited.
    try {
        std::vector<uint64_t> seen((nn + 63) / 64, 0ull);
        std::vector<std::pair<uint32_t, int32_t>> stack{{0u, 0}};
        seen[0] |= 1ull;
        while (!stack.empty()) {
            const uint32_t ni = stack.back().first;
            const int32_t depth = stack.back().second;
            stack.pop_back();
            const Node& n = t->nodes[ni];
            const uint32_t kind = node_kind(n.info);
            if (kind == K_BRICK && depth != levels - 1) SVO_FAIL(SVO_EIO, "svo_tree_load: brick node above the brick level");
            if (kind != K_INTERIOR) continue;
            if (depth >= levels - 1) SVO_FAIL(SVO_EIO, "svo_tree_load: interior node at the brick level");
            const uint32_t cnt = (uint32_t)__builtin_popcountll(n.mask);
            for (uint32_t c = 0; c < cnt; c++) {
                const uint32_t ci = n.ref + c;  // (in range: checked above)
                if ((seen[ci >> 6] >> (ci & 63u)) & 1ull) SVO_FAIL(SVO_EIO, "svo_tree_load: node reached twice (cycle or shared subtree)");
                seen[ci >> 6] |= 1ull << (ci & 63u);
                stack.push_back({ci, depth + 1});
            }
        }
    } catch (const std::bad_alloc&) {
        SVO_FAIL(SVO_ENOMEM, "svo_tree_load: out of memory");
    }
    *out = t.release();
    return SVO_OK;
}

// ================================================================================================
// Host helpers (the same code the kernel runs)
// ================================================================================================
extern "C" int svo_proj_plane(int32_t width, int32_t height, float* ppx, float* ppy) {
    if (width <= 0 || height <= 0 || !ppx || !ppy) SVO_FAIL(SVO_EINVAL, "svo_proj_plane: bad argument");
    // main.cpp:94: glm::tan(glm::radians(45.0)) in double, then the float uniforms
    const double t = tan(45.0 * 0.01745329251994329576923690768489);
    *ppx = (float)t;
    *ppy = (float)(t * (double)(float)height / (double)width);
    return SVO_OK;
}

extern "C" int svo_normalize(const float v[3], float o[3]) {
    if (!v || !o) SVO_FAIL(SVO_EINVAL, "svo_normalize: NULL argument");
    normalize3(v, o);
    return SVO_OK;
}

extern "C" int svo_pixel_dir(const float cam[3], float ppx, float ppy, int32_t w, int32_t h, int32_t px, int32_t py, float o[3]) {
    if (!cam || !o || w <= 0 || h <= 0) SVO_FAIL(SVO_EINVAL, "svo_pixel_dir: bad argument");
    RayGen g;
    raygen_init(g, cam, ppx, ppy, w, h);
    raygen_pixel(g, px, py, o);
    return SVO_OK;
}

extern "C" int svo_pixel_dirs(const float cam[3], float ppx, float ppy, int32_t w, int32_t h, float* out) {
    if (!cam || !out || w <= 0 || h <= 0) SVO_FAIL(SVO_EINVAL, "svo_pixel_dirs: bad argument");
    RayGen g;
    raygen_init(g, cam, ppx, ppy, w, h);
    parallel_for(h, 0, [&](int64_t b, int64_t e) {
        for (int64_t py = b; py < e; py++)
            for (int32_t px = 0; px < w; px++) raygen_pixel(g, px, (int32_t)py, out + 3 * ((size_t)py * w + px));
    });
    return SVO_OK;
}

extern "C" int svo_hemisphere(int32_t n, float* out) {
    if (n < 0 || n > 64 || (!out && n > 0)) SVO_FAIL(SVO_EINVAL, "svo_hemisphere: n must be in [0, 64]");
    hemisphere_table(n, out);
    return SVO_OK;
}

extern "C" int svo_noise2(int64_t seed, const double* x, const double* y, int64_t n, double* out) {
    if ((!x || !y || !out) && n > 0) SVO_FAIL(SVO_EINVAL, "svo_noise2: NULL argument");
    Simplex2 s;
    simplex2_seed(s, seed);
    for (int64_t i = 0; i < n; i++) out[i] = simplex2_eval(s.perm, x[i], y[i]);
    return SVO_OK;
}

extern "C" int svo_terrain_heights(int32_t width, int32_t length, int32_t nthreads, int32_t* out) {
    if (width < 0 || length < 0 || (!out && (int64_t)width * length > 0)) SVO_FAIL(SVO_EINVAL, "svo_terrain_heights: bad argument");
    Simplex2 n42, n64, n100;
    simplex2_seed(n42, 42);
    simplex2_seed(n64, 64);
    simplex2_seed(n100, 100);
    parallel_for(width, nthreads, [&](int64_t b, int64_t e) {
        for (int64_t x = b; x < e; x++)
            for (int32_t z = 0; z < length; z++) out[(size_t)x * length + z] = terrain_height(n42.perm, n64.perm, n100.perm, (int32_t)x, z);
    });
    return SVO_OK;
}

extern "C" int svo_get_blocks(const svo_world* w, const int32_t* xyz, int64_t n, svo_block* out) {
    if (!w || ((!xyz || !out) && n > 0)) SVO_FAIL(SVO_EINVAL, "svo_get_blocks: NULL argument");
    for (int64_t i = 0; i < n; i++) {
        int rc = svo_get_block(w, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], &out[i]);
        if (rc) return rc;
    }
    return SVO_OK;
}

extern "C" int svo_put_blocks(svo_world* w, const int32_t* xyz, const svo_block* b, int64_t n, int32_t level) {
    if (!w || ((!xyz || !b) && n > 0)) SVO_FAIL(SVO_EINVAL, "svo_put_blocks: NULL argument");
    for (int64_t i = 0; i < n; i++) {
        int rc = svo_put_block(w, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], &b[i], level);
        if (rc) return rc;
    }
    return SVO_OK;
}

extern "C" int svo_tree_get_blocks(const svo_tree* t, const int32_t* xyz, int64_t n, uint32_t* ids) {
    if (!t || ((!xyz || !ids) && n > 0)) SVO_FAIL(SVO_EINVAL, "svo_tree_get_blocks: NULL argument");
    for (int64_t i = 0; i < n; i++) {
        svo_block b;
        int rc = svo_tree_get_block(t, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], &b, &ids[i]);
        if (rc) return rc;
    }
    return SVO_OK;
}

// frames of a frame-mode desc (validated: 1 .. SVO_MAX_FRAMES, origins given for more than one)
static int desc_frames(const svo_cast_desc* d, const char* fn, int32_t* nf) {
    *nf = d->n_frames <= 1 ? 1 : d->n_frames;
    if (d->n_frames < 0 || d->n_frames > SVO_MAX_FRAMES) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": n_frames outside [0, SVO_MAX_FRAMES]");
    if (d->n_frames > 1 && !d->frame_origins) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": n_frames > 1 without frame_origins");
    return SVO_OK;
}

extern "C" int svo_cast_blocks(const svo_cast_desc* d, int64_t* n) {
    if (!d || !n) SVO_FAIL(SVO_EINVAL, "svo_cast_blocks: NULL argument");
    if (d->ray_dirs) {
        *n = d->n_rays > 0 ? ((int64_t)d->n_rays + 63) / 64 : 0;
        return SVO_OK;
    }
    if (d->width <= 0 || d->height <= 0 || d->tile_row_step <= 0 || d->tile_row_start < 0)
        SVO_FAIL(SVO_EINVAL, "svo_cast_blocks: bad frame geometry");
    int32_t nf = 1;
    int rc = desc_frames(d, "svo_cast_blocks", &nf);
    if (rc) return rc;
    const int32_t tile_rows = (d->height + 7) / 8;
    const int64_t rows = d->tile_row_start < tile_rows ? (tile_rows - d->tile_row_start + d->tile_row_step - 1) / d->tile_row_step : 0;
    const int32_t lh = svo::frame_wave_lh(d->flags), cols = svo::frame_wave_cols(d->width, lh);
    *n = (rows + svo::frame_half_rows((int32_t)rows, d->flags, lh, cols, nf)) * cols * nf;
    return SVO_OK;
}

extern "C" int svo_cast_count(const svo_cast_desc* d, int64_t* n) {
    if (!d || !n) SVO_FAIL(SVO_EINVAL, "svo_cast_count: NULL argument");
    if (d->ray_dirs) {
        *n = d->n_rays;
        return SVO_OK;
    }
    if (d->width <= 0 || d->height <= 0 || d->tile_row_step <= 0 || d->tile_row_start < 0)
        SVO_FAIL(SVO_EINVAL, "svo_cast_count: bad frame geometry");
    int32_t nf = 1;
    int rc = desc_frames(d, "svo_cast_count", &nf);
    if (rc) return rc;
    const int32_t tile_rows = (d->height + 7) / 8;
    int64_t rows = 0;
    for (int32_t r = d->tile_row_start; r < tile_rows; r += d->tile_row_step) rows += std::min(8, d->height - r * 8);
    *n = rows * d->width * nf;
    return SVO_OK;
}
