// Host code of libsvo_rt under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 "race detection /
// sanitizers": on host code only — GPU sanitizers are not available on the pool).  Built and run by
// tests/test_sanitizers.py from raytracing_test_amd/csrc/svo_world.cpp: world edits, every builder in
// both views, incremental updates (patch, growth, rebuild), lookups, export and the checkpoint round trip.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/svo_rt.h"
#include "../../raytracing_test_amd/csrc/svo_internal.h"

// the device half of the library (svo_cast.hip) is not built here: a tree is only ever host-side
extern "C" void svo_tree_destroy(svo_tree* t) { delete t; }

#define CHECK(x)                                                              \
    do {                                                                      \
        int rc_ = (x);                                                        \
        if (rc_) {                                                            \
            fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, svo_last_error()); \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

static void probe(const svo_tree* t, int n, unsigned seed) {
    std::vector<int32_t> xyz(3 * n);
    for (int i = 0; i < 3 * n; i++) xyz[i] = (int32_t)((seed = seed * 1103515245u + 12345u) >> 8) % 2048 - 512;
    std::vector<uint32_t> ids(n);
    std::vector<uint64_t> idx(n);
    CHECK(svo_tree_get_blocks(t, xyz.data(), n, ids.data()));
    CHECK(svo_tree_node_indices(t, xyz.data(), n, idx.data()));
}

int main(int argc, char** argv) {
    const char* ckpt = argc > 1 ? argv[1] : "/tmp/sanitize_tree.svo";
    svo_world* w = nullptr;
    CHECK(svo_world_create(5, &w));
    CHECK(svo_init_tetra_hexa_tree(w));
    CHECK(svo_gen_world(w, 200, 200));
    for (int view = 0; view < 2; view++) {
        svo_tree* t = nullptr;
        CHECK(svo_build_view(w, view, &t));
        probe(t, 20000, 7 + view);
        // edits: voxels, 4^3 blocks, deletes, far away (wrap), then enough to force a rebuild
        unsigned s = 99;
        for (int round = 0; round < 6; round++) {
            std::vector<int32_t> xyz;
            for (int i = 0; i < 40; i++) {
                s = s * 1664525u + 1013904223u;
                xyz.push_back((int32_t)(s >> 8) % 260 - 20);
                xyz.push_back((int32_t)(s >> 16) % 80);
                xyz.push_back((int32_t)(s >> 4) % 260 - 20);
            }
            const int level = round % 3 == 2 ? 5 : 6;
            for (size_t i = 0; i < xyz.size() / 3; i++) {
                if (round % 2) {
                    svo_block removed;
                    CHECK(svo_delete_block(w, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], level, &removed));
                } else {
                    const svo_block b{(uint32_t)(i % 3 == 0 ? 0x14 : 0x2), 12345u + i, 0.0f};
                    CHECK(svo_put_block(w, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], &b, level));
                }
            }
            CHECK(svo_tree_update(t, w, xyz.data(), (int64_t)(xyz.size() / 3), level));
            probe(t, 5000, s);
        }
        svo_tree_info info;
        CHECK(svo_tree_get_info(t, &info));
        std::vector<uint8_t> nodes(info.n_nodes * 16), mats(info.n_mat_bytes + 2);
        CHECK(svo_tree_export(t, nodes.data(), nodes.size(), mats.data(), mats.size()));
        CHECK(svo_tree_save(t, ckpt));
        svo_tree* u = nullptr;
        CHECK(svo_tree_load(ckpt, &u));
        probe(u, 5000, 3);
        svo_tree_destroy(u);
        svo_tree_destroy(t);
    }
    svo_world_destroy(w);
    // the column builders, both views, ragged widths, and the heightfield builder
    for (int view = 0; view < 2; view++) {
        svo_tree* t = nullptr;
        CHECK(svo_build_terrain_view(5, 300, 170, 4, view, &t));
        probe(t, 20000, 11);
        svo_tree_destroy(t);
    }
    std::vector<int32_t> h(97 * 33);
    for (size_t i = 0; i < h.size(); i++) h[i] = (int32_t)(((uint32_t)(i * 2654435761u) >> 7) % 60u);
    svo_tree* t = nullptr;
    CHECK(svo_build_heightfield(4, 97, 33, h.data(), 3, &t));
    probe(t, 5000, 5);
    svo_tree_destroy(t);
    // error paths return codes (no exits, no leaks)
    svo_world* bad = nullptr;
    if (svo_world_create(9, &bad) == 0) return 1;
    if (svo_tree_load("/nonexistent/file.svo", &t) != SVO_EIO) return 1;
    float out[3];
    const float v[3] = {1.0f, -0.45f, 1.0f};
    CHECK(svo_normalize(v, out));
    printf("host sanitize ok\n");
    return 0;
}
