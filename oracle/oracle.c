/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the product
 * (raytracing_test_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * it, and only as the checker / the timed CPU baseline.
 *
 * A clean-room CPU restatement (plain C11) of the hot path of reedthorngag/raytracing_test
 * (reference snapshot under /root/reference; paths below are relative to it):
 *
 *   - reference node / child-array pools, 4 MiB blocks   src/voxel_data/voxel_allocator.{hpp,cpp}
 *   - Node / Branch / Leaf encoding (16 B)               src/voxel_data/types.hpp:29-47
 *   - initTetraHexaTree (incl. the root-array aliasing)  src/voxel_data/tetrahexa_tree.cpp:13-41
 *   - getBlock                                           src/voxel_data/tetrahexa_tree.cpp:113-157
 *   - putBlock / deleteChildren                          src/voxel_data/tetrahexa_tree.cpp:159-291
 *   - genWorld (generalised to W x L)                    src/world_gen.cpp:13-42
 *   - OpenSimplex 2D (seed permutation, eval, extrap.)   include/OpenSimplexNoise.cpp:52-208,2518-2523
 *   - RGB_TO_U64 material colour packing                 src/types.hpp:6-9
 *   - buildRay + castRayFromCam (FP64 voxel DDA)         src/ray_caster.cpp:19-87
 *   - per-pixel primary ray generation                   src/shaders/low_res.frag:264-288, src/main.cpp:94
 *   - common-ancestor restart traffic model (E_child)    src/shaders/low_res.frag:493-531
 *   - shading over castRayFromCam hits (svo_shade_rays)  src/shaders/low_res.frag:139-252,319-391
 *
 * Parity pinning: the reference's GL/GLM/Win32-dependent translation units are unbuildable in this
 * image (no GLM, GLEW, GLFW or windows.h; stand-in headers are not allowed).  Only
 * include/OpenSimplexNoise.cpp builds from its own sources; oracle/Makefile compiles it into
 * oracle/_ref/ and tests pin orc_noise2() against it bit-for-bit.  The tree / DDA restatement is
 * pinned by the reference's own test.cpp known-answer vector and the structural facts recorded in
 * SURVEY.md (node/array counts, root bitmap, wrap behaviour) — see DESIGN.md §Oracle.
 *
 * Build: gcc -O3 -ffp-contract=off (no fast-math): every FP operation below is meant to round
 * exactly as the reference's g++ build (x86-64 SSE2, no FMA contraction) does.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------------------
 * Reference node encoding (types.hpp:29-47): 16 B; word0 = bitmap (branch) or packedColor (leaf),
 * flags at byte 8 (bit 0 = leaf), word3 = children array index (branch) or f32 metadata (leaf).
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
    uint64_t w0;
    uint32_t flags;
    uint32_t w1;
} onode;

typedef struct {
    uint32_t c[64];
} oarray;

/* voxel_allocator.hpp:12-21 — 4 MiB blocks, <=1024 blocks per pool, free lists of 4096 */
#define O_BLOCK_BITS 22
#define O_BLOCK_SIZE (1u << O_BLOCK_BITS)
#define O_MAX_BLOCKS 1024
#define O_FREE_LIST 4096
#define O_FREE_MASK (O_FREE_LIST - 1)

typedef struct {
    int max_depth; /* reference maxDepth (tetrahexa_tree.hpp:6) = levels + 1 */
    uint8_t* node_blocks[O_MAX_BLOCKS];
    uint8_t* array_blocks[O_MAX_BLOCKS];
    uint32_t node_next; /* byte offsets, as nodeNextAllocIndex / arrayNextAllocIndex */
    uint32_t array_next;
    uint32_t node_free[O_FREE_LIST];
    int node_free_pop, node_free_next, node_free_first;
    uint32_t array_free[O_FREE_LIST];
    int array_free_pop, array_free_next, array_free_first;
    uint32_t root;
    int error; /* set instead of the reference's exit(1) */
    uint64_t n_nodes_alloc, n_arrays_alloc;
} otree;

static inline onode* NODE(const otree* t, uint32_t i) {
    uint32_t b = i << 4; /* convertToPtr (voxel_allocator.hpp:93-95) */
    return (onode*)(t->node_blocks[b >> O_BLOCK_BITS] + (b & (O_BLOCK_SIZE - 1)));
}
static inline oarray* ARR(const otree* t, uint32_t i) {
    uint32_t b = i << 8; /* convertToArrayPtr (voxel_allocator.hpp:97-99) */
    return (oarray*)(t->array_blocks[b >> O_BLOCK_BITS] + (b & (O_BLOCK_SIZE - 1)));
}

static void* o_block_alloc(void) {
    /* the reference mallocs uninitialised blocks; calloc keeps runs deterministic (no reference
       path reads a slot before writing it except the aliased root array, restated explicitly) */
    void* p = calloc(1, O_BLOCK_SIZE);
    if (!p) {
        fprintf(stderr, "oracle: out of memory\n");
        abort();
    }
    return p;
}

/* allocNode (voxel_allocator.cpp:24-43) */
static uint32_t o_alloc_node(otree* t) {
    if (t->node_free_pop > 0) {
        t->node_free_pop--;
        uint32_t n = t->node_free[t->node_free_next++];
        t->node_free_next &= O_FREE_MASK;
        return n;
    }
    if (!t->node_blocks[t->node_next >> O_BLOCK_BITS]) t->node_blocks[t->node_next >> O_BLOCK_BITS] = o_block_alloc();
    uint32_t idx = t->node_next >> 4;
    t->node_next += 16;
    t->n_nodes_alloc++;
    return idx;
}

/* freeConsecNodes (voxel_allocator.cpp:84-96) */
static void o_free_consec(otree* t, uint32_t start, int n) {
    if (t->node_free_pop + n > O_FREE_LIST) return;
    t->node_free_pop += n;
    while (n--) {
        t->node_free[t->node_free_first++] = start++;
        t->node_free_first &= O_FREE_MASK;
    }
}

/* allocConsecNodes (voxel_allocator.cpp:68-82) */
static uint32_t o_alloc_consec(otree* t, int n) {
    if ((t->node_next & (O_BLOCK_SIZE - 1)) + ((uint32_t)n << 4) > O_BLOCK_SIZE) {
        o_free_consec(t, t->node_next >> 4, n);
        t->node_next += (uint32_t)n << 4;
        t->node_blocks[t->node_next >> O_BLOCK_BITS] = o_block_alloc();
    }
    if (!t->node_blocks[t->node_next >> O_BLOCK_BITS]) t->node_blocks[t->node_next >> O_BLOCK_BITS] = o_block_alloc();
    uint32_t idx = t->node_next >> 4;
    t->node_next += (uint32_t)n << 4;
    t->n_nodes_alloc += (uint64_t)n;
    return idx;
}

/* allocArray (voxel_allocator.cpp:45-66).  (The free-list branch returns convertToPtr in the
   reference — Appendix A defect; only reachable after deletions, never in static scenes.) */
static uint32_t o_alloc_array(otree* t) {
    if (t->array_free_pop > 0) {
        t->array_free_pop--;
        uint32_t a = t->array_free[t->array_free_next++];
        t->array_free_next &= O_FREE_MASK;
        return a;
    }
    if (!t->array_blocks[t->array_next >> O_BLOCK_BITS]) t->array_blocks[t->array_next >> O_BLOCK_BITS] = o_block_alloc();
    uint32_t idx = t->array_next >> 8;
    t->array_next += 256;
    t->n_arrays_alloc++;
    return idx;
}

static void o_free_node(otree* t, uint32_t i) {
    if (t->node_free_pop >= 1024) return; /* voxel_allocator.hpp:115-124 */
    t->node_free[t->node_free_first++] = i;
    t->node_free_first &= O_FREE_MASK;
    t->node_free_pop++;
}
static void o_free_array(otree* t, uint32_t i) {
    if (t->array_free_pop >= 1024) return;
    t->array_free[t->array_free_first++] = i;
    t->array_free_first &= O_FREE_MASK;
    t->array_free_pop++;
}

/* Pos >> n (types.hpp:11-17): the reference shifts by a negative count at the leaf depth (UB);
   x86 masks the count to 5 bits, which is what a -O0 build executes. */
static inline int o_shr(int v, int n) { return v >> (n & 31); }

static inline int o_child_index(int x, int y, int z, int off) {
    return ((o_shr(z, off) & 3) << 4) | ((o_shr(y, off) & 3) << 2) | (o_shr(x, off) & 3);
}

EXPORT otree* orc_tree_new(int levels) {
    otree* t = (otree*)calloc(1, sizeof(otree));
    t->max_depth = levels + 1;
    return t;
}

EXPORT void orc_tree_free(otree* t) {
    if (!t) return;
    for (int i = 0; i < O_MAX_BLOCKS; i++) {
        free(t->node_blocks[i]);
        free(t->array_blocks[i]);
    }
    free(t);
}

EXPORT int orc_tree_error(const otree* t) { return t->error; }
EXPORT uint64_t orc_tree_nodes(const otree* t) { return t->n_nodes_alloc; }
EXPORT uint64_t orc_tree_arrays(const otree* t) { return t->n_arrays_alloc; }
EXPORT uint64_t orc_root_bitmap(const otree* t) { return NODE(t, t->root)->w0; }
EXPORT uint32_t orc_root_children(const otree* t) { return NODE(t, t->root)->w1; }
EXPORT uint32_t orc_root_flags(const otree* t) { return NODE(t, t->root)->flags; }

/* getBlock (tetrahexa_tree.cpp:113-157).  Returns 0, or -1 where the reference exit(1)s. */
static inline int o_get_block(const otree* t, int x, int y, int z, uint32_t* flags, uint64_t* color, float* meta) {
    int off = (t->max_depth - 1) * 2;
    uint32_t cur = t->root;
    for (int depth = 0; depth < t->max_depth; depth++) {
        off -= 2;
        int idx = o_child_index(x, y, z, off);
        const onode* n = NODE(t, cur);
        if (n->flags & 1) {
            *flags = n->flags;
            *color = n->w0;
            memcpy(meta, &n->w1, 4);
            return 0;
        }
        if (!((n->w0 >> idx) & 1)) {
            *flags = 0;
            *color = ~0ull;
            *meta = 0.0f;
            return 0;
        }
        cur = ARR(t, n->w1)->c[idx];
    }
    return -1;
}

EXPORT int orc_get_block(const otree* t, int x, int y, int z, uint32_t* flags, uint64_t* color, float* meta) {
    return o_get_block(t, x, y, z, flags, color, meta);
}

/* deleteChildren (tetrahexa_tree.cpp:159-173) */
static void o_delete_children(otree* t, uint32_t node) {
    onode* n = NODE(t, node);
    if (n->flags & 1) return;
    oarray* a = ARR(t, n->w1);
    for (int i = 0; i < 64; i++) {
        if (a->c[i]) {
            o_delete_children(t, a->c[i]);
            o_free_node(t, a->c[i]);
        }
    }
    o_free_array(t, n->w1);
}

/* putBlock (tetrahexa_tree.cpp:175-291).  level 6 = one voxel at maxDepth 6. */
EXPORT int orc_put_block(otree* t, int x, int y, int z, uint32_t bflags, uint64_t color, float meta, int level) {
    level--;
    int off = (t->max_depth - 1) * 2;
    uint32_t stack[16];
    int depth = 0;
    stack[0] = t->root;
    uint32_t mbits;
    memcpy(&mbits, &meta, 4);
    while (depth < t->max_depth) {
        off -= 2;
        int idx = o_child_index(x, y, z, off);
        onode* n = NODE(t, stack[depth]);
        if (depth == level) {
            if (!(n->flags & 1)) o_delete_children(t, stack[depth]);
            n->w0 = color;
            n->flags = 1u | bflags;
            n->w1 = mbits;
            return 0;
        } else if (n->flags & 1) {
            /* split a leaf into 64 copies (tetrahexa_tree.cpp:221-247) */
            uint32_t lf = n->flags;
            uint64_t lc = n->w0;
            uint32_t lm = n->w1;
            uint32_t arr = o_alloc_array(t);
            memset(ARR(t, arr), 0, sizeof(oarray));
            uint32_t kids = o_alloc_consec(t, 64);
            for (int i = 0; i < 64; i++) {
                ARR(t, arr)->c[i] = kids + (uint32_t)i;
                onode* k = NODE(t, kids + (uint32_t)i);
                k->flags = lf;
                k->w0 = lc;
                k->w1 = lm;
            }
            n = NODE(t, stack[depth]);
            n->flags = 0;
            n->w0 = ~0ull;
            n->w1 = arr;
            stack[++depth] = ARR(t, arr)->c[idx];
        } else if (!((n->w0 >> idx) & 1)) {
            if (depth + 1 == level) {
                uint32_t leaf = o_alloc_node(t);
                onode* l = NODE(t, leaf);
                l->w0 = color;
                l->flags = 1u | bflags;
                l->w1 = mbits;
                n = NODE(t, stack[depth]);
                n->w0 |= 1ull << idx;
                ARR(t, n->w1)->c[idx] = leaf;
                return 0;
            }
            uint32_t child = o_alloc_node(t);
            uint32_t arr = o_alloc_array(t);
            memset(ARR(t, arr), 0, sizeof(oarray));
            onode* c = NODE(t, child);
            c->w0 = 0;
            c->flags = 0;
            c->w1 = arr;
            n = NODE(t, stack[depth]);
            n->w0 |= 1ull << idx;
            ARR(t, n->w1)->c[idx] = child;
            stack[++depth] = child;
        } else {
            stack[depth + 1] = ARR(t, n->w1)->c[idx];
            depth++;
        }
    }
    t->error = 1; /* reference: "hit max depth" exit(1) */
    return -1;
}

/* deleteBlock (tetrahexa_tree.cpp:293-359): walk to the depth-`level` node (splitting any leaf met
   above it into 64 copies, :309-333), take its block, free it and its subtree (deleteChildren +
   freeNode, :350-351) and clear its bit in the parent's bitmap.  The reference clears that bit with
   the int expression `1 << index` (:352): x86 masks the shift count to 5 bits and the int result is
   sign-extended to the u64 bitmap, so for index >= 31 it flips the wrong bits (index 31: bits 31-63;
   index 32-62: bit index-32).  ref_shift = 1 reproduces that; 0 clears bit `index` (the intended
   meaning, which libsvo_rt implements).  Returns 0, 1 when the position was already empty, or -1
   where the reference exit(1)s. */
EXPORT int orc_delete_block(otree* t, int x, int y, int z, int level, int ref_shift, uint32_t* flags, uint64_t* color, float* meta) {
    int off = (t->max_depth - 1) * 2;
    uint32_t stack[16];
    int depth = 0;
    stack[0] = t->root;
    while (depth < t->max_depth) {
        off -= 2;
        int idx = o_child_index(x, y, z, off);
        onode* n = NODE(t, stack[depth]);
        if (n->flags & 1) {
            uint32_t lf = n->flags;
            uint64_t lc = n->w0;
            uint32_t lm = n->w1;
            uint32_t arr = o_alloc_array(t);
            memset(ARR(t, arr), 0, sizeof(oarray));
            uint32_t kids = o_alloc_consec(t, 64);
            for (int i = 0; i < 64; i++) {
                ARR(t, arr)->c[i] = kids + (uint32_t)i;
                onode* k = NODE(t, kids + (uint32_t)i);
                k->flags = lf;
                k->w0 = lc;
                k->w1 = lm;
            }
            n = NODE(t, stack[depth]);
            n->flags = 0;
            n->w0 = ~0ull; /* bitmap = -1: all set */
            n->w1 = arr;
        } else if (!((n->w0 >> idx) & 1)) {
            *flags = 0;
            *color = ~0ull;
            *meta = 0.0f;
            return 1;
        }
        stack[depth + 1] = ARR(t, NODE(t, stack[depth])->w1)->c[idx];
        depth++;
        if (depth == level) {
            const onode* d = NODE(t, stack[depth]);
            *flags = d->flags;
            *color = d->w0;
            memcpy(meta, &d->w1, 4);
            o_delete_children(t, stack[depth]);
            o_free_node(t, stack[depth]);
            onode* p = NODE(t, stack[depth - 1]);
            if (ref_shift)
                p->w0 ^= (uint64_t)(int64_t)(int32_t)(1u << (idx & 31));
            else
                p->w0 &= ~(1ull << idx);
            return 0;
        }
    }
    t->error = 1; /* "hit max depth without finding leaf node!" exit(1) */
    return -1;
}

/* initTetraHexaTree (tetrahexa_tree.cpp:13-41), including its construction defect: the root's child
   array is taken from the NODE pool (allocConsecNodes(4) -> node index 1) but read through the
   ARRAY pool, i.e. it aliases child array #1 — the second array allocated, zeroed by that
   allocation. */
EXPORT void orc_init_tetra_hexa_tree(otree* t) {
    t->root = o_alloc_node(t);
    uint32_t aliased = o_alloc_consec(t, (int)((sizeof(uint32_t) * 64) / 16));
    /* memset(array.ptr, 0, 256) on node memory (nodes 1..16) — nothing reads those bytes later */
    if (!t->array_blocks[0]) t->array_blocks[0] = o_block_alloc(); /* array block 0 backs index 1 */
    onode* r = NODE(t, t->root);
    r->w0 = 0;
    r->flags = 0;
    r->w1 = aliased;
    const float zero = 0.0f;
    orc_put_block(t, 1000, 1000, 1000, 1, 0, zero, 5);
    orc_put_block(t, 10, 100, 10, 2, 0, zero, 6);
    orc_put_block(t, 100, 10, 100, 3, 0, zero, 6);
    orc_put_block(t, 20, 10, 200, 4, 0, zero, 5);
    orc_put_block(t, 1, 10, 10, 5, 0, zero, 6);
    orc_put_block(t, 2, 10, 10, 6, 0, zero, 6);
    orc_put_block(t, 3, 10, 10, 7, 0, zero, 6);
    orc_put_block(t, 4, 10, 10, 8, 0, zero, 6);
}

/* A clean root (no aliasing) — for worlds the reference cannot build (depth-12/14 terrain). */
EXPORT void orc_init_clean_root(otree* t) {
    t->root = o_alloc_node(t);
    uint32_t arr = o_alloc_array(t);
    memset(ARR(t, arr), 0, sizeof(oarray));
    onode* r = NODE(t, t->root);
    r->w0 = 0;
    r->flags = 0;
    r->w1 = arr;
}

/* ------------------------------------------------------------------------------------------------
 * OpenSimplex 2D — restated from include/OpenSimplexNoise.cpp (a 2019 C++ port of KdotJPG's
 * OpenSimplex gist; vendored in the reference).  Constants are the reference's literals.
 * ---------------------------------------------------------------------------------------------- */
#define OS_STRETCH (-0.211324865405187)
#define OS_SQUISH (0.366025403784439)
#define OS_NORM (47.0)

typedef struct {
    short perm[256];
} onoise;

static const signed char OS_GRAD2[16] = {5, 2, 2, 5, -5, 2, -2, 5, 5, -2, 2, -5, -5, -2, -2, -5};

/* Noise(int64_t seed) (OpenSimplexNoise.cpp:52-75): LCG-driven Fisher-Yates */
static void onoise_seed(onoise* n, int64_t seed) {
    short src[256];
    for (int i = 0; i < 256; i++) src[i] = (short)i;
    const uint64_t A = 6364136223846793005ull, C = 1442695040888963407ull;
    uint64_t s = (uint64_t)seed;
    s = s * A + C;
    s = s * A + C;
    s = s * A + C;
    for (int i = 255; i >= 0; i--) {
        s = s * A + C;
        int64_t q = (int64_t)(s + 31u);
        int r = (int)(q % (int64_t)(i + 1));
        if (r < 0) r += i + 1;
        n->perm[i] = src[r];
        src[r] = src[i];
    }
}

/* extrapolate 2D (OpenSimplexNoise.cpp:2518-2523) */
static inline double onoise_grad(const onoise* n, int xsb, int ysb, double dx, double dy) {
    int g = n->perm[(n->perm[xsb & 0xFF] + ysb) & 0xFF] & 0x0E;
    return (double)OS_GRAD2[g] * dx + (double)OS_GRAD2[g + 1] * dy;
}

/* eval(x, y) (OpenSimplexNoise.cpp:77-208) */
static double onoise_eval(const onoise* n, double x, double y) {
    double so = (x + y) * OS_STRETCH;
    double xs = x + so, ys = y + so;
    int xsb = (int)floor(xs), ysb = (int)floor(ys);
    double sq = (double)(xsb + ysb) * OS_SQUISH;
    double xb = (double)xsb + sq, yb = (double)ysb + sq;
    double xins = xs - (double)xsb, yins = ys - (double)ysb;
    double in_sum = xins + yins;
    double dx0 = x - xb, dy0 = y - yb;
    double dxe, dye;
    int xe, ye;
    double v = 0;

    double dx1 = dx0 - 1 - OS_SQUISH, dy1 = dy0 - 0 - OS_SQUISH;
    double a1 = 2 - dx1 * dx1 - dy1 * dy1;
    if (a1 > 0) {
        a1 *= a1;
        v += a1 * a1 * onoise_grad(n, xsb + 1, ysb + 0, dx1, dy1);
    }
    double dx2 = dx0 - 0 - OS_SQUISH, dy2 = dy0 - 1 - OS_SQUISH;
    double a2 = 2 - dx2 * dx2 - dy2 * dy2;
    if (a2 > 0) {
        a2 *= a2;
        v += a2 * a2 * onoise_grad(n, xsb + 0, ysb + 1, dx2, dy2);
    }
    if (in_sum <= 1) {
        double zins = 1 - in_sum;
        if (zins > xins || zins > yins) {
            if (xins > yins) {
                xe = xsb + 1; ye = ysb - 1; dxe = dx0 - 1; dye = dy0 + 1;
            } else {
                xe = xsb - 1; ye = ysb + 1; dxe = dx0 + 1; dye = dy0 - 1;
            }
        } else {
            xe = xsb + 1; ye = ysb + 1;
            dxe = dx0 - 1 - 2 * OS_SQUISH; dye = dy0 - 1 - 2 * OS_SQUISH;
        }
    } else {
        double zins = 2 - in_sum;
        if (zins < xins || zins < yins) {
            if (xins > yins) {
                xe = xsb + 2; ye = ysb + 0;
                dxe = dx0 - 2 - 2 * OS_SQUISH; dye = dy0 + 0 - 2 * OS_SQUISH;
            } else {
                xe = xsb + 0; ye = ysb + 2;
                dxe = dx0 + 0 - 2 * OS_SQUISH; dye = dy0 - 2 - 2 * OS_SQUISH;
            }
        } else {
            dxe = dx0; dye = dy0; xe = xsb; ye = ysb;
        }
        xsb += 1;
        ysb += 1;
        dx0 = dx0 - 1 - 2 * OS_SQUISH;
        dy0 = dy0 - 1 - 2 * OS_SQUISH;
    }
    double a0 = 2 - dx0 * dx0 - dy0 * dy0;
    if (a0 > 0) {
        a0 *= a0;
        v += a0 * a0 * onoise_grad(n, xsb, ysb, dx0, dy0);
    }
    double ae = 2 - dxe * dxe - dye * dye;
    if (ae > 0) {
        ae *= ae;
        v += ae * ae * onoise_grad(n, xe, ye, dxe, dye);
    }
    return v / OS_NORM;
}

EXPORT double orc_noise2(int64_t seed, double x, double y) {
    onoise n;
    onoise_seed(&n, seed);
    return onoise_eval(&n, x, y);
}

EXPORT void orc_noise_perm(int64_t seed, int16_t* out256) {
    onoise n;
    onoise_seed(&n, seed);
    memcpy(out256, n.perm, sizeof(n.perm));
}

/* ------------------------------------------------------------------------------------------------
 * Terrain (world_gen.cpp:13-42) and materials (types.hpp:6-9, globals.hpp:68-74)
 * ---------------------------------------------------------------------------------------------- */
#define F_REFRACTIVE 0x4u
#define F_LIQUID 0x10u

/* RGB_TO_U64: ((u64)((float)c/255.0 * RGB_RANGE) & RGB_MASK) per channel (types.hpp:6-9) */
static uint64_t o_cs(int c) { return (uint64_t)((double)(float)c / 255.0 * (double)((1 << 21) - 1)) & ((1u << 21) - 1); }
EXPORT uint64_t orc_rgb(int r, int g, int b) { return (o_cs(r) << 42) | (o_cs(g) << 21) | o_cs(b); }

/* column height (world_gen.cpp:22) */
static int o_height(const onoise* n1, const onoise* n2, const onoise* n3, int x, int z) {
    double h = round(onoise_eval(n1, x * 0.005, z * 0.005) * 30) + round(onoise_eval(n2, x * 0.05, z * 0.05) * 5) +
               round(onoise_eval(n3, x * 0.1, z * 0.1) * 3) + 32;
    return (int)h;
}

typedef struct {
    onoise n1, n2, n3;
} oterrain;

static void o_terrain_init(oterrain* T) {
    onoise_seed(&T->n1, 42);
    onoise_seed(&T->n2, 64);
    onoise_seed(&T->n3, 100);
}

/* heights for x in [0,W), z in [0,L); out[x*L + z] */
typedef struct {
    const oterrain* T;
    int W, L, x0, x1;
    int32_t* out;
} o_hjob;
static void* o_height_worker(void* p) {
    o_hjob* j = (o_hjob*)p;
    for (int x = j->x0; x < j->x1; x++)
        for (int z = 0; z < j->L; z++) j->out[(size_t)x * j->L + z] = o_height(&j->T->n1, &j->T->n2, &j->T->n3, x, z);
    return NULL;
}
EXPORT void orc_heights(int W, int L, int32_t* out, int nthreads) {
    oterrain T;
    o_terrain_init(&T);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    o_hjob jobs[64];
    for (int i = 0; i < nthreads; i++) {
        jobs[i] = (o_hjob){&T, W, L, (int)((int64_t)W * i / nthreads), (int)((int64_t)W * (i + 1) / nthreads), out};
        pthread_create(&th[i], NULL, o_height_worker, &jobs[i]);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
}

/* genWorld (world_gen.cpp:13-42) generalised to W x L columns; the reference is W = L = 200. */
EXPORT void orc_gen_world(otree* t, int W, int L) {
    oterrain T;
    o_terrain_init(&T);
    const uint64_t GRASS = orc_rgb(0, 150, 10), DIRT = orc_rgb(45, 18, 0), STONE = orc_rgb(33, 33, 33);
    for (int x = 0; x < W; x++) {
        for (int z = 0; z < L; z++) {
            int y = o_height(&T.n1, &T.n2, &T.n3, x, z);
            if (y < 20) {
                for (int i = 20; i > y; i--) orc_put_block(t, x, i, z, F_REFRACTIVE | F_LIQUID, GRASS, 0.0f, t->max_depth);
                orc_put_block(t, x, y, z, 0, DIRT, 0.0f, t->max_depth);
            } else
                orc_put_block(t, x, y, z, 0, GRASS, 0.0f, t->max_depth);
            y--;
            for (int i = 3; y > 0 && i; i--, y--) orc_put_block(t, x, y, z, 0, DIRT, 0.0f, t->max_depth);
            for (; y > 0; y--) orc_put_block(t, x, y, z, 0, STONE, 0.0f, t->max_depth);
        }
    }
}

/* ------------------------------------------------------------------------------------------------
 * Collapse-builder: builds a reference-format tree (same node / array encoding, leaves allowed at
 * any level as putBlock level<6 makes them) directly from the terrain columns, collapsing uniform
 * regions.  getBlock over it equals getBlock over the putBlock-built tree voxel for voxel (tested);
 * it exists because the reference layout cannot hold depth-12/14 terrain voxel by voxel.
 * Column model for top height h (world_gen.cpp:22-39): water (h, 20] if h < 20; top voxel dirt
 * (h < 20) or grass; 3 dirt below while y > 0; stone down to y = 1.
 * Material codes: 0 air, 1 water, 2 grass, 3 dirt, 4 stone.
 * ---------------------------------------------------------------------------------------------- */
static inline int o_col_mat(int h, int y) {
    if (y == h) return h < 20 ? 3 : 2;
    if (y > h) return (h < 20 && y <= 20) ? 1 : 0;
    if (y <= 0) return 0;
    if (y >= h - 3) return 3;
    return 4;
}

typedef struct {
    otree* t;
    const int32_t* hgt; /* [x*L + z] */
    int W, L;
    uint64_t mcolor[5];
    uint32_t mflags[5];
} ocbuild;

/* uniform material of a region, or -1 when mixed.  Columns outside [0,W)x[0,L) are air. */
static int o_region_uniform(const ocbuild* B, int x0, int y0, int z0, int s) {
    int m = -2;
    for (int x = x0; x < x0 + s; x++) {
        for (int z = z0; z < z0 + s; z++) {
            if (x >= B->W || z >= B->L) { /* no column: air at every height */
                if (m == -2) m = 0;
                else if (m != 0) return -1;
                continue;
            }
            int h = B->hgt[(size_t)x * B->L + z];
            int lo = o_col_mat(h, y0), hi = o_col_mat(h, y0 + s - 1);
            if (lo != hi) return -1;
            /* a column is uniform over [y0, y0+s) iff its materials at both ends agree and no
               boundary lies strictly inside: boundaries sit at 0/1, h-4/h-3, h-1/h, h/h+1, 20/21 */
            int b[5] = {1, h - 3, h, h + 1, 21};
            for (int k = 0; k < 5; k++)
                if (b[k] > y0 && b[k] <= y0 + s - 1) return -1;
            if (m == -2) m = lo;
            else if (m != lo) return -1;
        }
    }
    return m;
}

static void o_cbuild(ocbuild* B, uint32_t node, int x0, int y0, int z0, int s) {
    /* node is a branch with a zeroed child array; fill its 64 children */
    int cs = s / 4;
    for (int i = 0; i < 64; i++) {
        int cx = x0 + (i & 3) * cs, cy = y0 + ((i >> 2) & 3) * cs, cz = z0 + ((i >> 4) & 3) * cs;
        int m = o_region_uniform(B, cx, cy, cz, cs);
        if (m == 0) continue;
        uint32_t c = o_alloc_node(B->t);
        NODE(B->t, node)->w0 |= 1ull << i;
        ARR(B->t, NODE(B->t, node)->w1)->c[i] = c;
        onode* cn = NODE(B->t, c);
        if (m > 0) {
            cn->w0 = B->mcolor[m];
            cn->flags = 1u | B->mflags[m];
            cn->w1 = 0;
        } else {
            uint32_t a = o_alloc_array(B->t);
            memset(ARR(B->t, a), 0, sizeof(oarray));
            cn = NODE(B->t, c);
            cn->w0 = 0;
            cn->flags = 0;
            cn->w1 = a;
            o_cbuild(B, c, cx, cy, cz, cs);
        }
    }
}

/* terrain only (no initTetraHexaTree debug puts); needs W, L <= extent and 0 <= h, max(h,20) < extent-1 */
EXPORT int orc_build_terrain_collapsed(otree* t, const int32_t* heights, int W, int L) {
    int levels = t->max_depth - 1;
    int E = 1 << (2 * levels);
    if (W > E || L > E) return -1;
    for (size_t i = 0; i < (size_t)W * L; i++)
        if (heights[i] < 0 || heights[i] >= E - 1 || 21 >= E) return -2;
    orc_init_clean_root(t);
    ocbuild B;
    B.t = t;
    B.hgt = heights;
    B.W = W;
    B.L = L;
    B.mcolor[0] = ~0ull;
    B.mflags[0] = 0;
    B.mcolor[1] = orc_rgb(0, 150, 10);
    B.mflags[1] = F_REFRACTIVE | F_LIQUID;
    B.mcolor[2] = orc_rgb(0, 150, 10);
    B.mflags[2] = 0;
    B.mcolor[3] = orc_rgb(45, 18, 0);
    B.mflags[3] = 0;
    B.mcolor[4] = orc_rgb(33, 33, 33);
    B.mflags[4] = 0;
    o_cbuild(&B, t->root, 0, 0, 0, E);
    return 0;
}

/* ------------------------------------------------------------------------------------------------
 * Ray generation (low_res.frag:264-288; projPlaneSize main.cpp:94; GLM vector ops, no contraction)
 * ---------------------------------------------------------------------------------------------- */
static inline void o_cross(const float a[3], const float b[3], float o[3]) {
    /* glm::cross */
    o[0] = a[1] * b[2] - b[1] * a[2];
    o[1] = a[2] * b[0] - b[2] * a[0];
    o[2] = a[0] * b[1] - b[0] * a[1];
}
static inline void o_normalize(const float v[3], float o[3]) {
    /* glm::normalize = v * inversesqrt(dot(v, v)); dot = (x*x + y*y) + z*z; inversesqrt = 1/sqrt */
    float d = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
    float r = 1.0f / sqrtf(d);
    o[0] = v[0] * r;
    o[1] = v[1] * r;
    o[2] = v[2] * r;
}
EXPORT void orc_normalize(const float v[3], float o[3]) { o_normalize(v, o); }

/* pixel (px, py) with py counted from the bottom row (gl_FragCoord convention) */
static inline void o_pixel_dir(const float cam[3], float ppx, float ppy, float rw, float rh, int px, int py, float d[3]) {
    const float up[3] = {0.0f, 1.0f, 0.0f};
    float fx = ((float)px + 0.5f) * rw;
    float fy = ((float)py + 0.5f) * rh;
    float L[3], U[3], v[3];
    o_cross(cam, up, L);
    o_cross(cam, L, U);
    float sl = -(ppx * (fx - 0.5f));
    float su = -fy + 0.5f;
    for (int a = 0; a < 3; a++) {
        float lt = L[a] * sl;
        float ut = (U[a] * su) * ppy;
        v[a] = (cam[a] + lt) + ut;
    }
    o_normalize(v, d);
}

EXPORT void orc_pixel_dir(const float cam[3], float ppx, float ppy, int W, int H, int px, int py, float d[3]) {
    o_pixel_dir(cam, ppx, ppy, 1.0f / (float)W, 1.0f / (float)H, px, py, d);
}

/* projPlaneSize (main.cpp:94): (tan(radians(45.0)), tan(radians(45.0)) * (float)height / width) */
EXPORT void orc_proj_plane(int W, int H, float* ppx, float* ppy) {
    double t = tan(45.0 * 0.01745329251994329576923690768489);
    *ppx = (float)t;
    *ppy = (float)(t * (double)(float)H / (double)W);
}

/* ------------------------------------------------------------------------------------------------
 * castRayFromCam (ray_caster.cpp:19-87) with explicit origin / direction instead of the globals.
 * Outputs the reference RayResult {pos, lastPos, steps} plus the build-defined extras: hit flag,
 * last stepped axis, t = deltaPos[axis] before its increment, and the block at pos.
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
    int32_t pos[3];
    int32_t last[3];
    int32_t steps;
    int32_t hit;
    int32_t axis; /* -1 when no step was taken */
    uint32_t flags;
    uint64_t color;
    float meta;
    double t;
    int32_t err;
    uint32_t n_dda; /* DDA steps executed */
} orayres;

typedef int (*o_getblock_fn)(const void* world, int x, int y, int z, uint32_t* f, uint64_t* c, float* m);

static int o_gb_tree(const void* w, int x, int y, int z, uint32_t* f, uint64_t* c, float* m) {
    return o_get_block((const otree*)w, x, y, z, f, c, m);
}

/* dense u8 grid (config C1): material codes per o_col_mat, coordinates & (n-1) */
typedef struct {
    const uint8_t* vox; /* [z][y][x] */
    int n;              /* power of two */
    uint64_t mcolor[256];
    uint32_t mflags[256];
} odense;
static int o_gb_dense(const void* w, int x, int y, int z, uint32_t* f, uint64_t* c, float* m) {
    const odense* D = (const odense*)w;
    int k = D->n - 1;
    uint8_t v = D->vox[((size_t)(z & k) * D->n + (y & k)) * D->n + (x & k)];
    *f = D->mflags[v];
    *c = D->mcolor[v];
    *m = 0.0f;
    return 0;
}

static inline double o_gabs(double v) { return v >= 0 ? v : -v; } /* glm::abs */

static void o_cast(o_getblock_fn gb, const void* world, const float org[3], const float dir[3], int steps, orayres* R) {
    int st[3];
    double dl[3], ad[3], ex[3], dp[3];
    int r[3], last[3];
    for (int a = 0; a < 3; a++) {
        st[a] = dir[a] < 0 ? -1 : 1;
        dl[a] = (double)(1.0f / dir[a]);
        ad[a] = o_gabs(dl[a]);
    }
    for (int a = 0; a < 3; a++) {
        r[a] = (int)truncf(org[a]);
        ex[a] = (double)org[a];
        if (st[a] < 0) ex[a] -= 1;
    }
    for (int a = 0; a < 3; a++) dp[a] = ad[a] - (ex[a] - (double)r[a]) * dl[a];
    memset(R, 0, sizeof(*R));
    R->axis = -1;
    for (int a = 0; a < 3; a++) last[a] = r[a];
    R->t = 0.0;
    while (steps--) {
        int ax;
        for (int a = 0; a < 3; a++) last[a] = r[a];
        if (dp[0] < dp[1] && dp[0] < dp[2]) ax = 0;
        else if (dp[1] < dp[2]) ax = 1;
        else ax = 2;
        r[ax] += st[ax];
        R->t = dp[ax];
        dp[ax] += ad[ax];
        R->axis = ax;
        R->n_dda++;
        uint32_t f;
        uint64_t c;
        float m;
        if (gb(world, r[0], r[1], r[2], &f, &c, &m)) {
            R->err = 1;
            break;
        }
        if (c != ~0ull && (f & 0x10) == 0) {
            memcpy(R->pos, r, sizeof(r));
            memcpy(R->last, last, sizeof(last));
            R->steps = steps;
            R->hit = 1;
            R->flags = f;
            R->color = c;
            R->meta = m;
            return;
        }
    }
    memcpy(R->pos, r, sizeof(r));
    memcpy(R->last, last, sizeof(last));
    R->steps = 0;
    R->hit = 0;
    R->flags = 0; /* miss: no material reported */
    R->color = ~0ull;
    R->meta = 0.0f;
}

EXPORT void orc_cast_ray(const otree* t, const float org[3], const float dir[3], int steps, orayres* R) {
    o_cast(o_gb_tree, t, org, dir, steps, R);
}

/* test.cpp known-answer vector: the same DDA with no tree, 500 steps (test.cpp:78-134) */
EXPORT void orc_dda_free(const float org[3], const float dir[3], int steps, int32_t out_pos[3], int32_t* out_last_axis) {
    int st[3];
    double dl[3], ad[3], ex[3], dp[3];
    int r[3];
    for (int a = 0; a < 3; a++) {
        st[a] = dir[a] < 0 ? -1 : 1;
        dl[a] = (double)(1.0f / dir[a]);
        ad[a] = o_gabs(dl[a]);
        r[a] = (int)truncf(org[a]);
        ex[a] = (double)org[a];
        if (st[a] < 0) ex[a] -= 1;
    }
    for (int a = 0; a < 3; a++) dp[a] = ad[a] - (ex[a] - (double)r[a]) * dl[a];
    int lastHit = 0;
    while (steps--) {
        if (dp[0] < dp[1] && dp[0] < dp[2]) { r[0] += st[0]; dp[0] += ad[0]; lastHit = 0; }
        else if (dp[1] < dp[2]) { r[1] += st[1]; dp[1] += ad[1]; lastHit = 1; }
        else { r[2] += st[2]; dp[2] += ad[2]; lastHit = 2; }
    }
    memcpy(out_pos, r, sizeof(r));
    *out_last_axis = lastHit;
}

/* ------------------------------------------------------------------------------------------------
 * Frame cast: every pixel of a W x H frame (optionally a pixel subset), multi-threaded over
 * interleaved rows.  Output arrays are in pixel order idx = py * W + px.
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
    o_getblock_fn gb;
    const void* world;
    float org[3], cam[3];
    float ppx, ppy, rw, rh;
    int W, H, steps;
    const int64_t* pix; /* optional subset of pixel indices */
    int64_t n;
    int tid, nthreads;
    int32_t* pos;   /* [n*3] */
    int32_t* last;  /* [n*3] */
    int32_t* stp;   /* [n] */
    int32_t* hit;   /* [n] */
    double* t;      /* [n] */
    uint64_t* color;
    uint32_t* flags;
    int32_t* axis;
    uint64_t dda_total;
    int err;
} o_fjob;

static void* o_frame_worker(void* p) {
    o_fjob* j = (o_fjob*)p;
    uint64_t dda = 0;
    for (int64_t k = j->tid; k < j->n; k += j->nthreads) {
        int64_t pi = j->pix ? j->pix[k] : k;
        int px = (int)(pi % j->W), py = (int)(pi / j->W);
        float d[3];
        o_pixel_dir(j->cam, j->ppx, j->ppy, j->rw, j->rh, px, py, d);
        orayres R;
        o_cast(j->gb, j->world, j->org, d, j->steps, &R);
        dda += R.n_dda;
        if (R.err) j->err = 1;
        if (j->pos) memcpy(j->pos + 3 * k, R.pos, 12);
        if (j->last) memcpy(j->last + 3 * k, R.last, 12);
        if (j->stp) j->stp[k] = R.steps;
        if (j->hit) j->hit[k] = R.hit;
        if (j->t) j->t[k] = R.t;
        if (j->color) j->color[k] = R.color;
        if (j->flags) j->flags[k] = R.flags;
        if (j->axis) j->axis[k] = R.axis;
    }
    j->dda_total = dda;
    return NULL;
}

static int o_frame(o_getblock_fn gb, const void* world, const float org[3], const float cam[3], float ppx, float ppy, int W, int H,
                   int steps, const int64_t* pix, int64_t n, int nthreads, int32_t* pos, int32_t* last, int32_t* stp, int32_t* hit,
                   double* t, uint64_t* color, uint32_t* flags, int32_t* axis, uint64_t* dda_total) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    o_fjob* jobs = (o_fjob*)calloc((size_t)nthreads, sizeof(o_fjob));
    for (int i = 0; i < nthreads; i++) {
        o_fjob* j = &jobs[i];
        j->gb = gb;
        j->world = world;
        memcpy(j->org, org, 12);
        memcpy(j->cam, cam, 12);
        j->ppx = ppx;
        j->ppy = ppy;
        j->rw = 1.0f / (float)W;
        j->rh = 1.0f / (float)H;
        j->W = W;
        j->H = H;
        j->steps = steps;
        j->pix = pix;
        j->n = pix ? n : (int64_t)W * H;
        j->tid = i;
        j->nthreads = nthreads;
        j->pos = pos; j->last = last; j->stp = stp; j->hit = hit; j->t = t; j->color = color; j->flags = flags; j->axis = axis;
        if (nthreads > 1) pthread_create(&th[i], NULL, o_frame_worker, j);
    }
    int err = 0;
    uint64_t dda = 0;
    if (nthreads == 1) o_frame_worker(&jobs[0]);
    for (int i = 0; i < nthreads; i++) {
        if (nthreads > 1) pthread_join(th[i], NULL);
        err |= jobs[i].err;
        dda += jobs[i].dda_total;
    }
    free(jobs);
    if (dda_total) *dda_total = dda;
    return err ? -1 : 0;
}

EXPORT int orc_cast_frame(const otree* t, const float org[3], const float cam[3], float ppx, float ppy, int W, int H, int steps,
                          const int64_t* pix, int64_t n, int nthreads, int32_t* pos, int32_t* last, int32_t* stp, int32_t* hit,
                          double* tt, uint64_t* color, uint32_t* flags, int32_t* axis, uint64_t* dda_total) {
    return o_frame(o_gb_tree, t, org, cam, ppx, ppy, W, H, steps, pix, n, nthreads, pos, last, stp, hit, tt, color, flags, axis,
                   dda_total);
}

/* dense grid world for config C1: materialise [0,n)^3 of a tree via getBlock into material codes */
EXPORT odense* orc_dense_from_tree(const otree* t, int n) {
    odense* D = (odense*)calloc(1, sizeof(odense));
    uint8_t* vox = (uint8_t*)malloc((size_t)n * n * n);
    int nm = 1;
    D->mcolor[0] = ~0ull;
    D->mflags[0] = 0;
    for (int z = 0; z < n; z++)
        for (int y = 0; y < n; y++)
            for (int x = 0; x < n; x++) {
                uint32_t f;
                uint64_t c;
                float m;
                o_get_block(t, x, y, z, &f, &c, &m);
                int code = 0;
                if (c != ~0ull || f != 0) {
                    for (code = 1; code < nm; code++)
                        if (D->mcolor[code] == c && D->mflags[code] == f) break;
                    if (code == nm && nm < 256) {
                        D->mcolor[nm] = c;
                        D->mflags[nm] = f;
                        nm++;
                    }
                }
                vox[((size_t)z * n + y) * n + x] = (uint8_t)code;
            }
    D->vox = vox;
    D->n = n;
    return D;
}
EXPORT void orc_dense_free(odense* D) {
    if (!D) return;
    free((void*)D->vox);
    free(D);
}
EXPORT int orc_cast_frame_dense(const odense* D, const float org[3], const float cam[3], float ppx, float ppy, int W, int H, int steps,
                                int nthreads, int32_t* pos, int32_t* stp, int32_t* hit, uint64_t* color, uint64_t* dda_total) {
    return o_frame(o_gb_dense, D, org, cam, ppx, ppy, W, H, steps, NULL, 0, nthreads, pos, NULL, stp, hit, NULL, color, NULL, NULL,
                   dda_total);
}

/* ------------------------------------------------------------------------------------------------
 * Algorithmic-traffic model: node entries along the reference DDA path under the
 * shader's common-ancestor restart (low_res.frag:493-531): per DDA step the lookup restarts at the
 * deepest common ancestor of the previous and the new voxel (never deeper than where the previous
 * lookup stopped) and descends; every descent is one 4 B child-slot read + one 16 B node read.
 * Returns the summed E_child over the rays of a frame (plus the frame's DDA step count).
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
    uint32_t stack[16];
    int depth;   /* depth of the node where the previous lookup stopped */
    int prev[3]; /* the previously looked-up voxel */
    int have_prev;
} o_estate;

/* walk one ray (ray_caster.cpp:19-87 DDA) and count node entries under the restart model, continuing
   from S (the lookup state a previous ray left); *hit / pos / last / axis describe where it ended */
static uint64_t o_walk_entries(const otree* t, o_estate* S, const float org[3], const float dir[3], int steps, int* hit, int pos[3],
                               int last[3], int* axis) {
    int L = t->max_depth - 1;
    int st[3];
    double dl[3], ad[3], ex[3], dp[3];
    int r[3];
    for (int a = 0; a < 3; a++) {
        st[a] = dir[a] < 0 ? -1 : 1;
        dl[a] = (double)(1.0f / dir[a]);
        ad[a] = o_gabs(dl[a]);
        r[a] = (int)truncf(org[a]);
        ex[a] = (double)org[a];
        if (st[a] < 0) ex[a] -= 1;
    }
    for (int a = 0; a < 3; a++) dp[a] = ad[a] - (ex[a] - (double)r[a]) * dl[a];
    uint64_t entries = 0;
    *hit = 0;
    *axis = -1;
    while (steps--) {
        int ax;
        if (dp[0] < dp[1] && dp[0] < dp[2]) ax = 0;
        else if (dp[1] < dp[2]) ax = 1;
        else ax = 2;
        memcpy(last, r, sizeof(r));
        r[ax] += st[ax];
        dp[ax] += ad[ax];
        *axis = ax;
        /* common ancestor depth: number of leading levels whose 2-bit digits agree */
        int n = 0;
        if (S->have_prev) {
            for (n = 0; n < L; n++) {
                int off = 2 * (L - 1 - n);
                if (o_child_index(r[0], r[1], r[2], off) != o_child_index(S->prev[0], S->prev[1], S->prev[2], off)) break;
            }
        }
        if (n < S->depth) S->depth = n;
        /* descend from stack[depth] */
        uint32_t f = 0;
        uint64_t c = ~0ull;
        for (;;) {
            const onode* nd = NODE(t, S->stack[S->depth]);
            if (nd->flags & 1) {
                f = nd->flags;
                c = nd->w0;
                break;
            }
            if (S->depth >= L) break; /* corrupted (root-63 region): stop counting */
            int off = 2 * (L - 1 - S->depth);
            int idx = o_child_index(r[0], r[1], r[2], off);
            if (!((nd->w0 >> idx) & 1)) break;
            S->stack[S->depth + 1] = ARR(t, nd->w1)->c[idx];
            S->depth++;
            entries++;
        }
        memcpy(S->prev, r, sizeof(r));
        S->have_prev = 1;
        if (c != ~0ull && (f & 0x10) == 0) {
            *hit = 1;
            break;
        }
    }
    memcpy(pos, r, sizeof(r));
    return entries;
}

static uint64_t o_count_entries(const otree* t, const float org[3], const float dir[3], int steps) {
    o_estate S;
    memset(&S, 0, sizeof(S));
    S.stack[0] = t->root;
    int hit, pos[3], last[3], axis;
    return o_walk_entries(t, &S, org, dir, steps, &hit, pos, last, &axis);
}

static inline void o_ao_dir(const float h[3], int ax, int sg, float d[3]);
EXPORT void orc_hemisphere(int n, float* out);

/* §8(d) "for AO: add <= 5 steps x E per sample": the node entries of a hit's AO rays (A8: from the
   centre of lastPos, the table turned to the hit face), each continuing the restart model from the
   lookup state the primary ray left (the shader-style stack of the hit voxel) */
static uint64_t o_count_entries_ao(const otree* t, const float org[3], const float dir[3], int steps, const float* table, int n_ao,
                                   int ao_steps) {
    o_estate S;
    memset(&S, 0, sizeof(S));
    S.stack[0] = t->root;
    int hit, pos[3], last[3], axis;
    (void)o_walk_entries(t, &S, org, dir, steps, &hit, pos, last, &axis);
    if (!hit || axis < 0) return 0;
    int sg = last[axis] - pos[axis];
    float o2[3] = {(float)last[0] + 0.5f, (float)last[1] + 0.5f, (float)last[2] + 0.5f};
    uint64_t e = 0;
    for (int i = 0; i < n_ao; i++) {
        float d[3];
        o_ao_dir(table + 3 * i, axis, sg, d);
        o_estate A = S;
        int h2, p2[3], l2[3], a2;
        e += o_walk_entries(t, &A, o2, d, ao_steps, &h2, p2, l2, &a2);
    }
    return e;
}

typedef struct {
    const otree* t;
    float org[3], cam[3], ppx, ppy, rw, rh;
    int W, H, steps, tid, nthreads, n_ao, ao_steps;
    const float* table;
    const int64_t* pix;
    int64_t n;
    uint64_t sum;
} o_ejob;
static void* o_entries_worker(void* p) {
    o_ejob* j = (o_ejob*)p;
    uint64_t s = 0;
    for (int64_t k = j->tid; k < j->n; k += j->nthreads) {
        int64_t pi = j->pix ? j->pix[k] : k;
        float d[3];
        o_pixel_dir(j->cam, j->ppx, j->ppy, j->rw, j->rh, (int)(pi % j->W), (int)(pi / j->W), d);
        s += j->n_ao ? o_count_entries_ao(j->t, j->org, d, j->steps, j->table, j->n_ao, j->ao_steps)
                     : o_count_entries(j->t, j->org, d, j->steps);
    }
    j->sum = s;
    return NULL;
}
static uint64_t o_frame_entries(const otree* t, const float org[3], const float cam[3], float ppx, float ppy, int W, int H, int steps,
                                int n_ao, int ao_steps, const int64_t* pix, int64_t n, int nthreads) {
    float table[3 * 64];
    if (n_ao > 64) n_ao = 64;
    if (n_ao > 0) orc_hemisphere(n_ao, table);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    o_ejob* jobs = (o_ejob*)calloc((size_t)nthreads, sizeof(o_ejob));
    for (int i = 0; i < nthreads; i++) {
        o_ejob* j = &jobs[i];
        j->t = t;
        memcpy(j->org, org, 12);
        memcpy(j->cam, cam, 12);
        j->ppx = ppx; j->ppy = ppy;
        j->rw = 1.0f / (float)W; j->rh = 1.0f / (float)H;
        j->W = W; j->H = H; j->steps = steps;
        j->n_ao = n_ao > 0 ? n_ao : 0; j->ao_steps = ao_steps; j->table = table;
        j->pix = pix;
        j->n = pix ? n : (int64_t)W * H;
        j->tid = i;
        j->nthreads = nthreads;
        pthread_create(&th[i], NULL, o_entries_worker, j);
    }
    uint64_t s = 0;
    for (int i = 0; i < nthreads; i++) {
        pthread_join(th[i], NULL);
        s += jobs[i].sum;
    }
    free(jobs);
    return s;
}
EXPORT uint64_t orc_frame_entries(const otree* t, const float org[3], const float cam[3], float ppx, float ppy, int W, int H, int steps,
                                  const int64_t* pix, int64_t n, int nthreads) {
    return o_frame_entries(t, org, cam, ppx, ppy, W, H, steps, 0, 0, pix, n, nthreads);
}
/* the AO rays' entries only (summed over the frame's hits), see o_count_entries_ao */
EXPORT uint64_t orc_frame_entries_ao(const otree* t, const float org[3], const float cam[3], float ppx, float ppy, int W, int H,
                                     int steps, int n_ao, int ao_steps, const int64_t* pix, int64_t n, int nthreads) {
    return o_frame_entries(t, org, cam, ppx, ppy, W, H, steps, n_ao, ao_steps, pix, n, nthreads);
}

/* FNV-1a digest of getBlock over a box (material identity = (flags, color)) */
EXPORT uint64_t orc_digest_box(const otree* t, int x0, int y0, int z0, int nx, int ny, int nz) {
    uint64_t h = 1469598103934665603ull;
    for (int z = z0; z < z0 + nz; z++)
        for (int y = y0; y < y0 + ny; y++)
            for (int x = x0; x < x0 + nx; x++) {
                uint32_t f;
                uint64_t c;
                float m;
                if (o_get_block(t, x, y, z, &f, &c, &m)) f = 0xFFFFFFFFu, c = 0x5A5A5A5A5A5A5A5Aull;
                h = (h ^ f) * 1099511628211ull;
                h = (h ^ c) * 1099511628211ull;
            }
    return h;
}

/* dump getBlock over a box into arrays (flags, color) for voxel-by-voxel comparisons */
EXPORT int orc_dump_box(const otree* t, int x0, int y0, int z0, int nx, int ny, int nz, uint32_t* flags, uint64_t* color) {
    size_t k = 0;
    int err = 0;
    for (int z = z0; z < z0 + nz; z++)
        for (int y = y0; y < y0 + ny; y++)
            for (int x = x0; x < x0 + nx; x++, k++) {
                float m;
                if (o_get_block(t, x, y, z, &flags[k], &color[k], &m)) {
                    flags[k] = 0xFFFFFFFFu;
                    color[k] = 0;
                    err = 1;
                }
            }
    return err ? -1 : 0;
}

/* ------------------------------------------------------------------------------------------------
 * Hemisphere AO (light_scattering.frag:133-154,175-236; gen_hemisphare_distrib.py)
 * Table: phi = arccos(1 - (i+0.5)*0.85/N), theta = pi*(1+sqrt 5)*(i+0.5); (cos th sin ph,
 * sin th sin ph, cos ph) in double, rounded to float; component 2 is the pole (the shader reads the
 * printed (x, z, y) back through .xzy, so its pole is +z).  The reference computes an orientation
 * matrix but never applies it (light_scattering.frag:224 vs :231); this build orients the pole to
 * the hit face's normal by an exact signed axis permutation.  Each AO ray starts at the centre of
 * lastPos and is a castRayFromCam with a 5-step budget (light_scattering.frag:231); the pixel's
 * result is the number of AO rays that hit.
 * ---------------------------------------------------------------------------------------------- */
EXPORT void orc_hemisphere(int n, float* out) {
    const double PI = 3.141592653589793;
    for (int i = 0; i < n; i++) {
        double idx = (double)i + 0.5;
        double phi = acos(1.0 - idx * 0.85 / (double)n);
        double theta = PI * (1.0 + sqrt(5.0)) * idx;
        out[3 * i + 0] = (float)(cos(theta) * sin(phi));
        out[3 * i + 1] = (float)(sin(theta) * sin(phi));
        out[3 * i + 2] = (float)cos(phi);
    }
}

/* AO direction for a face normal on axis `ax` with sign `sg` (+1/-1): pole -> ax, then the two
   tangent components to the cyclically following axes */
static inline void o_ao_dir(const float h[3], int ax, int sg, float d[3]) {
    d[ax] = sg > 0 ? h[2] : -h[2];
    d[(ax + 1) % 3] = h[0];
    d[(ax + 2) % 3] = h[1];
}

static int o_ao_count(o_getblock_fn gb, const void* world, const orayres* P, const float* table, int n, int steps) {
    if (!P->hit || P->axis < 0) return 0;
    int ax = P->axis;
    int sg = P->last[ax] - P->pos[ax]; /* normal points from the hit voxel towards lastPos */
    float org[3] = {(float)P->last[0] + 0.5f, (float)P->last[1] + 0.5f, (float)P->last[2] + 0.5f};
    int cnt = 0;
    for (int i = 0; i < n; i++) {
        float d[3];
        o_ao_dir(table + 3 * i, ax, sg, d);
        orayres R;
        o_cast(gb, world, org, d, steps, &R);
        cnt += R.hit != 0;
    }
    return cnt;
}

typedef struct {
    const otree* t;
    float org[3], cam[3], ppx, ppy, rw, rh;
    int W, H, steps, tid, nthreads, n_ao, ao_steps;
    const float* table;
    const int64_t* pix;
    int64_t n;
    uint8_t* ao;
    int32_t* hit;
} o_aojob;
static void* o_ao_worker(void* p) {
    o_aojob* j = (o_aojob*)p;
    for (int64_t k = j->tid; k < j->n; k += j->nthreads) {
        int64_t pi = j->pix ? j->pix[k] : k;
        float d[3];
        o_pixel_dir(j->cam, j->ppx, j->ppy, j->rw, j->rh, (int)(pi % j->W), (int)(pi / j->W), d);
        orayres R;
        o_cast(o_gb_tree, j->t, j->org, d, j->steps, &R);
        j->ao[k] = (uint8_t)o_ao_count(o_gb_tree, j->t, &R, j->table, j->n_ao, j->ao_steps);
        if (j->hit) j->hit[k] = R.hit;
    }
    return NULL;
}
EXPORT void orc_cast_frame_ao(const otree* t, const float org[3], const float cam[3], float ppx, float ppy, int W, int H, int steps,
                              int n_ao, int ao_steps, const int64_t* pix, int64_t n, int nthreads, uint8_t* ao, int32_t* hit) {
    float table[3 * 64];
    if (n_ao > 64) n_ao = 64;
    orc_hemisphere(n_ao, table);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    o_aojob* jobs = (o_aojob*)calloc((size_t)nthreads, sizeof(o_aojob));
    for (int i = 0; i < nthreads; i++) {
        o_aojob* j = &jobs[i];
        j->t = t;
        memcpy(j->org, org, 12);
        memcpy(j->cam, cam, 12);
        j->ppx = ppx; j->ppy = ppy;
        j->rw = 1.0f / (float)W; j->rh = 1.0f / (float)H;
        j->W = W; j->H = H; j->steps = steps; j->n_ao = n_ao; j->ao_steps = ao_steps;
        j->table = table;
        j->pix = pix;
        j->n = pix ? n : (int64_t)W * H;
        j->tid = i; j->nthreads = nthreads;
        j->ao = ao; j->hit = hit;
        pthread_create(&th[i], NULL, o_ao_worker, j);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(jobs);
}

/* ------------------------------------------------------------------------------------------------
 * Shading, restating include/svo_rt.h's svo_shade_rays contract: low_res.frag's
 * colour model (genSkyBox :157-168, calcLightIntensity :242-252, shadow ray :373-391, highlight
 * :340-343, reflectRay :170-189, refractRay :196-240 for non-liquid blocks) over castRayFromCam hits.  Single precision, shader op order.
 * ---------------------------------------------------------------------------------------------- */
/* refractRay(vec3, vec3, float, float) (:196-209) with n1 = 1.0, n2 = 1.1; dot as ((x + y) + z),
   no fused operations. */
static void o_refract_dir(float d[3], const float nin[3]) {
    const float r = 1.0f / 1.1f;
    float n[3] = {nin[0], nin[1], nin[2]};
    float c1 = (n[0] * d[0] + n[1] * d[1]) + n[2] * d[2];
    if (c1 < 0.0f) {
        for (int a = 0; a < 3; a++) n[a] = -n[a];
        c1 = (n[0] * d[0] + n[1] * d[1]) + n[2] * d[2];
    }
    const float c2 = sqrtf(1.0f - r * r * (1.0f - c1 * c1));
    const float k = r * c1 - c2;
    for (int a = 0; a < 3; a++) d[a] = r * d[a] + k * n[a];
}

/* GLSL sin for the liquid wobble (:226): defined here (and in the product, svo_common.h sin_f32)
   as sin evaluated in double and rounded once to float — Cody-Waite reduction by pi/2, Taylor
   polynomials on [-pi/4, pi/4] — the same double operations on both sides (no contraction). */
static float o_sin_f32(float xf) {
    // (beyond the exact reduction range the argument is first taken modulo fl(2 pi) — an exact remainder
    // on host and device alike — so the value stays a bounded sine of an equal argument on both)
    const double x0 = (double)xf;
    const double x = __builtin_fabs(x0) < 524288.0 ? x0 : __builtin_fmod(x0, 6.283185307179586);
    const double k = rint(x * 0.63661977236758134308);
    const double r = (x - k * 1.57079632673412561417e+00) - k * 6.07710050650619224932e-11;
    const double r2 = r * r;
    const double sn = r + (r * r2) * (-1.6666666666666666e-01 + r2 * (8.3333333333333332e-03 + r2 * (-1.9841269841269841e-04 +
                                     r2 * (2.7557319223985893e-06 + r2 * (-2.5052108385441720e-08 + r2 * 1.6059043836821613e-10)))));
    const double cs = 1.0 + r2 * (-0.5 + r2 * (4.1666666666666664e-02 + r2 * (-1.3888888888888889e-03 + r2 * (2.4801587301587302e-05 +
                                  r2 * (-2.7557319223985888e-07 + r2 * (2.0876756987868100e-09 + r2 * -1.1470745597729725e-11))))));
    // quadrant k mod 4 without an integer conversion of k (undefined for non-finite or huge k): exact
    // for every finite k (k * 0.25, its floor and 4 * that are exact; k >= 2^54 is a multiple of 4), 0
    // for NaN / infinite k, whose result is NaN anyway.  The reduction is exact for |k| < 2^20, which
    // holds on the direct path (|x| < 2^19); host and device take the same operations everywhere.
    const double kq = k - 4.0 * floor(k * 0.25);
    const int q = (kq >= 0.0 && kq < 4.0) ? (int)kq : 0;
    const double v = (q & 1) ? cs : sn;
    return (float)((q & 2) ? -v : v);
}
EXPORT float orc_sin_f32(float x) { return o_sin_f32(x); }

/* o_cast with reflections and refractions.  A hit on a block with (flags & 7) == 3 while steps
   remain undoes the last crossing on the hit axis, flips that axis's step and direction, and
   continues (reflectRay :170-189).  A hit on a non-liquid block with (flags & 7) == 5 (liquid is
   empty in castRayFromCam) while steps remain tints by 0.95 and continues; the first one also
   bends the ray (refractRay :211-240): the origin-based exact position (never advanced by the DDA,
   as in the shader) gets +1 on the other axes with a negative step, the direction is refracted, the
   ray rebuilt (A1), exact += min(step, 0) and deltaPos = absDelta - (exact - round) * delta from
   the current cell.  mod = finalColorMod (0.94 per reflection, 0.95 per refractive block, in
   order).  liquid != 0: liquid blocks are not empty but blocks like any other (low_res.frag's
   getBlock, :312-333): refractive liquid (flags & 7 == 5, the terrain's water 0x15) tints by
   (0.94, 0.97, 1.0) (:214) and, when it is the first refractive block, bends the ray with the
   normal's wobble x += sin((time + exact.x * 0.2 - exact.z * 0.1) * 10) * 0.2, renormalised
   (:225-229; exact as float). */
static void o_cast_refl(o_getblock_fn gb, const void* world, const float org[3], const float dir_in[3], int steps, orayres* R,
                        float dir[3], int* nrefl, float mod[3], int liquid, float time) {
    int st[3];
    double dl[3], ad[3], ex[3], dp[3];
    int r[3], last[3];
    int bent = 0;
    for (int a = 0; a < 3; a++) {
        dir[a] = dir_in[a];
        st[a] = dir[a] < 0 ? -1 : 1;
        dl[a] = (double)(1.0f / dir[a]);
        ad[a] = o_gabs(dl[a]);
        r[a] = (int)truncf(org[a]);
        ex[a] = (double)org[a];
        if (st[a] < 0) ex[a] -= 1;
    }
    for (int a = 0; a < 3; a++) dp[a] = ad[a] - (ex[a] - (double)r[a]) * dl[a];
    memset(R, 0, sizeof(*R));
    R->axis = -1;
    *nrefl = 0;
    mod[0] = mod[1] = mod[2] = 1.0f;
    for (int a = 0; a < 3; a++) last[a] = r[a];
    while (steps--) {
        int ax;
        for (int a = 0; a < 3; a++) last[a] = r[a];
        if (dp[0] < dp[1] && dp[0] < dp[2]) ax = 0;
        else if (dp[1] < dp[2]) ax = 1;
        else ax = 2;
        r[ax] += st[ax];
        R->t = dp[ax];
        dp[ax] += ad[ax];
        R->axis = ax;
        uint32_t f;
        uint64_t c;
        float m;
        if (gb(world, r[0], r[1], r[2], &f, &c, &m)) {
            R->err = 1;
            break;
        }
        const int liq = (f & 0x10) != 0;
        if (c != ~0ull && (liquid || !liq)) {
            if ((f & 7u) == 3u && steps > 0) {
                dp[ax] -= ad[ax];
                st[ax] = -st[ax];
                dir[ax] = -dir[ax];
                (*nrefl)++;
                for (int k = 0; k < 3; k++) mod[k] *= 0.94f;
                continue;
            }
            if ((f & 7u) == 5u && steps > 0) {
                mod[0] *= liq ? 0.94f : 0.95f;
                mod[1] *= liq ? 0.97f : 0.95f;
                mod[2] *= liq ? 1.0f : 0.95f;
                if (!bent) {
                    bent = 1;
                    for (int a = 0; a < 3; a++)
                        if (a != ax && st[a] < 0) ex[a] += 1;
                    float nrm[3] = {0.0f, 0.0f, 0.0f};
                    nrm[ax] = (float)st[ax];
                    if (liq) {
                        const float arg = ((time + (float)ex[0] * 0.2f) - (float)ex[2] * 0.1f) * 10.0f;
                        nrm[0] += o_sin_f32(arg) * 0.2f;
                        o_normalize(nrm, nrm);
                    }
                    o_refract_dir(dir, nrm);
                    for (int a = 0; a < 3; a++) {
                        st[a] = dir[a] < 0 ? -1 : 1;
                        dl[a] = (double)(1.0f / dir[a]);
                        ad[a] = o_gabs(dl[a]);
                        if (st[a] < 0) ex[a] -= 1;
                    }
                    for (int a = 0; a < 3; a++) dp[a] = ad[a] - (ex[a] - (double)r[a]) * dl[a];
                }
                continue;
            }
            memcpy(R->pos, r, sizeof(r));
            memcpy(R->last, last, sizeof(last));
            R->steps = steps;
            R->hit = 1;
            R->flags = f;
            R->color = c;
            R->meta = m;
            return;
        }
    }
    memcpy(R->pos, r, sizeof(r));
    memcpy(R->last, last, sizeof(last));
    R->steps = 0;
    R->hit = 0;
    R->flags = 0;
    R->color = ~0ull;
    R->meta = 0.0f;
}

static void o_color(uint64_t c, float o[3]) {
    const double sc = 1.0 / 2097152.0;
    o[0] = (float)((double)(c >> 42) * sc);
    o[1] = (float)((double)((c >> 21) & 0x1FFFFFull) * sc);
    o[2] = (float)((double)(c & 0x1FFFFFull) * sc);
}

static float o_sigmoid(float x, float scale, float k) { return 1.0f / (1.0f + expf(-x * k)) * scale; }
static float o_clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

static void o_sky(const float d[3], const float sun[3], float o[3]) {
    float dy = d[1];
    if (dy < 0.0f) dy *= 1.4f;
    float haze = (0.1f - fabsf(o_clampf(dy, -0.3f, 0.3f))) * 0.8f + 0.1f;
    float modifier = o_clampf(o_sigmoid(1.0f - (haze * 2.0f), 1.0f, 2.0f), 0.0f, 1.0f);
    float ex = d[0] - sun[0], ey = dy - sun[1], ez = d[2] - sun[2];
    float b = sqrtf((ex * ex + ey * ey) + ez * ez) * 50.0f;
    float sv = o_sigmoid(1.5f - b, 1.0f, 1.6f);
    float h3 = o_clampf(haze, 0.0f, 1.0f) * 3.0f;
    o[0] = (0.2f + h3) * modifier + sv;
    o[1] = (0.4f + h3) * modifier + sv;
    o[2] = (1.0f + h3) * modifier + 0.0f;
}

static void o_shade(o_getblock_fn gb, const void* world, const float org[3], const float d0[3], int steps, const float sun[3],
                    const int32_t* look, int shadow_steps, int liquid, float time, float out[4], int* shadow_ray) {
    orayres R;
    if (shadow_ray) *shadow_ray = 0;
    float dir[3];
    int nrefl;
    float m[3];
    o_cast_refl(gb, world, org, d0, steps, &R, dir, &nrefl, m, liquid, time);
    float c[3];
    if (look && R.pos[0] == look[0] && R.pos[1] == look[1] && R.pos[2] == look[2]) {
        float b[3];
        o_color(R.color, b);
        for (int k = 0; k < 3; k++) c[k] = b[k] * 2.0f + 0.3f;
    } else if (!R.hit) {
        float sk[3];
        o_sky(dir, sun, sk);
        for (int k = 0; k < 3; k++) c[k] = sk[k] * m[k];
    } else {
        float col[3];
        o_color(R.color, col);
        int ax = R.axis;
        int sg = R.pos[ax] - R.last[ax];
        float l = sun[ax] * (float)(-sg);
        int facing = l > 0.0f;
        float inten = fminf(fmaxf(0.0f, l) + 0.4f + (facing ? 0.15f : 0.0f), 1.0f);
        for (int k = 0; k < 3; k++) c[k] = col[k] * inten * m[k];
        int dark = 0;
        if (nrefl == 0) {
            if (!facing) {
                dark = 1;
            } else {
                float so[3] = {(float)R.last[0] + 0.5f, (float)R.last[1] + 0.5f, (float)R.last[2] + 0.5f};
                orayres S;
                o_cast(gb, world, so, sun, shadow_steps, &S);
                dark = S.hit != 0;
                if (shadow_ray) *shadow_ray = 1;
            }
        }
        if (dark)
            for (int k = 0; k < 3; k++) c[k] = col[k] * 0.3f * m[k];
    }
    out[0] = c[0];
    out[1] = c[1];
    out[2] = c[2];
    out[3] = 0.0f;
}

typedef struct {
    const otree* t;
    float org[3], cam[3], ppx, ppy, rw, rh, sun[3], time;
    int W, H, steps, shadow_steps, tid, nthreads, liquid;
    const int32_t* look;
    const int64_t* pix;
    int64_t n;
    float* rgba;
} o_shjob;
static void* o_shade_worker(void* p) {
    o_shjob* j = (o_shjob*)p;
    for (int64_t k = j->tid; k < j->n; k += j->nthreads) {
        int64_t pi = j->pix ? j->pix[k] : k;
        float d[3];
        o_pixel_dir(j->cam, j->ppx, j->ppy, j->rw, j->rh, (int)(pi % j->W), (int)(pi / j->W), d);
        o_shade(o_gb_tree, j->t, j->org, d, j->steps, j->sun, j->look, j->shadow_steps, j->liquid, j->time, j->rgba + 4 * k, NULL);
    }
    return NULL;
}
EXPORT void orc_shade_frame(const otree* t, const float org[3], const float cam[3], float ppx, float ppy, int W, int H, int steps,
                            const float sun[3], const int32_t* look, int shadow_steps, const int64_t* pix, int64_t n, int nthreads,
                            float* rgba, int liquid, float time) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    o_shjob* jobs = (o_shjob*)calloc((size_t)nthreads, sizeof(o_shjob));
    for (int i = 0; i < nthreads; i++) {
        o_shjob* j = &jobs[i];
        j->t = t;
        memcpy(j->org, org, 12);
        memcpy(j->cam, cam, 12);
        memcpy(j->sun, sun, 12);
        j->ppx = ppx; j->ppy = ppy;
        j->rw = 1.0f / (float)W; j->rh = 1.0f / (float)H;
        j->W = W; j->H = H; j->steps = steps; j->shadow_steps = shadow_steps;
        j->look = look;
        j->liquid = liquid;
        j->time = time;
        j->pix = pix;
        j->n = pix ? n : (int64_t)W * H;
        j->tid = i; j->nthreads = nthreads;
        j->rgba = rgba;
        pthread_create(&th[i], NULL, o_shade_worker, j);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(jobs);
}

/* §8(d) for the shading pass (bench.py --shade): node entries of every lookup the pass's rays make under
   the same common-ancestor restart model as o_walk_entries — the primary ray with its reflections and
   refractions (o_cast_refl: one lookup per DDA step, the DDA continuing after each bounce) and the 75-step
   shadow ray of a lit, unreflected hit, which continues from the lookup state the primary left (as the AO
   rays do, o_count_entries_ao).  The block each lookup returns is o_get_block's, so the walk is the shading
   pass itself; the counter only rides along.  out[0] = entries, out[1] = shadow rays, out[2] = DDA lookups. */
typedef struct {
    const otree* t;
    o_estate S;
    uint64_t entries, lookups;
} o_ecount;
static int o_gb_count(const void* w, int x, int y, int z, uint32_t* f, uint64_t* c, float* m) {
    o_ecount* E = (o_ecount*)w;
    const otree* t = E->t;
    o_estate* S = &E->S;
    const int L = t->max_depth - 1;
    const int r[3] = {x, y, z};
    int n = 0;
    if (S->have_prev) {
        for (n = 0; n < L; n++) {
            int off = 2 * (L - 1 - n);
            if (o_child_index(r[0], r[1], r[2], off) != o_child_index(S->prev[0], S->prev[1], S->prev[2], off)) break;
        }
    }
    if (n < S->depth) S->depth = n;
    for (;;) {
        const onode* nd = NODE(t, S->stack[S->depth]);
        if (nd->flags & 1) break;
        if (S->depth >= L) break;
        int off = 2 * (L - 1 - S->depth);
        int idx = o_child_index(r[0], r[1], r[2], off);
        if (!((nd->w0 >> idx) & 1)) break;
        S->stack[S->depth + 1] = ARR(t, nd->w1)->c[idx];
        S->depth++;
        E->entries++;
    }
    memcpy(S->prev, r, sizeof(r));
    S->have_prev = 1;
    E->lookups++;
    return o_get_block(t, x, y, z, f, c, m);
}
typedef struct {
    const otree* t;
    float org[3], cam[3], ppx, ppy, rw, rh, sun[3], time;
    int W, H, steps, shadow_steps, tid, nthreads, liquid;
    const int64_t* pix;
    int64_t n;
    uint64_t out[3];
} o_sejob;
static void* o_shade_entries_worker(void* p) {
    o_sejob* j = (o_sejob*)p;
    for (int64_t k = j->tid; k < j->n; k += j->nthreads) {
        int64_t pi = j->pix ? j->pix[k] : k;
        float d[3], rgba[4];
        o_pixel_dir(j->cam, j->ppx, j->ppy, j->rw, j->rh, (int)(pi % j->W), (int)(pi / j->W), d);
        o_ecount E;
        memset(&E, 0, sizeof(E));
        E.t = j->t;
        E.S.stack[0] = j->t->root;
        int sh = 0;
        o_shade(o_gb_count, &E, j->org, d, j->steps, j->sun, NULL, j->shadow_steps, j->liquid, j->time, rgba, &sh);
        j->out[0] += E.entries;
        j->out[1] += (uint64_t)sh;
        j->out[2] += E.lookups;
    }
    return NULL;
}
EXPORT void orc_shade_entries(const otree* t, const float org[3], const float cam[3], float ppx, float ppy, int W, int H, int steps,
                              const float sun[3], int shadow_steps, const int64_t* pix, int64_t n, int nthreads, int liquid, float time,
                              uint64_t out[3]) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    o_sejob* jobs = (o_sejob*)calloc((size_t)nthreads, sizeof(o_sejob));
    for (int i = 0; i < nthreads; i++) {
        o_sejob* j = &jobs[i];
        j->t = t;
        memcpy(j->org, org, 12);
        memcpy(j->cam, cam, 12);
        memcpy(j->sun, sun, 12);
        j->ppx = ppx; j->ppy = ppy;
        j->rw = 1.0f / (float)W; j->rh = 1.0f / (float)H;
        j->W = W; j->H = H; j->steps = steps; j->shadow_steps = shadow_steps;
        j->liquid = liquid;
        j->time = time;
        j->pix = pix;
        j->n = pix ? n : (int64_t)W * H;
        j->tid = i; j->nthreads = nthreads;
        pthread_create(&th[i], NULL, o_shade_entries_worker, j);
    }
    out[0] = out[1] = out[2] = 0;
    for (int i = 0; i < nthreads; i++) {
        pthread_join(th[i], NULL);
        for (int k = 0; k < 3; k++) out[k] += jobs[i].out[k];
    }
    free(jobs);
}
