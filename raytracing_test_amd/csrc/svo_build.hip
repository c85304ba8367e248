// svo_build.hip — on-device world generation and tree build.
//
// genWorld's column tops (world_gen.cpp:22, OpenSimplex 2D from include/OpenSimplexNoise.cpp:77-208)
// are evaluated one column per lane, then the same canonical breadth-first tree the host terrain
// builder emits (svo_world.cpp build_from_heights) is built level by level on the GPU:
//   * a min/max height pyramid over aligned 4^k column footprints classifies any aligned region
//     in O(1) (EMPTY / uniform SOLID / MIXED, the host's classify_region);
//   * one wavefront per region, one lane per child slot (or per voxel at the brick level):
//     ballots give the child mask, the MIXED children and the solid voxels; exclusive scans over
//     the regions (hipCUB) place every child block and material run; a second pass writes them.
// The node array is identical, byte for byte, to svo_build_terrain's (tests), and it stays in HBM
// (adopted as the uploaded copy); the host image is copied back for host queries and edits.
#include <hip/hip_runtime.h>
#include <string.h>

#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <memory>
#include <vector>

#include "../../include/svo_rt.h"
#include "svo_hip.h"
#include "svo_internal.h"
#include "svo_noise.h"

using namespace svo;

namespace {

constexpr uint32_t G_EMPTY = 0u;
constexpr uint32_t G_MIXED = 0xFFFFFFFFu;
constexpr int kMaxPyr = 8;

struct DevTerrain {
    int32_t levels, E, W, L;
    const int16_t* h;  // [x*L + z]
    const int16_t* hmin[kMaxPyr];
    const int16_t* hmax[kMaxPyr];
    int32_t dimz[kMaxPyr];
    uint32_t id_of[5];
    int32_t view;  // SVO_VIEW_SOLID / SVO_VIEW_ALL
};

struct Region {
    int32_t x0, y0, z0;
    uint32_t node;  // index of the region's record in the node array
};

__device__ __forceinline__ uint32_t g_solid_class(const DevTerrain& T, int32_t h, int32_t y) {
    return T.id_of[terrain_material(h, y)];
}

// svo_world.cpp classify_region: class of the aligned region [x0,x0+s)x[y0,y0+s)x[z0,z0+s), s = 4^k
__device__ uint32_t g_classify(const DevTerrain& T, int32_t x0, int32_t y0, int32_t z0, int32_t s, int k) {
    const int32_t y1 = y0 + s - 1;
    if (x0 >= T.W || z0 >= T.L) return G_EMPTY;
    const bool partial = (x0 + s > T.W) || (z0 + s > T.L);
    const size_t ci = (size_t)(x0 >> (2 * k)) * T.dimz[k] + (z0 >> (2 * k));
    const int32_t hmin = T.hmin[k][ci], hmax = T.hmax[k][ci];
    if (terrain_region_empty(T.view, hmax, y0, y1)) return G_EMPTY;
    if (partial) return G_MIXED;
    return terrain_region_class(T.id_of, T.view, hmin, hmax, y0, y1, G_EMPTY, G_MIXED);
}

__global__ void k_heights(const uint8_t* perms, int32_t W, int32_t L, int16_t* h, int32_t* bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)W * L) return;
    const int32_t x = (int32_t)(i / L), z = (int32_t)(i - (int64_t)x * L);
    const int32_t v = terrain_height(perms, perms + 256, perms + 512, x, z);
    if (v < 0 || v > 32767) atomicOr(bad, 1);
    h[i] = (int16_t)v;
}

__global__ void k_pyramid(const int16_t* pmn, const int16_t* pmx, int32_t px, int32_t pz, int16_t* mn, int16_t* mx, int32_t dx,
                          int32_t dz) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)dx * dz) return;
    const int32_t cx = (int32_t)(i / dz), cz = (int32_t)(i - (int64_t)cx * dz);
    int16_t a = 32767, c = -32768;
    for (int u = 0; u < 4; u++)
        for (int v = 0; v < 4; v++) {
            const int64_t sx = (int64_t)cx * 4 + u, sz = (int64_t)cz * 4 + v;
            if (sx >= px || sz >= pz) continue;
            a = min(a, pmn[sx * pz + sz]);
            c = max(c, pmx[sx * pz + sz]);
        }
    mn[i] = a;
    mx[i] = c;
}

// one wavefront per region, lane = child slot: counts of non-empty and MIXED children
__global__ void k_count(DevTerrain T, const Region* cur, int64_t r0, int64_t n, int32_t cs, int k, uint32_t* nkid, uint32_t* nmix) {
    const int64_t r = r0 + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t sl = threadIdx.x & 63u;
    if (r >= n) return;  // whole waves exit together (n is per wave)
    const Region R = cur[r];
    const uint32_t c = g_classify(T, R.x0 + (int32_t)(sl & 3u) * cs, R.y0 + (int32_t)((sl >> 2) & 3u) * cs,
                                  R.z0 + (int32_t)(sl >> 4) * cs, cs, k);
    const uint64_t kid = __ballot(c != G_EMPTY), mix = __ballot(c == G_MIXED);
    if (sl == 0) {
        nkid[r] = (uint32_t)__popcll(kid);
        nmix[r] = (uint32_t)__popcll(mix);
    }
}

// second pass: the region's INTERIOR record, its SOLID children, the next level's MIXED regions
__global__ void k_write(DevTerrain T, const Region* cur, int64_t r0, int64_t n, int32_t cs, int k, const uint64_t* koff, const uint64_t* moff,
                        uint64_t base, Node* nodes, Region* next) {
    const int64_t r = r0 + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t sl = threadIdx.x & 63u;
    if (r >= n) return;
    const Region R = cur[r];
    const int32_t x = R.x0 + (int32_t)(sl & 3u) * cs, y = R.y0 + (int32_t)((sl >> 2) & 3u) * cs, z = R.z0 + (int32_t)(sl >> 4) * cs;
    const uint32_t c = g_classify(T, x, y, z, cs, k);
    const uint64_t kid = __ballot(c != G_EMPTY), mix = __ballot(c == G_MIXED);
    const uint64_t below = (1ull << sl) - 1ull;
    const uint64_t kpos = base + koff[r] + (uint64_t)__popcll(kid & below);
    if (c == G_MIXED) {
        next[moff[r] + (uint64_t)__popcll(mix & below)] = Region{x, y, z, (uint32_t)kpos};
    } else if (c != G_EMPTY) {
        nodes[kpos] = Node{~0ull, 0u, K_SOLID | (c << 16)};
    }
    if (sl == 0) nodes[R.node] = Node{kid, (uint32_t)(base + koff[r]), K_INTERIOR};
}

// bricks: one wavefront per brick region, lane = voxel (z<<4 | y<<2 | x)
__device__ __forceinline__ uint32_t g_voxel(const DevTerrain& T, const Region& R, uint32_t v) {
    const int32_t x = R.x0 + (int32_t)(v & 3u), y = R.y0 + (int32_t)((v >> 2) & 3u), z = R.z0 + (int32_t)(v >> 4);
    if (x >= T.W || z >= T.L) return G_EMPTY;
    return g_solid_class(T, T.h[(size_t)x * T.L + z], y);
}

__device__ __forceinline__ bool g_uniform(uint32_t c, uint64_t solid) {
    const uint32_t first = (uint32_t)__shfl((int)c, (int)__builtin_ctzll(solid | (1ull << 63)));
    return __ballot(c != G_EMPTY && c != first) == 0ull;
}

__global__ void k_brick_count(DevTerrain T, const Region* cur, int64_t r0, int64_t n, uint32_t* nmat) {
    const int64_t r = r0 + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t v = threadIdx.x & 63u;
    if (r >= n) return;
    const uint32_t c = g_voxel(T, cur[r], v);
    const uint64_t solid = __ballot(c != G_EMPTY);
    const bool uni = g_uniform(c, solid);
    if (v == 0) nmat[r] = uni ? 0u : (uint32_t)__popcll(solid);
}

__global__ void k_brick_write(DevTerrain T, const Region* cur, int64_t r0, int64_t n, const uint64_t* moff, Node* nodes, uint16_t* mats) {
    const int64_t r = r0 + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t v = threadIdx.x & 63u;
    if (r >= n) return;
    const Region R = cur[r];
    const uint32_t c = g_voxel(T, R, v);
    const uint64_t solid = __ballot(c != G_EMPTY);
    const bool uni = g_uniform(c, solid);
    const uint32_t first = (uint32_t)__shfl((int)c, (int)__builtin_ctzll(solid | (1ull << 63)));
    if (!uni && c != G_EMPTY) mats[moff[r] + (uint64_t)__popcll(solid & ((1ull << v) - 1ull))] = (uint16_t)c;
    if (v == 0) nodes[R.node] = uni ? Node{solid, 0u, K_BRICK | K_UNIFORM | (first << 16)} : Node{solid, (uint32_t)moff[r], K_BRICK};
}

// exclusive scan of n counts; returns the total
int scan(const uint32_t* in, uint64_t* out, int64_t n, uint64_t* total, std::vector<void*>& tmp_pool) {
    if (n == 0) {
        *total = 0;
        return SVO_OK;
    }
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, (int)n), SVO_EDEVICE);
    void* tmp = nullptr;
    HIP_TRY(hipMalloc(&tmp, std::max<size_t>(tb, 16)), SVO_ENOMEM);
    tmp_pool.push_back(tmp);
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, in, out, (int)n), SVO_EDEVICE);
    uint64_t last = 0;
    uint32_t lastc = 0;
    HIP_TRY(hipMemcpy(&last, out + n - 1, 8, hipMemcpyDeviceToHost), SVO_EDEVICE);
    HIP_TRY(hipMemcpy(&lastc, in + n - 1, 4, hipMemcpyDeviceToHost), SVO_EDEVICE);
    *total = last + lastc;
    return SVO_OK;
}

// device allocations of one build, freed on every exit
struct Pool {
    std::vector<void*> p;
    ~Pool() {
        for (void* x : p)
            if (x) (void)hipFree(x);
    }
    template <class T>
    int alloc(T** out, size_t n) {
        void* x = nullptr;
        HIP_TRY(hipMalloc(&x, std::max<size_t>(n * sizeof(T), 16)), SVO_ENOMEM);
        p.push_back(x);
        *out = reinterpret_cast<T*>(x);
        return SVO_OK;
    }
    void release(void* x) {  // hand over ownership
        for (auto& y : p)
            if (y == x) y = nullptr;
    }
};

inline uint32_t blocks_for(int64_t threads, int bs) { return (uint32_t)((threads + bs - 1) / bs); }

// A dispatch holds fewer than 2^32 work-items (the HSA packet's grid size is 32-bit): the one-wave-per-
// region kernels run over chunks of at most 2^24 regions (2^30 work-items).
constexpr int64_t kRegionChunk = (int64_t)1 << 24;
template <class F>
int for_region_chunks(int64_t n, F&& launch) {
    for (int64_t r0 = 0; r0 < n; r0 += kRegionChunk) {
        const int64_t m = std::min(kRegionChunk, n - r0);
        launch(r0, dim3(blocks_for(m * 64, 256)));
        HIP_TRY(hipGetLastError(), SVO_EDEVICE);
    }
    return SVO_OK;
}

int build_on_device(int32_t levels, int32_t W, int32_t L, int16_t* dh, Pool& pool, int32_t device, int32_t view, svo_tree** out) {
    const int32_t E = 1 << (2 * levels);
    DevTerrain T;
    memset(&T, 0, sizeof(T));
    T.levels = levels;
    T.E = E;
    T.W = W;
    T.L = L;
    T.h = dh;
    T.id_of[TM_AIR] = G_EMPTY;
    T.id_of[TM_WATER] = view ? 4u : G_EMPTY;
    T.view = view;
    T.id_of[TM_GRASS] = 1;
    T.id_of[TM_DIRT] = 2;
    T.id_of[TM_STONE] = 3;
    // ---- min / max pyramid
    T.hmin[0] = T.hmax[0] = dh;
    T.dimz[0] = L;
    int32_t px = W, pz = L;
    for (int k = 1; k <= levels; k++) {
        const int32_t dx = (px + 3) / 4, dz = (pz + 3) / 4;
        int16_t *mn, *mx;
        int rc = pool.alloc(&mn, (size_t)dx * dz);
        if (!rc) rc = pool.alloc(&mx, (size_t)dx * dz);
        if (rc) return rc;
        hipLaunchKernelGGL(k_pyramid, dim3(blocks_for((int64_t)dx * dz, 256)), dim3(256), 0, nullptr, T.hmin[k - 1], T.hmax[k - 1], px, pz,
                           mn, mx, dx, dz);
        HIP_TRY(hipGetLastError(), SVO_EDEVICE);
        T.hmin[k] = mn;
        T.hmax[k] = mx;
        T.dimz[k] = dz;
        px = dx;
        pz = dz;
    }
    int16_t top_max = 0;
    HIP_TRY(hipMemcpy(&top_max, T.hmax[levels], 2, hipMemcpyDeviceToHost), SVO_EDEVICE);
    if (top_max + 1 >= E || 21 >= E)
        SVO_FAIL(SVO_ERANGE, "svo_build_terrain_gpu: a column top falls outside [0, extent-2] (wrap not supported here)");

    svo_tree* t = new (std::nothrow) svo_tree();
    if (!t) SVO_FAIL(SVO_ENOMEM, "svo_build_terrain_gpu: out of memory");
    std::unique_ptr<svo_tree> guard(t);
    t->levels = levels;
    t->view = view;
    t->palette.push_back(Material{0, ~0ull, 0.0f});
    t->palette.push_back(Material{1u, rgb_to_u64(0, 150, 10), 0.0f});         // 1 grass
    t->palette.push_back(Material{1u, rgb_to_u64(45, 18, 0), 0.0f});          // 2 dirt
    t->palette.push_back(Material{1u, rgb_to_u64(33, 33, 33), 0.0f});         // 3 stone
    t->palette.push_back(Material{1u | 0x14u, rgb_to_u64(0, 150, 10), 0.0f});  // 4 water (LIQUID)

    // node array: grown per level (capacity doubling, device copies)
    uint64_t cap = 1 << 16, used = 1;
    Node* nodes;
    int rc = pool.alloc(&nodes, cap);
    if (rc) return rc;
    auto reserve = [&](uint64_t need) -> int {
        if (need <= cap) return SVO_OK;
        uint64_t nc = cap;
        while (nc < need) nc *= 2;
        Node* nn;
        int r2 = pool.alloc(&nn, nc);
        if (r2) return r2;
        HIP_TRY(hipMemcpy(nn, nodes, used * sizeof(Node), hipMemcpyDeviceToDevice), SVO_EDEVICE);
        pool.release(nodes);
        (void)hipFree(nodes);
        nodes = nn;
        cap = nc;
        return SVO_OK;
    };
    uint16_t* mats = nullptr;
    uint64_t n_mats = 0;
    std::vector<void*> tmp;

    // root: classified on the host side of the pyramid's top
    Region root{0, 0, 0, 0};
    Region* cur;
    rc = pool.alloc(&cur, 1);
    if (rc) return rc;
    HIP_TRY(hipMemcpy(cur, &root, sizeof(Region), hipMemcpyHostToDevice), SVO_EDEVICE);
    int64_t ncur = 1;
    t->nodes_per_level[0] = 1;
    const Node empty_root{0, 0, K_INTERIOR};
    HIP_TRY(hipMemcpy(nodes, &empty_root, sizeof(Node), hipMemcpyHostToDevice), SVO_EDEVICE);
    for (int d = 0; d < levels && ncur > 0; d++) {
        const int32_t cs = 1 << (2 * (levels - d - 1));
        if (d == levels - 1) {
            uint32_t* nmat;
            uint64_t* moff;
            rc = pool.alloc(&nmat, ncur);
            if (!rc) rc = pool.alloc(&moff, ncur);
            if (rc) return rc;
            rc = for_region_chunks(ncur, [&](int64_t r0, dim3 g) {
                hipLaunchKernelGGL(k_brick_count, g, dim3(256), 0, nullptr, T, cur, r0, ncur, nmat);
            });
            if (rc) return rc;
            rc = scan(nmat, moff, ncur, &n_mats, tmp);
            if (rc) return rc;
            rc = pool.alloc(&mats, n_mats + 1);
            if (rc) return rc;
            rc = for_region_chunks(ncur, [&](int64_t r0, dim3 g) {
                hipLaunchKernelGGL(k_brick_write, g, dim3(256), 0, nullptr, T, cur, r0, ncur, moff, nodes, mats);
            });
            if (rc) return rc;
            t->n_bricks = (uint64_t)ncur;
            break;
        }
        uint32_t *nkid, *nmix;
        uint64_t *koff, *moff, nk = 0, nm = 0;
        rc = pool.alloc(&nkid, ncur);
        if (!rc) rc = pool.alloc(&nmix, ncur);
        if (!rc) rc = pool.alloc(&koff, ncur);
        if (!rc) rc = pool.alloc(&moff, ncur);
        if (rc) return rc;
        // the root is a region like any other (its record may become SOLID: handled below)
        rc = for_region_chunks(ncur, [&](int64_t r0, dim3 g) {
            hipLaunchKernelGGL(k_count, g, dim3(256), 0, nullptr, T, cur, r0, ncur, cs, levels - d - 1, nkid, nmix);
        });
        if (rc) return rc;
        rc = scan(nkid, koff, ncur, &nk, tmp);
        if (!rc) rc = scan(nmix, moff, ncur, &nm, tmp);
        if (rc) return rc;
        if (used + nk > 0xFFFFFFFFull) SVO_FAIL(SVO_ERANGE, "svo_build_terrain_gpu: tree exceeds 2^32 nodes");
        rc = reserve(used + nk);
        if (rc) return rc;
        Region* next;
        rc = pool.alloc(&next, nm);
        if (rc) return rc;
        rc = for_region_chunks(ncur, [&](int64_t r0, dim3 g) {
            hipLaunchKernelGGL(k_write, g, dim3(256), 0, nullptr, T, cur, r0, ncur, cs, levels - d - 1, koff, moff, used, nodes, next);
        });
        if (rc) return rc;
        t->nodes_per_level[d + 1] = nk;
        used += nk;
        cur = next;
        ncur = (int64_t)nm;
    }
    HIP_TRY(hipDeviceSynchronize(), SVO_EDEVICE);
    for (void* x : tmp) (void)hipFree(x);
    // (the root is never uniform SOLID: the extent reaches above every column, checked above)
    // host image + adoption of the device arrays (with slack for edits)
    const uint64_t ncap = std::min<uint64_t>(used + used / 8 + 65536, 1ull << 32), mcap = std::min<uint64_t>(n_mats + n_mats / 8 + 65536, 1ull << 32);
    Node* dn;
    uint16_t* dm;
    rc = pool.alloc(&dn, ncap);
    if (!rc) rc = pool.alloc(&dm, mcap);
    if (rc) return rc;
    HIP_TRY(hipMemcpy(dn, nodes, used * sizeof(Node), hipMemcpyDeviceToDevice), SVO_EDEVICE);
    if (n_mats) HIP_TRY(hipMemcpy(dm, mats, n_mats * sizeof(uint16_t), hipMemcpyDeviceToDevice), SVO_EDEVICE);
    t->nodes.resize(used);
    t->mats.resize(n_mats);
    HIP_TRY(hipMemcpy(t->nodes.data(), dn, used * sizeof(Node), hipMemcpyDeviceToHost), SVO_EDEVICE);
    if (n_mats) HIP_TRY(hipMemcpy(t->mats.data(), dm, n_mats * sizeof(uint16_t), hipMemcpyDeviceToHost), SVO_EDEVICE);
    pool.release(dn);
    pool.release(dm);
    rc = adopt_device(t, device, dn, ncap, dm, mcap);
    if (rc) {
        (void)hipFree(dn);
        (void)hipFree(dm);
        return rc;
    }
    *out = guard.release();
    return SVO_OK;
}

}  // namespace

extern "C" int svo_build_terrain_gpu(int32_t levels, int32_t width, int32_t length, int32_t device, svo_tree** out) {
    return svo_build_terrain_gpu_view(levels, width, length, device, SVO_VIEW_SOLID, out);
}

extern "C" int svo_build_terrain_gpu_view(int32_t levels, int32_t width, int32_t length, int32_t device, int32_t view, svo_tree** out) {
    if (!out) SVO_FAIL(SVO_EINVAL, "svo_build_terrain_gpu: out is NULL");
    if (view != SVO_VIEW_SOLID && view != SVO_VIEW_ALL) SVO_FAIL(SVO_EINVAL, "svo_build_terrain_gpu: unknown view");
    if (levels < 2 || levels > 7) SVO_FAIL(SVO_EINVAL, "svo_build_terrain_gpu: levels must be in [2, 7]");
    const int32_t E = 1 << (2 * levels);
    if (width < 1 || length < 1 || width > E || length > E) SVO_FAIL(SVO_EINVAL, "svo_build_terrain_gpu: columns must fit the extent");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev), SVO_EDEVICE);
    if (device < 0 || device >= ndev) SVO_FAIL(SVO_EDEVICE, "svo_build_terrain_gpu: no such HIP device");
    HIP_TRY(hipSetDevice(device), SVO_EDEVICE);
    Pool pool;
    uint8_t perms[768];
    {
        Simplex2 a, b, c;
        simplex2_seed(a, 42);
        simplex2_seed(b, 64);
        simplex2_seed(c, 100);
        memcpy(perms, a.perm, 256);
        memcpy(perms + 256, b.perm, 256);
        memcpy(perms + 512, c.perm, 256);
    }
    uint8_t* dperm;
    int16_t* dh;
    int32_t* dbad;
    int rc = pool.alloc(&dperm, 768);
    if (!rc) rc = pool.alloc(&dh, (size_t)width * length);
    if (!rc) rc = pool.alloc(&dbad, 1);
    if (rc) return rc;
    HIP_TRY(hipMemcpy(dperm, perms, 768, hipMemcpyHostToDevice), SVO_EDEVICE);
    HIP_TRY(hipMemset(dbad, 0, 4), SVO_EDEVICE);
    hipLaunchKernelGGL(k_heights, dim3(blocks_for((int64_t)width * length, 256)), dim3(256), 0, nullptr, dperm, width, length, dh, dbad);
    HIP_TRY(hipGetLastError(), SVO_EDEVICE);
    int32_t bad = 0;
    HIP_TRY(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost), SVO_EDEVICE);
    if (bad) SVO_FAIL(SVO_ERANGE, "svo_build_terrain_gpu: a column top falls outside [0, 32767]");
    return build_on_device(levels, width, length, dh, pool, device, view, out);
}

extern "C" int svo_build_heightfield_gpu(int32_t levels, int32_t width, int32_t length, const int32_t* heights, int32_t device,
                                         svo_tree** out) {
    if (!out || !heights) SVO_FAIL(SVO_EINVAL, "svo_build_heightfield_gpu: NULL argument");
    if (levels < 2 || levels > 7) SVO_FAIL(SVO_EINVAL, "svo_build_heightfield_gpu: levels must be in [2, 7]");
    const int32_t E = 1 << (2 * levels);
    if (width < 1 || length < 1 || width > E || length > E) SVO_FAIL(SVO_EINVAL, "svo_build_heightfield_gpu: columns must fit the extent");
    std::vector<int16_t> hg((size_t)width * length);
    for (size_t i = 0; i < hg.size(); i++) {
        if (heights[i] < 0 || heights[i] > 32767) SVO_FAIL(SVO_ERANGE, "svo_build_heightfield_gpu: heights must be in [0, extent-2]");
        hg[i] = (int16_t)heights[i];
    }
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev), SVO_EDEVICE);
    if (device < 0 || device >= ndev) SVO_FAIL(SVO_EDEVICE, "svo_build_heightfield_gpu: no such HIP device");
    HIP_TRY(hipSetDevice(device), SVO_EDEVICE);
    Pool pool;
    int16_t* dh;
    int rc = pool.alloc(&dh, hg.size());
    if (rc) return rc;
    HIP_TRY(hipMemcpy(dh, hg.data(), hg.size() * sizeof(int16_t), hipMemcpyHostToDevice), SVO_EDEVICE);
    return build_on_device(levels, width, length, dh, pool, device, SVO_VIEW_SOLID, out);
}
