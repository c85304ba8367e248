// svo_cast.hip — gfx950 kernels of libsvo_rt: the primary-ray SVO traversal that replaces
// RAY_CASTER::castRayFromCam (src/ray_caster.cpp:54-87) and the DDA + tree walk of
// src/shaders/low_res.frag:256-333,446-531, plus device upload (the updateSsboData analogue,
// src/voxel_data/voxel_allocator.hpp:38-91) and the cast entry points of include/svo_rt.h.
//
// Semantics are castRayFromCam's, bit for bit: FP64 DDA from trunc(origin), strict-< axis choice
// with ties / NaN falling to z, one voxel per step, the start voxel never tested, LIQUID and empty
// blocks passed through, coordinates wrapped modulo the extent.  What the kernel changes is how a
// step finds its block: the ray keeps the deepest region it knows (an empty child region of some
// level, or a 4^3 brick whose 64-bit solid mask sits in registers) and only walks the tree again
// when a step leaves that region, so most steps touch no memory.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "../../include/svo_rt.h"
#include "svo_internal.h"

using namespace svo;

#define SVO_FAIL(code, msg)     \
    do {                        \
        svo::set_error(msg);    \
        return (code);          \
    } while (0)

#define HIP_TRY(expr, code)                                                                    \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            svo::set_error(std::string(#expr " failed: ") + hipGetErrorString(e_));            \
            return (code);                                                                     \
        }                                                                                      \
    } while (0)

namespace {

enum : int32_t { MODE_FRAME = 0, MODE_EXPLICIT = 1, MODE_SINGLE = 2 };

struct CastParams {
    const Node* nodes;
    const uint16_t* mats;
    int32_t levels;
    uint32_t wmask;
    int32_t mode;
    int32_t steps;
    // frame mode
    RayGen rg;
    float org[3];
    float sdir[3];
    int32_t width, height, tiles_x, tile_row_start, tile_row_step, tile_rows_local;
    // explicit mode
    const float* rdir;
    const float* rorg;
    int64_t n_rays;
    // outputs
    int32_t* pos;
    float* t;
    uint32_t* info;
};

constexpr int kBlock = 256;

struct Hit {
    int32_t x, y, z, steps_left;
    float t;
    uint32_t info;
};

// One ray, castRayFromCam semantics.  Region cache: (cwx,cwy,cwz) >> cshift identifies the region
// the last lookup ended in: an empty child region (no memory access while inside it) or a brick
// (solid mask in registers).
__device__ __forceinline__ Hit trace(const CastParams& P, const float o[3], const float d[3]) {
    const Dda1 ax = dda_axis(o[0], d[0]);
    const Dda1 ay = dda_axis(o[1], d[1]);
    const Dda1 az = dda_axis(o[2], d[2]);
    int32_t rx = ax.cell, ry = ay.cell, rz = az.cell;
    double tx = ax.dpos, ty = ay.dpos, tz = az.dpos;
    int32_t steps = P.steps;
    uint32_t axis = 3u;
    double tlast = 0.0;
    bool hit = false;
    uint32_t mat = 0;
    bool cvalid = false, cbrick = false;
    uint32_t cwx = 0, cwy = 0, cwz = 0, cshift = 0;
    uint64_t bmask = 0;
    uint32_t bref = 0, binfo = 0;
    const uint32_t wm = P.wmask;
    while (steps > 0) {
        // ray_caster.cpp:71-80
        const bool sx = (tx < ty) && (tx < tz);
        const bool sy = !sx && (ty < tz);
        if (sx) {
            rx += ax.step;
            tlast = tx;
            tx += ax.adelta;
            axis = 0u;
        } else if (sy) {
            ry += ay.step;
            tlast = ty;
            ty += ay.adelta;
            axis = 1u;
        } else {
            rz += az.step;
            tlast = tz;
            tz += az.adelta;
            axis = 2u;
        }
        steps--;
        const uint32_t wx = (uint32_t)rx & wm, wy = (uint32_t)ry & wm, wz = (uint32_t)rz & wm;
        if (!cvalid || (((wx ^ cwx) | (wy ^ cwy) | (wz ^ cwz)) >> cshift) != 0u) {
            // walk from the root (tetrahexa_tree.cpp:124-152 / low_res.frag:493-531)
            cvalid = true;
            cbrick = false;
            cwx = wx;
            cwy = wy;
            cwz = wz;
            cshift = 0u;
            uint32_t ni = 0u;
            for (int32_t dd = 0; dd < P.levels; dd++) {
                const Node n = P.nodes[ni];
                const uint32_t kind = n.info & K_KIND_MASK;
                if (kind == K_SOLID) {
                    hit = true;
                    mat = n.info >> 16;
                    break;
                }
                if (kind == K_BRICK) {
                    cbrick = true;
                    bmask = n.mask;
                    bref = n.ref;
                    binfo = n.info;
                    cshift = 2u;
                    break;
                }
                const uint32_t sh = (uint32_t)(2 * (P.levels - 1 - dd));
                const uint32_t sl = child_slot(wx, wy, wz, sh);
                if (!((n.mask >> sl) & 1ull)) {
                    cshift = sh;
                    break;
                }
                ni = n.ref + (uint32_t)__popcll(n.mask & ((1ull << sl) - 1ull));
            }
            if (hit) break;
        }
        if (cbrick) {
            const uint32_t v = child_slot(wx, wy, wz, 0u);
            if ((bmask >> v) & 1ull) {
                hit = true;
                mat = (binfo & K_UNIFORM) ? (binfo >> 16) : (uint32_t)P.mats[bref + (uint32_t)__popcll(bmask & ((1ull << v) - 1ull))];
                break;
            }
        }
    }
    Hit h;
    h.x = rx;
    h.y = ry;
    h.z = rz;
    h.steps_left = hit ? steps : 0;
    h.t = (float)tlast;
    uint32_t neg = 0u;
    if (axis == 0u) neg = ax.step < 0;
    else if (axis == 1u) neg = ay.step < 0;
    else if (axis == 2u) neg = az.step < 0;
    h.info = (hit ? HIT_BIT : 0u) | (axis << AXIS_SHIFT) | (neg ? NEG_BIT : 0u) | (mat & MAT_MASK);
    return h;
}

__global__ __launch_bounds__(kBlock) void k_cast(const CastParams P) {
    const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    float o[3], d[3];
    int64_t out;
    if (P.mode == MODE_FRAME) {
        // 8x8 pixel tiles, one wavefront (64 lanes) per tile: tile-coherent rays share nodes
        const int64_t tile = g >> 6;
        const int32_t lane = (int32_t)(g & 63);
        const int32_t trl = (int32_t)(tile / P.tiles_x);
        const int32_t tx = (int32_t)(tile - (int64_t)trl * P.tiles_x);
        if (trl >= P.tile_rows_local) return;
        const int32_t tr = P.tile_row_start + trl * P.tile_row_step;
        const int32_t px = tx * 8 + (lane & 7), py = tr * 8 + (lane >> 3);
        if (px >= P.width || py >= P.height) return;
        raygen_pixel(P.rg, px, py, d);
        o[0] = P.org[0];
        o[1] = P.org[1];
        o[2] = P.org[2];
        out = ((int64_t)trl * 8 + (lane >> 3)) * P.width + px;
    } else if (P.mode == MODE_EXPLICIT) {
        if (g >= P.n_rays) return;
        d[0] = P.rdir[3 * g + 0];
        d[1] = P.rdir[3 * g + 1];
        d[2] = P.rdir[3 * g + 2];
        if (P.rorg) {
            o[0] = P.rorg[3 * g + 0];
            o[1] = P.rorg[3 * g + 1];
            o[2] = P.rorg[3 * g + 2];
        } else {
            o[0] = P.org[0];
            o[1] = P.org[1];
            o[2] = P.org[2];
        }
        out = g;
    } else {
        if (g != 0) return;
        for (int a = 0; a < 3; a++) {
            d[a] = P.sdir[a];
            o[a] = P.org[a];
        }
        out = 0;
    }
    const Hit h = trace(P, o, d);
    reinterpret_cast<int4*>(P.pos)[out] = make_int4(h.x, h.y, h.z, h.steps_left);
    P.t[out] = h.t;
    P.info[out] = h.info;
}

int fill_params(const svo_tree* t, const svo_cast_desc* d, const svo_hits* o, CastParams& P, int64_t& nthreads) {
    memset(&P, 0, sizeof(P));
    P.nodes = reinterpret_cast<const Node*>(t->d_nodes);
    P.mats = reinterpret_cast<const uint16_t*>(t->d_mats);
    P.levels = t->levels;
    P.wmask = (1u << (2 * t->levels)) - 1u;
    P.steps = d->steps;
    P.org[0] = d->origin[0];
    P.org[1] = d->origin[1];
    P.org[2] = d->origin[2];
    P.pos = o->pos_steps;
    P.t = o->t;
    P.info = o->info;
    if (d->ray_dirs) {
        P.mode = MODE_EXPLICIT;
        P.rdir = d->ray_dirs;
        P.rorg = d->ray_origins;
        P.n_rays = d->n_rays;
        nthreads = d->n_rays;
        return SVO_OK;
    }
    P.mode = MODE_FRAME;
    raygen_init(P.rg, d->cam_dir, d->ppx, d->ppy, d->width, d->height);
    P.width = d->width;
    P.height = d->height;
    P.tiles_x = (d->width + 7) / 8;
    P.tile_row_start = d->tile_row_start;
    P.tile_row_step = d->tile_row_step;
    const int32_t tile_rows = (d->height + 7) / 8;
    P.tile_rows_local = d->tile_row_start < tile_rows ? (tile_rows - d->tile_row_start + d->tile_row_step - 1) / d->tile_row_step : 0;
    nthreads = (int64_t)P.tile_rows_local * P.tiles_x * 64;
    return SVO_OK;
}

}  // namespace

// ================================================================================================
// device residency
// ================================================================================================
void svo::tree_release_device(svo_tree* t) {
    if (!t || t->device < 0) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(t->device);
    if (t->d_nodes) (void)hipFree(t->d_nodes);
    if (t->d_mats) (void)hipFree(t->d_mats);
    if (t->d_work) (void)hipFree(t->d_work);
    (void)hipSetDevice(prev);
    t->d_nodes = t->d_mats = t->d_work = nullptr;
    t->device = -1;
    t->device_bytes = 0;
}

extern "C" void svo_tree_destroy(svo_tree* t) {
    if (!t) return;
    tree_release_device(t);
    delete t;
}

extern "C" int svo_upload(svo_tree* t, int32_t device) {
    if (!t) SVO_FAIL(SVO_EINVAL, "svo_upload: NULL tree");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev), SVO_EDEVICE);
    if (device < 0 || device >= ndev) SVO_FAIL(SVO_EDEVICE, "svo_upload: no such HIP device");
    tree_release_device(t);
    HIP_TRY(hipSetDevice(device), SVO_EDEVICE);
    const size_t nb = t->nodes.size() * sizeof(Node);
    const size_t mb = std::max<size_t>(t->mats.size() * sizeof(uint16_t), 16);
    const size_t wb = 4096;
    HIP_TRY(hipMalloc(&t->d_nodes, nb), SVO_ENOMEM);
    HIP_TRY(hipMalloc(&t->d_mats, mb), SVO_ENOMEM);
    HIP_TRY(hipMalloc(&t->d_work, wb), SVO_ENOMEM);
    HIP_TRY(hipMemcpy(t->d_nodes, t->nodes.data(), nb, hipMemcpyHostToDevice), SVO_EDEVICE);
    if (!t->mats.empty()) HIP_TRY(hipMemcpy(t->d_mats, t->mats.data(), t->mats.size() * sizeof(uint16_t), hipMemcpyHostToDevice), SVO_EDEVICE);
    HIP_TRY(hipMemset(t->d_work, 0, wb), SVO_EDEVICE);
    t->device = device;
    t->device_bytes = nb + mb + wb;
    t->work_slots = (uint32_t)(wb / sizeof(uint32_t));
    t->work_next = 0;
    return SVO_OK;
}

// ================================================================================================
// casting
// ================================================================================================
extern "C" int svo_cast_rays(const svo_tree* t, const svo_cast_desc* d, const svo_hits* o, void* stream) {
    if (!t || !d || !o) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: NULL argument");
    if (!o->pos_steps || !o->t || !o->info) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: NULL output buffer");
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, "svo_cast_rays: tree not uploaded (svo_upload)");
    if (d->steps < 0) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: negative step budget");
    if (d->ray_dirs) {
        if (d->n_rays < 0) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: negative ray count");
    } else if (d->width <= 0 || d->height <= 0 || d->tile_row_step <= 0 || d->tile_row_start < 0) {
        SVO_FAIL(SVO_EINVAL, "svo_cast_rays: bad frame geometry");
    }
    CastParams P;
    int64_t n = 0;
    int rc = fill_params(t, d, o, P, n);
    if (rc) return rc;
    if (n == 0) return SVO_OK;
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    const int64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks > 0x7FFFFFFF) SVO_FAIL(SVO_ERANGE, "svo_cast_rays: too many rays for one launch");
    hipLaunchKernelGGL(k_cast, dim3((uint32_t)blocks), dim3(kBlock), 0, (hipStream_t)stream, P);
    HIP_TRY(hipGetLastError(), SVO_EDEVICE);
    return SVO_OK;
}

extern "C" int svo_cast_ray_from_cam(const svo_tree* t, const float pos[3], const float dir[3], int32_t steps, svo_ray_result* out,
                                     svo_block* block) {
    if (!t || !pos || !dir || !out) SVO_FAIL(SVO_EINVAL, "svo_cast_ray_from_cam: NULL argument");
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, "svo_cast_ray_from_cam: tree not uploaded (svo_upload)");
    if (steps < 0) SVO_FAIL(SVO_EINVAL, "svo_cast_ray_from_cam: negative step budget");
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    void* buf = nullptr;
    HIP_TRY(hipMalloc(&buf, 64), SVO_ENOMEM);
    CastParams P;
    memset(&P, 0, sizeof(P));
    P.nodes = reinterpret_cast<const Node*>(t->d_nodes);
    P.mats = reinterpret_cast<const uint16_t*>(t->d_mats);
    P.levels = t->levels;
    P.wmask = (1u << (2 * t->levels)) - 1u;
    P.mode = MODE_SINGLE;
    P.steps = steps;
    for (int a = 0; a < 3; a++) {
        P.org[a] = pos[a];
        P.sdir[a] = dir[a];
    }
    P.pos = reinterpret_cast<int32_t*>(buf);
    P.t = reinterpret_cast<float*>(reinterpret_cast<char*>(buf) + 16);
    P.info = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(buf) + 32);
    hipLaunchKernelGGL(k_cast, dim3(1), dim3(kBlock), 0, nullptr, P);
    unsigned char host[64];
    hipError_t e = hipMemcpy(host, buf, 64, hipMemcpyDeviceToHost);
    (void)hipFree(buf);
    if (e != hipSuccess) SVO_FAIL(SVO_EDEVICE, std::string("svo_cast_ray_from_cam: ") + hipGetErrorString(e));
    int32_t p4[4];
    uint32_t info;
    memcpy(p4, host, 16);
    memcpy(&info, host + 32, 4);
    for (int a = 0; a < 3; a++) out->pos[a] = out->last_pos[a] = p4[a];
    out->steps = p4[3];
    const uint32_t axis = (info >> AXIS_SHIFT) & 3u;
    if (axis < 3u) out->last_pos[axis] -= (info & NEG_BIT) ? -1 : 1;
    if (block) {
        const Material& m = t->palette[(info & HIT_BIT) ? (info & MAT_MASK) : 0u];
        *block = svo_block{m.flags, m.color, m.meta};
    }
    return SVO_OK;
}

extern "C" int svo_sync(void* stream) {
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream), SVO_EDEVICE);
    return SVO_OK;
}
