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
    int32_t flags;
    unsigned long long* stats;
    uint32_t lds_nodes;
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
constexpr uint32_t kLdsNodes = 512;  // 8 KB of LDS per block

struct Hit {
    int32_t x, y, z, steps_left;
    float t;
    uint32_t info;
};

// ------------------------------------------------------------------------------------------------
// Exact closed-form skipping.  castRayFromCam's axis choice (ray_caster.cpp:71-80) is, for non-NaN
// values, the lexicographic minimum of (T_axis, rank) with rank z < y < x: x wins only when
// strictly smallest, y beats z only when strictly smaller.  Each axis' crossings form the sequence
// T, T+a, T+2a, ... (deltaPos += absDelta).  absDelta is an f32 reciprocal widened to f64, so it
// carries 24 significant bits; when every partial sum a ray can reach (<= budget+2 terms) stays
// below 2^(lsb+53) — lsb = lowest set bit of T and a — every sum is exact and T + k*a computed
// directly equals the k-fold accumulation bit for bit.  Such a ray ("fast") crosses an empty
// region in O(1): the first event to leave the region is the lexicographic minimum of the three
// per-axis exit events, and the events before it on the other axes are counted by division
// (with an exact +-1 fix-up).  Rays that fail the test step voxel by voxel (still without memory
// traffic inside known-empty regions).  Both paths give identical results (tests).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int dbl_lsb(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const int ef = (int)((b >> 52) & 0x7FF);
    uint64_t m = b & 0xFFFFFFFFFFFFFull;
    if (ef == 0) return m ? -1074 + __builtin_ctzll(m) : (1 << 20);
    return ef - 1075 + __builtin_ctzll(m | (1ull << 52));
}

__device__ __forceinline__ int dbl_ilogb(double x) {  // x > 0, normal
    return (int)(((uint64_t)__double_as_longlong(x) >> 52) & 0x7FF) - 1023;
}

__device__ __forceinline__ bool exact_axis(double T, double a, int32_t budget) {
    if (!__builtin_isfinite(T) || !__builtin_isfinite(a) || !(a > 0.0)) return false;
    const int u = min(dbl_lsb(T), dbl_lsb(a));
    const double bound = __builtin_fabs(T) + (double)(budget + 2) * a;
    return dbl_ilogb(bound) + 1 <= u + 52;  // bound < 2^(u+52): the unrounded bound < 2^(u+53)
}

// #{ j >= 0 : T + j*a < V }  and  #{ j >= 0 : T + j*a <= V }, exact under exact_axis.  q = (V-T)/a
// is estimated to within 1 (relative error ~2^-51), k0 = floor(q), and the exact remainder
// r0 = V - (T + k0*a) (both terms on the ray's 2^lsb grid, below 2^(lsb+53)) picks k0, k0+1 or k0+2.
// A count above the budget may be off, but then the skip is rejected anyway (total > steps).
__device__ __forceinline__ int32_t count_lt(double T, double a, double inva, double V) {
    if (!(T < V)) return 0;
    const int32_t k0 = (int32_t)((V - T) * inva);
    const double r0 = V - (T + (double)k0 * a);
    return k0 + (r0 > 0.0 ? 1 : 0) + (r0 > a ? 1 : 0);
}
__device__ __forceinline__ int32_t count_le(double T, double a, double inva, double V) {
    if (T > V) return 0;
    const int32_t k0 = (int32_t)((V - T) * inva);
    const double r0 = V - (T + (double)k0 * a);
    return k0 + (r0 >= 0.0 ? 1 : 0) + (r0 >= a ? 1 : 0);
}

struct Ray {
    int32_t rx, ry, rz;
    double tx, ty, tz;  // next crossing per axis (deltaPos)
    double ax, ay, az;  // absDelta
    int32_t sx, sy, sz;
    int32_t steps;
    uint32_t axis;
    double tlast;
};

// one DDA step (ray_caster.cpp:70-80)
__device__ __forceinline__ void dda_step(Ray& R) {
    const bool cx = (R.tx < R.ty) && (R.tx < R.tz);
    const bool cy = !cx && (R.ty < R.tz);
    if (cx) {
        R.rx += R.sx;
        R.tlast = R.tx;
        R.tx += R.ax;
        R.axis = 0u;
    } else if (cy) {
        R.ry += R.sy;
        R.tlast = R.ty;
        R.ty += R.ay;
        R.axis = 1u;
    } else {
        R.rz += R.sz;
        R.tlast = R.tz;
        R.tz += R.az;
        R.axis = 2u;
    }
    R.steps--;
}

// steps along one axis until the wrapped coordinate w leaves its aligned 2^sh cell
__device__ __forceinline__ int32_t exit_steps(uint32_t w, int32_t s, uint32_t sh) {
    const uint32_t lo = w & ~((1u << sh) - 1u);
    return s > 0 ? (int32_t)(lo + (1u << sh) - w) : (int32_t)(w - lo + 1u);
}

// Cross the empty aligned cell of size 2^sh containing the current voxel in one move.  Returns
// false (state unchanged) when the budget ends inside the cell.
__device__ __forceinline__ bool skip_cell(Ray& R, uint32_t wx, uint32_t wy, uint32_t wz, uint32_t sh, double iax, double iay,
                                          double iaz) {
    const int32_t lim = R.steps + 1;  // exits beyond the budget are clamped (safe: total > steps)
    const int32_t ex = min(exit_steps(wx, R.sx, sh), lim);
    const int32_t ey = min(exit_steps(wy, R.sy, sh), lim);
    const int32_t ez = min(exit_steps(wz, R.sz, sh), lim);
    const double Ex = R.tx + (double)(ex - 1) * R.ax;
    const double Ey = R.ty + (double)(ey - 1) * R.ay;
    const double Ez = R.tz + (double)(ez - 1) * R.az;
    int32_t cx, cy, cz, total;
    if ((Ex < Ey) && (Ex < Ez)) {  // x leaves first; y, z events tied with it come before it
        cy = count_le(R.ty, R.ay, iay, Ex);
        cz = count_le(R.tz, R.az, iaz, Ex);
        total = ex + cy + cz;
        if (total > R.steps) return false;
        R.rx += R.sx * ex;
        R.ry += R.sy * cy;
        R.rz += R.sz * cz;
        R.ty += (double)cy * R.ay;
        R.tz += (double)cz * R.az;
        R.tlast = Ex;
        R.tx = Ex + R.ax;
        R.axis = 0u;
    } else if (Ey < Ez) {  // y first; tied x events come after it, tied z events before
        cx = count_lt(R.tx, R.ax, iax, Ey);
        cz = count_le(R.tz, R.az, iaz, Ey);
        total = ey + cx + cz;
        if (total > R.steps) return false;
        R.rx += R.sx * cx;
        R.ry += R.sy * ey;
        R.rz += R.sz * cz;
        R.tx += (double)cx * R.ax;
        R.tz += (double)cz * R.az;
        R.tlast = Ey;
        R.ty = Ey + R.ay;
        R.axis = 1u;
    } else {  // z first; tied x and y events come after it
        cx = count_lt(R.tx, R.ax, iax, Ez);
        cy = count_lt(R.ty, R.ay, iay, Ez);
        total = ez + cx + cy;
        if (total > R.steps) return false;
        R.rx += R.sx * cx;
        R.ry += R.sy * cy;
        R.rz += R.sz * ez;
        R.tx += (double)cx * R.ax;
        R.ty += (double)cy * R.ay;
        R.tlast = Ez;
        R.tz = Ez + R.az;
        R.axis = 2u;
    }
    R.steps -= total;
    return true;
}

// Region lookup of a wrapped voxel: SOLID hit, an empty child cell (returns its shift), or the
// brick holding the voxel (mask / ref / info returned).  tetrahexa_tree.cpp:124-152 on the
// breadth-first layout.
enum : uint32_t { R_EMPTY = 0u, R_BRICK = 1u, R_SOLID = 2u };

struct Stats {
    uint32_t lookups, loads, skips, skip_out, brick_steps, plain_steps;
};

// wave-wide max / sum (diagnostics only)
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

// The interior node whose child region holds the ray's current cell, kept in registers: a move to
// a sibling region reads the cached child mask (no load when the sibling is empty) and restarts
// the descent at most one level down; leaving the parent's region restarts at the root, whose top
// levels are staged in LDS.
struct Parent {
    uint64_t mask;
    uint32_t ref;
    uint32_t sh;  // child shift: a child region is 2^sh voxels wide, the parent's 2^(sh+2)
    uint32_t wx, wy, wz;
    bool valid;
};

template <bool STATS>
__device__ __forceinline__ uint32_t lookup(const CastParams& P, const Node* __restrict__ lds, uint32_t nlds, uint32_t wx,
                                           uint32_t wy, uint32_t wz, Parent& par, uint32_t& sh_out, uint64_t& bmask,
                                           uint32_t& bref, uint32_t& binfo, Stats& st) {
    uint32_t ni = 0u;
    int32_t dd = 0;
    if (STATS) st.lookups++;
    if (par.valid && ((((wx ^ par.wx) | (wy ^ par.wy) | (wz ^ par.wz)) >> (par.sh + 2u)) == 0u)) {
        const uint32_t sl = child_slot(wx, wy, wz, par.sh);
        if (!((par.mask >> sl) & 1ull)) {
            sh_out = par.sh;
            return R_EMPTY;
        }
        ni = par.ref + (uint32_t)__popcll(par.mask & ((1ull << sl) - 1ull));
        dd = P.levels - (int32_t)(par.sh >> 1);  // depth of that child
    }
    for (; dd < P.levels; dd++) {
        const Node n = ni < nlds ? lds[ni] : P.nodes[ni];
        if (STATS) st.loads += ni < nlds ? 0u : 1u;
        const uint32_t kind = n.info & K_KIND_MASK;
        if (kind == K_SOLID) {
            binfo = n.info;
            return R_SOLID;
        }
        if (kind == K_BRICK) {
            bmask = n.mask;
            bref = n.ref;
            binfo = n.info;
            sh_out = 2u;
            return R_BRICK;
        }
        const uint32_t sh = (uint32_t)(2 * (P.levels - 1 - dd));
        par.mask = n.mask;
        par.ref = n.ref;
        par.sh = sh;
        par.wx = wx;
        par.wy = wy;
        par.wz = wz;
        par.valid = true;
        const uint32_t sl = child_slot(wx, wy, wz, sh);
        if (!((n.mask >> sl) & 1ull)) {
            sh_out = sh;
            return R_EMPTY;
        }
        ni = n.ref + (uint32_t)__popcll(n.mask & ((1ull << sl) - 1ull));
    }
    sh_out = 0u;  // malformed tree: treat as a one-voxel empty cell
    return R_EMPTY;
}

__device__ __forceinline__ uint32_t brick_material(const CastParams& P, uint64_t mask, uint32_t ref, uint32_t info, uint32_t v) {
    return (info & K_UNIFORM) ? (info >> 16) : (uint32_t)P.mats[ref + (uint32_t)__popcll(mask & ((1ull << v) - 1ull))];
}

// One ray with castRayFromCam semantics.
template <bool STATS, bool FLAT>
__device__ __forceinline__ Hit trace(const CastParams& P, const Node* __restrict__ lds, uint32_t nlds, const float o[3],
                                     const float d[3]) {
    Ray R;
    {
        const Dda1 ax = dda_axis(o[0], d[0]);
        const Dda1 ay = dda_axis(o[1], d[1]);
        const Dda1 az = dda_axis(o[2], d[2]);
        R.rx = ax.cell;
        R.ry = ay.cell;
        R.rz = az.cell;
        R.tx = ax.dpos;
        R.ty = ay.dpos;
        R.tz = az.dpos;
        R.ax = ax.adelta;
        R.ay = ay.adelta;
        R.az = az.adelta;
        R.sx = ax.step;
        R.sy = ay.step;
        R.sz = az.step;
    }
    R.steps = P.steps;
    R.axis = 3u;
    R.tlast = 0.0;
    const bool fast = !(P.flags & SVO_CAST_ITERATIVE) && exact_axis(R.tx, R.ax, P.steps) && exact_axis(R.ty, R.ay, P.steps) &&
                      exact_axis(R.tz, R.az, P.steps);
    const double iax = 1.0 / R.ax, iay = 1.0 / R.ay, iaz = 1.0 / R.az;
    bool hit = false;
    uint32_t mat = 0u;
    const uint32_t wm = P.wmask;
    Stats st = {0, 0, 0, 0, 0, 0};
    Parent par;
    par.valid = false;
    par.mask = 0ull;
    par.ref = par.sh = par.wx = par.wy = par.wz = 0u;
    if (FLAT) {
    // one action per iteration and lane (keeps the 64 lanes of a tile in step): a lookup of the voxel
    // just entered (+ an O(1) crossing when it lies in an empty cell), or one voxel step in a brick
    enum : uint32_t { M_LOOKUP = 0u, M_BRICK = 1u, M_DONE = 2u };
    uint32_t mode = M_DONE;
    if (R.steps > 0) {
        dda_step(R);
        mode = M_LOOKUP;
    }
    uint64_t bmask = 0ull;
    uint32_t bref = 0u, binfo = 0u, cwx = 0u, cwy = 0u, cwz = 0u;
    while (mode != M_DONE) {
        uint32_t wx = (uint32_t)R.rx & wm, wy = (uint32_t)R.ry & wm, wz = (uint32_t)R.rz & wm;
        if (mode == M_BRICK) {
            // one voxel step inside the brick, solid mask in registers
            dda_step(R);
            if (STATS) st.brick_steps++;
            wx = (uint32_t)R.rx & wm;
            wy = (uint32_t)R.ry & wm;
            wz = (uint32_t)R.rz & wm;
            if ((((wx ^ cwx) | (wy ^ cwy) | (wz ^ cwz)) >> 2) != 0u) {
                mode = M_LOOKUP;
                continue;
            }
            const uint32_t v = child_slot(wx, wy, wz, 0u);
            if ((bmask >> v) & 1ull) {
                hit = true;
                mat = brick_material(P, bmask, bref, binfo, v);
                mode = M_DONE;
            } else if (R.steps <= 0) {
                mode = M_DONE;
            }
            continue;
        }
        // M_LOOKUP: the voxel just entered is untested
        uint32_t sh = 0u;
        const uint32_t kind = lookup<STATS>(P, lds, nlds, wx, wy, wz, par, sh, bmask, bref, binfo, st);
        if (kind == R_SOLID) {
            hit = true;
            mat = binfo >> 16;
            mode = M_DONE;
        } else if (kind == R_BRICK) {
            cwx = wx;
            cwy = wy;
            cwz = wz;
            const uint32_t v = child_slot(wx, wy, wz, 0u);
            if ((bmask >> v) & 1ull) {
                hit = true;
                mat = brick_material(P, bmask, bref, binfo, v);
                mode = M_DONE;
            } else {
                mode = R.steps > 0 ? M_BRICK : M_DONE;
            }
        } else if (R.steps <= 0) {
            mode = M_DONE;
        } else if (fast && skip_cell(R, wx, wy, wz, sh, iax, iay, iaz)) {
            if (STATS) st.skips++;  // still M_LOOKUP: the exit voxel is untested
        } else {
            // budget ends inside the cell, or a non-exact ray: step through it without lookups
            if (STATS && fast) st.skip_out++;
            const uint32_t ewx = wx, ewy = wy, ewz = wz;
            bool left = false;
            while (R.steps > 0) {
                dda_step(R);
                if (STATS) st.plain_steps++;
                wx = (uint32_t)R.rx & wm;
                wy = (uint32_t)R.ry & wm;
                wz = (uint32_t)R.rz & wm;
                if ((((wx ^ ewx) | (wy ^ ewy) | (wz ^ ewz)) >> sh) != 0u) {
                    left = true;
                    break;
                }
            }
            mode = left ? M_LOOKUP : M_DONE;
        }
    }
    } else {
    if (R.steps > 0) {
        dda_step(R);
        for (;;) {
            // the voxel just entered is untested
            uint32_t wx = (uint32_t)R.rx & wm, wy = (uint32_t)R.ry & wm, wz = (uint32_t)R.rz & wm;
            uint32_t sh = 0u, bref = 0u, binfo = 0u;
            uint64_t bmask = 0ull;
            const uint32_t kind = lookup<STATS>(P, lds, nlds, wx, wy, wz, par, sh, bmask, bref, binfo, st);
            if (kind == R_SOLID) {
                hit = true;
                mat = binfo >> 16;
                break;
            }
            if (kind == R_BRICK) {
                // voxel steps inside the brick, solid mask in registers
                const uint32_t cwx = wx, cwy = wy, cwz = wz;
                bool left = false;
                for (;;) {
                    const uint32_t v = child_slot(wx, wy, wz, 0u);
                    if ((bmask >> v) & 1ull) {
                        hit = true;
                        mat = brick_material(P, bmask, bref, binfo, v);
                        break;
                    }
                    if (R.steps <= 0) break;
                    dda_step(R);
                    if (STATS) st.brick_steps++;
                    wx = (uint32_t)R.rx & wm;
                    wy = (uint32_t)R.ry & wm;
                    wz = (uint32_t)R.rz & wm;
                    if ((((wx ^ cwx) | (wy ^ cwy) | (wz ^ cwz)) >> 2) != 0u) {
                        left = true;
                        break;
                    }
                }
                if (hit || !left) break;
                continue;
            }
            // empty cell of size 2^sh around the voxel
            if (R.steps <= 0) break;
            if (fast) {
                if (skip_cell(R, wx, wy, wz, sh, iax, iay, iaz)) {
                    if (STATS) st.skips++;
                    continue;
                }
                if (STATS) st.skip_out++;
            }
            // step through the cell without lookups (budget ends inside it, or not exact)
            const uint32_t ewx = wx, ewy = wy, ewz = wz;
            bool left = false;
            while (R.steps > 0) {
                dda_step(R);
                if (STATS) st.plain_steps++;
                wx = (uint32_t)R.rx & wm;
                wy = (uint32_t)R.ry & wm;
                wz = (uint32_t)R.rz & wm;
                if ((((wx ^ ewx) | (wy ^ ewy) | (wz ^ ewz)) >> sh) != 0u) {
                    left = true;
                    break;
                }
            }
            if (!left) break;
        }
    }
    }
    if (STATS) {
        // SIMD efficiency: a lane's work units (lookups + voxel steps) against the wave's maximum
        const uint32_t work = st.lookups + st.brick_steps + st.plain_steps;
        const uint32_t wmax = wave_max(work), wsum = wave_sum(work);
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(P.stats + 7, (unsigned long long)wsum);
            atomicAdd(P.stats + 8, (unsigned long long)wmax * 64ull);
        }
        atomicAdd(P.stats + 0, 1ull);
        atomicAdd(P.stats + 1, (unsigned long long)st.lookups);
        atomicAdd(P.stats + 2, (unsigned long long)st.loads);
        atomicAdd(P.stats + 3, (unsigned long long)st.skips);
        atomicAdd(P.stats + 4, (unsigned long long)st.skip_out);
        atomicAdd(P.stats + 5, (unsigned long long)st.brick_steps);
        atomicAdd(P.stats + 6, (unsigned long long)st.plain_steps);
    }
    Hit h;
    h.x = R.rx;
    h.y = R.ry;
    h.z = R.rz;
    h.steps_left = hit ? R.steps : 0;
    h.t = (float)R.tlast;
    uint32_t neg = 0u;
    if (R.axis == 0u) neg = R.sx < 0;
    else if (R.axis == 1u) neg = R.sy < 0;
    else if (R.axis == 2u) neg = R.sz < 0;
    h.info = (hit ? HIT_BIT : 0u) | (R.axis << AXIS_SHIFT) | (neg ? NEG_BIT : 0u) | (mat & MAT_MASK);
    return h;
}

template <bool STATS, bool FLAT>
__global__ __launch_bounds__(kBlock) void k_cast(const CastParams P) {
    // diagnostics: block start / end stamps (100 MHz s_memrealtime) after the 16 counters
    unsigned long long t_start = 0;
    if (STATS && threadIdx.x == 0) t_start = __builtin_amdgcn_s_memrealtime();
    // top of the breadth-first array (root + the first levels) staged in LDS
    __shared__ Node lds[kLdsNodes];
    const uint32_t nlds = P.lds_nodes;
    for (uint32_t i = threadIdx.x; i < nlds; i += kBlock) lds[i] = P.nodes[i];
    __syncthreads();
    int64_t blk = blockIdx.x;
    if (P.flags & SVO_CAST_XCD_SWIZZLE) {
        // blocks are dealt round-robin to the 8 XCDs (blk % 8 share an L2): give each XCD one
        // contiguous band of tiles so neighbouring tiles hit the same L2
        const int64_t nb = gridDim.x, per = (nb + 7) / 8, x = blk & 7, k = blk >> 3;
        const int64_t full = nb - (per - 1) * 8;  // XCDs 0..full-1 receive `per` blocks
        blk = x < full ? x * per + k : full * per + (x - full) * (per - 1) + k;
    }
    const int64_t g = blk * kBlock + threadIdx.x;
    float o[3] = {0.0f, 0.0f, 0.0f}, d[3] = {0.0f, 0.0f, 0.0f};
    int64_t out = -1;
    if (P.mode == MODE_FRAME) {
        // 8x8 pixel tiles, one wavefront (64 lanes) per tile: tile-coherent rays share nodes
        const int64_t tile = g >> 6;
        const int32_t lane = (int32_t)(g & 63);
        int32_t trl = (int32_t)(tile / P.tiles_x);
        if (P.flags & SVO_CAST_TOP_FIRST) trl = P.tile_rows_local - 1 - trl;
        const int32_t tx = (int32_t)(tile - (int64_t)(tile / P.tiles_x) * P.tiles_x);
        const int32_t tr = P.tile_row_start + trl * P.tile_row_step;
        const int32_t px = tx * 8 + (lane & 7), py = tr * 8 + (lane >> 3);
        if (trl >= 0 && trl < P.tile_rows_local && px < P.width && py < P.height) {
            raygen_pixel(P.rg, px, py, d);
            o[0] = P.org[0];
            o[1] = P.org[1];
            o[2] = P.org[2];
            out = ((int64_t)trl * 8 + (lane >> 3)) * P.width + px;
        }
    } else if (P.mode == MODE_EXPLICIT) {
        if (g < P.n_rays) {
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
        }
    } else if (g == 0) {
        for (int a = 0; a < 3; a++) {
            d[a] = P.sdir[a];
            o[a] = P.org[a];
        }
        out = 0;
    }
    if (out >= 0) {
        const Hit h = trace<STATS, FLAT>(P, lds, nlds, o, d);
        reinterpret_cast<int4*>(P.pos)[out] = make_int4(h.x, h.y, h.z, h.steps_left);
        P.t[out] = h.t;
        P.info[out] = h.info;
    }
    if (STATS) {
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
            P.stats[16 + 2 * blockIdx.x] = t_start;
            P.stats[16 + 2 * blockIdx.x + 1] = t_end;
        }
    }
}

int fill_params(const svo_tree* t, const svo_cast_desc* d, const svo_hits* o, CastParams& P, int64_t& nthreads) {
    memset(&P, 0, sizeof(P));
    P.nodes = reinterpret_cast<const Node*>(t->d_nodes);
    P.mats = reinterpret_cast<const uint16_t*>(t->d_mats);
    P.levels = t->levels;
    P.wmask = (1u << (2 * t->levels)) - 1u;
    P.steps = d->steps;
    P.flags = d->flags;
    P.stats = reinterpret_cast<unsigned long long*>(d->stats);
    P.lds_nodes = t->lds_nodes;
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
    // stage whole levels from the top while they fit kLdsNodes
    uint64_t acc = 0;
    for (int lv = 0; lv < t->levels && lv < 8; lv++) {
        if (acc + t->nodes_per_level[lv] > kLdsNodes) break;
        acc += t->nodes_per_level[lv];
    }
    t->lds_nodes = (uint32_t)std::min<uint64_t>(acc, t->nodes.size());
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
    if ((d->flags & SVO_CAST_STATS) && !d->stats) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: SVO_CAST_STATS without a stats buffer");
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
    const bool flat = (P.flags & SVO_CAST_FLAT) != 0;
    if (P.flags & SVO_CAST_STATS) {
        if (flat) hipLaunchKernelGGL((k_cast<true, true>), dim3((uint32_t)blocks), dim3(kBlock), 0, (hipStream_t)stream, P);
        else hipLaunchKernelGGL((k_cast<true, false>), dim3((uint32_t)blocks), dim3(kBlock), 0, (hipStream_t)stream, P);
    } else {
        if (flat) hipLaunchKernelGGL((k_cast<false, true>), dim3((uint32_t)blocks), dim3(kBlock), 0, (hipStream_t)stream, P);
        else hipLaunchKernelGGL((k_cast<false, false>), dim3((uint32_t)blocks), dim3(kBlock), 0, (hipStream_t)stream, P);
    }
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
    P.lds_nodes = t->lds_nodes;
    for (int a = 0; a < 3; a++) {
        P.org[a] = pos[a];
        P.sdir[a] = dir[a];
    }
    P.pos = reinterpret_cast<int32_t*>(buf);
    P.t = reinterpret_cast<float*>(reinterpret_cast<char*>(buf) + 16);
    P.info = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(buf) + 32);
    hipLaunchKernelGGL((k_cast<false, false>), dim3(1), dim3(kBlock), 0, nullptr, P);
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
