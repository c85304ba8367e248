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
#include <array>
#include <type_traits>
#include <string>
#include <utility>
#include <vector>

#include "../../include/svo_rt.h"
#include "svo_hip.h"
#include "svo_internal.h"
#include "svo_wire.h"

using namespace svo;

namespace {

enum : int32_t { MODE_FRAME = 0, MODE_EXPLICIT = 1, MODE_SINGLE = 2 };

// dda_axis for a ray from origin o along a direction whose step signs are known: cell = trunc(o)
// and frac = exact - cell (exact = o, or o - 1 when the step is negative), both exact; a ray's
// first crossing is then adelta - frac * delta (frac * delta exact in double: one rounding, as
// dda_axis' product and difference)
struct FrameAxes {
    double frac[3];
    int32_t cell[3];
};

struct CastParams {
    const Node* nodes;
    const uint16_t* mats;
    int32_t levels;
    uint32_t wmask;
    int32_t mode;
    int32_t steps;
    int32_t flags;
    unsigned long long* stats;
    // frame mode
    RayGen rg;
    float org[3];
    float sdir[3];
    int32_t width, height, tiles_x, tile_row_start, tile_row_step, tile_rows_local;
    int32_t tile_lh;  // log2 of a wavefront's pixel rows (frame_wave_lh)
    int32_t half_rows;  // the first tile rows dispatched, cast by half footprints (frame_half_rows: small launches)
    int32_t n_frames;        // frames in this launch (>= 1); frame f casts from frame_org[3f..]
    int64_t frame_records;   // records of one frame (this shard)
    float frame_org[3 * SVO_MAX_FRAMES];
    // octant instances (frame_dirs): dda_axis' per-axis set-up of each frame origin, hoisted to the
    // host (the same for every ray of the frame: the steps' signs are the octant's)
    FrameAxes fax[SVO_MAX_FRAMES];
    // explicit mode
    const float* rdir;
    const float* rorg;
    int64_t n_rays;
    // outputs
    int32_t* pos;
    float* t;
    uint32_t* info;
    uint8_t* ao;
    uint32_t* wire;        // svo_cast_wire: the wire record of each ray instead of its hit record (svo_wire.h)
    int32_t wire_compact;  // 8-B records
    // hemisphere AO (A8)
    int32_t ao_n, ao_steps;
    float ao_tab[3 * 64];
    const uint32_t* ao_plan;  // device AO plan (ao_plan_get) or null
    // shading: palette colours / flags, sun, highlighted block, shadow budget
    const uint64_t* mat_color;
    const uint32_t* mat_flags;
    float4* rgba;
    float sun[3];
    int32_t sun_dirs;  // the shadow rays' step-sign octant (dirs_sign numbering, 1..8): every shadow ray steps with the sun's signs
    int32_t look[3];
    int32_t look_valid, shadow_steps;
    int32_t look_empty;         // the host look-at voxel is not stored in the scene (an escaped ray could end on it)
    const int32_t* look_dev;    // device lookingAtBlock record (svo_ray_result: pos first) or null
    float time;                 // deltaTime of the liquid wobble (low_res.frag:226)
    const Node* snodes;         // shading: the solid-view tree the shadow rays walk (nodes: the scene)
    const uint16_t* smats;
    // the highest stored voxel row of the scene / of the solid tree (tree_top_y; casts: top_solid); a ray
    // moving up above it that cannot wrap in y before its budget ends can hit nothing more
    int32_t top_scene, top_solid;
    // column ceilings of the tree the rays walk (the scene, for shading): two levels of the tree's table
    // (set_ceilings), blocks 2^ceil_sh[j] columns wide, row-major at ceil + ceil_off[j] (svo_internal.h
    // tree_ceilings); ceil_levels: how many of the two the tree has
    const int16_t* ceil;
    int32_t ceil_levels;
    uint32_t ceil_sh[2];
    int64_t ceil_off[2];
    const uint32_t* ceilp;  // the launch's two levels paired (svo_tree.d_ceilp at its first level's offset)
    const uint32_t* sceilp;  // shading: the same pairs of the solid-view tree the shadow rays walk (trace CEIL 3)
    int32_t sceil_levels;
    const uint64_t* ceilq;  // every level per finest block (svo_tree.d_ceilq; trace CEIL == 2)
    uint32_t* guard_trips;  // the tree's counter of progress-guard trips (svo_tree_guard_trips)
    // frame schedule (sched_attach): launch block b casts frame block sched_order[b] (null: b) and, with sched_cost,
    // writes its duration (100 MHz ticks) to sched_cost[frame block]
    const uint32_t* sched_order;
    uint32_t* sched_cost;
};

constexpr int kBlock = 64;    // threads per block: one wavefront per tile footprint
constexpr int kSchedGroup = SVO_SCHED_GROUP;  // frame schedules order groups of this many consecutive blocks (sched_attach)
// (round 3's A/B switches — ceiling caching and packing, wave-gated boxes, XCD grouping, issue priority —
// were resolved to their measured winners and removed from the source; the losing sides are in git history
// (DESIGN.md cites the commits) and build_variant.py --rev rebuilds them.  The critical-path diagnostics
// (an iteration cap, dropping the top tile rows) are patches: tools/variants/*.patch, build_variant.py --patch)
// waves per SIMD of the shading instances on the camera's octant: 72 VGPRs (0-4 spilled).  The LDS allows 7 blocks per
// SIMD when the launch's path depth is its own (dynamic, path_lds: 3.75 KB for 6 levels) and the bounce state packs into
// 28 B per lane: 7 waves measured 4 % faster than 6 (80 VGPRs), which was 0.7 % faster than 5 (85 VGPRs) with the straight
// trace on the camera's octant (profiles/r05/shade_split_ab.json); 8 with the bounce state in registers spilled 22 VGPRs.
// The generic-sign instance (no octant) runs 6 (80 VGPRs: 7 would spill 29)
constexpr int kShadeWaves = 7;

struct Hit {
    int32_t x, y, z, steps_left;
    float t;
    uint32_t info;
};

// ------------------------------------------------------------------------------------------------
// Exact closed-form skipping.  castRayFromCam's axis choice (ray_caster.cpp:71-80) is, for non-NaN
// values, the lexicographic minimum of (T_axis, rank) with rank z < y < x: x wins only when
// strictly smallest, y beats z only when strictly smaller.  Each axis' crossings form the sequence
// T, fl(T+a), fl(fl(T+a)+a), ... (deltaPos += absDelta in double).  absDelta is an f32 value
// widened to f64: 24 significant bits, a multiple of 2^(ea-23).
//  * Linear rays: when every partial sum a ray can reach (<= budget+2 terms) stays below
//    2^(lsb+53) — lsb = lowest set bit of T and a — every sum is exact and T + k*a computed directly
//    equals the k-fold accumulation bit for bit (e.g. always from integral camera positions).
//  * Every other ray (budget < 2^20, finite values): |T| stays below 2^(ea+22), so a is a multiple
//    of ulp(T) and every crossing below B = 2^(e+1) (e = the binade of |T|) is an exact,
//    representable multiple of ulp(T); the first crossing at or above B is that exact sum rounded
//    once, which fma(k, a, T) also computes.  Only later crossings (one more rounding per binade
//    entered) drift from the closed form, so the crossings are exact segment by segment
//    (seg_cap), and an empty region is crossed in a few moves (skip_box<true>).
// A ray crosses an empty region in O(1): the first event to leave the region is the lexicographic
// minimum of the three per-axis exit events, and the events before it on the other axes are
// counted by division (with an exact fix-up).  Rays outside both domains step voxel by voxel
// (still without memory traffic inside known-empty regions).  All paths give identical results
// (tests).
// ------------------------------------------------------------------------------------------------
// lowest set bit (power of two) of |x|: x finite and nonzero; denormals -> 1 << 20 ("not fast")
__device__ __forceinline__ int dbl_lsb(uint32_t hi, uint32_t lo) {
    const int e = (int)((hi >> 20) & 0x7FFu);
    const uint32_t mh = (hi & 0xFFFFFu) | 0x100000u;  // hidden bit
    const int tz = lo ? (int)__builtin_ctz(lo) : 32 + (int)__builtin_ctz(mh);
    return e == 0 ? (1 << 20) : e - 1075 + tz;
}

// a: positive, normal, finite; T: finite (the closed forms' domain)
__device__ __forceinline__ bool axis_ok(double T, double a) {
    const uint32_t th = (uint32_t)((uint64_t)__double_as_longlong(T) >> 32) & 0x7FFFFFFFu;
    const uint32_t ah = (uint32_t)((uint64_t)__double_as_longlong(a) >> 32);
    const uint32_t et = th >> 20, ea = (ah >> 20) & 0x7FFu;
    return ((unsigned)((ah >> 31) == 0u) & (unsigned)(ea - 1u < 0x7FEu) & (unsigned)(et != 0x7FFu)) != 0u;  // (branch-free)
}

// every partial sum exact ("linear" axis: no rounding at all); axis_ok(T, a) holds
__device__ __forceinline__ bool exact_axis(double T, double a, int32_t budget) {
    const uint32_t th = (uint32_t)((uint64_t)__double_as_longlong(T) >> 32) & 0x7FFFFFFFu, tl = (uint32_t)__double_as_longlong(T);
    const uint32_t ah = (uint32_t)((uint64_t)__double_as_longlong(a) >> 32), al = (uint32_t)__double_as_longlong(a);
    const int u = (th | tl) ? min(dbl_lsb(th, tl), dbl_lsb(ah, al)) : dbl_lsb(ah, al);
    const double bound = __builtin_fabs(T) + (double)(budget + 2) * a;
    const int eb = (int)((uint32_t)((uint64_t)__double_as_longlong(bound) >> 52) & 0x7FFu) - 1023;
    return eb + 1 <= u + 52;  // bound < 2^(u+52): the unrounded bound < 2^(u+53)
}

struct Ray {
    int32_t r[3];   // current voxel (unwrapped)
    double T[3];    // next crossing per axis (deltaPos)
    float af[3];    // absDelta: an f32 value widened to f64 by the reference (ray_caster.cpp:35-41)
    int32_t s[3];   // step
    int32_t steps;  // budget left
    uint32_t axis;  // axis of the last step (3: none)
    double tlast;   // crossing value of the last step (converted to the f32 output once, at the end)
    float ia[3];    // f32 estimate of 1/absDelta (crossing counts only estimate with it)
    int32_t rb[3];  // segment-cached instances (skip_box RB): the cell of each axis' last exact crossing
    __device__ __forceinline__ float inv_a(int k) const { return ia[k]; }
    __device__ __forceinline__ double a(int k) const { return (double)af[k]; }
};

// T + k*a for a fast ray: exact (exact_axis), so one fused operation gives the same double
__device__ __forceinline__ double on_grid(double T, int32_t k, double a) {
    return __builtin_fma((double)k, a, T);
}

// The f32 count estimates (count_est) need every exit event V in f32 range: V is at most the
// smallest absDelta times budget + 2 (< 2^21), so a ray whose every absDelta is 2^100 or more (a
// direction vector with every component below 2^-100) takes the stepping path.  (Frame rays have unit
// directions: their smallest absDelta is at most sqrt(3).)
__device__ __forceinline__ bool span_ok(const Ray& R) {
    return __builtin_fminf(__builtin_fminf(R.af[0], R.af[1]), R.af[2]) < 0x1p100f;
}

// one DDA step (ray_caster.cpp:70-80), branch-free
__device__ __forceinline__ void dda_step(Ray& R) {
    const bool cx = (R.T[0] < R.T[1]) && (R.T[0] < R.T[2]);
    const bool cy = !cx && (R.T[1] < R.T[2]);
    const bool cz = !cx && !cy;
    R.tlast = cx ? R.T[0] : (cy ? R.T[1] : R.T[2]);
    R.axis = cx ? 0u : (cy ? 1u : 2u);
    R.r[0] += cx ? R.s[0] : 0;
    R.r[1] += cy ? R.s[1] : 0;
    R.r[2] += cz ? R.s[2] : 0;
    R.T[0] = cx ? R.T[0] + R.a(0) : R.T[0];
    R.T[1] = cy ? R.T[1] + R.a(1) : R.T[1];
    R.T[2] = cz ? R.T[2] + R.a(2) : R.T[2];
    R.steps--;
}

// Wave-uniform step directions per axis: 1 = every active lane steps +, 2 = every one steps -,
// 0 = mixed.  Lanes only retire while a ray runs, so flags taken at its start stay true.
__device__ __forceinline__ void dir_flags(const int32_t s[3], uint32_t ud[3]) {
    const uint64_t ex = __builtin_amdgcn_read_exec();
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint64_t b = __ballot(s[k] > 0);
        ud[k] = b == ex ? 1u : (b == 0ull ? 2u : 0u);
    }
}

// r + n or r - n by the step sign s; ud: wave-uniform sign (dir_flags) or 0
__device__ __forceinline__ int32_t step_by(int32_t r, int32_t n, int32_t s, uint32_t ud) {
    if (ud == 1u) return r + n;
    if (ud == 2u) return r - n;
    return s > 0 ? r + n : r - n;  // (s * n as a 24-bit multiply-add became v_mad_u64_u32)
}

// A run of free cells through a 4-cell line (occupancy bits 0-3; higher bits are ignored) from the
// ray's cell c (free itself) in its step direction: t = cells in the run (>= 1), m = their slots.
// A sentinel bit stands for the end of the line: one ctz (up) or one clz (down) finds the run.
// ((1 << w) - 1) << o in one v_bfm_b32 (clang emits a shift, a not and a shift)
__device__ __forceinline__ uint32_t bfm(uint32_t w, uint32_t o) {
    uint32_t r;
    asm("v_bfm_b32 %0, %1, %2" : "=v"(r) : "v"(w), "v"(o));
    return r;
}
__device__ __forceinline__ void run_up(uint32_t occ, uint32_t c, uint32_t& t, uint32_t& m) {
    t = (uint32_t)__builtin_ctz((occ | 16u) >> c);
    m = bfm(t, c);
}
__device__ __forceinline__ void run_down(uint32_t occ, uint32_t c, uint32_t& t, uint32_t& m) {
    // slots below c at bits 1..c, the sentinel at bit 0: the highest set bit is the run's first slot
    const uint32_t lo = 31u - (uint32_t)__builtin_clz(__builtin_amdgcn_ubfe((occ << 1) | 1u, 0u, c + 1u));
    t = c + 1u - lo;
    m = bfm(t, lo);
}
__device__ __forceinline__ void run_fwd(uint32_t occ, uint32_t c, bool pos, uint32_t ud, uint32_t& t, uint32_t& m) {
    if (ud == 1u) {
        run_up(occ, c, t, m);
    } else if (ud == 2u) {
        run_down(occ, c, t, m);
    } else {
        uint32_t t0, m0, t1, m1;
        run_up(occ, c, t0, m0);
        run_down(occ, c, t1, m1);
        t = pos ? t0 : t1;
        m = pos ? m0 : m1;
    }
}

// per 16-bit half of v: 1 if it is nonzero — one packed min (clang scalarises the vector form)
__device__ __forceinline__ uint32_t nonzero16(uint32_t v) {
    uint32_t r;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(v), "s"(0x00010001u));
    return r;
}

// Grow the ray's empty child slot into a forward box of empty sibling slots (greedy: the run along x
// from the mask row, then whole rows along z; one cell in y), all from the parent's 64-bit child
// mask in registers, without loops.  Returns per-axis steps to leave it, less one (the index of the
// step that leaves).
__device__ __forceinline__ void box_exits(const uint32_t w[3], const int32_t s[3], uint32_t sh, uint64_t pmask, const uint32_t ud[3],
                                          int32_t e[3]) {
    const uint32_t cx = __builtin_amdgcn_ubfe(w[0], sh, 2u), cy = __builtin_amdgcn_ubfe(w[1], sh, 2u), cz = __builtin_amdgcn_ubfe(w[2], sh, 2u);
    const bool px = s[0] > 0, py = s[1] > 0, pz = s[2] > 0;
    const uint32_t lo = (uint32_t)pmask, hi = (uint32_t)(pmask >> 32);
    uint32_t tx, xm, tz, zm;
    // x run through the row (cy, cz)
    run_fwd((uint32_t)(pmask >> (16u * cz + 4u * cy)), cx, px, ud[0], tx, xm);
    // rows (cy, z) over the x run: bit z (bits 0, 16 -> 0, 1 of the low half, 2, 3 of the high) =
    // the row holds a solid slot
    const uint32_t xs = xm << (4u * cy);
    const uint32_t xl = xs | (xs << 16);
    const uint32_t zc = nonzero16(lo & xl) | (nonzero16(hi & xl) << 2);
    run_fwd(zc | (zc >> 15), cz, pz, ud[2], tz, zm);
    (void)zm;
    // (growing the box along y as well — whole planes over the x run x z run — cost more per crossing
    // than it saved in crossings: without it C3 2.7 %, C5 3.7 %, C2 0.5-2.7 % faster; x runs alone
    // were 16 % slower at C3 / C5)
    const uint32_t ty = 1u;
    // steps to leave: t cells of 2^sh voxels, less the part of the current cell behind the ray;
    // less one: x + ~y = x - y - 1
    const uint32_t m = (1u << sh) - 1u;
    e[0] = (int32_t)((tx << sh) + ~((px ? w[0] : ~w[0]) & m));
    e[1] = (int32_t)((ty << sh) + ~((py ? w[1] : ~w[1]) & m));
    e[2] = (int32_t)((tz << sh) + ~((pz ? w[2] : ~w[2]) & m));
}

// The child mask shifted so that slot sl's bit lands on bit 63 (m << (63 - sl)): its sign is the
// occupancy, and one more shift leaves exactly the lower slots' bits, whose popcount is the
// child's rank among its siblings.
__device__ __forceinline__ uint64_t slot_top(uint64_t m, uint32_t sl) { return m << (sl ^ 63u); }
// popcount(x) + acc through the accumulating v_bcnt_u32_b32 (clang adds acc separately)
__device__ __forceinline__ uint32_t popc_add(uint64_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"((uint32_t)x), "v"(acc));
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"((uint32_t)(x >> 32)), "v"(r));
    return r;
}

// #{ j >= 0 : T + j*a < V } or #{ j >= 0 : T + j*a <= V } = m + [E < V] or m + [E <= V] with
// E = T + m*a and the estimate m = floor((V-T)/a + 1/2) (for <=, the count is floor(x) + 1 with
// x = (V-T)/a, and m is that or one less)
// per-lane selects and a carry-in add on a wave mask held in SGPRs
__device__ __forceinline__ uint32_t sel32(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
__device__ __forceinline__ double sel64(uint64_t m, double a, double b) {
    const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
    const uint32_t lo = sel32(m, (uint32_t)ua, (uint32_t)ub), hi = sel32(m, (uint32_t)(ua >> 32), (uint32_t)(ub >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ int32_t add_bit(int32_t x, uint64_t m) {
    int32_t r;
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(co) : "v"(x), "s"(m));
    return r;
}
// The difference V - T is taken in f32 from f32 copies of both (one conversion of V serves the three
// axes; V < 2^121 by span_ok, so its copy is finite, and a T beyond the f32 range only makes the
// estimate 0, its count): T / a and V / a stay below budget + 2 < 2^20 + 2 (V is at most T + steps * a on every axis),
// so the two conversions, the subtraction, the 1-ulp reciprocal and the fma move the estimate by less
// than 6 * 2^20 * 2^-24 = 3/8 < 1/2 — m stays c - 1 or c
// V, or nextup(V) on the lanes of m (V >= 0 and finite: the bits plus one)
__device__ __forceinline__ double next_if(double V, uint64_t m) {
    const uint64_t b = (uint64_t)__double_as_longlong(V);
    uint32_t lo, hi;
    uint64_t c, c2;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(lo), "=s"(c) : "v"((uint32_t)b), "s"(m));
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(hi), "=s"(c2) : "v"((uint32_t)(b >> 32)), "s"(c));
    (void)c2;
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ int32_t count_est(double T, double a, float inva, double V, float Vf, double& E) {
    uint32_t mu;
    asm("v_cvt_u32_f32 %0, %1" : "=v"(mu) : "v"(__builtin_fmaf(Vf - (float)T, inva, 0.5f)));
    E = on_grid(T, (int32_t)mu, a);
    return (int32_t)mu;
}

// Exact segments.  From any state (T, a), the crossings T + i*a are multiples of 2^v, v = the lower
// of the lowest set bits of T and a, so every crossing below B = 2^(v+53) is exact and representable,
// and the first one at or above B is that sum rounded once, as fma(i, a, T) computes it too.  B is at
// least 2^(e+1) (e = the binade of |T|: T is a multiple of ulp(T), and a of 2^(ea-23) > ulp(T) as
// |T| < 2^(ea+22)); for a ray from a non-integral origin it is typically hundreds of crossings away,
// and past it each binade the crossings enter costs one rounding.  seg_cap returns an index of a
// crossing below B (at most the last one): the crossings 0 .. seg_cap + 1 are fma-exact.
// lowest set bit exponent of |T| (zero: none, 2^20; subnormal: -1074, a safe underestimate)
__device__ __forceinline__ int32_t lsb_exp(double T) {
    const uint64_t b = (uint64_t)__double_as_longlong(T);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    const int32_t e = (int32_t)((hi >> 20) & 0x7FFu);
    const int32_t tz = lo ? (int32_t)__builtin_ctz(lo) : 32 + (int32_t)__builtin_ctz((hi & 0xFFFFFu) | 0x100000u);
    return e != 0 ? e - 1075 + tz : ((b << 1) == 0ull ? (1 << 20) : -1074);
}
// A ray is linear, by a cheap sufficient test on its origin, when every coordinate is integral or
// half-integral: dda_axis then starts at T = a, 0, a/2, 3a/2 or -a/2 (a multiple of half of a's
// lowest set bit, 2^(la-1)), and with a budget below 2^20 every sum stays below 2^(la-1+53) — the
// camera positions of integral poses, and the cell centres shadow and AO rays start from.
__device__ __forceinline__ bool lin_origin(float o) {
    const float o2 = o + o;
    return o2 == __builtin_truncf(o2) && __builtin_fabsf(o) < 1073741824.0f;
}

// x = (B - T)/a is estimated as x~ within 2^-22 relative (f32 roundings, the 1-ulp reciprocal), so
// floor(x~ * (1 - 2^-20)) < x: at most the count of crossings below B, less one (almost always equal)
__device__ __forceinline__ int32_t seg_cap(double T, float af, float inva) {
    const uint32_t ab = __float_as_uint(af);
    const int32_t la = (int32_t)((ab >> 23) & 0xFFu) - 150 + (int32_t)__builtin_ctz(ab | 0x800000u);  // a: normal
    const int32_t be = min(max(min(lsb_exp(T), la) + 53 + 1023, 1), 0x7FF);  // biased exponent of B (0x7FF: inf)
    const double B = __longlong_as_double((long long)((uint64_t)(uint32_t)(be << 20) << 32));
    uint32_t c;
    asm("v_cvt_u32_f32 %0, %1" : "=v"(c) : "v"((float)(B - T) * inva * 0.99999905f));  // saturates (inf: 2^32 - 1)
    return (int32_t)min(c, 1u << 30);  // (never negative: every skip takes at least its exit step)
}

// Cross an empty box, branch-free over the exit axis: ex[k] = steps along axis k that leave the box,
// less one.  Returns false (state unchanged) when the budget ends inside the box.  seg (wave-uniform:
// the wave holds rays that are not linear): each axis' exit event is also held to its exact segment (seg_cap); an exit on such a
// bound is a virtual one inside the box (the next lookup finds the same empty cell in the parent's
// mask, without a load, and the crossing continues).
// RB: segment bounds cached as cells (R.rb): crossing i of axis k from the current state is the one
// into cell r + s*i, so the bound seg_cap gave at some earlier state stays s*(rb - r) crossings ahead
// while the ray has not passed it (every sum up to there is exact, from any state on the way); a
// negative count means it has, and seg_cap is taken again from the current state
template <bool TRACK = true, bool RB = false>
__device__ __forceinline__ bool skip_box(Ray& R, const int32_t ex[3], bool seg) {
    // exits beyond the budget are clamped (safe: total > steps)
    int32_t e[3];
#pragma unroll
    for (int k = 0; k < 3; k++) e[k] = min(ex[k], R.steps);
    if (seg && RB) {  // wave-uniform
        int32_t cap[3];
#pragma unroll
        for (int k = 0; k < 3; k++)  // (wrapping differences: |cap| < 2^31)
            cap[k] = (int32_t)(R.s[k] > 0 ? (uint32_t)R.rb[k] - (uint32_t)R.r[k] : (uint32_t)R.r[k] - (uint32_t)R.rb[k]);
        if (__ballot(min(min(cap[0], cap[1]), cap[2]) < 0) != 0ull) {
#pragma unroll
            for (int k = 0; k < 3; k++) {
                if (cap[k] < 0) {
                    cap[k] = seg_cap(R.T[k], R.af[k], R.inv_a(k));
                    R.rb[k] = (int32_t)(R.s[k] > 0 ? (uint32_t)R.r[k] + (uint32_t)cap[k] : (uint32_t)R.r[k] - (uint32_t)cap[k]);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 3; k++) e[k] = min(e[k], cap[k]);
    } else if (seg) {  // wave-uniform
#pragma unroll
        for (int k = 0; k < 3; k++) e[k] = min(e[k], seg_cap(R.T[k], R.af[k], R.inv_a(k)));
    }
    double E[3];
#pragma unroll
    for (int k = 0; k < 3; k++) E[k] = on_grid(R.T[k], e[k], R.a(k));
    // lexicographic minimum of (E, rank) with rank z < y < x (the DDA rule applied to exits)
    // exit flags as lane masks (SGPRs): selects and tie terms read them directly
    // (ballots of single compares are the compare masks themselves)
    const uint64_t mx = __ballot(E[0] < E[1]) & __ballot(E[0] < E[2]);
    const uint64_t my = __ballot(E[1] < E[2]) & ~mx;
    const double V = sel64(mx, E[0], sel64(my, E[1], E[2]));
    // Events of another axis k that precede the exit event: T + j*a < V when k loses ties
    // (rank_k > rank_b, i.e. k < b), else T + j*a <= V, which on doubles is < nextup(V).
    // strict: x only when the exit is on y or z, y only when it is on z, z never.  On the exit
    // axis b, E = V exactly (V is its e_b-th crossing, m = e_b): there the tie term is the flag b_b
    // itself, so x and y need no second compare of their own for it.
    int32_t n[3];
    double F[3];
    const float Vf = (float)V;
    n[0] = count_est(R.T[0], R.a(0), R.inv_a(0), V, Vf, F[0]);
    n[1] = count_est(R.T[1], R.a(1), R.inv_a(1), V, Vf, F[1]);
    n[2] = count_est(R.T[2], R.a(2), R.inv_a(2), V, Vf, F[2]);
    // (the terms of one axis are disjoint: a tie term implies F = V)
    n[0] = add_bit(n[0], __ballot(F[0] < V) | mx);
    // y's tie term: exit on x counts y's events <= V, i.e. < nextup(V) (V >= 0 finite: its bits + 1),
    // taken by one integer add with the carry-in on mx instead of a second f64 compare
    n[1] = add_bit(n[1], __ballot(F[1] < next_if(V, mx)) | my);
    n[2] = add_bit(n[2], __ballot(F[2] <= V));
    const int32_t total = n[0] + n[1] + n[2];
    if (total > R.steps) return false;  // (a wrong count cannot hang the launch either: trace's progress guard)
#pragma unroll
    for (int k = 0; k < 3; k++) {
        R.T[k] = on_grid(R.T[k], n[k], R.a(k));
        // a compile-time step (sign octant instances) adds or subtracts; else a 24-bit multiply-add
        // (full rate; s = +-1, |n| < 2^21)
        R.r[k] += __builtin_constant_p(R.s[k]) ? (R.s[k] > 0 ? n[k] : -n[k]) : __mul24(R.s[k], n[k]);
    }
    if (TRACK) R.tlast = V;  // (else recovered at the end of the ray: trace)
    R.axis = sel32(mx, 0u, sel32(my, 1u, 2u));
    R.steps -= total;
    return true;
}

struct Stats {
    uint32_t lookups, loads, skips, skip_out, brick_steps, plain_steps;
    uint32_t skip_by_sh[4];  // crossings whose box is made of 2^sh cells: sh = 2, 4, 6, >= 8
    uint32_t bricks;         // brick visits
    uint32_t wv_iters, wv_brick;  // wave-level executions (counted on the first active lane): outer
                                  // loop iterations, brick voxel steps
    uint32_t root_starts, cache_empty;  // lookups started at the root; lookups answered by the
                                        // parent mask
    uint32_t path_starts;                          // lookups restarted from the LDS path
    uint32_t wv_skips, wv_descents;                // wave-level crossings, descent levels
    uint32_t no_progress;                          // loop iterations that consumed no budget (the guard's trips: 0)
    uint32_t ceil_moves;                           // crossings of a column-ceiling box (no lookup)
    uint32_t iters;                                // this lane's traversal iterations
    uint32_t above_top;                            // iterations that start above the tree's highest stored row
    uint32_t bends;                                // reflections and refractions (shading)
    uint32_t tints, tint_iters;                    // refractive voxels passed; iterations that ended passing one
};

// true on one lane of the active lanes (wave-level counters)
__device__ __forceinline__ bool wave_lead() {
    return (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec());
}

// wave-wide max / sum (diagnostics only)
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

// Region lookup of a wrapped voxel: SOLID hit, an empty child cell (returns its shift), or the
// brick holding the voxel (mask / ref / info returned).  tetrahexa_tree.cpp:124-152 on the
// breadth-first layout.
enum : uint32_t { R_EMPTY = 0u, R_BRICK = 1u, R_SOLID = 2u, R_CEIL = 3u };
// Hit.info of a shading ray that left the loop early (ESCAPE): a miss whose remaining steps are all in empty voxels
// (never written to a hit record: escaping is off when records are requested)
constexpr uint32_t ESC_BIT = 1u << 19;

// The interior node whose child region holds the ray's current cell, kept in registers: a move to
// a sibling region reads the cached child mask (no load when the sibling is empty) and restarts
// the descent at most one level down; leaving the parent's region restarts at the root, whose top
// levels are staged in LDS.
// per-lane path of the last descent in LDS
struct Path {
    // [depth][mask low, mask high, first child][lane] dwords: one address per depth (the three
    // words at +0, +256, +512 bytes: ds_write2st64 / ds_read2st64 and one more)
    uint32_t* __restrict__ w;
    __device__ __forceinline__ void put(int32_t d, uint64_t mask, uint32_t ref) const {
        uint32_t* e = w + d * (3 * kBlock);
        e[0] = (uint32_t)mask;
        e[kBlock] = (uint32_t)(mask >> 32);
        e[2 * kBlock] = ref;
    }
    __device__ __forceinline__ uint64_t mask(int32_t d) const {
        const uint32_t* e = w + d * (3 * kBlock);
        return (uint64_t)e[0] | ((uint64_t)e[kBlock] << 32);
    }
    __device__ __forceinline__ uint32_t ref(int32_t d) const { return w[d * (3 * kBlock) + 2 * kBlock]; }
};

struct Parent {
    uint64_t mask;
    uint32_t ref;
    uint32_t sh;  // child shift: a child region is 2^sh voxels wide, the parent's 2^(sh+2)
};

// Node reads.  Trees of up to kNarrowNodes nodes (4 GiB) read through a buffer resource with 32-bit
// byte offsets (one shift per load, and buffer loads are never merged with the LDS path); larger
// trees — the builders accept up to 2^32 nodes, 64 GiB — through 64-bit global addresses.  The host
// picks the instance per tree (svo_cast.hip: node_addressing), so no index can wrap or fall outside
// the resource and read zeros (an empty node) silently.
// Loads take "one past" indices: ni1 = node index + 1 = first child + rank + 1, which is the popcount
// of the child mask shifted so the child's own bit stays in (slot_top: no further shift), and the
// bases sit one node before the array.
constexpr uint64_t kNarrowNodes = 1ull << 28;  // below it, ni1 << 4 stays below 2^32

struct BufNodes {
    __amdgpu_buffer_rsrc_t rsrc;
    const Node* __restrict__ base;
    __device__ __forceinline__ explicit BufNodes(const Node* p)
        : rsrc(__builtin_amdgcn_make_buffer_rsrc(const_cast<Node*>(p - 1), (short)0, (int)0xFFFFFFFFu, (int)0x00020000)), base(p) {}
    __device__ __forceinline__ Node root() const { return base[0]; }  // (uniform: a scalar load)
    __device__ __forceinline__ Node load(uint32_t ni) const {  // node ni - 1
        const uint32_t off = ni << 4;
        Node n;
        n.mask = ((uint64_t)(uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0)) |
                 ((uint64_t)(uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4, 0, 0) << 32);
        n.ref = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 8, 0, 0);
        n.info = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 12, 0, 0);
        return n;
    }
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct WideNodes {
    const __attribute__((address_space(1))) u32x4* p;
    const Node* __restrict__ base;
    __device__ __forceinline__ explicit WideNodes(const Node* q) : p((const __attribute__((address_space(1))) u32x4*)(q - 1)), base(q) {}
    __device__ __forceinline__ Node root() const { return base[0]; }  // (uniform: a scalar load)
    __device__ __forceinline__ Node load(uint32_t ni) const {  // node ni - 1
        const u32x4 v = p[ni];  // 64-bit address: base + (u64)ni * 16
        Node n;
        n.mask = (uint64_t)v.x | ((uint64_t)v.y << 32);
        n.ref = v.z;
        n.info = v.w;
        return n;
    }
};

// SPLIT: the levels above the bricks hold interior nodes or SOLID regions only; a SOLID region ends
// the ray, so the parent may be overwritten by it, and those levels need no leaf branch and no
// copies of the loaded node (the shading pass, whose callers read the final parent's regions, keeps
// the general loop).  PSH (AO instances: ao_count_plan reads the final parent's shift only): a SOLID
// region above the bricks leaves the shift of its own parent, so no path entry at or below the
// SOLID node is read back
template <bool STATS, bool SPLIT, bool PSH, class Mem>
__device__ __forceinline__ uint32_t lookup(const CastParams& P, const Mem& mem, const Path& path,
                                           const uint32_t w[3], uint32_t moved, Parent& par, uint32_t& sh_out, uint64_t& bmask,
                                           uint32_t& bref, uint32_t& binfo, Stats& st) {
    uint32_t ni = 0u;
    int32_t dd = 0;
    if (STATS) st.lookups++;
    {
        // the previous voxel lies in the parent's region (every move starts inside it), so the
        // bits in which the last step changed the stepped coordinate tell whether the ray left it
        const uint32_t diff = moved;
        if (diff >= (4u << par.sh)) {  // a bit at or above the parent region's size changed
            // left the parent's region: the deepest node of the last descent whose region also
            // holds this cell (depth levels-1-floor(h/2), h = highest differing bit) becomes the
            // parent, read back from the per-lane path in LDS
            const int32_t da = P.levels - 1 - (int32_t)((31u - (uint32_t)__builtin_clz(diff)) >> 1);  // (diff != 0)
            par.mask = path.mask(da);
            par.ref = path.ref(da);
            par.sh = (uint32_t)(2 * (P.levels - 1 - da));
            if (STATS) st.path_starts++;
        }
        sh_out = par.sh;
        const uint64_t t = slot_top(par.mask, child_slot(w[0], w[1], w[2], par.sh));
        if ((int64_t)t >= 0) {
            if (STATS) st.cache_empty++;
            return R_EMPTY;
        }
        ni = popc_add(t, par.ref);  // (one past: BufNodes)
        dd = P.levels - (int32_t)(par.sh >> 1);  // depth of that child
        if (STATS && dd == 0) st.root_starts++;
    }
    // descend (one exit: no per-exit register copies)
    uint32_t res = R_EMPTY;
    if (SPLIT) {
        bool pend = true;  // node ni - 1 occupies the cell and is not loaded yet
        bool more = dd < P.levels - 1;
        while (more) {
            if (STATS) {
                st.wv_descents += wave_lead();
                st.loads++;
            }
            const Node n = mem.load(ni);
            const uint32_t sh = (uint32_t)(2 * (P.levels - 1 - dd));
            path.put(dd, n.mask, n.ref);
            par.mask = n.mask;
            par.ref = n.ref;
            binfo = n.info;
            const uint64_t t = slot_top(n.mask, child_slot(w[0], w[1], w[2], sh));
            const bool occ = (int64_t)t < 0;
            const bool solid = (n.info & K_KIND_MASK) == K_SOLID;
            par.sh = PSH && solid ? sh + 2u : sh;
            ni = popc_add(t, n.ref);
            dd++;
            pend = occ && !solid;
            more = pend && dd < P.levels - 1;
            sh_out = occ ? 0u : sh;
            res = solid ? R_SOLID : R_EMPTY;
        }
        if (pend) {  // the brick level: a BRICK or SOLID leaf
            if (STATS) {
                st.wv_descents += wave_lead();
                st.loads++;
            }
            const Node n = mem.load(ni);
            bmask = n.mask;
            bref = n.ref;
            binfo = n.info;
            sh_out = 2u;
            res = (n.info & K_KIND_MASK) == K_SOLID ? R_SOLID : R_BRICK;
        }
        return res;
    }
    bool more = dd < P.levels;
    while (more) {
        if (STATS) {
            st.wv_descents += wave_lead();
            st.loads++;
        }
        const Node n = mem.load(ni);
        const uint32_t kind = n.info & K_KIND_MASK;
        // (read only for BRICK / SOLID results: written on every load, so the previous values need
        // no copies around it)
        bmask = n.mask;
        bref = n.ref;
        binfo = n.info;
        if (kind == K_INTERIOR) {
            const uint32_t sh = (uint32_t)(2 * (P.levels - 1 - dd));
            path.put(dd, n.mask, n.ref);
            par.mask = n.mask;
            par.ref = n.ref;
            par.sh = sh;
            const uint64_t t = slot_top(n.mask, child_slot(w[0], w[1], w[2], sh));
            const bool occ = (int64_t)t < 0;
            ni = popc_add(t, n.ref);
            dd++;
            more = occ && dd < P.levels;
            sh_out = occ ? 0u : sh;  // (occupied at the last level only in a malformed tree: one voxel)
        } else {
            sh_out = 2u;
            res = kind == K_SOLID ? R_SOLID : R_BRICK;
            more = false;
        }
    }
    return res;
}

__device__ __forceinline__ uint32_t brick_material(const uint16_t* mats, uint64_t mask, uint32_t ref, uint32_t info, uint32_t v) {
    return (info & K_UNIFORM) ? (info >> 16) : (uint32_t)mats[ref + (uint32_t)__popcll(mask & ((1ull << v) - 1ull))];
}

__device__ __forceinline__ void wrap3(const Ray& R, uint32_t wm, uint32_t w[3]) {
    w[0] = (uint32_t)R.r[0] & wm;
    w[1] = (uint32_t)R.r[1] & wm;
    w[2] = (uint32_t)R.r[2] & wm;
}

// One ray with castRayFromCam semantics.
// Voxel steps through a brick on its register mask (see trace): returns the voxel index reached;
// `left` = per-axis steps left in the brick (bytes 0-2, a zero byte = left the brick), `solid` =
// stopped on a solid voxel.  The crossing value of every step is kept (recovering it after the
// walk as T - a, exact for fast rays, measured no faster).
// TRACK: keep the crossing value of every step (R.tlast); without it trace recovers the last one
// once, at the end of the ray (exact sums: T - a).  (A wave-uniform runtime flag in this loop
// measured 1.6 % slower than tracking always.)
// (Skipping the per-step budget test for waves with budget for a whole walk, at most 10 steps,
// measured equal.)
template <bool STATS, bool TRACK>
__device__ __forceinline__ uint32_t brick_walk(Ray& R, uint64_t bmask, const uint32_t w[3], uint32_t left0, uint32_t& left, bool& solid,
                                               Stats& st) {
    // 127 - voxel index (byte 0: the 64-bit shift reads its low 6 bits, 63 - v, which moves the
    // voxel's bit to bit 63 — one shift and a sign test; the +-1/4/16 moves of a walk stay within
    // 48..143, so byte 0 never borrows) and steps left (bytes 1-3, biased: 0x80 + left - 1, so a
    // byte leaves the brick by clearing its top bit, without a borrow) in one register.  The step
    // keeps its delta instead of the axis: the axis follows from the last delta after the walk.
    uint32_t pk = (left0 << 8) | (127u - child_slot(w[0], w[1], w[2], 0u));
    const uint32_t d0 = (uint32_t)(-R.s[0]) - 0x100u, d1 = (uint32_t)(-R.s[1] * 4) - 0x10000u, d2 = (uint32_t)(-R.s[2] * 16) - 0x1000000u;
    uint32_t dl = 0u;
    bool go;
    do {  // one exit: the compiler keeps the state in place (no per-exit copies)
        solid = (int64_t)(bmask << (pk & 63u)) < 0;
        go = !solid && R.steps > 0;
        if (go) {
            // one DDA step (ray_caster.cpp:70-80) without position updates
            const bool cx = (R.T[0] < R.T[1]) && (R.T[0] < R.T[2]);
            const bool cy = !cx && (R.T[1] < R.T[2]);
            if (TRACK) R.tlast = cx ? R.T[0] : (cy ? R.T[1] : R.T[2]);
            R.T[0] = cx ? R.T[0] + R.a(0) : R.T[0];
            R.T[1] = cy ? R.T[1] + R.a(1) : R.T[1];
            R.T[2] = (cx || cy) ? R.T[2] : R.T[2] + R.a(2);  // (a mask or, not a fourth f64 compare)
            R.steps--;
            dl = cx ? d0 : (cy ? d1 : d2);
            pk += dl;
            if (STATS) {
                st.brick_steps++;
                st.wv_brick += wave_lead();
            }
            go = (pk & 0x80808000u) == 0x80808000u;  // every steps-left byte above its bias: inside
        }
    } while (go);
    if (dl != 0u) R.axis = dl == d0 ? 0u : (dl == d1 ? 1u : 2u);
    left = pk >> 8;
    return 63u - (pk & 63u);
}

// Column-ceiling march (round 5).  A descending ray above the ceiling of its 16-column block crosses, cell by cell,
// only empty voxels until its row reaches that ceiling or it leaves the block; castRayFromCam's DDA (ray_caster.cpp:71-80)
// takes its x / z / y steps at the crossing values T_k + j * a_k, so every event that matters here is one fma of an
// integer index: the x (z) event entering the next block, j = the cells left in the block on that axis, and the y event
// entering the ceiling row c, j = y - 1 - c.  The march walks the blocks the ray's column path crosses (their order
// follows from the x / z boundary events alone) comparing exact event values, one 32-bit ceiling load per block (the
// next block's load issued before this one is judged), until the ceiling event comes first or the ray enters a block
// at or below its ceiling; every voxel entered before that event is then empty, and one closed-form crossing
// (skip_box) moves the ray to the state right after it — the cell that event enters is the loop's next untested
// voxel.  This replaces the chain of per-block ceiling moves of a ray's descent (C3: ~6 of its ~11 loop iterations,
// each a full iteration with its own exact crossing) by one crossing and a few integer / fma steps per block.
// Linear rays only (every sum exact: `fast` in the non-segment instances), stepping down (R.s[1] < 0); a tie between
// the x and z boundary events (a block corner) or between a boundary and the ceiling event stops the march there.
// Returns whether the ray moved.
// The march's end: ex (skip_box's exits) of the first event whose voxel it could not prove empty.  Returns false when
// nothing beyond the current voxel is proven (its own row is at or below its block's ceiling).
template <bool STATS>
__device__ __forceinline__ bool ceil_march(const CastParams& P, const uint32_t* __restrict__ ceilp, const Ray& R, uint32_t wm, int32_t ex[3],
                                           Stats& st) {
    const uint32_t lsh = P.ceil_sh[0];  // the finest level's blocks: 2^lsh columns
    const uint32_t bm = (1u << lsh) - 1u, rows = (wm + 1u) >> lsh, rm = rows - 1u;
    const int32_t wy = (int32_t)((uint32_t)R.r[1] & wm);
    const uint32_t wx = (uint32_t)R.r[0] & wm, wz = (uint32_t)R.r[2] & wm;
    // per axis the next block-boundary event: its index from the current state (the cells left in the block) and value
    int32_t jx = (int32_t)(R.s[0] > 0 ? bm - (wx & bm) : (wx & bm)), jz = (int32_t)(R.s[2] > 0 ? bm - (wz & bm) : (wz & bm));
    double Ex = on_grid(R.T[0], jx, R.a(0)), Ez = on_grid(R.T[2], jz, R.a(2));
    uint32_t bx = wx >> lsh, bz = wz >> lsh;
    const uint32_t dx = R.s[0] > 0 ? 1u : rm, dz = R.s[2] > 0 ? 1u : rm;  // (one block on, wrapped)
    uint32_t cv = ceilp[__umul24(bz, rows) + bx];
    double Ein = -__builtin_inf();  // the event that entered the current block (none for the first)
    int32_t ein_axis = -1, ein_j = 0, stop_axis = -1, stop_j = 0;
    for (int32_t it = 0;; it++) {
        const bool xn = Ex < Ez;
        // the next block's ceiling, loaded before this block is judged (the blocks' order follows from x / z alone)
        const uint32_t nbx = xn ? (bx + dx) & rm : bx, nbz = xn ? bz : (bz + dz) & rm;
        const uint32_t ncv = ceilp[__umul24(nbz, rows) + nbx];
        const int32_t jy = wy - 1 - (int32_t)(int16_t)(cv & 0xFFFFu);  // the y event entering the ceiling row
        const double tc = jy >= 0 ? on_grid(R.T[1], jy, R.a(1)) : -__builtin_inf();
        if (!(tc > Ein) || it == 1024) {  // the voxel entering this block is at or below its ceiling: end before that event
            stop_axis = ein_axis;        // (and a bound on the march: its blocks so far are proven)
            stop_j = ein_j;
            break;
        }
        const double Eexit = xn ? Ex : Ez;
        // the next boundary lies beyond the budget: only the ceiling event can come first within it
        const bool far = (xn ? jx : jz) > R.steps;
        if (!(Eexit < tc) || Ex == Ez || far) {
            if (far || (!(Ez <= tc && Ez <= Ex) && tc <= Ex)) {  // the first unproven event, in the DDA's order at ties: z, y, x
                stop_axis = 1;
                stop_j = jy;
            } else if (Ez <= tc && Ez <= Ex) {
                stop_axis = 2;
                stop_j = jz;
            } else {
                stop_axis = 0;
                stop_j = jx;
            }
            break;
        }
        if (STATS) st.ceil_moves++;
        Ein = Eexit;  // on into the next block
        if (xn) {
            ein_axis = 0;
            ein_j = jx;
            jx += (int32_t)bm + 1;
            Ex = on_grid(R.T[0], jx, R.a(0));
        } else {
            ein_axis = 2;
            ein_j = jz;
            jz += (int32_t)bm + 1;
            Ez = on_grid(R.T[2], jz, R.a(2));
        }
        bx = nbx;
        bz = nbz;
        cv = ncv;
    }
    // (selects on values: a dynamically indexed register array would go through scratch)
    ex[0] = stop_axis == 0 ? stop_j : R.steps;
    ex[1] = stop_axis == 1 ? stop_j : R.steps;
    ex[2] = stop_axis == 2 ? stop_j : R.steps;
    return stop_axis >= 0;
}

// A shading ray's DDA state on entering the first block it hits (the cell, crossing values, budget and last step axis):
// the straight trace before any bounce hands it to the reflection / refraction trace, which resumes from it (trace XS)
struct RayState {
    double T[3];
    int32_t r[3];
    int32_t steps;
    uint32_t axis;
};

// Reflections and refractions of the shading pass (reflectRay / refractRay, low_res.frag:170-240):
// direction after them, reflection count, finalColorMod (a vec3: liquid tints per channel), and
// whether the ray was bent (kBent, a bit of the reflection count's word: 28 B per lane in LDS, which with the launch's own
// path depth lets the shading instances run 7 waves per SIMD).
constexpr int32_t kBent = 1 << 30;
struct Bounce {
    float d[3];
    int32_t n;  // reflections | kBent
    float m[3];
};

// refractRay(vec3, vec3, float, float) (low_res.frag:196-209), n1 = 1.0, n2 = 1.1; dot as
// ((x + y) + z), no fused operations (-ffp-contract=off)
__device__ __forceinline__ void refract_dir(float d[3], const float nin[3]) {
    const float r = 1.0f / 1.1f;
    float n[3] = {nin[0], nin[1], nin[2]};
    float c1 = (n[0] * d[0] + n[1] * d[1]) + n[2] * d[2];
    if (c1 < 0.0f) {
#pragma unroll
        for (int k = 0; k < 3; k++) n[k] = -n[k];
        c1 = (n[0] * d[0] + n[1] * d[1]) + n[2] * d[2];
    }
    const float c2 = svo::sqrt_rn(1.0f - r * r * (1.0f - c1 * c1));
    const float kf = r * c1 - c2;
#pragma unroll
    for (int k = 0; k < 3; k++) d[k] = r * d[k] + kf * n[k];
}

// par_out: receives the parent of the region the ray ended in (it holds the final voxel; the LDS
// path holds its ancestors at depths 0 .. levels-1-sh/2).  KEEPPAR (AO): only its shift is exact
// (lookup: PSH) — a ray ending in a SOLID region above the bricks leaves that region's mask and ref
// ESCAPE (shading rays whose end position is not output): a ray moving up above the highest stored
// voxel row `top` (wrapped) whose budget cannot carry it past the extent in y leaves the loop as a
// miss at once — it can only enter empty space — and skips its remaining steps (top < 0: off); so does
// a ray whose budget ends inside an empty box; and with CEIL, a ray above `top` crosses the whole
// half-space above it (every x and z) in one move.
// DIRS (1..8): every ray of the launch steps with the signs dirs_sign(DIRS, k) (frame_dirs proves it
// on the host): the steps are compile-time constants and the sign branches of the crossings and brick
// walks fold away; 0: per-wave sign flags (dir_flags)
// NO_T: no crossing value is output (shading launches without hit records), so none is tracked per step.
// XS (round 5, the shading pass): 1 — on a hit, store the DDA state the ray entered its block with in *xs (RayState);
// 2 — start from *xs instead of the origin's first step (the flags fast / lin still from the origin and direction),
// with no pre-top box and no march: the straight trace of a shading ray hands its first hit on to the bouncing one
__host__ __device__ constexpr int32_t dirs_sign(int DIRS, int k) { return DIRS == 0 ? 0 : (((DIRS - 1) >> k) & 1) ? -1 : 1; }

template <bool STATS, bool REFLECT = false, bool ESCAPE = false, bool SEG = false, int DIRS = 0, bool KEEPPAR = false, int CEIL = 0,
          bool NO_T = false, int XS = 0, class Mem>
__device__ __forceinline__ Hit trace(const CastParams& P, const Mem& mem, const uint16_t* mats, const Path& path, const float o[3],
                                     const float d[3], int32_t budget, unsigned long long* ray_work = nullptr,
                                     Bounce* bounce = nullptr, Parent* par_out = nullptr, int32_t top = -1, int32_t pre_top = -1,
                                     const FrameAxes* fx = nullptr, RayState* xs = nullptr) {
    Ray R;
    if (DIRS != 0 && fx) {
        // a frame ray of an octant instance: the origin's part of dda_axis is the frame's (fx)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const float df = rcp_rn(d[k]);
            const double delta = (double)df;
            R.r[k] = fx->cell[k];
            R.T[k] = __builtin_fma(-fx->frac[k], delta, __builtin_fabs(delta));
            R.af[k] = __builtin_fabsf(df);
            R.s[k] = dirs_sign(DIRS, k);
            R.ia[k] = __builtin_amdgcn_rcpf(R.af[k]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const Dda1 ax = dda_axis(o[k], d[k]);
            R.r[k] = ax.cell;
            R.T[k] = ax.dpos;
            R.af[k] = (float)ax.adelta;  // exact: adelta is |f32 quotient|
            R.s[k] = ax.step;
            R.ia[k] = __builtin_amdgcn_rcpf((float)ax.adelta);
        }
    }
    R.steps = budget;
    R.axis = 3u;
    R.tlast = 0.0;
    // closed-form crossings (fast): budget < 2^20 also keeps the f32 count estimates within 3/8 of
    // the truth (count_est, seg_cap); linear rays need no segment bounds, and a wave of linear rays
    // takes the cheaper crossing.  Origins within 2^30 (an exact start cell: deltaPos starts in
    // [0, 2 absDelta]); beyond them castRayFromCam's int conversion is undefined, and those rays step
    // voxel by voxel (no closed form over a start cell the conversion clamped)
    // (bitwise ands: one straight-line computation, no branch per term)
    bool fast = ((unsigned)!(P.flags & SVO_CAST_ITERATIVE) & (unsigned)(budget < (1 << 20)) & (unsigned)axis_ok(R.T[0], R.a(0)) &
                 (unsigned)axis_ok(R.T[1], R.a(1)) & (unsigned)axis_ok(R.T[2], R.a(2)) & (unsigned)((DIRS != 0 && fx) || span_ok(R)) &  // (frame rays: unit directions)
                 (unsigned)(!SEG || (__builtin_fabsf(o[0]) < 0x1p30f && __builtin_fabsf(o[1]) < 0x1p30f &&
                                     __builtin_fabsf(o[2]) < 0x1p30f))) != 0u;  // (!SEG: need_seg bounds the origins)
    // SEG: the instance carries segment-bounded crossings (the host picks it when rays can be
    // non-linear: need_seg).  The other one runs exact-origin rays only; it re-tests them cheaply
    // (lin_origin) and steps any other ray voxel by voxel.
    bool lin = SEG ? fast && exact_axis(R.T[0], R.a(0), budget) && exact_axis(R.T[1], R.a(1), budget) && exact_axis(R.T[2], R.a(2), budget)
                   : (DIRS != 0 && fx) ? fast  // (need_seg: this instance's frame origins are exact)
                   : ((unsigned)fast & (unsigned)lin_origin(o[0]) & (unsigned)lin_origin(o[1]) & (unsigned)lin_origin(o[2])) != 0u;
    if (!SEG) fast = lin;
    const bool wseg = SEG && __ballot(fast && !lin) != 0ull;  // wave-uniform (REFLECT: taken per crossing)
    // octant segment instances cache their segment bounds (skip_box RB); none yet (cap -1)
    constexpr bool RB = SEG && DIRS != 0 && !REFLECT;
    if (RB) {
#pragma unroll
        for (int k = 0; k < 3; k++) R.rb[k] = R.r[k] - R.s[k];
    }
    // Instances without segments run rays from integral / half-integral origins only (need_seg):
    // every sum they take is exact, so they recover the output crossing value once at the end
    // (T - a on the last step's axis) instead of keeping it on every brick step
    // (NO_T: no crossing value is output — shading launches without hit records — so none is kept)
    constexpr bool TRACK = (REFLECT || SEG) && !NO_T;
    uint32_t ud[3];
    if (DIRS != 0) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            R.s[k] = dirs_sign(DIRS, k);  // (equal to dda_axis' step: frame_dirs)
            ud[k] = dirs_sign(DIRS, k) > 0 ? 1u : 2u;
        }
    } else {
        dir_flags(R.s, ud);
    }
    // the hit is mat != kNoHit (a flag of its own costs lane-mask upkeep every iteration)
    uint32_t mat = kNoHit;
    const uint32_t wm = P.wmask;
    Stats st = {0, 0, 0, 0, 0, 0, {0, 0, 0, 0}, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    Parent par;
    // the root (node 0 of the tree this trace walks; uniform, one scalar load) is the first parent and stands in the
    // per-lane path at depth 0, so the first lookup starts at the root's child slot instead of loading the root (one
    // dependent load fewer per ray; every later restart at depth 0 reads the same node from the path: C3 -0.8 %, C4
    // -0.6 %, C5 -1.1 %, shaded -0.5 %, profiles/r06/ab_root_seed_*.txt).  A root that is not interior (a one-level
    // tree, a uniform world) keeps the virtual parent above it.
    const Node rn = mem.root();
    if (P.levels >= 2 && (rn.info & K_KIND_MASK) == K_INTERIOR) {  // (uniform)
        path.put(0, rn.mask, rn.ref);
        par.mask = rn.mask;
        par.ref = rn.ref;
        par.sh = 2u * (uint32_t)(P.levels - 1);
    } else {
        // a virtual parent above the root (its one child region, slot 0 of the wrapped coordinates, is
        // the whole world = node 0): the first lookup takes the same path as every later one
        par.mask = 1ull;
        par.ref = 0u;
        par.sh = 2u * (uint32_t)P.levels;
    }
    // XS 2: resume a ray from the state its straight trace (XS 1) stopped in — the cell it entered, untested; the
    // flags above (fast, lin: from the origin and direction) are the ones that trace had
    bool done = R.steps <= 0;
    if (XS == 2) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            R.T[k] = xs->T[k];
            R.r[k] = xs->r[k];
        }
        R.steps = xs->steps;
        R.axis = xs->axis;
        done = false;
    } else if (!done) {
        dda_step(R);
    }
    // pre_top (>= 0: the tree's highest stored voxel row, tree_top_y): a ray starting above it is in
    // one empty region {y > pre_top} (every x, z; up to the wrap in y) and crosses it in one move,
    // exactly like a box (false: its budget ends up there, state unchanged, the loop walks it)
    if (XS != 2 && pre_top >= 0 && fast && !done) {
        uint32_t w[3];
        wrap3(R, wm, w);
        if ((int32_t)w[1] > pre_top) {
            const int32_t ex[3] = {R.steps, R.s[1] < 0 ? (int32_t)w[1] - pre_top - 1 : (int32_t)(wm - w[1]), R.steps};
            skip_box<TRACK, RB>(R, ex, wseg);
        }
    }
    // one back-edge: every path through the body ends at the loop latch
    bool escaped = false;
    uint32_t bref = 0u, binfo = 0u;
    uint64_t bmask = 0ull;
    // coordinate bits changed since the last voxel known to lie in the parent's region, by ceiling moves since
    // the last lookup and the step before them (the lookup's restart depth)
    uint32_t jump = 0u;
    // CEIL 1: the launch's two levels of the column ceilings (P.ceilp pairs); 2: every level, the coarsest block the ray is
    // above (P.ceilq: a max-mipmap walk of the ceilings); 3: as 1 on P.sceilp
    // (CEIL 3: CEIL 1 on the pairs of the solid-view tree of a shading launch, P.sceilp — the shadow rays)
    const bool ceil_on = CEIL != 0 && (CEIL == 3 ? P.sceil_levels : P.ceil_levels) > 0;  // (uniform)
    const uint32_t* const ceilp = CEIL == 3 ? P.sceilp : P.ceilp;
    uint32_t ckey = 0xFFFFFFFFu, cval = 0u;  // the lane's 16-column block (key) and its ceilings (c0 | c1 << 16)
    uint64_t cq = 0ull;                      // (CEIL 2: the ceilings of the blocks of every level holding the lane's 16-column block)
    // the descent through the air above the terrain in one march (ceil_march): linear primary / AO rays stepping down
    // (the voxel it ends in is untested, even when the budget ends with it: the loop tests it)
    // (primary / AO casts, and the shading pass's rays before any bounce; exact-sum lanes only: `lin` in segment instances)
    constexpr bool MARCH = CEIL == 1 || CEIL == 2;
    if (XS != 2 && MARCH && ceil_on && !done && (SEG ? lin : fast) && R.s[1] < 0 && R.steps > 0) {
        int32_t ex[3];
        if (ceil_march<STATS>(P, ceilp, R, wm, ex, st)) (void)skip_box<TRACK, RB>(R, ex, wseg);
    }
    while (!done) {
        // the voxel just entered is untested
        if (STATS) {
            st.wv_iters += wave_lead();
            st.iters++;
        }
        const int32_t steps_in = R.steps;  // (the progress guard below)
        uint32_t w[3];
        wrap3(R, wm, w);
        if (STATS && pre_top >= 0 && (int32_t)w[1] > pre_top) st.above_top++;
        if (ESCAPE && top >= 0 && R.s[1] > 0 && (int32_t)w[1] > top && (int64_t)w[1] + R.steps <= (int64_t)wm) {
            escaped = true;  // only empty voxels ahead: a miss
            break;
        }
        uint32_t sh = 0u;
        bool pend = false;  // the lookup found a brick: step through it below
        const uint32_t ax = R.axis;
        const uint32_t wa = ax == 0u ? w[0] : (ax == 1u ? w[1] : w[2]);
        const int32_t sa = ax == 0u ? R.s[0] : (ax == 1u ? R.s[1] : R.s[2]);
        const uint32_t moved = jump | (wa ^ ((wa - (uint32_t)sa) & wm));  // bits the last step(s) changed
        // Column ceilings: a ray above the highest stored row of the 256- (then 64-) column block it is in
        // has only empty voxels between it and that row, and above it up to the top of the world, over the
        // whole block: that box is crossed without a lookup (R_CEIL; the next lookup restarts from the
        // per-lane path at the depth the moves since the last lookup left intact)
        int32_t cex[3] = {0, 0, 0};
        bool cl = false, any_cl = false, gt = false;
        int32_t c0 = -1, c1 = 32767;  // the ceilings of the lane's blocks at the launch's two levels (set_ceilings)
        uint32_t lv = 0u;             // (CEIL 2) how many levels' ceilings the ray is above: its box is a block of level lv - 1
        if (CEIL == 2 && ceil_on && fast && R.steps > 0) {
            const int32_t y = (int32_t)w[1];
            constexpr uint32_t lsh0 = 2u * kCeilK0;
            const uint32_t rows0 = (wm + 1u) >> lsh0;
            const uint32_t key = __umul24(w[2] >> lsh0, rows0) + (w[0] >> lsh0);
            if (key != ckey) {
                ckey = key;
                cq = P.ceilq[key];
            }
            // (the ceilings grow with the level: a block's holds its children's)
            lv = (uint32_t)(y > (int32_t)(int16_t)cq) + (uint32_t)(y > (int32_t)(int16_t)(cq >> 16)) +
                 (uint32_t)(y > (int32_t)(int16_t)(cq >> 32)) + (uint32_t)(y > (int32_t)(int16_t)(cq >> 48));
            cl = lv != 0u;
            if (ESCAPE) gt = top >= 0 && y > top;
        } else if (ceil_on && fast && R.steps > 0) {
            const int32_t y = (int32_t)w[1];
            const uint32_t lsh0 = P.ceil_sh[0], rows0 = (wm + 1u) >> lsh0;
            const uint32_t key = __umul24(w[2] >> lsh0, rows0) + (w[0] >> lsh0);  // (< 2^28: 2^14 x 2^14 blocks at most)
            // (the lane's block and its ceilings stay in registers until it moves to another block; both
            // ceilings come from one 32-bit load of svo_tree.d_ceilp: the block's ceiling and its parent block's)
            if (key != ckey) {
                ckey = key;
                cval = ceilp[key];
            }
            c0 = (int32_t)(int16_t)(cval & 0xFFFFu);
            c1 = (int32_t)cval >> 16;
            const bool p1 = y > c1;
            cl = p1 || y > c0;
            // above the tree's highest stored row (ESCAPE instances: top): every column is empty from there up to the
            // top of the world, so the box spans every x and z (a ray climbing out of the terrain band crosses it in one
            // move instead of one per 256-column block; its budget ends in it or it wraps in y)
            if (ESCAPE) gt = top >= 0 && y > top;
        }
        // (the box exits are taken only when a lane of the wave moves — wave-uniform; with the forward boxes gated
        // the same way, 1.1 % faster at C3 than per-lane selects: profiles/r03/ab_r03_x_*.log)
        any_cl = ceil_on && __ballot(cl) != 0ull;
        if (any_cl) {
            const int32_t y = (int32_t)w[1];
            const bool p1 = y > c1;
            uint32_t bmk = (1u << (p1 ? P.ceil_sh[1] : P.ceil_sh[0])) - 1u;  // block width - 1
            int32_t c = p1 ? c1 : c0;
            if (CEIL == 2) {
                const uint32_t l = (lv - 1u) & 3u;  // (lanes with lv 0 take no box)
                bmk = (1u << (2u * (kCeilK0 + l))) - 1u;
                c = (int32_t)(int16_t)(cq >> (16u * l));
            }
            // steps to leave the box, less one: the block's faces in x / z, the ceiling (down) or the top
            // of the world (up) in y
            cex[0] = gt ? R.steps : (int32_t)(R.s[0] > 0 ? bmk - (w[0] & bmk) : (w[0] & bmk));
            cex[1] = R.s[1] < 0 ? y - (gt ? top : c) - 1 : (int32_t)(wm - w[1]);
            cex[2] = gt ? R.steps : (int32_t)(R.s[2] > 0 ? bmk - (w[2] & bmk) : (w[2] & bmk));
        }
        uint32_t kind = R_CEIL;
        if (!cl) {
            kind = lookup<STATS, !REFLECT, KEEPPAR>(P, mem, path, w, moved, par, sh, bmask, bref, binfo, st);
            jump = 0u;
        }
        if (kind == R_SOLID) {
            mat = binfo >> 16;
            done = true;
        } else if (kind == R_BRICK) {
            if (STATS) st.bricks++;
            pend = true;
        } else if (R.steps <= 0) {
            done = true;
        } else if (!(fast && [&] {
                       int32_t ex[3];
                       if (REFLECT) dir_flags(R.s, ud);  // reflections and refractions flip steps
                       // (a wave whose every crossing is a ceiling move — the air above the terrain — skips the forward
                       // boxes: wave-uniform)
                       if (!any_cl || __ballot(!cl) != 0ull) {
                           box_exits(w, R.s, sh, par.mask, ud, ex);
                           if (any_cl) {
#pragma unroll
                               for (int k = 0; k < 3; k++) ex[k] = cl ? cex[k] : ex[k];
                           }
                       } else {
#pragma unroll
                           for (int k = 0; k < 3; k++) ex[k] = cex[k];
                       }
                       const bool moved_ok = skip_box<TRACK, RB>(R, ex, REFLECT ? SEG && __ballot(!lin) != 0ull : wseg);
                       if (ceil_on && cl && moved_ok) {
                           // (the voxel this move started from need not lie in the parent's region: the step
                           // that entered it — `moved` — counts too)
                           uint32_t wn[3];
                           wrap3(R, wm, wn);
                           jump = moved | (w[0] ^ wn[0]) | (w[1] ^ wn[1]) | (w[2] ^ wn[2]);
                           if (STATS) st.ceil_moves++;
                       }
                       return moved_ok;
                   }())) {
            if (STATS && fast) st.skip_out++;
            if (fast) {
                done = true;  // the budget ends inside this empty box: steps after the loop
                // (ESCAPE: where a ray without a hit ends is not output — a miss whose budget ends in empty space skips them)
                if (ESCAPE && top >= 0) escaped = true;
            } else {
                // not exact: voxel steps to the end of this (empty) 4^3 brick, then a lookup
                pend = true;
                bmask = 0ull;
            }
        } else if (STATS) {
            st.skips++;
            st.wv_skips += wave_lead();
            st.skip_by_sh[min(3u, (sh >> 1) - 1u)]++;
        }
        if (pend) {
            // voxel steps inside the brick, solid mask in registers.  (Postponing bricks until
            // more lanes hold one, or bounding the steps per iteration, measured slower.)
            uint32_t w[3];
            wrap3(R, wm, w);
            // Voxel index v and per-axis steps left in the brick (one byte each) are stepped
            // instead of positions; positions follow from the step counts when the brick ends.
            // Steps left: 4 - c stepping up, c + 1 stepping down (c = the cell in the brick), i.e.
            // (c ^ 3) + 1 or c + 1 — all three bytes at once, biased by 0x7F (brick_walk).
            const uint32_t up3 = (R.s[0] > 0 ? 3u : 0u) | (R.s[1] > 0 ? 0x300u : 0u) | (R.s[2] > 0 ? 0x30000u : 0u);
            const uint32_t left0 = (((w[0] & 3u) | ((w[1] & 3u) << 8) | ((w[2] & 3u) << 16)) ^ up3) + 0x808080u;
            uint32_t left, v;
            bool solid;
            v = brick_walk<STATS, TRACK>(R, bmask, w, left0, left, solid, st);
            if (solid) {
                mat = brick_material(mats, bmask, bref, binfo, v);
                done = true;
            } else if (R.steps <= 0 && (left & 0x808080u) == 0x808080u) {
                done = true;  // budget ended inside the brick
            }
            const uint32_t dn = left0 - left;  // steps taken per axis, one byte each (no borrows)
            R.r[0] = step_by(R.r[0], (int32_t)(dn & 0xFFu), R.s[0], REFLECT ? 0u : ud[0]);
            R.r[1] = step_by(R.r[1], (int32_t)((dn >> 8) & 0xFFu), R.s[1], REFLECT ? 0u : ud[1]);
            R.r[2] = step_by(R.r[2], (int32_t)(dn >> 16), R.s[2], REFLECT ? 0u : ud[2]);
        }
        const uint32_t mfl = REFLECT && mat != kNoHit ? P.mat_flags[mat] : 0u;
        const uint32_t mflags = mfl & 7u;
        if (REFLECT && R.steps > 0 && mflags == 3u) {
            // a reflective block (flags & 7 == 3) with budget left: undo the last crossing on the
            // hit axis, mirror that axis (step and direction) and take the next DDA step from the
            // block, as low_res.frag:170-189 + :319-331 do
            const uint32_t ax = R.axis;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                if (ax == (uint32_t)k) {
                    R.T[k] -= R.a(k);
                    R.s[k] = -R.s[k];
                    bounce->d[k] = -bounce->d[k];
                }
            }
            bounce->n++;
            if (STATS) st.bends++;
#pragma unroll
            for (int k = 0; k < 3; k++) bounce->m[k] *= 0.94f;
            dda_step(R);
            done = false;
            mat = kNoHit;
        } else if (REFLECT && R.steps > 0 && mflags == 5u) {
            // a refractive block (glass, or liquid when the scene tree holds it) with budget left:
            // tint (liquid (0.94, 0.97, 1.0), else 0.95) and pass; the first one bends the ray
            // (refractRay, :211-240).  The shader's exact position is never advanced by its DDA: it
            // is the origin (minus 1 on axes with a negative initial step), +1 on the other axes with
            // a negative step, then min(new step, 0); deltaPos restarts from the current cell.
            const bool liquid = (mfl & 0x10u) != 0u;
            const float t0 = liquid ? 0.94f : 0.95f, t1 = liquid ? 0.97f : 0.95f, t2 = liquid ? 1.0f : 0.95f;
            if (STATS) {
                st.tints++;
                st.tint_iters++;
            }
            bounce->m[0] *= t0;
            bounce->m[1] *= t1;
            bounce->m[2] *= t2;
            uint32_t wr[3];
            wrap3(R, wm, wr);  // the refractive voxel (its region, when uniform, is passed below)
            if (!(bounce->n & kBent)) {
                bounce->n |= kBent;
                if (STATS) st.bends++;
                const uint32_t ax = R.axis;
                double ex[3];
                float nrm[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    ex[k] = (double)o[k];
                    if (d[k] < 0.0f) ex[k] -= 1.0;
                    if (ax != (uint32_t)k && R.s[k] < 0) ex[k] += 1.0;
                    if (ax == (uint32_t)k) nrm[k] = (float)R.s[k];
                }
                if (liquid) {
                    // the wave wobble (:225-229) at the shader's (float) exact position
                    const float arg = ((P.time + (float)ex[0] * 0.2f) - (float)ex[2] * 0.1f) * 10.0f;
                    nrm[0] += svo::sin_f32(arg) * 0.2f;
                    normalize3(nrm, nrm);
                }
                refract_dir(bounce->d, nrm);
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const float dk = bounce->d[k];
                    const int32_t s = dk < 0.0f ? -1 : 1;
                    const double delta = (double)svo::rcp_rn(dk);
                    const double ad = delta >= 0.0 ? delta : -delta;
                    if (s < 0) ex[k] -= 1.0;
                    R.T[k] = ad - (ex[k] - (double)R.r[k]) * delta;
                    R.s[k] = s;
                    R.af[k] = (float)ad;
                    R.ia[k] = __builtin_amdgcn_rcpf((float)ad);
                }
                // (deltaPos restarts from the shader's origin, not the current cell: |T| / absDelta
                // is bounded by the distance travelled, so the initial budget is held below 2^19 to
                // keep the count estimates within 1/2 — count_est)
                fast = !(P.flags & SVO_CAST_ITERATIVE) && budget < (1 << 19) && axis_ok(R.T[0], R.a(0)) && axis_ok(R.T[1], R.a(1)) &&
                       axis_ok(R.T[2], R.a(2)) && span_ok(R);
                lin = fast && exact_axis(R.T[0], R.a(0), R.steps) && exact_axis(R.T[1], R.a(1), R.steps) && exact_axis(R.T[2], R.a(2), R.steps);
                if (!SEG) fast = lin;  // (REFLECT runs in SEG instances)
            }
            dda_step(R);
            done = false;
            const uint32_t keep = mat;
            mat = kNoHit;
            if (kind == R_SOLID) {
                // the rest of a uniform refractive region (a lake's body): the same block voxel after
                // voxel — tint and step without lookups; its 2^sh-wide aligned region is the child
                // slot of `par` the lookup ended in.  A voxel reached with no budget left is the hit.
                for (;;) {
                    uint32_t w[3];
                    wrap3(R, wm, w);
                    if (((w[0] ^ wr[0]) | (w[1] ^ wr[1]) | (w[2] ^ wr[2])) >> par.sh) break;
                    if (R.steps <= 0) {
                        mat = keep;
                        done = true;
                        break;
                    }
                    bounce->m[0] *= t0;
                    bounce->m[1] *= t1;
                    bounce->m[2] *= t2;
                    if (STATS) st.tints++;
                    dda_step(R);
                }
            } else if (kind == R_BRICK) {
                // the rest of the brick (a lake's surface layer: water and air in one brick): its voxel mask and
                // materials are at hand, so refractive voxels are passed (each tints with its own block) and empty
                // ones stepped without lookups; any other block ends the ray there (a mirror with budget left is
                // left to the next iteration, which reflects it), and leaving the brick ends the pass (a lookup)
                for (;;) {
                    uint32_t w[3];
                    wrap3(R, wm, w);
                    if (((w[0] ^ wr[0]) | (w[1] ^ wr[1]) | (w[2] ^ wr[2])) >> 2) break;
                    const uint32_t v = child_slot(w[0], w[1], w[2], 0u);
                    if ((bmask >> v) & 1ull) {
                        const uint32_t m2 = brick_material(mats, bmask, bref, binfo, v);
                        const uint32_t f2 = P.mat_flags[m2];
                        if ((f2 & 7u) != 5u || R.steps <= 0) {
                            if ((f2 & 7u) != 3u || R.steps <= 0) {
                                mat = m2;  // the hit
                                done = true;
                            }
                            break;
                        }
                        const bool lq = (f2 & 0x10u) != 0u;
                        bounce->m[0] *= lq ? 0.94f : 0.95f;
                        bounce->m[1] *= lq ? 0.97f : 0.95f;
                        bounce->m[2] *= lq ? 1.0f : 0.95f;
                        if (STATS) st.tints++;
                    } else if (R.steps <= 0) {
                        done = true;  // the budget ends in an empty voxel
                        break;
                    }
                    dda_step(R);
                }
            }
        }
        // Progress guard, by construction: every iteration that does not end the ray takes at least one
        // DDA step (a crossing takes its exit step, a brick walk its first step, a reflection / refraction
        // its next one), so the budget strictly decreases.  An iteration that left the budget where it was,
        // or grew it — only a wrong crossing count could (a saturated or wrapped estimate, as before commit
        // 1a85dd6) — ends the ray: the launch always ends.  (STATS counts the trips: 0 in every test.)
        if (R.steps >= steps_in && !done) {
            if (STATS) st.no_progress++;
            R.steps = -1;  // marked in every build: the record's steps_left is -1 and the tree's trip counter counts it
            done = true;
        }
    }
    const bool hit = mat != kNoHit;
    // (out of the loop, so the stepping loop's state copies stay off every skip, and the lanes
    // whose budget ends in empty space take their last steps together).  Every other way out of
    // the loop without a hit has spent the budget.
    if (!hit && !escaped) {
        while (R.steps > 0) {
            dda_step(R);
            if (STATS) st.plain_steps++;
        }
    }
    if (par_out) *par_out = par;
    if (XS == 1 && hit) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            xs->T[k] = R.T[k];
            xs->r[k] = R.r[k];
        }
        xs->steps = R.steps;
        xs->axis = R.axis;
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
        for (int k = 0; k < 4; k++) atomicAdd(P.stats + 9 + k, (unsigned long long)st.skip_by_sh[k]);
        atomicAdd(P.stats + 13, (unsigned long long)st.bricks);
        atomicAdd(P.stats + 14, (unsigned long long)st.wv_iters);
        atomicAdd(P.stats + 15, (unsigned long long)st.wv_brick);
        atomicAdd(P.stats + 17, (unsigned long long)st.root_starts);
        atomicAdd(P.stats + 18, (unsigned long long)st.cache_empty);
        atomicAdd(P.stats + 19, (unsigned long long)st.wv_skips);
        atomicAdd(P.stats + 20, (unsigned long long)st.wv_descents);
        atomicAdd(P.stats + 21, (unsigned long long)st.path_starts);
        if (st.no_progress) atomicAdd(P.stats + 16, (unsigned long long)st.no_progress);
        atomicAdd(P.stats + 23, (unsigned long long)st.ceil_moves);
        atomicAdd(P.stats + 24, (unsigned long long)st.above_top);
        atomicAdd(P.stats + 25, (unsigned long long)st.bends);
        atomicAdd(P.stats + 26, (unsigned long long)st.tints);
        atomicAdd(P.stats + 27, (unsigned long long)st.tint_iters);
        // per-ray work (offline analysis, bench.py SVO_RAY_WORK): 16-bit fields, lookups | iterations | brick steps | node loads
        if (ray_work)
            *ray_work = (unsigned long long)min(st.lookups, 65535u) | ((unsigned long long)min(st.iters, 65535u) << 16) |
                        ((unsigned long long)min(st.brick_steps, 65535u) << 32) | ((unsigned long long)min(st.loads, 65535u) << 48);
    }
    if (!TRACK && !NO_T && R.axis < 3u) {
        // the last step's crossing: T - a exactly (exact sums); an infinite absDelta only comes
        // with an infinite crossing (deltaPos = inf - frac * inf), which stays inf
        const double Ta = R.axis == 0u ? R.T[0] : (R.axis == 1u ? R.T[1] : R.T[2]);
        const float aa = R.axis == 0u ? R.af[0] : (R.axis == 1u ? R.af[1] : R.af[2]);
        R.tlast = __builtin_isinf(aa) ? Ta : Ta - (double)aa;
    }
    Hit h;
    h.x = R.r[0];
    h.y = R.r[1];
    h.z = R.r[2];
    // (a miss has spent its budget or escaped: 0; a progress-guard trip: -1)
    h.steps_left = hit ? R.steps : min(R.steps, 0);
    if (R.steps < 0 && P.guard_trips) atomicAdd(P.guard_trips, 1u);
    h.t = (float)R.tlast;  // (one rounding of the same double as before)
    const int32_t sa = R.axis == 0u ? R.s[0] : (R.axis == 1u ? R.s[1] : R.s[2]);
    const uint32_t neg = (R.axis < 3u && sa < 0) ? 1u : 0u;
    h.info = (hit ? HIT_BIT : 0u) | (R.axis << AXIS_SHIFT) | (neg ? NEG_BIT : 0u) | (hit ? mat & MAT_MASK : 0u);
    if (ESCAPE && escaped) h.info |= ESC_BIT;  // (its position is where the escape began, not where the budget ends)
    return h;
}


// ------------------------------------------------------------------------------------------------
// Shading: low_res.frag's colour model over castRayFromCam hits — sky
// (genSkyBox :157-168), sun lighting (calcLightIntensity :242-252), 75-step shadow ray (:373-391),
// the looked-at block highlight (:340-343), reflections (:170-189) and refractions of solids
// (:196-240); the last two are applied inside trace.
// Single precision in the shader's operation order (-ffp-contract=off).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float3 color_of(uint64_t c) {  // color_int_to_vec3 (:139-145)
    const double sc = 1.0 / 2097152.0;
    return make_float3((float)((double)(c >> 42) * sc), (float)((double)((c >> 21) & 0x1FFFFFull) * sc),
                       (float)((double)(c & 0x1FFFFFull) * sc));
}

__device__ __forceinline__ float sigmoidf(float x, float scale, float k) { return 1.0f / (1.0f + expf(-x * k)) * scale; }

__device__ __forceinline__ float3 sky_color(const float d[3], const float sun[3]) {
    float dy = d[1];
    if (dy < 0.0f) dy *= 1.4f;
    const float haze = (0.1f - fabsf(fminf(fmaxf(dy, -0.3f), 0.3f))) * 0.8f + 0.1f;
    const float modifier = fminf(fmaxf(sigmoidf(1.0f - (haze * 2.0f), 1.0f, 2.0f), 0.0f), 1.0f);
    const float ex = d[0] - sun[0], ey = dy - sun[1], ez = d[2] - sun[2];
    const float b = sqrtf((ex * ex + ey * ey) + ez * ez) * 50.0f;
    const float sv = sigmoidf(1.5f - b, 1.0f, 1.6f);
    const float h3 = fminf(fmaxf(haze, 0.0f), 1.0f) * 3.0f;
    return make_float3((0.2f + h3) * modifier + sv, (0.4f + h3) * modifier + sv, (1.0f + h3) * modifier + 0.0f);
}

// ------------------------------------------------------------------------------------------------
// Hemisphere AO from a plan (A8).  An AO ray starts at the centre of lastPos: for a cell c >= 0,
// dda_axis gives deltaPos = absDelta - (+-0.5) * delta whatever c is, so the voxels a ray of
// direction d visits are lastPos + a fixed offset sequence, and the ray hits iff one of its
// ao_steps voxels is solid (castRayFromCam never tests the start voxel).  The host simulates the
// DDA of every (sample, hit face) once (ao_plan_get); per face the distinct offsets, each with the
// mask of samples passing through it, are grouped by the 4^3 brick they fall in — which depends on
// where lastPos sits in its brick, so there is one group list per (face, alignment).  Per hit,
// each brick is looked up once (skipped when all its samples already hit), starting at the deepest
// node of the primary ray's LDS path holding both the hit voxel and the brick; its solid plan voxels
// add their samples.  The count is the popcount of the samples hit.
// Plan layout (u32 words): [2g, 2g+1] = first record (16-B units), bricks, for g = face*64 + align
// (face = 2*axis + (sign < 0), align = lastPos & 3 per axis as z<<4|y<<2|x); per brick: {packed
// brick offset (bx+128 | by+128 << 8 | bz+128 << 16), 0, voxel mask lo, hi}, {union of its sample
// masks lo, hi, 0, 0}, then one u64 sample mask per voxel of the voxel mask in bit order (padded
// to 16 B).
// ------------------------------------------------------------------------------------------------
// A plan brick's lookup starts at the deepest node of the primary ray's LDS path holding both the hit voxel and the
// brick's corner w (mask / ref / child shift); an empty or SOLID region of any level covers whole bricks (0 or ~0)
__device__ __forceinline__ void brick_start(const CastParams& P, const Path& path, const uint32_t w[3], const uint32_t hw[3], int32_t dmax,
                                            uint64_t& mask, uint32_t& ref, uint32_t& sh) {
    const uint32_t diff = ((w[0] ^ hw[0]) | (w[1] ^ hw[1]) | (w[2] ^ hw[2])) | 1u;
    const int32_t da = min(P.levels - 1 - (int32_t)((31u - (uint32_t)__builtin_clz(diff)) >> 1), dmax);  // (diff != 0)
    mask = path.mask(da);
    ref = path.ref(da);
    sh = (uint32_t)(2 * (P.levels - 1 - da));
}

// loads: node loads of the plan's brick lookups (counted for SVO_CAST_STATS; dead code elsewhere)
template <class Mem>
__device__ __forceinline__ uint32_t ao_count_plan(const CastParams& P, const Mem& mem, const Path& path,
                                                  const Parent& pfin, const Hit& h, const int32_t l[3], uint32_t ax, int32_t sg,
                                                  uint32_t& loads) {
    const uint32_t face = 2u * ax + (sg < 0 ? 1u : 0u);
    const uint32_t al = ((uint32_t)l[0] & 3u) | (((uint32_t)l[1] & 3u) << 2) | (((uint32_t)l[2] & 3u) << 4);
    const uint2 hd = reinterpret_cast<const uint2*>(P.ao_plan)[face * 64u + al];
    const uint4* r = reinterpret_cast<const uint4*>(P.ao_plan) + hd.x;
    const uint32_t wm = P.wmask;
    const uint32_t hw[3] = {(uint32_t)h.x & wm, (uint32_t)h.y & wm, (uint32_t)h.z & wm};
    const uint32_t hb[3] = {(uint32_t)l[0] >> 2, (uint32_t)l[1] >> 2, (uint32_t)l[2] >> 2};
    const int32_t dmax = P.levels - 1 - (int32_t)(pfin.sh >> 1);
    const uint64_t all = P.ao_n >= 64 ? ~0ull : ((1ull << P.ao_n) - 1ull);
    uint64_t hits = 0ull;
    // the plan's bricks two at a time: both lookups descend in one loop, so their node loads are in flight together
    // (C4 -1.2 %, 20 AO rays -1.5 %: profiles/r06/ab_aopair_*.txt; three or four at a time spill 38 / 72 VGPRs).  A brick
    // whose samples all hit before its pair started is not looked up; one the pair's first brick would have covered is
    // looked up anyway — the union of the samples hit, the count, is the same
    for (uint32_t j = 0; j < hd.y && hits != all; j += 2u) {
        const uint4 e0 = r[0], u0 = r[1];
        const uint64_t vm0 = (uint64_t)e0.z | ((uint64_t)e0.w << 32), um0 = (uint64_t)u0.x | ((uint64_t)u0.y << 32);
        const uint2* sm0 = reinterpret_cast<const uint2*>(r + 2);
        r += 2u + (((uint32_t)__popcll(vm0) + 1u) >> 1);
        const bool has1 = j + 1u < hd.y;
        uint4 e1 = make_uint4(0u, 0u, 0u, 0u), u1 = make_uint4(0u, 0u, 0u, 0u);
        const uint2* sm1 = nullptr;
        if (has1) {
            e1 = r[0];
            u1 = r[1];
            sm1 = reinterpret_cast<const uint2*>(r + 2);
            r += 2u + (((uint32_t)__popcll((uint64_t)e1.z | ((uint64_t)e1.w << 32)) + 1u) >> 1);
        }
        const uint64_t vm1 = (uint64_t)e1.z | ((uint64_t)e1.w << 32), um1 = (uint64_t)u1.x | ((uint64_t)u1.y << 32);
        bool more0 = (hits & um0) != um0, more1 = has1 && (hits & um1) != um1;
        uint64_t mk0 = 0ull, mk1 = 0ull, res0 = 0ull, res1 = 0ull;
        uint32_t rf0 = 0u, rf1 = 0u, sh0 = 0u, sh1 = 0u, w0[3], w1[3];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            w0[k] = ((hb[k] + ((e0.x >> (8 * k)) & 255u) - 128u) << 2) & wm;
            w1[k] = ((hb[k] + ((e1.x >> (8 * k)) & 255u) - 128u) << 2) & wm;
        }
        if (more0) brick_start(P, path, w0, hw, dmax, mk0, rf0, sh0);
        if (more1) brick_start(P, path, w1, hw, dmax, mk1, rf1, sh1);
        while (more0 || more1) {
            Node n0, n1;
            bool ld0 = false, ld1 = false;
            if (more0) {
                const uint64_t t = slot_top(mk0, child_slot(w0[0], w0[1], w0[2], sh0));
                ld0 = (int64_t)t < 0;
                if (ld0) n0 = mem.load(popc_add(t, rf0));
                more0 = false;
            }
            if (more1) {
                const uint64_t t = slot_top(mk1, child_slot(w1[0], w1[1], w1[2], sh1));
                ld1 = (int64_t)t < 0;
                if (ld1) n1 = mem.load(popc_add(t, rf1));
                more1 = false;
            }
            if (ld0) {
                loads++;
                const uint32_t kind = n0.info & K_KIND_MASK;
                if (kind == K_INTERIOR) {
                    mk0 = n0.mask;
                    rf0 = n0.ref;
                    sh0 -= 2u;
                    more0 = true;
                } else {
                    res0 = kind == K_SOLID ? ~0ull : n0.mask;
                }
            }
            if (ld1) {
                loads++;
                const uint32_t kind = n1.info & K_KIND_MASK;
                if (kind == K_INTERIOR) {
                    mk1 = n1.mask;
                    rf1 = n1.ref;
                    sh1 -= 2u;
                    more1 = true;
                } else {
                    res1 = kind == K_SOLID ? ~0ull : n1.mask;
                }
            }
        }
        uint64_t m = res0 & vm0;
        while (m) {  // the plan voxels of this brick that are solid: their samples hit
            const uint32_t v = (uint32_t)__builtin_ctzll(m);
            const uint2 smv = sm0[__popcll(vm0 & ((1ull << v) - 1ull))];
            hits |= (uint64_t)smv.x | ((uint64_t)smv.y << 32);
            m &= m - 1ull;
        }
        m = res1 & vm1;
        while (m) {
            const uint32_t v = (uint32_t)__builtin_ctzll(m);
            const uint2 smv = sm1[__popcll(vm1 & ((1ull << v) - 1ull))];
            hits |= (uint64_t)smv.x | ((uint64_t)smv.y << 32);
            m &= m - 1ull;
        }
    }
    return (uint32_t)__popcll(hits);
}

// WIDE: 64-bit node addresses (trees above kNarrowNodes nodes, or SVO_CAST_WIDE_ADDR)
// The shading of a finished ray (low_res.frag:319-391 over castRayFromCam hits): its hit record (when requested) and its
// colour — the looked-at highlight, the sky of its final direction, or the lit / shadowed block (a 75-step shadow ray
// from the centre of lastPos through the solid view, smem); bn: its reflections / refraction (Bounce).  DIRS: the sun's
// step octant (0: per-wave sign flags)
template <int DIRS, class Mem>
__device__ __forceinline__ void shade_out(const CastParams& P, const Mem& smem, const Path& path, const Hit& h, const Bounce& bn, int64_t out) {
        if (P.pos) {
        reinterpret_cast<int4*>(P.pos)[out] = make_int4(h.x, h.y, h.z, h.steps_left);
        P.t[out] = h.t;
        P.info[out] = h.info;
    }
    const bool hit = (h.info & HIT_BIT) != 0u;
    const float* m = bn.m;  // finalColorMod
    float3 c;
    int32_t lk[3] = {P.look[0], P.look[1], P.look[2]};
    bool lv = P.look_valid != 0;
    if (P.look_dev) {  // (uniform: the pick ray's record, written on this stream before the launch)
        lk[0] = P.look_dev[0];
        lk[1] = P.look_dev[1];
        lk[2] = P.look_dev[2];
        lv = true;
    }
    // (an escaped ray's position is not its end; it can only end on a voxel the scene does not store, and the launch lets
    // rays escape only when the look-at voxel is stored: k_cast's `esc`)
    if (lv && !(h.info & ESC_BIT) && h.x == lk[0] && h.y == lk[1] && h.z == lk[2]) {
        const float3 b = color_of(P.mat_color[hit ? (h.info & MAT_MASK) : 0u]);
        c = make_float3(b.x * 2.0f + 0.3f, b.y * 2.0f + 0.3f, b.z * 2.0f + 0.3f);
    } else if (!hit) {
        const float3 sk = sky_color(bn.d, P.sun);
        c = make_float3(sk.x * m[0], sk.y * m[1], sk.z * m[2]);
    } else {
        const float3 col = color_of(P.mat_color[h.info & MAT_MASK]);
        const uint32_t ax = (h.info >> AXIS_SHIFT) & 3u;
        const int32_t sg = (h.info & NEG_BIT) ? -1 : 1;  // the ray's step on the hit axis
        const float l = (ax == 0u ? P.sun[0] : (ax == 1u ? P.sun[1] : P.sun[2])) * (float)(-sg);
        const bool facing = l > 0.0f;
        const float inten = fminf(fmaxf(0.0f, l) + 0.4f + (facing ? 0.15f : 0.0f), 1.0f);
        c = make_float3(col.x * inten * m[0], col.y * inten * m[1], col.z * inten * m[2]);
        bool dark = false;
        if ((bn.n & ~kBent) == 0) {  // (not reflected)
            if (!facing) {
                dark = true;
            } else {
                // shadow ray towards the sun from the centre of lastPos, through empty and liquid
                const float so[3] = {(float)(h.x - (ax == 0u ? sg : 0)) + 0.5f, (float)(h.y - (ax == 1u ? sg : 0)) + 0.5f,
                                     (float)(h.z - (ax == 2u ? sg : 0)) + 0.5f};
                // (DIRS: a sign octant every shadow ray of the launch steps with; shading launches pass 0 — their instances are
                // specialised on the camera's octant instead, k_cast)
                // the reference's sun, normalize(2, 1, 4) (globals.cpp:23; uniform), steps + on every axis: its octant is
                // compiled into a second copy of the shadow trace (shaded C3 -3.0 %, profiles/r06/ab_sun_octant_shadows.txt);
                // any other sun takes per-wave sign flags
                if (DIRS == 0 && P.sun_dirs == 1)
                    dark = (trace<false, false, true, false, 1, false, 3>(P, smem, P.smats, path, so, P.sun, P.shadow_steps, nullptr, nullptr, nullptr,
                                                                          P.top_solid).info & HIT_BIT) != 0u;
                else
                dark = (trace<false, false, true, false, DIRS, false, 3>(P, smem, P.smats, path, so, P.sun, P.shadow_steps, nullptr, nullptr, nullptr, P.top_solid)
                            .info & HIT_BIT) != 0u;
            }
        }
        if (dark) c = make_float3(col.x * 0.3f * m[0], col.y * 0.3f * m[1], col.z * 0.3f * m[2]);
    }
    P.rgba[out] = make_float4(c.x, c.y, c.z, 0.0f);
}

// Frame mode: the pixel of this lane of launch block blk (its ray o, d and record index out; out = -1 for lanes past the
// frame's edge).  8-pixel tile rows, one wavefront per 2^(6-lh) x 2^lh footprint; frames interleave wave by wave (every
// frame's long top rows first); the frame and tile indices are wave-uniform: their divisions run on the scalar unit.
__device__ __forceinline__ void frame_pixel(const CastParams& P, int64_t blk, float o[3], float d[3], int64_t& out, uint32_t& frm,
                                            int32_t* pxy = nullptr) {
    const uint32_t wv = (uint32_t)blk * (kBlock / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t fr = wv % (uint32_t)P.n_frames, tile = wv / (uint32_t)P.n_frames;
    frm = fr;
    const int32_t lane = (int32_t)(threadIdx.x & 63u);
    // (small launches: the first half_rows tile rows dispatched are cast by half footprints — two adjacent waves of 32
    // lanes per footprint, 2^(lh-1) pixel rows each; frame_half_rows)
    const uint32_t h2 = (uint32_t)P.half_rows * 2u * (uint32_t)P.tiles_x;
    uint32_t tq, tx_;
    int32_t half = -1;
    if (tile < h2) {
        tq = tile / (2u * (uint32_t)P.tiles_x);
        const uint32_t t2 = tile - tq * 2u * (uint32_t)P.tiles_x;
        tx_ = t2 >> 1;
        half = (int32_t)(t2 & 1u);
    } else {
        const uint32_t t = tile - h2 + (uint32_t)P.half_rows * (uint32_t)P.tiles_x;
        tq = t / (uint32_t)P.tiles_x;
        tx_ = t - tq * (uint32_t)P.tiles_x;
    }
    int32_t trl = (int32_t)tq;
    // default order: top tile rows first (rays nearest the horizon travel furthest; dispatching
    // them first keeps the long tiles out of the launch's tail)
    if (!(P.flags & SVO_CAST_BOTTOM_FIRST)) trl = P.tile_rows_local - 1 - trl;
    const int32_t tx = (int32_t)tx_;
    const int32_t tr = P.tile_row_start + trl * P.tile_row_step;
    // the wavefront's 2^(6-lh) x 2^lh pixels of its 8-pixel tile row (lh = 3: an 8x8 tile); the
    // sub-rows of one column of footprints are adjacent waves
    const int32_t lh = P.tile_lh, lw = 6 - lh, sub = 3 - lh;
    const int32_t rr = ((tx & ((1 << sub) - 1)) << lh) + (half >= 0 ? (half << (lh - 1)) : 0) + (lane >> lw);
    const int32_t px = ((tx >> sub) << lw) + (lane & ((1 << lw) - 1)), py = tr * 8 + rr;
    if (trl >= 0 && trl < P.tile_rows_local && px < P.width && py < P.height && !(half >= 0 && lane >= 32)) {
        raygen_pixel(P.rg, px, py, d);
        o[0] = P.frame_org[3 * fr + 0];
        o[1] = P.frame_org[3 * fr + 1];
        o[2] = P.frame_org[3 * fr + 2];
        out = (int64_t)fr * P.frame_records + ((int64_t)trl * 8 + rr) * P.width + px;
        if (pxy) {
            pxy[0] = px;
            pxy[1] = py;
        }
    }
}

template <bool STATS, bool STAMPS, bool AO, bool SHADE, bool WIDE, bool SEG, int DIRS = 0, bool NOREC = false>
// primary rays: 64 VGPRs = 8 waves per SIMD without spills; the AO instances run 8 waves too (4 spilled VGPRs; with
// the hemisphere table read from the kernel arguments instead of LDS, the LDS allows 8 waves: C4 0.2441 -> 0.2311 ms
// against 6 waves at 79 VGPRs, 0.2349 at 7); the diagnostics instances 6; the shading instances 7 waves on the camera's
// octant (kShadeWaves), 6 with generic signs
__global__ __launch_bounds__(kBlock, STATS ? 6 : (SHADE ? (DIRS != 0 ? kShadeWaves : 6) : 8)) void k_cast(const CastParams P) {
    using Mem = typename std::conditional<WIDE, WideNodes, BufNodes>::type;
    const Mem mem(P.nodes);
    const Mem smem(SHADE ? P.snodes : P.nodes);  // shading: shadow rays walk the solid view
    // diagnostics: block start / end stamps (100 MHz s_memrealtime) after the 16 counters
    // (frame schedules: shading instances only — sched_attach; the primary instances compile without the hooks)
    const bool sched = SHADE && P.sched_cost;
    const unsigned long long t_start = (STAMPS || sched) ? __builtin_amdgcn_s_memrealtime() : 0ull;
    // per-lane node path (mask and first-child index of the interior node at each depth of the
    // last descent), [depth][lane]
    // (dynamic LDS: the launch's own depth, path_lds — a 6-level tree's shading launch fits 7 blocks per SIMD)
    extern __shared__ uint32_t path_words[];
    const Path path = {path_words + threadIdx.x};
    // (the hemisphere AO sample set is read from the kernel arguments: uniform loads, no LDS)
    __shared__ Bounce shade_bn[SHADE ? kBlock : 1];  // shading: the rays' bounce state (k_cast SHADE below)
    int64_t blk = blockIdx.x;
    // (frame mode: the schedule's group of kSchedGroup blocks at this dispatch slot's group)
    if (SHADE && P.sched_order) blk = (int64_t)P.sched_order[blockIdx.x / kSchedGroup] * kSchedGroup + blockIdx.x % kSchedGroup;
    const int64_t g = blk * kBlock + threadIdx.x;
    float o[3] = {0.0f, 0.0f, 0.0f}, d[3] = {0.0f, 0.0f, 0.0f};
    int64_t out = -1;
    uint32_t frm = 0u;  // the wave's frame (frame mode)
    if (P.mode == MODE_FRAME) {
        frame_pixel(P, blk, o, d, out, frm);
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
    if (SHADE && out >= 0) {
        // the ray's bounce state lives in LDS: the trace touches it only at reflections / refractions, and in registers
        // it cost the loop spills (22 VGPRs at 8 waves; 0.4748 -> 0.4660 ms per shaded C3 frame at 5 waves without them)
        Bounce& bn = shade_bn[threadIdx.x];
        bn = {{d[0], d[1], d[2]}, 0, {1.0f, 1.0f, 1.0f}};
        // rays may escape (stop early once only empty voxels lie ahead) unless their end position is output (hit records)
        // or could be the highlighted lookingAtBlock (low_res.frag:347 compares every ray's end, misses too): a look-at
        // voxel the scene may not store — the host's, checked on the host, or a device pick record that is not a sure hit
        // (stepsLeft 0: a miss or a hit on the last step) (uniform)
        const bool look_risk = P.look_dev ? P.look_dev[6] <= 0 : (P.look_valid && P.look_empty);
        const int32_t esc = (P.pos || look_risk) ? -1 : P.top_scene;
        unsigned long long* const rw = P.stats ? P.stats + SVO_STATS_HEADER + 2 * (int64_t)gridDim.x * (kBlock / 64) + out : nullptr;
        if (STATS || STAMPS) {  // (diagnostics: one trace, bounces included)
            const Hit h = trace<STATS, true, true, SEG, 0, false, 2, NOREC>(P, mem, P.mats, path, o, d, P.steps, rw, &bn, nullptr, esc, P.top_scene);
            shade_out<0>(P, smem, path, h, bn, out);
        } else {
            // the straight trace to the first block hit — no reflection / refraction upkeep per step, on the camera's step
            // octant (DIRS) — and only a mirror or a refractive block with budget left hands its state on to the bouncing
            // trace, which resumes there (shaded C3 0.3103 -> 0.3027 ms, then 0.2914 with the octant; the straight trace's
            // state on its first hit is the one the bouncing trace from the origin reaches: both take castRayFromCam's
            // exact steps).  Its column ceilings: the launch's two levels (CEIL 1, as primary casts: 0.8 % faster than the walk
            // over every level, CEIL 2, which the bouncing trace keeps)
            RayState xs;
            Hit h = trace<false, false, true, SEG, DIRS, false, 1, NOREC, 1>(P, mem, P.mats, path, o, d, P.steps, nullptr, nullptr, nullptr,
                                                                             esc, P.top_scene, DIRS != 0 ? &P.fax[frm] : nullptr, &xs);
            const uint32_t mf = ((h.info & HIT_BIT) && h.steps_left > 0) ? P.mat_flags[h.info & MAT_MASK] & 7u : 0u;
            if (mf == 3u || mf == 5u)
                h = trace<false, true, true, true, 0, false, 2, NOREC, 2>(P, mem, P.mats, path, o, d, P.steps, nullptr, &bn, nullptr, esc,
                                                                     P.top_scene, nullptr, &xs);
            shade_out<0>(P, smem, path, h, bn, out);
        }
    } else if (out >= 0) {
        Parent pfin;
        const Hit h = trace<STATS, false, false, SEG, DIRS, AO, 1>(P, mem, P.mats, path, o, d, P.steps, P.stats ? P.stats + SVO_STATS_HEADER + 2 * (int64_t)gridDim.x * (kBlock / 64) + out : nullptr,
                                   nullptr, AO ? &pfin : nullptr, -1, P.top_solid, DIRS != 0 ? &P.fax[frm] : nullptr);
        if (!SHADE && P.wire) {  // (wave-uniform: one launch writes one kind of record)
            wire_put(P.wire, P.wire_compact != 0, out, o, h.x, h.y, h.z, h.t, h.info);
        } else {
            reinterpret_cast<int4*>(P.pos)[out] = make_int4(h.x, h.y, h.z, h.steps_left);
            P.t[out] = h.t;
            P.info[out] = h.info;
        }
        if (AO) {
            // AO rays from the centre of lastPos, pole turned to the hit face's normal (A8)
            uint32_t cnt = 0u;
            if (h.info & HIT_BIT) {
                const uint32_t ax = (h.info >> AXIS_SHIFT) & 3u;
                const int32_t st = (h.info & NEG_BIT) ? -1 : 1;  // step on the hit axis
                const int32_t lx = h.x - (ax == 0u ? st : 0), ly = h.y - (ax == 1u ? st : 0), lz = h.z - (ax == 2u ? st : 0);
                const int32_t l[3] = {lx, ly, lz};
                if (P.ao_plan && pfin.sh < 2u * (uint32_t)P.levels && (uint32_t)lx < (1u << 23) && (uint32_t)ly < (1u << 23) && (uint32_t)lz < (1u << 23)) {
                    uint32_t aol = 0u;
                    cnt = ao_count_plan(P, mem, path, pfin, h, l, ax, -st, aol);
                    if (STATS) atomicAdd(P.stats + 22, (unsigned long long)aol);
                } else {
                const float ao_o[3] = {(float)lx + 0.5f, (float)ly + 0.5f, (float)lz + 0.5f};
                for (int32_t i = 0; i < P.ao_n; i++) {
                    const float hv[3] = {P.ao_tab[3 * i], P.ao_tab[3 * i + 1], P.ao_tab[3 * i + 2]};
                    float ad[3];
                    ao_dir(hv, ax, -st, ad);
                    const Hit a = trace<false>(P, mem, P.mats, path, ao_o, ad, P.ao_steps);
                    cnt += (a.info & HIT_BIT) ? 1u : 0u;
                }
                }
            }
            P.ao[out] = (uint8_t)cnt;
        }
    }
    if (STAMPS || sched) {
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();  // (one wavefront per block: every lane is done)
        if (threadIdx.x == 0) {
            if (STAMPS) {
                P.stats[SVO_STATS_HEADER + 2 * blockIdx.x] = t_start;
                P.stats[SVO_STATS_HEADER + 2 * blockIdx.x + 1] = t_end;
            }
            if (sched) P.sched_cost[blk] = (uint32_t)std::min(t_end - t_start, 0xFFFFFFFFull);
        }
    }
}

// The next frame's dispatch order from this frame's block durations (one workgroup): a counting sort, longest first, of
// groups of kSchedGroup consecutive blocks (a group's duration: its longest block's) on 256 logarithmic buckets (8 per
// octave: durations within 12.5 % share one; groups within a bucket in any order).  Its cost is the LDS atomics, which
// serialise on a bucket (most blocks share a few): per block 24 us for a 1080p frame, per group of 4 a quarter; the
// groups also keep 64 x 4-pixel strips of a tile row together.  All of a thread's loads go out together (kSchedBatch
// per thread, kept in registers for the scatter up to 32768 groups).  The key is a function of the duration alone,
// and every group index lands once: the order is a permutation whatever the durations.
constexpr int kSchedThreads = 1024, kSchedBuckets = 256, kSchedBatch = 32;
__device__ __forceinline__ uint32_t sched_key(uint32_t c) {
    // bits 20.. of the f32 value: exponent and 3 mantissa bits; c >= 1 gives 0 .. 255 from 1 to 2^32 (c near 2^32 rounds
    // to 2^32: 256, clamped)
    if (c == 0u) return (uint32_t)(kSchedBuckets - 1);
    return (uint32_t)(kSchedBuckets - 1) - std::min((__float_as_uint((float)c) >> 20) - (127u << 3), (uint32_t)(kSchedBuckets - 1));
}
// the duration of group i: its longest block (kSchedGroup == 4: one 16-B load)
__device__ __forceinline__ void sched_load(const uint32_t* __restrict__ cost, uint32_t n, uint32_t base, uint32_t (&c)[kSchedBatch]) {
    static_assert(kSchedGroup == 4, "one uint4 per group");
#pragma unroll
    for (int j = 0; j < kSchedBatch; j++) {
        const uint32_t i = base + (uint32_t)j * kSchedThreads + threadIdx.x;
        const uint4 q = i < n ? reinterpret_cast<const uint4*>(cost)[i] : make_uint4(0u, 0u, 0u, 0u);
        c[j] = std::max(std::max(q.x, q.y), std::max(q.z, q.w));
    }
}
// n: groups
__global__ __launch_bounds__(kSchedThreads) void k_sched_order(const uint32_t* __restrict__ cost, uint32_t* __restrict__ order, uint32_t n) {
    __shared__ uint32_t hist[kSchedBuckets];
    __shared__ uint32_t wsum[kSchedBuckets / 64];
    const uint32_t tid = threadIdx.x;
    constexpr uint32_t kRound = (uint32_t)kSchedThreads * kSchedBatch;
    uint32_t c[kSchedBatch];
    sched_load(cost, n, 0u, c);
    if (tid < kSchedBuckets) hist[tid] = 0u;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += kRound) {
        if (base) sched_load(cost, n, base, c);
#pragma unroll
        for (int j = 0; j < kSchedBatch; j++)
            if (base + (uint32_t)j * kSchedThreads + tid < n) atomicAdd(&hist[sched_key(c[j])], 1u);
    }
    __syncthreads();
    // exclusive scan of the histogram: per wavefront, then the wavefronts' totals
    uint32_t v = 0u, inc = 0u;
    if (tid < kSchedBuckets) {
        v = hist[tid];
        inc = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)inc, o);
            if ((tid & 63u) >= (uint32_t)o) inc += u;
        }
        if ((tid & 63u) == 63u) wsum[tid >> 6] = inc;
    }
    __syncthreads();
    if (tid < kSchedBuckets) {
        uint32_t b = 0u;
        for (uint32_t w = 0; w < (tid >> 6); w++) b += wsum[w];
        hist[tid] = b + inc - v;
    }
    __syncthreads();
    for (uint32_t base = 0; base < n; base += kRound) {
        if (n > kRound) sched_load(cost, n, base, c);  // (one round: the durations are still in c)
#pragma unroll
        for (int j = 0; j < kSchedBatch; j++) {
            const uint32_t i = base + (uint32_t)j * kSchedThreads + tid;
            if (i < n) order[atomicAdd(&hist[sched_key(c[j])], 1u)] = i;
        }
    }
}

// The AO plan of (n samples, `steps`) (see ao_count_plan): every (sample, face) ray simulated with
// the kernel's DDA from the centre of cell 0 — dda_axis, then dda_step's axis rule in double.
// Offsets are listed by step index, then sample, first appearance only.  Cached on the tree.
static int ao_plan_get(const svo_tree* t, int32_t n, int32_t steps, const float* tab, const uint32_t** out) {
    *out = nullptr;
    if (steps > 127 || n > 64) return SVO_OK;  // offsets are packed in bytes, masks in 64 bits: rays
    if (t->d_ao_plan && t->ao_plan_n == n && t->ao_plan_steps == steps) {
        *out = reinterpret_cast<const uint32_t*>(t->d_ao_plan);
        return SVO_OK;
    }
    std::vector<std::vector<std::pair<uint32_t, uint64_t>>> faces(6);
    for (int face = 0; face < 6; face++) {
        const uint32_t ax = (uint32_t)face >> 1;
        const int32_t sg = (face & 1) ? -1 : 1;
        std::vector<std::vector<uint32_t>> seq(n);
        for (int32_t i = 0; i < n; i++) {
            float dir[3];
            ao_dir(tab + 3 * i, ax, sg, dir);
            double T[3], A[3];
            int32_t st[3], pos[3] = {0, 0, 0};
            for (int k = 0; k < 3; k++) {
                const Dda1 a = dda_axis(0.5f, dir[k]);
                T[k] = a.dpos;
                A[k] = (double)(float)a.adelta;
                st[k] = a.step;
            }
            for (int32_t j = 0; j < steps; j++) {
                const bool cx = (T[0] < T[1]) && (T[0] < T[2]);
                const bool cy = !cx && (T[1] < T[2]);
                const int k = cx ? 0 : (cy ? 1 : 2);
                pos[k] += st[k];
                T[k] = T[k] + A[k];
                seq[i].push_back((uint32_t)(pos[0] + 128) | ((uint32_t)(pos[1] + 128) << 8) | ((uint32_t)(pos[2] + 128) << 16));
            }
        }
        auto& f = faces[face];
        for (int32_t j = 0; j < steps; j++)
            for (int32_t i = 0; i < n; i++) {
                const uint32_t key = seq[i][j];
                size_t e = 0;
                while (e < f.size() && f[e].first != key) e++;
                if (e == f.size()) f.push_back({key, 0ull});
                f[e].second |= 1ull << i;
            }
    }
    struct Brick {
        uint32_t key;
        uint64_t vm, um, sm[64];
    };
    std::vector<uint32_t> img(2 * 6 * 64, 0u);
    for (int face = 0; face < 6; face++)
        for (int al = 0; al < 64; al++) {
            const int32_t a[3] = {al & 3, (al >> 2) & 3, al >> 4};
            std::vector<Brick> bricks;  // in order of first use
            for (const auto& f : faces[face]) {
                uint32_t key = 0u, v = 0u;
                for (int k = 0; k < 3; k++) {
                    const int32_t p = a[k] + (int32_t)((f.first >> (8 * k)) & 255u) - 128;  // from lastPos's brick corner
                    key |= (uint32_t)((p >> 2) + 128) << (8 * k);                            // floor division
                    v |= (uint32_t)(p & 3) << (2 * k);
                }
                size_t b = 0;
                while (b < bricks.size() && bricks[b].key != key) b++;
                if (b == bricks.size()) {
                    bricks.push_back(Brick{});
                    bricks.back().key = key;
                }
                bricks[b].vm |= 1ull << v;
                bricks[b].um |= f.second;
                bricks[b].sm[v] |= f.second;
            }
            const size_t g = (size_t)face * 64 + (size_t)al;
            img[2 * g] = (uint32_t)(img.size() / 4);
            img[2 * g + 1] = (uint32_t)bricks.size();
            for (const Brick& b : bricks) {
                const uint32_t rec[8] = {b.key, 0u, (uint32_t)b.vm, (uint32_t)(b.vm >> 32), (uint32_t)b.um, (uint32_t)(b.um >> 32), 0u, 0u};
                img.insert(img.end(), rec, rec + 8);
                for (int v = 0; v < 64; v++)
                    if ((b.vm >> v) & 1ull) {
                        img.push_back((uint32_t)b.sm[v]);
                        img.push_back((uint32_t)(b.sm[v] >> 32));
                    }
                while (img.size() % 4) img.push_back(0u);
            }
        }
    if (t->d_ao_plan) (void)hipFree(t->d_ao_plan);
    t->d_ao_plan = nullptr;
    t->ao_plan_steps = -1;
    HIP_TRY(hipMalloc(&t->d_ao_plan, img.size() * sizeof(uint32_t)), SVO_ENOMEM);
    HIP_TRY(hipMemcpy(t->d_ao_plan, img.data(), img.size() * sizeof(uint32_t), hipMemcpyHostToDevice), SVO_EDEVICE);
    t->ao_plan_n = n;
    t->ao_plan_steps = steps;
    *out = reinterpret_cast<const uint32_t*>(t->d_ao_plan);
    return SVO_OK;
}

// node addressing of a cast over t: 64-bit when its device allocation holds more nodes than a 32-bit
// buffer offset reaches (or on request)
bool wide_nodes(const svo_tree* t, int32_t flags) { return t->dev_node_cap >= kNarrowNodes || (flags & SVO_CAST_WIDE_ADDR); }

// The per-lane LDS path of k_cast (Path): 3 dwords per interior depth (levels - 1 of them) per lane of the block
size_t path_lds(const CastParams& P) { return (size_t)(P.levels > 1 ? P.levels - 1 : 1) * 3 * kBlock * sizeof(uint32_t); }

// The sign-octant instances (dirs 1..8, frame_dirs) of one family, as a table built at compile time: launch block b of the
// primary casts (AO or not, SEG or not) and of the shading pass's straight trace (with / without hit records) picks its
// kernel by index instead of a hand-written case per octant
using CastKernel = void (*)(CastParams);
template <bool AO, bool SHADE, bool SEG, bool NOREC, size_t... I>
constexpr std::array<CastKernel, sizeof...(I)> octant_kernels(std::index_sequence<I...>) {
    return {{&k_cast<false, false, AO, SHADE, false, SEG, (int)I + 1, NOREC>...}};
}
template <bool AO, bool SHADE, bool SEG, bool NOREC = false>
void launch_octant(int dirs, dim3 grid, dim3 block, hipStream_t st, const CastParams& P) {
    static constexpr std::array<CastKernel, 8> tab = octant_kernels<AO, SHADE, SEG, NOREC>(std::make_index_sequence<8>());
    CastParams arg = P;
    void* args[] = {&arg};
    (void)hipLaunchKernel(reinterpret_cast<const void*>(tab[(dirs >= 1 && dirs <= 8 ? dirs : 8) - 1]), grid, block, args, path_lds(P), st);
}
template <bool STATS, bool STAMPS, bool AO, bool SHADE>
void launch_cast(bool wide, bool seg, dim3 grid, dim3 block, hipStream_t st, const CastParams& P, int dirs = 0) {
    if (!STATS && !STAMPS && !SHADE && !wide && dirs) {  // (narrow trees: below 2^28 nodes)
        if (seg) launch_octant<AO, false, true>(dirs, grid, block, st, P);
        else launch_octant<AO, false, false>(dirs, grid, block, st, P);
        return;
    }
    // the camera's octant (the straight trace of the shading rays); without hit records, a launch whose every origin is
    // exact (seg: need_seg false) takes the straight trace without segment bounds (the bouncing trace keeps them)
    if (SHADE && !STATS && !wide && dirs) {
        if (P.pos) launch_octant<false, true, true>(dirs, grid, block, st, P);
        else if (seg) launch_octant<false, true, true, true>(dirs, grid, block, st, P);
        else launch_octant<false, true, false, true>(dirs, grid, block, st, P);
        return;
    }
    if (SHADE || seg) {
        if (wide) hipLaunchKernelGGL((k_cast<STATS, STAMPS, AO, SHADE, true, true>), grid, block, path_lds(P), st, P);
        else hipLaunchKernelGGL((k_cast<STATS, STAMPS, AO, SHADE, false, true>), grid, block, path_lds(P), st, P);
    } else {
        if (wide) hipLaunchKernelGGL((k_cast<STATS, STAMPS, AO, false, true, false>), grid, block, path_lds(P), st, P);
        else hipLaunchKernelGGL((k_cast<STATS, STAMPS, AO, false, false, false>), grid, block, path_lds(P), st, P);
    }
}

// The launch's step-sign octant (1..8, dirs_sign) when every frame ray has the same step signs, else 0.
// A pixel's direction before normalisation (raygen_pixel) is an affine function of the pixel, so its
// extremes are at the frame's corners; a corner value beyond 1e-4 of the terms' magnitudes keeps
// every pixel's rounded value (errors of a few ulps of those terms) on the same side of zero, and
// normalisation keeps the sign.  Explicit rays: 0.
static int frame_dirs(const CastParams& P) {
    if (P.mode != MODE_FRAME || (P.flags & SVO_CAST_NO_OCTANT)) return 0;
    int code = 1;
    for (int a = 0; a < 3; a++) {
        int pos = 0, neg = 0;
        for (int c = 0; c < 4; c++) {
            const int32_t px = (c & 1) ? P.width - 1 : 0, py = (c & 2) ? P.height - 1 : 0;
            const float fx = ((float)px + 0.5f) * P.rg.rw, fy = ((float)py + 0.5f) * P.rg.rh;
            const float sl = -(P.rg.ppx * (fx - 0.5f)), su = -fy + 0.5f;
            const float lt = P.rg.l[a] * sl, ut = (P.rg.u[a] * su) * P.rg.ppy;
            const float v = (P.rg.c[a] + lt) + ut;
            const float mag = fabsf(P.rg.c[a]) + fabsf(P.rg.l[a]) * fabsf(P.rg.ppx) + fabsf(P.rg.u[a] * P.rg.ppy);
            if (v > 1e-4f * mag) pos++;
            else if (v < -1e-4f * mag) neg++;
        }
        if (pos == 4) continue;
        if (neg == 4) code += 1 << a;
        else return 0;
    }
    return code;
}

// Can the launch hold rays that are not linear (svo_cast.hip, "Exact closed-form skipping")?  From an
// integral or half-integral origin every ray is (lin_origin, with budgets below 2^28 every sum it
// takes is exact); explicit rays are not inspected.  The instance without segments relies on it
// (trace: TRACK); SVO_CAST_SEGMENTS forces the other one (the same results).
static bool need_seg(const CastParams& P) {
    if (P.flags & SVO_CAST_SEGMENTS) return true;
    if (P.mode == MODE_EXPLICIT || P.steps >= (1 << 28)) return true;
    const int32_t nf = P.mode == MODE_FRAME ? P.n_frames : 1;
    const float* org = P.mode == MODE_FRAME ? P.frame_org : P.org;
    for (int32_t i = 0; i < 3 * nf; i++)
        if (!(2.0f * org[i] == __builtin_truncf(2.0f * org[i]) && __builtin_fabsf(org[i]) < 1073741824.0f)) return true;
    return false;
}

// the octant's frame set-up (FrameAxes) for every frame of the launch
static void frame_axes(CastParams& P, int dirs) {
    if (dirs == 0) return;
    for (int32_t f = 0; f < P.n_frames; f++)
        for (int k = 0; k < 3; k++) {
            const float o = P.frame_org[3 * f + k];
            const int32_t cell = (int32_t)__builtin_truncf(o);
            const double exact = ((dirs - 1) >> k) & 1 ? (double)o - 1.0 : (double)o;
            P.fax[f].cell[k] = cell;
            P.fax[f].frac[k] = exact - (double)cell;
        }
}

// The two ceiling levels a launch checks, as levels of the tree's table (4^(kCeilK0 + j) columns per block).
// Primary casts: 16 and 64 columns (C3 0.1824 -> 0.1787 ms, C5 0.562 -> 0.543 against 64 / 256; 16 / 256 was
// slower than both: profiles/r03/ab_j_*.log).  The shading pass walks every level (trace CEIL 2: P.ceilq); its
// pair levels are unused.
constexpr int kCeilPrimary[2] = {0, kCeilPairStep}, kCeilShade[2] = {0, kCeilPairStep};
// (a launch's second level is read from the pair table, whose high half is level lv[0] + kCeilPairStep: the box of
// level lv[1] must come with the ceiling of a block that holds it)
static_assert(kCeilPrimary[1] - kCeilPrimary[0] == kCeilPairStep && kCeilShade[1] - kCeilShade[0] == kCeilPairStep,
              "ceiling pairs: the second level must be the pair table's partner level");

static void set_ceilings(const svo_tree* t, const svo_cast_desc* d, CastParams& P, const int lv[2]) {
    P.ceil = nullptr;
    P.ceil_levels = 0;
    if (d->flags & SVO_CAST_NO_CEILINGS) return;
    P.ceil = reinterpret_cast<const int16_t*>(t->d_ceil);
    P.ceil_levels = t->ceil_levels > lv[1] ? 2 : (t->ceil_levels > lv[0] ? 1 : 0);
    // (the pair table of level lv[0] holds lv[0] + kCeilPairStep = lv[1] when the tree has it, else its coarsest level, whose
    // blocks hold level lv[0]'s: with one level the kernel's second box is then level lv[0]'s — as below — under a ceiling
    // at least as high as that block's own, which is safe)
    P.ceilp = P.ceil_levels > 0 ? reinterpret_cast<const uint32_t*>(t->d_ceilp) + t->ceilp_off[lv[0]] : nullptr;
    P.ceilq = P.ceil_levels > 0 ? reinterpret_cast<const uint64_t*>(t->d_ceilq) : nullptr;
    for (int j = 0; j < 2; j++) {
        // (one level only: the second is a copy of the first, so the kernel may read both unconditionally)
        const int l = j < P.ceil_levels ? lv[j] : lv[0];
        P.ceil_sh[j] = 2u * (uint32_t)(kCeilK0 + l);
        P.ceil_off[j] = t->ceil_off[l];
    }
}

// the tree's progress-guard trip counter: a u32 in its device side buffer (svo_internal.h kSideGuard)
uint32_t* guard_word(const svo_tree* t) { return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(t->d_pick) + kSideGuard); }

int fill_params(const svo_tree* t, const svo_cast_desc* d, const svo_hits* o, CastParams& P, int64_t& nthreads) {
    memset(&P, 0, sizeof(P));
    P.nodes = reinterpret_cast<const Node*>(t->d_nodes);
    P.mats = reinterpret_cast<const uint16_t*>(t->d_mats);
    P.mat_color = reinterpret_cast<const uint64_t*>(t->d_pal);
    P.mat_flags = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(t->d_pal) + t->dev_pal_n * 8);
    P.levels = t->levels;
    P.wmask = (1u << (2 * t->levels)) - 1u;
    P.top_solid = t->dev_top_y;  // the empty region above the tree's highest voxel row (trace: pre_top)
    P.guard_trips = guard_word(t);
    set_ceilings(t, d, P, kCeilPrimary);
    P.steps = d->steps;
    P.flags = d->flags;
    P.stats = reinterpret_cast<unsigned long long*>(d->stats);
    P.org[0] = d->origin[0];
    P.org[1] = d->origin[1];
    P.org[2] = d->origin[2];
    P.pos = o->pos_steps;
    P.t = o->t;
    P.info = o->info;
    P.ao = o->ao;
    P.ao_n = d->ao_samples;
    P.ao_steps = d->ao_steps;
    if (P.ao_n > 0) {
        hemisphere_table(P.ao_n, P.ao_tab);
        if (!(P.flags & SVO_CAST_AO_TRACE)) {
            int rc = ao_plan_get(t, P.ao_n, P.ao_steps, P.ao_tab, &P.ao_plan);
            if (rc) return rc;
        }
    }
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
    // wavefronts per tile row: one per 16x4 footprint (or 8x8 / 32x2: svo_rt.h)
    P.tile_lh = frame_wave_lh(d->flags);
    P.tiles_x = frame_wave_cols(d->width, P.tile_lh);
    P.tile_row_start = d->tile_row_start;
    P.tile_row_step = d->tile_row_step;
    const int32_t tile_rows = (d->height + 7) / 8;
    P.tile_rows_local = d->tile_row_start < tile_rows ? (tile_rows - d->tile_row_start + d->tile_row_step - 1) / d->tile_row_step : 0;
    if (d->n_frames < 0 || d->n_frames > SVO_MAX_FRAMES) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: n_frames outside [0, SVO_MAX_FRAMES]");
    if (d->n_frames > 1 && !d->frame_origins) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: n_frames > 1 without frame_origins");
    P.n_frames = d->n_frames > 1 ? d->n_frames : 1;
    P.half_rows = frame_half_rows(P.tile_rows_local, d->flags, P.tile_lh, P.tiles_x, P.n_frames);
    for (int32_t f = 0; f < P.n_frames; f++)
        for (int k = 0; k < 3; k++) P.frame_org[3 * f + k] = d->n_frames > 1 ? d->frame_origins[3 * f + k] : d->origin[k];
    int64_t per_frame = 0;
    for (int32_t r = d->tile_row_start; r < tile_rows; r += d->tile_row_step) per_frame += std::min(8, d->height - r * 8);
    P.frame_records = per_frame * d->width;
    // (a dispatch holds fewer than 2^32 work-items: the HSA packet's grid size is 32-bit)
    if ((int64_t)(P.tile_rows_local + P.half_rows) * P.tiles_x * P.n_frames >= (int64_t)1 << 26)
        SVO_FAIL(SVO_ERANGE, "svo_cast_rays: frame too large (2^26 wavefronts or more in one launch)");
    nthreads = (int64_t)(P.tile_rows_local + P.half_rows) * P.tiles_x * P.n_frames * 64;
    return SVO_OK;
}

// Frame schedules: a shading launch of more than SVO_SCHED_MIN_BLOCKS blocks finds the schedule of its (stream, kind)
// and, when the frame geometry matches the last one, dispatches in its order; every block writes its duration, and
// sched_order() (after the launch, same stream) sorts them into the next frame's order.  One schedule per stream:
// launches on one stream run in order, so the sort never overlaps a launch reading its order.
// Measured (r04_at, 1080p frames): the shaded C3 frame 0.4667 -> 0.3782 ms — its bent-ray waves (up to 250 us) start at
// once instead of mid-launch, and the launch packs to its work (span 363 us against 340 us of block time per wave
// slot).  Primary casts keep the default order (kinds 0 / 1 are not scheduled): their longest waves are already
// dispatched first (top tile rows), and the sorted order loses the neighbouring tiles' shared node reads — C3 0.1678 ->
// 0.1941 ms, C4 0.2314 -> 0.2569, C5 0.5078 -> 0.6209 when scheduled.
constexpr size_t kSchedMax = 16;  // schedules per tree (least recently used replaced)
// A schedule predicts a frame from the last one: a camera that turned more than kSchedTurn or moved more than kSchedMove
// voxels since runs the default order (and re-primes).  Measured (tools/shade_motion.py, r04_ax): a still view 0.462 ->
// 0.368 ms; 0.25 deg + 0.14 voxels per frame 0.400 -> 0.395; 2 deg per frame 0.292 -> 0.374 and a cut every frame
// 0.308 -> 0.358 when a stale order was used — a wrong order is worse than the default one.  A frame far from the last
// one is not sorted after either (the sort costs ~9 us): the schedule comes back one frame after the camera settles.
constexpr float kSchedTurnCos = 0.99996f;  // cos(0.5 deg)
// A still camera's order holds for the next frames too: a scheduled frame writes its durations and is sorted after only
// every kSchedEvery-th frame (the sort, one workgroup for ~9 us between two launches, is otherwise on every frame's path)
constexpr int32_t kSchedEvery = 4;
constexpr float kSchedMove = 1.0f;
struct SchedUse {  // a launch's schedule (sched_attach), by value: the tree's list may change under other threads
    uint32_t* base = nullptr;
    int64_t blocks = 0;
    int32_t kind = 0;
};
// `lock` (the tree's sched_mu) is taken here and stays held by the caller until the launch and its sort are queued
// (sched_order): the buffer handed out cannot be freed by another thread's eviction or resize before the work that uses
// it is on its stream (hipFree synchronises the device, which protects queued work only)
SchedUse sched_attach(const svo_tree* t, const svo_cast_desc* d, CastParams& P, int32_t kind, int64_t blocks, hipStream_t st,
                      std::unique_lock<std::mutex>& lock) {
    if (P.mode != MODE_FRAME || (P.flags & (SVO_CAST_NO_SCHEDULE | SVO_CAST_STATS)) || blocks <= SVO_SCHED_MIN_BLOCKS ||
        blocks > 0x7FFFFFFFll || blocks % kSchedGroup)
        return SchedUse{};
    const int64_t sig[7] = {P.width, P.height, P.n_frames, P.tile_row_start, P.tile_row_step, P.tile_lh, (int64_t)(P.flags & SVO_CAST_BOTTOM_FIRST)};
    lock = std::unique_lock<std::mutex>(t->sched_mu);
    svo_tree::Sched* s = nullptr;
    for (auto& e : t->scheds)
        if (e.stream == (void*)st && e.kind == kind) s = &e;
    if (!s) {
        if (t->scheds.size() >= kSchedMax) {
            auto lru = std::min_element(t->scheds.begin(), t->scheds.end(),
                                        [](const svo_tree::Sched& a, const svo_tree::Sched& b) { return a.last_use < b.last_use; });
            (void)hipFree(lru->d_buf);  // (synchronises the device: no launch still reads it)
            t->scheds.erase(lru);
        }
        t->scheds.push_back(svo_tree::Sched{(void*)st, kind, {0}, 0, nullptr, 0, false, 0, {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f},
                                            {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f}});
        s = &t->scheds.back();
    }
    s->last_use = ++t->sched_clock;
    if (s->blocks != blocks || !std::equal(sig, sig + 7, s->sig)) {
        if (s->blocks < blocks) {
            if (s->d_buf) (void)hipFree(s->d_buf);
            s->d_buf = nullptr;
            s->blocks = 0;
            if (hipMalloc(&s->d_buf, (size_t)blocks * 8) != hipSuccess) {  // (no schedule; the launch runs unscheduled)
                (void)hipGetLastError();
                s->d_buf = nullptr;
                return SchedUse{};
            }
        }
        s->blocks = blocks;
        std::copy(sig, sig + 7, s->sig);
        s->primed = false;
    }
    const float cam[6] = {P.frame_org[0], P.frame_org[1], P.frame_org[2], d->cam_dir[0], d->cam_dir[1], d->cam_dir[2]};
    const auto close = [&](const float* c) {
        const float dx = cam[0] - c[0], dy = cam[1] - c[1], dz = cam[2] - c[2];
        return dx * dx + dy * dy + dz * dz <= kSchedMove * kSchedMove && cam[3] * c[3] + cam[4] * c[4] + cam[5] * c[5] >= kSchedTurnCos;
    };
    const bool near_last = close(s->last_cam);            // (a frame far from the last one is not sorted after)
    const bool near_sorted = s->primed && close(s->cam);  // (the order is used only near the frame it was sorted from)
    std::copy(cam, cam + 6, s->last_cam);
    uint32_t* base = reinterpret_cast<uint32_t*>(s->d_buf);
    P.sched_order = near_sorted ? base : nullptr;
    if (!near_last) {  // (a moving camera: no sort after this frame; the first frame near it sorts for the next)
        P.sched_cost = nullptr;
        s->primed = false;
        return SchedUse{nullptr, blocks, kind};
    }
    // sorted after this frame: an order missing or sorted from a camera this one has drifted from, else every
    // kSchedEvery-th frame.  Only the frames sorted after write their durations, so the stored order is always the sort of
    // the stored durations (svo_tree_schedule)
    const bool sort = !near_sorted || ++s->since >= kSchedEvery;
    if (sort) {
        s->since = 0;
        std::copy(cam, cam + 6, s->cam);
    }
    P.sched_cost = sort ? base + blocks : nullptr;
    return SchedUse{sort ? base : nullptr, blocks, kind};
}
// after the launch of a scheduled frame: the next frame's order (the schedule counts as sorted once the sort is queued);
// called with sched_attach's lock still held
int sched_order(const svo_tree* t, const SchedUse& u, hipStream_t st) {
    if (!u.base) return SVO_OK;
    hipLaunchKernelGGL(k_sched_order, dim3(1), dim3(kSchedThreads), 0, st, u.base + u.blocks, u.base, (uint32_t)(u.blocks / kSchedGroup));
    HIP_TRY(hipGetLastError(), SVO_EDEVICE);
    for (auto& e : t->scheds)
        if (e.stream == (void*)st && e.kind == u.kind && e.d_buf == (void*)u.base && e.blocks == u.blocks) e.primed = true;
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
    if (t->d_pal) (void)hipFree(t->d_pal);
    if (t->d_pick) (void)hipFree(t->d_pick);
    if (t->d_ao_plan) (void)hipFree(t->d_ao_plan);
    if (t->d_ceil) (void)hipFree(t->d_ceil);
    if (t->d_ceilp) (void)hipFree(t->d_ceilp);
    if (t->d_ceilq) (void)hipFree(t->d_ceilq);
    t->d_ceil = t->d_ceilp = t->d_ceilq = nullptr;
    for (auto& e : t->scheds)
        if (e.d_buf) (void)hipFree(e.d_buf);
    t->scheds.clear();
    t->ceil_levels = 0;
    t->ceil_dev_n = 0;
    t->d_ao_plan = nullptr;
    t->ao_plan_steps = -1;
    (void)hipSetDevice(prev);
    t->d_nodes = t->d_mats = t->d_pick = t->d_pal = nullptr;
    t->dev_node_cap = t->dev_mat_cap = t->dev_pal_n = 0;
    t->device = -1;
    t->device_bytes = 0;
}

extern "C" void svo_tree_destroy(svo_tree* t) {
    if (!t) return;
    tree_release_device(t);
    delete t;
}

// The ceiling pairs of level j (its block's ceiling, low 16 bits; its level-(j + kCeilPairStep) block's, high, or the coarsest
// level's when the tree has fewer) over the blocks holding columns [x0, x1) x [z0, z1) — widened to whole parent blocks, whose change reaches
// every child's pair.  Returns per level the first and last row written (level j's rows of blocks, row-major [z][x]).
static void ceil_pairs(svo_tree* t, int32_t n, int64_t x0, int64_t z0, int64_t x1, int64_t z1, int64_t zr[kCeilMax][2]) {
    for (int32_t j = 0; j < n; j++) {
        const int64_t rows = (int64_t)1 << (2 * (t->levels - kCeilK0 - j));
        const int32_t up = std::min(j + kCeilPairStep, n - 1), sh = 2 * (up - j);
        const int32_t ush = 2 * (kCeilK0 + up), bsh = 2 * (kCeilK0 + j);
        const int64_t rows_up = rows >> sh;
        const int64_t bz0 = (z0 >> ush) << (ush - bsh), bz1 = std::min(rows, (((z1 - 1) >> ush) + 1) << (ush - bsh));
        const int64_t bx0 = (x0 >> ush) << (ush - bsh), bx1 = std::min(rows, (((x1 - 1) >> ush) + 1) << (ush - bsh));
        const int16_t* c = t->ceil_host.data();
        for (int64_t z = bz0; z < bz1; z++)
            for (int64_t x = bx0; x < bx1; x++)
                t->ceilp_host[t->ceil_off[j] + z * rows + x] = (uint32_t)(uint16_t)c[t->ceil_off[j] + z * rows + x] |
                                                                 ((uint32_t)(uint16_t)c[t->ceil_off[up] + (z >> sh) * rows_up + (x >> sh)] << 16);
        zr[j][0] = bz0;
        zr[j][1] = bz1;
    }
}

// The ceiling quads (svo_tree.d_ceilq) of the level-0 blocks holding columns [x0, x1) x [z0, z1), widened to whole blocks of
// the coarsest level (whose change reaches every level-0 block inside it).  Returns the first and last row written.
static void ceil_quads(svo_tree* t, int32_t n, int64_t x0, int64_t z0, int64_t x1, int64_t z1, int64_t zr[2]) {
    const int64_t rows = (int64_t)1 << (2 * (t->levels - kCeilK0));
    const int32_t tsh = 2 * (n - 1);  // the coarsest level's blocks, in level-0 blocks (log2)
    const int32_t bsh = 2 * kCeilK0 + tsh;
    const int64_t bz0 = (z0 >> bsh) << tsh, bz1 = std::min(rows, (((z1 - 1) >> bsh) + 1) << tsh);
    const int64_t bx0 = (x0 >> bsh) << tsh, bx1 = std::min(rows, (((x1 - 1) >> bsh) + 1) << tsh);
    const int16_t* c = t->ceil_host.data();
    for (int64_t z = bz0; z < bz1; z++)
        for (int64_t x = bx0; x < bx1; x++) {
            uint64_t q = 0;
            for (int32_t j = 0; j < kCeilMax; j++) {
                const int16_t v = j < n ? c[t->ceil_off[j] + (z >> (2 * j)) * (rows >> (2 * j)) + (x >> (2 * j))] : (int16_t)0x7FFF;
                q |= (uint64_t)(uint16_t)v << (16 * j);
            }
            t->ceilq_host[z * rows + x] = q;
        }
    zr[0] = bz0;
    zr[1] = bz1;
}

// the column ceilings of the host image (tree_ceilings), their pairs and quads, replacing the device copies (the device
// buffers are kept when their size is unchanged)
static int upload_ceilings(svo_tree* t) {
    int32_t n = 0;
    int64_t zr[kCeilMax][2];
    try {
        int64_t off[kCeilMax] = {0, 0, 0, 0};
        n = tree_ceilings(t, t->ceil_host, off);
        for (int j = 0; j < kCeilMax; j++) t->ceil_off[j] = t->ceilp_off[j] = off[j];
        t->ceilp_host.assign(t->ceil_host.size(), 0u);
        t->ceilq_host.clear();
        if (n > 0) {
            const int64_t e = (int64_t)1 << (2 * t->levels);
            ceil_pairs(t, n, 0, 0, e, e, zr);
            t->ceilq_host.assign((size_t)1 << (4 * (t->levels - kCeilK0)), 0ull);
            int64_t qr[2];
            ceil_quads(t, n, 0, 0, e, e, qr);
        }
    } catch (const std::bad_alloc&) {
        t->ceil_host.clear();
        t->ceilp_host.clear();
        t->ceilq_host.clear();
        n = -1;
    }
    t->ceil_dirty.clear();
    if (n <= 0 || (int64_t)t->ceil_host.size() != t->ceil_dev_n) {
        if (t->d_ceil) (void)hipFree(t->d_ceil);
        if (t->d_ceilp) (void)hipFree(t->d_ceilp);
        if (t->d_ceilq) (void)hipFree(t->d_ceilq);
        t->d_ceil = t->d_ceilp = t->d_ceilq = nullptr;
        t->ceil_dev_n = 0;
    }
    t->ceil_levels = 0;
    if (n < 0) SVO_FAIL(SVO_ENOMEM, "column ceilings: out of host memory");
    if (n == 0) return SVO_OK;
    const size_t m = t->ceil_host.size();
    if (!t->d_ceil) {
        HIP_TRY(hipMalloc(&t->d_ceil, m * sizeof(int16_t)), SVO_ENOMEM);
        HIP_TRY(hipMalloc(&t->d_ceilp, m * sizeof(uint32_t)), SVO_ENOMEM);
        HIP_TRY(hipMalloc(&t->d_ceilq, t->ceilq_host.size() * sizeof(uint64_t)), SVO_ENOMEM);
        t->ceil_dev_n = (int64_t)m;
    }
    HIP_TRY(hipMemcpy(t->d_ceil, t->ceil_host.data(), m * sizeof(int16_t), hipMemcpyHostToDevice), SVO_EDEVICE);
    HIP_TRY(hipMemcpy(t->d_ceilp, t->ceilp_host.data(), m * sizeof(uint32_t), hipMemcpyHostToDevice), SVO_EDEVICE);
    HIP_TRY(hipMemcpy(t->d_ceilq, t->ceilq_host.data(), t->ceilq_host.size() * sizeof(uint64_t), hipMemcpyHostToDevice), SVO_EDEVICE);
    t->ceil_levels = n;
    return SVO_OK;
}

// after edits: only the columns svo_tree_update touched are recomputed (tree walks restricted to them), and only the
// rows of the tables that changed travel, into the device buffers already there
static int sync_ceilings(svo_tree* t) {
    if (t->ceil_dirty.empty()) return SVO_OK;
    if (t->ceil_levels == 0 || !t->d_ceil) {
        t->ceil_dirty.clear();
        return SVO_OK;
    }
    const int32_t n = t->ceil_levels;
    std::vector<std::array<int64_t, 4>> rects;
    rects.swap(t->ceil_dirty);
    for (const auto& r : rects) {
        int64_t zr[kCeilMax][2], qr[2];
        try {
            ceilings_update_rect(t, t->ceil_host, t->ceil_off, n, r[0], r[1], r[2], r[3]);
            ceil_pairs(t, n, r[0], r[1], r[2], r[3], zr);
            ceil_quads(t, n, r[0], r[1], r[2], r[3], qr);
        } catch (const std::bad_alloc&) {
            SVO_FAIL(SVO_ENOMEM, "svo_tree_sync: column ceilings: out of host memory");
        }
        {
            const int64_t rows = (int64_t)1 << (2 * (t->levels - kCeilK0));
            const int64_t lo = qr[0] * rows, cnt = (qr[1] - qr[0]) * rows;
            if (cnt > 0)
                HIP_TRY(hipMemcpy(reinterpret_cast<uint64_t*>(t->d_ceilq) + lo, t->ceilq_host.data() + lo, cnt * sizeof(uint64_t),
                                  hipMemcpyHostToDevice), SVO_EDEVICE);
        }
        for (int32_t j = 0; j < n; j++) {
            const int64_t rows = (int64_t)1 << (2 * (t->levels - kCeilK0 - j));
            const int64_t lo = t->ceil_off[j] + zr[j][0] * rows, cnt = (zr[j][1] - zr[j][0]) * rows;
            if (cnt <= 0) continue;
            HIP_TRY(hipMemcpy(reinterpret_cast<int16_t*>(t->d_ceil) + lo, t->ceil_host.data() + lo, cnt * sizeof(int16_t),
                              hipMemcpyHostToDevice), SVO_EDEVICE);
            HIP_TRY(hipMemcpy(reinterpret_cast<uint32_t*>(t->d_ceilp) + lo, t->ceilp_host.data() + lo, cnt * sizeof(uint32_t),
                              hipMemcpyHostToDevice), SVO_EDEVICE);
        }
    }
    return SVO_OK;
}

static int upload_palette(svo_tree* t) {
    // palette colours (u64[n]) then flags (u32[n]) for the shading pass
    const size_t np = std::max<size_t>(t->palette.size(), 1);
    std::vector<uint8_t> pal(np * 12, 0);
    for (size_t i = 0; i < t->palette.size(); i++) {
        memcpy(&pal[i * 8], &t->palette[i].color, 8);
        memcpy(&pal[np * 8 + i * 4], &t->palette[i].flags, 4);
    }
    if (t->d_pal) (void)hipFree(t->d_pal);
    t->d_pal = nullptr;
    HIP_TRY(hipMalloc(&t->d_pal, pal.size()), SVO_ENOMEM);
    HIP_TRY(hipMemcpy(t->d_pal, pal.data(), pal.size(), hipMemcpyHostToDevice), SVO_EDEVICE);
    t->dev_pal_n = np;
    t->palette_dirty = false;
    return SVO_OK;
}

extern "C" int svo_upload(svo_tree* t, int32_t device) {
    if (!t) SVO_FAIL(SVO_EINVAL, "svo_upload: NULL tree");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev), SVO_EDEVICE);
    if (device < 0 || device >= ndev) SVO_FAIL(SVO_EDEVICE, "svo_upload: no such HIP device");
    tree_release_device(t);
    HIP_TRY(hipSetDevice(device), SVO_EDEVICE);
    // capacity for appended edit blocks (svo_tree_update / svo_tree_sync) without reallocation
    // (node and material indices are 32-bit: no room beyond 2^32 elements)
    const uint64_t ncap = std::min<uint64_t>(t->nodes.size() + t->nodes.size() / 8 + 65536, 1ull << 32);
    const uint64_t mcap = std::min<uint64_t>(t->mats.size() + t->mats.size() / 8 + 65536, 1ull << 32);
    const size_t nb = ncap * sizeof(Node), mb = mcap * sizeof(uint16_t);
    const size_t wb = kSideBytes;
    HIP_TRY(hipMalloc(&t->d_nodes, nb), SVO_ENOMEM);
    HIP_TRY(hipMalloc(&t->d_mats, mb), SVO_ENOMEM);
    HIP_TRY(hipMalloc(&t->d_pick, wb), SVO_ENOMEM);
    HIP_TRY(hipMemcpy(t->d_nodes, t->nodes.data(), t->nodes.size() * sizeof(Node), hipMemcpyHostToDevice), SVO_EDEVICE);
    if (!t->mats.empty()) HIP_TRY(hipMemcpy(t->d_mats, t->mats.data(), t->mats.size() * sizeof(uint16_t), hipMemcpyHostToDevice), SVO_EDEVICE);
    HIP_TRY(hipMemset(t->d_pick, 0, wb), SVO_EDEVICE);
    int rc = upload_palette(t);
    if (rc) return rc;
    t->device = device;
    t->device_bytes = nb + mb + wb + t->dev_pal_n * 12;
    t->dev_node_cap = ncap;
    t->dev_mat_cap = mcap;
    t->synced_nodes = t->nodes.size();
    t->dev_top_y = tree_top_y(t);
    t->synced_mats = t->mats.size();
    t->dirty_nodes.clear();
    t->full_upload = false;
    return upload_ceilings(t);
}

int svo::adopt_device(svo_tree* t, int32_t device, void* d_nodes, uint64_t node_cap, void* d_mats, uint64_t mat_cap) {
    tree_release_device(t);
    HIP_TRY(hipSetDevice(device), SVO_EDEVICE);
    const size_t wb = kSideBytes;
    t->d_nodes = d_nodes;
    t->d_mats = d_mats;
    HIP_TRY(hipMalloc(&t->d_pick, wb), SVO_ENOMEM);
    HIP_TRY(hipMemset(t->d_pick, 0, wb), SVO_EDEVICE);
    int rc = upload_palette(t);
    if (rc) return rc;
    t->device = device;
    t->device_bytes = node_cap * sizeof(Node) + mat_cap * sizeof(uint16_t) + wb + t->dev_pal_n * 12;
    t->dev_node_cap = node_cap;
    t->dev_mat_cap = mat_cap;
    t->synced_nodes = t->nodes.size();
    t->dev_top_y = tree_top_y(t);
    t->synced_mats = t->mats.size();
    t->dirty_nodes.clear();
    t->full_upload = false;
    return upload_ceilings(t);
}

// updateSsboData after edits (voxel_allocator.hpp:38-78): only the appended tail and the records
// rewritten in place travel; a rebuilt or outgrown tree is uploaded whole
extern "C" int svo_tree_sync(svo_tree* t) {
    if (!t) SVO_FAIL(SVO_EINVAL, "svo_tree_sync: NULL tree");
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, "svo_tree_sync: tree not uploaded (svo_upload)");
    if (t->full_upload || t->nodes.size() > t->dev_node_cap || t->mats.size() > t->dev_mat_cap) return svo_upload(t, t->device);
    if (t->nodes.size() == t->synced_nodes && t->mats.size() == t->synced_mats && t->dirty_nodes.empty() && !t->palette_dirty &&
        t->ceil_dirty.empty())
        return SVO_OK;  // nothing changed since the last upload / sync
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    // the records, ceilings and palette below are rewritten in place: every cast over the tree must be over first, on any
    // stream (null-stream copies do not wait for non-blocking streams; a frame reading lowered ceilings against old nodes
    // could skip blocks still stored).  As the reference's updateSsboData, this runs between frames.
    HIP_TRY(hipDeviceSynchronize(), SVO_EDEVICE);
    Node* dn = reinterpret_cast<Node*>(t->d_nodes);
    if (t->nodes.size() > t->synced_nodes)
        HIP_TRY(hipMemcpy(dn + t->synced_nodes, t->nodes.data() + t->synced_nodes, (t->nodes.size() - t->synced_nodes) * sizeof(Node),
                          hipMemcpyHostToDevice), SVO_EDEVICE);
    if (t->mats.size() > t->synced_mats)
        HIP_TRY(hipMemcpy(reinterpret_cast<uint16_t*>(t->d_mats) + t->synced_mats, t->mats.data() + t->synced_mats,
                          (t->mats.size() - t->synced_mats) * sizeof(uint16_t), hipMemcpyHostToDevice), SVO_EDEVICE);
    std::sort(t->dirty_nodes.begin(), t->dirty_nodes.end());
    for (size_t i = 0; i < t->dirty_nodes.size();) {  // runs of consecutive rewritten records
        size_t j = i + 1;
        while (j < t->dirty_nodes.size() && t->dirty_nodes[j] <= t->dirty_nodes[j - 1] + 1) j++;
        const uint32_t lo = t->dirty_nodes[i], hi = t->dirty_nodes[j - 1];
        HIP_TRY(hipMemcpy(dn + lo, t->nodes.data() + lo, (size_t)(hi - lo + 1) * sizeof(Node), hipMemcpyHostToDevice), SVO_EDEVICE);
        i = j;
    }
    if (t->palette_dirty) {
        int rc = upload_palette(t);
        if (rc) return rc;
    }
    t->dirty_nodes.clear();
    t->synced_nodes = t->nodes.size();
    t->dev_top_y = tree_top_y(t);
    t->synced_mats = t->mats.size();
    return sync_ceilings(t);
}

// ================================================================================================
// casting
// ================================================================================================
extern "C" int svo_shade_rays(const svo_tree* t, const svo_cast_desc* d, const svo_shade_desc* sd, float* rgba,
                              const svo_hits* o, void* stream) {
    if (!t || !d || !sd || !rgba) SVO_FAIL(SVO_EINVAL, "svo_shade_rays: NULL argument");
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, "svo_shade_rays: tree not uploaded (svo_upload)");
    if (t->view != SVO_VIEW_SOLID) SVO_FAIL(SVO_EINVAL, "svo_shade_rays: t must be a solid-view tree (the scene goes in svo_shade_desc.scene)");
    if (d->steps < 0 || sd->shadow_steps < 0) SVO_FAIL(SVO_EINVAL, "svo_shade_rays: negative step budget");
    if (d->ao_samples != 0) SVO_FAIL(SVO_EINVAL, "svo_shade_rays: AO is a separate pass (ao_samples must be 0)");
    if ((d->flags & (SVO_CAST_STATS | SVO_CAST_TIMELINE)) && !d->stats)
        SVO_FAIL(SVO_EINVAL, "svo_shade_rays: SVO_CAST_STATS / TIMELINE without a stats buffer");
    if (o && (!o->pos_steps || !o->t || !o->info)) SVO_FAIL(SVO_EINVAL, "svo_shade_rays: incomplete hit buffers");
    if (d->ray_dirs) {
        if (d->n_rays < 0) SVO_FAIL(SVO_EINVAL, "svo_shade_rays: negative ray count");
    } else if (d->width <= 0 || d->height <= 0 || d->tile_row_step <= 0 || d->tile_row_start < 0) {
        SVO_FAIL(SVO_EINVAL, "svo_shade_rays: bad frame geometry");
    }
    const svo_tree* sc = sd->scene ? sd->scene : t;
    if (sc->device != t->device) SVO_FAIL(SVO_ESTATE, "svo_shade_rays: scene tree not uploaded to the tree's device");
    if (sc->levels != t->levels) SVO_FAIL(SVO_EINVAL, "svo_shade_rays: scene and tree differ in levels");
    const svo_hits none = {nullptr, nullptr, nullptr, nullptr};
    CastParams P;
    int64_t n = 0;
    int rc = fill_params(sc, d, o ? o : &none, P, n);
    if (rc) return rc;
    set_ceilings(sc, d, P, kCeilShade);
    // shadow rays walk t: its own column ceilings (the scene's hold for the scene's voxels, which is t's world only when
    // both trees are synced to the same edits), and t's guard-trip counter (svo_tree_guard_trips counts launches over t)
    {
        CastParams S{};  // (set_ceilings leaves it untouched under SVO_CAST_NO_CEILINGS: compared zeroed)
        set_ceilings(t, d, S, kCeilShade);
        const bool same = S.ceil_levels == P.ceil_levels && S.ceil_sh[0] == P.ceil_sh[0] && S.ceil_sh[1] == P.ceil_sh[1];
        P.sceilp = same ? S.ceilp : nullptr;
        P.sceil_levels = same ? S.ceil_levels : 0;  // (shadow rays then walk the tree)
    }
    P.guard_trips = guard_word(t);
    P.snodes = reinterpret_cast<const Node*>(t->d_nodes);
    P.smats = reinterpret_cast<const uint16_t*>(t->d_mats);
    P.time = sd->time;
    P.top_scene = sc->dev_top_y;
    P.top_solid = t->dev_top_y;
    P.rgba = reinterpret_cast<float4*>(rgba);
    P.sun_dirs = (d->flags & SVO_CAST_NO_OCTANT) ? 0 : 1;  // (0: per-wave sign flags for the shadow rays as well)
    for (int k = 0; k < 3; k++) {
        P.sun[k] = sd->sun_dir[k];
        if (P.sun_dirs) P.sun_dirs += (sd->sun_dir[k] < 0.0f ? 1 : 0) << k;  // (dda_axis' step: -1 only below zero; -0.0, NaN: +)
        P.look[k] = sd->look_at[k];
    }
    P.look_valid = sd->look_at_valid != 0;
    if (P.look_valid && !sd->look_at_dev) {
        svo_block b;
        uint32_t mid = 0;
        rc = svo_tree_get_block(sc, sd->look_at[0], sd->look_at[1], sd->look_at[2], &b, &mid);
        if (rc) return rc;
        // (palette entry 0: no block).  The host image runs ahead of HBM between svo_tree_update and svo_tree_sync: with
        // edits not yet synced the device scene may still lack (or hold) that voxel, so it is taken as possibly empty
        // there — no shading ray escapes early then, and an escaped miss cannot lose the highlight
        const bool unsynced = sc->nodes.size() != sc->synced_nodes || !sc->dirty_nodes.empty() || sc->palette_dirty;
        P.look_empty = mid == 0u || unsynced;
    }
    P.look_dev = reinterpret_cast<const int32_t*>(sd->look_at_dev);
    P.shadow_steps = sd->shadow_steps;
    if (n == 0) return SVO_OK;
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    const int64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks * kBlock > 0xFFFFFFFFll) SVO_FAIL(SVO_ERANGE, "svo_shade_rays: too many rays for one launch");
    const bool wide = wide_nodes(t, d->flags) || wide_nodes(sc, d->flags);
    std::unique_lock<std::mutex> sched_lock;  // (held from here until the launch and the sort are queued)
    const SchedUse sch = sched_attach(t, d, P, 2, blocks, (hipStream_t)stream, sched_lock);
    if (P.flags & SVO_CAST_STATS) launch_cast<true, true, false, true>(wide, true, dim3((uint32_t)blocks), dim3(kBlock), (hipStream_t)stream, P);
    else if (P.flags & SVO_CAST_TIMELINE) launch_cast<false, true, false, true>(wide, true, dim3((uint32_t)blocks), dim3(kBlock), (hipStream_t)stream, P);
    else {
        // the straight trace runs on the camera's step octant (frame launches whose every pixel steps with it: frame_dirs;
        // shaded C3 0.3050 -> 0.2914 ms against generic sign flags, with the shadow rays' sun-octant instances given up
        // for it: profiles/r05/shade_split_ab.json); its segment bounds only when an origin needs them (0.2887 -> 0.2831)
        const int dirs = frame_dirs(P);
        frame_axes(P, dirs);
        launch_cast<false, false, false, true>(wide, need_seg(P), dim3((uint32_t)blocks), dim3(kBlock), (hipStream_t)stream, P, dirs);
    }
    HIP_TRY(hipGetLastError(), SVO_EDEVICE);
    return sched_order(t, sch, (hipStream_t)stream);
}

static int cast_launch(const svo_tree* t, const svo_cast_desc* d, const svo_hits* o, void* wire, void* stream);

extern "C" int svo_cast_rays(const svo_tree* t, const svo_cast_desc* d, const svo_hits* o, void* stream) {
    if (!t || !d || !o) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: NULL argument");
    if (!o->pos_steps || !o->t || !o->info) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: NULL output buffer");
    return cast_launch(t, d, o, nullptr, stream);
}

extern "C" int svo_cast_wire(const svo_tree* t, const svo_cast_desc* d, void* wire, uint8_t* ao, void* stream) {
    if (!t || !d || !wire) SVO_FAIL(SVO_EINVAL, "svo_cast_wire: NULL argument");
    if (d->flags & (SVO_CAST_STATS | SVO_CAST_TIMELINE)) SVO_FAIL(SVO_EINVAL, "svo_cast_wire: no diagnostics (svo_cast_rays has them)");
    WireParams Q;
    int rc = wire_params(t, d, "svo_cast_wire", Q);  // (the wire formats' limits)
    if (rc) return rc;
    const svo_hits o = {nullptr, nullptr, nullptr, ao};
    return cast_launch(t, d, &o, wire, stream);
}

static int cast_launch(const svo_tree* t, const svo_cast_desc* d, const svo_hits* o, void* wire, void* stream) {
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, "svo_cast_rays: tree not uploaded (svo_upload)");
    if (t->view != SVO_VIEW_SOLID) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: castRayFromCam semantics need a solid-view tree");
    if (d->steps < 0) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: negative step budget");
    if ((d->flags & (SVO_CAST_STATS | SVO_CAST_TIMELINE)) && !d->stats)
        SVO_FAIL(SVO_EINVAL, "svo_cast_rays: SVO_CAST_STATS / TIMELINE without a stats buffer");
    if (d->ao_samples < 0 || d->ao_samples > 64) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: ao_samples must be in [0, 64]");
    if (d->ao_samples > 0 && (!o->ao || d->ao_steps < 0)) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: AO needs an ao buffer and ao_steps >= 0");
    if (d->ray_dirs) {
        if (d->n_rays < 0) SVO_FAIL(SVO_EINVAL, "svo_cast_rays: negative ray count");
    } else if (d->width <= 0 || d->height <= 0 || d->tile_row_step <= 0 || d->tile_row_start < 0) {
        SVO_FAIL(SVO_EINVAL, "svo_cast_rays: bad frame geometry");
    }
    CastParams P;
    int64_t n = 0;
    int rc = fill_params(t, d, o, P, n);
    if (rc) return rc;
    P.wire = reinterpret_cast<uint32_t*>(wire);
    P.wire_compact = wire && wire_bytes_for(t, d) == 8;
    if (n == 0) return SVO_OK;
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    const int64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks * kBlock > 0xFFFFFFFFll) SVO_FAIL(SVO_ERANGE, "svo_cast_rays: too many rays for one launch");
    const dim3 grid((uint32_t)blocks), block(kBlock);
    hipStream_t st = (hipStream_t)stream;
    const bool wide = wide_nodes(t, d->flags), seg = need_seg(P);
    const int dirs = frame_dirs(P);
    frame_axes(P, dirs);
    const SchedUse sch = {};  // (primary casts: the default order; see sched_attach)
    if (P.ao_n > 0) {
        if (P.flags & SVO_CAST_STATS) launch_cast<true, true, true, false>(wide, seg, grid, block, st, P);
        else launch_cast<false, false, true, false>(wide, seg, grid, block, st, P, dirs);
    } else if (P.flags & SVO_CAST_STATS) {
        launch_cast<true, true, false, false>(wide, seg, grid, block, st, P);
    } else if (P.flags & SVO_CAST_TIMELINE) {
        launch_cast<false, true, false, false>(wide, seg, grid, block, st, P);
    } else {
        launch_cast<false, false, false, false>(wide, seg, grid, block, st, P, dirs);
    }
    HIP_TRY(hipGetLastError(), SVO_EDEVICE);
    return sched_order(t, sch, st);
}

namespace {
// one pick ray's hit record (int4 pos + steps, f32 t, u32 info at +0 / +16 / +20 of buf) on `stream`
int pick_launch(const svo_tree* t, const float pos[3], const float dir[3], int32_t steps, void* buf, hipStream_t stream, const char* fn) {
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, std::string(fn) + ": tree not uploaded (svo_upload)");
    if (t->view != SVO_VIEW_SOLID) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": castRayFromCam semantics need a solid-view tree");
    if (steps < 0) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": negative step budget");
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    CastParams P;
    memset(&P, 0, sizeof(P));
    P.nodes = reinterpret_cast<const Node*>(t->d_nodes);
    P.mats = reinterpret_cast<const uint16_t*>(t->d_mats);
    P.levels = t->levels;
    P.wmask = (1u << (2 * t->levels)) - 1u;
    P.mode = MODE_SINGLE;
    P.top_solid = t->dev_top_y;
    P.guard_trips = guard_word(t);
    P.steps = steps;
    for (int a = 0; a < 3; a++) {
        P.org[a] = pos[a];
        P.sdir[a] = dir[a];
    }
    P.pos = reinterpret_cast<int32_t*>(buf);
    P.t = reinterpret_cast<float*>(reinterpret_cast<char*>(buf) + 16);
    P.info = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(buf) + 20);
    launch_cast<false, false, false, false>(wide_nodes(t, 0), need_seg(P), dim3(1), dim3(kBlock), stream, P);
    HIP_TRY(hipGetLastError(), SVO_EDEVICE);
    return SVO_OK;
}

// the hit record at r (pick_launch) rewritten in place as a RayResult {pos, lastPos, steps} (ray_caster.hpp:6-10)
__global__ __launch_bounds__(64) void k_pick_result(int32_t* r) {
    if (threadIdx.x != 0) return;
    const int32_t x = r[0], y = r[1], z = r[2], st = r[3];
    const uint32_t info = (uint32_t)r[5];
    int32_t last[3] = {x, y, z};
    const uint32_t axis = (info >> AXIS_SHIFT) & 3u;
    if (axis < 3u) last[axis] -= (info & NEG_BIT) ? -1 : 1;
    r[0] = x;
    r[1] = y;
    r[2] = z;
    r[3] = last[0];
    r[4] = last[1];
    r[5] = last[2];
    r[6] = st;
}
}  // namespace

extern "C" int svo_cast_ray_from_cam_async(const svo_tree* t, const float pos[3], const float dir[3], int32_t steps, svo_ray_result* d_result,
                                           void* stream) {
    if (!t || !pos || !dir || !d_result) SVO_FAIL(SVO_EINVAL, "svo_cast_ray_from_cam_async: NULL argument");
    if (reinterpret_cast<uintptr_t>(d_result) & 15u) SVO_FAIL(SVO_EINVAL, "svo_cast_ray_from_cam_async: d_result not 16-byte aligned");
    int rc = pick_launch(t, pos, dir, steps, d_result, (hipStream_t)stream, "svo_cast_ray_from_cam_async");
    if (rc) return rc;
    hipLaunchKernelGGL(k_pick_result, dim3(1), dim3(64), 0, (hipStream_t)stream, reinterpret_cast<int32_t*>(d_result));
    HIP_TRY(hipGetLastError(), SVO_EDEVICE);
    return SVO_OK;
}

extern "C" int svo_cast_ray_from_cam(const svo_tree* t, const float pos[3], const float dir[3], int32_t steps, svo_ray_result* out,
                                     svo_block* block) {
    if (!t || !pos || !dir || !out) SVO_FAIL(SVO_EINVAL, "svo_cast_ray_from_cam: NULL argument");
    // the tree's own result record: no allocation per pick (the reference casts one every frame, main.cpp:81);
    // one synchronous pick at a time per tree
    std::lock_guard<std::mutex> lock(t->pick_mu);
    void* buf = reinterpret_cast<char*>(t->d_pick) + kSidePick;
    int rc = pick_launch(t, pos, dir, steps, buf, nullptr, "svo_cast_ray_from_cam");
    if (rc) return rc;
    unsigned char host[32];
    hipError_t e = hipMemcpy(host, buf, 32, hipMemcpyDeviceToHost);
    if (e != hipSuccess) SVO_FAIL(SVO_EDEVICE, std::string("svo_cast_ray_from_cam: ") + hipGetErrorString(e));
    int32_t p4[4];
    uint32_t info;
    memcpy(p4, host, 16);
    memcpy(&info, host + 20, 4);
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

extern "C" int svo_tree_device_ceilings(const svo_tree* t, int16_t* ceil, uint32_t* pairs, int64_t cap, int32_t* levels, int64_t* n) {
    if (!t || !levels || !n) SVO_FAIL(SVO_EINVAL, "svo_tree_device_ceilings: NULL argument");
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, "svo_tree_device_ceilings: tree not uploaded (svo_upload)");
    *levels = t->ceil_levels;
    *n = t->ceil_levels > 0 ? t->ceil_dev_n : 0;
    if ((ceil || pairs) && cap < *n) SVO_FAIL(SVO_ERANGE, "svo_tree_device_ceilings: buffer too small");
    if (*n == 0) return SVO_OK;
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    if (ceil) HIP_TRY(hipMemcpy(ceil, t->d_ceil, *n * sizeof(int16_t), hipMemcpyDeviceToHost), SVO_EDEVICE);
    if (pairs) HIP_TRY(hipMemcpy(pairs, t->d_ceilp, *n * sizeof(uint32_t), hipMemcpyDeviceToHost), SVO_EDEVICE);
    return SVO_OK;
}

extern "C" int svo_tree_device_ceiling_quads(const svo_tree* t, uint64_t* quads, int64_t cap, int64_t* n) {
    if (!t || !n) SVO_FAIL(SVO_EINVAL, "svo_tree_device_ceiling_quads: NULL argument");
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, "svo_tree_device_ceiling_quads: tree not uploaded (svo_upload)");
    *n = t->ceil_levels > 0 && t->d_ceilq ? (int64_t)t->ceilq_host.size() : 0;
    if (quads && cap < *n) SVO_FAIL(SVO_ERANGE, "svo_tree_device_ceiling_quads: buffer too small");
    if (*n == 0 || !quads) return SVO_OK;
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    HIP_TRY(hipMemcpy(quads, t->d_ceilq, *n * sizeof(uint64_t), hipMemcpyDeviceToHost), SVO_EDEVICE);
    return SVO_OK;
}

extern "C" int svo_tree_schedule(const svo_tree* t, void* stream, int32_t kind, uint32_t* order, uint32_t* cost, int64_t cap, int64_t* n) {
    if (!t || !n) SVO_FAIL(SVO_EINVAL, "svo_tree_schedule: NULL argument");
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, "svo_tree_schedule: tree not uploaded (svo_upload)");
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream), SVO_EDEVICE);
    std::lock_guard<std::mutex> lock(t->sched_mu);
    *n = 0;
    for (const auto& e : t->scheds) {
        if (e.stream != stream || e.kind != kind || !e.primed) continue;
        *n = e.blocks;
        if ((order || cost) && cap < *n) SVO_FAIL(SVO_ERANGE, "svo_tree_schedule: buffer too small");
        const uint32_t* base = reinterpret_cast<const uint32_t*>(e.d_buf);
        if (order) HIP_TRY(hipMemcpy(order, base, *n / kSchedGroup * sizeof(uint32_t), hipMemcpyDeviceToHost), SVO_EDEVICE);
        if (cost) HIP_TRY(hipMemcpy(cost, base + e.blocks, *n * sizeof(uint32_t), hipMemcpyDeviceToHost), SVO_EDEVICE);
    }
    return SVO_OK;
}

extern "C" int svo_ceiling_layout(int32_t* k0, int32_t* pair_step) {
    if (k0) *k0 = kCeilK0;
    if (pair_step) *pair_step = kCeilPairStep;
    return SVO_OK;
}

extern "C" int svo_tree_guard_trips(const svo_tree* t, uint64_t* trips, int32_t reset) {
    if (!t || !trips) SVO_FAIL(SVO_EINVAL, "svo_tree_guard_trips: NULL argument");
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, "svo_tree_guard_trips: tree not uploaded (svo_upload)");
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    uint32_t v = 0;
    // every launch over t finished, on whatever stream (a null-stream copy does not wait for non-blocking streams)
    HIP_TRY(hipDeviceSynchronize(), SVO_EDEVICE);
    HIP_TRY(hipMemcpy(&v, guard_word(t), sizeof(v), hipMemcpyDeviceToHost), SVO_EDEVICE);
    if (reset) HIP_TRY(hipMemset(guard_word(t), 0, sizeof(v)), SVO_EDEVICE);
    *trips = v;
    return SVO_OK;
}

extern "C" int svo_sync(void* stream) {
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream), SVO_EDEVICE);
    return SVO_OK;
}

// ================================================================================================
// wire records of the tile-row gather (svo_wire.h: 8 B compact, 12 B general)
// ================================================================================================
// 8-B records for frame descs from integral / half-integral camera positions (every crossing sum exact)
int32_t svo::wire_bytes_for(const svo_tree* t, const svo_cast_desc* d) {
    if (d->ray_dirs || d->steps > 32767 || t->palette.size() > 4096) return 12;
    const int32_t nf = d->n_frames > 1 ? d->n_frames : 1;
    for (int32_t f = 0; f < nf; f++)
        for (int k = 0; k < 3; k++) {
            const float o = nf > 1 ? d->frame_origins[3 * f + k] : d->origin[k];
            if (!(2.0f * o == __builtin_truncf(2.0f * o) && __builtin_fabsf(o) < 1073741824.0f)) return 12;
        }
    return 8;
}

int svo::wire_params(const svo_tree* t, const svo_cast_desc* d, const char* fn, WireParams& Q) {
    if (!t || !d) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": NULL argument");
    if (t->device < 0) SVO_FAIL(SVO_ESTATE, std::string(fn) + ": tree not uploaded (svo_upload)");
    if (d->steps < 0 || d->steps > 32767) SVO_FAIL(SVO_ERANGE, std::string(fn) + ": the wire formats need steps <= 32767");
    if (t->palette.size() > 4096) SVO_FAIL(SVO_ERANGE, std::string(fn) + ": the wire formats need at most 4096 materials");
    memset(&Q, 0, sizeof(Q));
    int64_t n = 0;
    int rc = svo_cast_count(d, &n);
    if (rc) return rc;
    if (n >= ((int64_t)1 << 32) - 256) SVO_FAIL(SVO_ERANGE, std::string(fn) + ": too many records for one launch");
    Q.n = n;
    Q.steps = d->steps;
    Q.explicit_mode = d->ray_dirs != nullptr;
    Q.compact = wire_bytes_for(t, d) == 8;
    const int32_t nf = (!Q.explicit_mode && d->n_frames > 1) ? d->n_frames : 1;
    Q.frame_records = std::max<int64_t>(1, n / nf);
    for (int32_t f = 0; f < nf; f++)
        for (int k = 0; k < 3; k++) Q.frame_org[3 * f + k] = nf > 1 ? d->frame_origins[3 * f + k] : d->origin[k];
    Q.rorg = Q.explicit_mode ? d->ray_origins : nullptr;
    if (!Q.explicit_mode) {
        raygen_init(Q.rg, d->cam_dir, d->ppx, d->ppy, d->width, d->height);
        Q.width = d->width;
        Q.tile_row_start = d->tile_row_start;
        Q.tile_row_step = d->tile_row_step;
        Q.frame_pixels = (int64_t)d->width * d->height;
    }
    return SVO_OK;
}

namespace {

__global__ __launch_bounds__(256) void k_hits_pack(const WireParams Q) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= Q.n) return;
    float o[3];
    wire_origin(Q, i, o);
    const int4 ps = reinterpret_cast<const int4*>(Q.pos)[i];
    wire_put(Q.wire, Q.compact != 0, i, o, ps.x, ps.y, ps.z, Q.t[i], Q.info[i]);
}

__global__ __launch_bounds__(256) void k_hits_unpack(const WireParams Q) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= Q.n) return;
    wire_get(Q, i);
}

int hits_check(const svo_hits* h, const char* fn) {
    if (!h || !h->pos_steps || !h->t || !h->info) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": NULL hit buffer");
    return SVO_OK;
}

}  // namespace

extern "C" int svo_wire_bytes(const svo_tree* t, const svo_cast_desc* d, int32_t* bytes) {
    if (!t || !d || !bytes) SVO_FAIL(SVO_EINVAL, "svo_wire_bytes: NULL argument");
    *bytes = wire_bytes_for(t, d);
    return SVO_OK;
}

extern "C" int svo_hits_pack(const svo_tree* t, const svo_cast_desc* d, const svo_hits* hits, void* wire, void* stream) {
    WireParams Q;
    int rc = wire_params(t, d, "svo_hits_pack", Q);
    if (!rc) rc = hits_check(hits, "svo_hits_pack");
    if (rc) return rc;
    if (!wire) SVO_FAIL(SVO_EINVAL, "svo_hits_pack: NULL wire buffer");
    Q.pos = hits->pos_steps;
    Q.t = hits->t;
    Q.info = hits->info;
    Q.wire = reinterpret_cast<uint32_t*>(wire);
    if (Q.n == 0) return SVO_OK;
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    hipLaunchKernelGGL(k_hits_pack, dim3((uint32_t)((Q.n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, Q);
    HIP_TRY(hipGetLastError(), SVO_EDEVICE);
    return SVO_OK;
}

// unpack into record order (scatter = 0) or into the whole frames at pixel positions (scatter = 1)
static int wire_decode(const svo_tree* t, const svo_cast_desc* d, const void* wire, const uint8_t* ao, const svo_hits* hits, void* stream,
                       int32_t scatter, const char* fn) {
    WireParams Q;
    int rc = wire_params(t, d, fn, Q);
    if (!rc) rc = hits_check(hits, fn);
    if (rc) return rc;
    if (!wire) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": NULL wire buffer");
    if (scatter && Q.explicit_mode) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": explicit rays have no pixels to scatter to");
    if (ao && !hits->ao) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": AO counts without an ao buffer");
    Q.wire = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(wire));
    Q.pos = hits->pos_steps;
    Q.t = hits->t;
    Q.info = hits->info;
    Q.ao_in = ao;
    Q.ao_out = ao ? hits->ao : nullptr;
    Q.scatter = scatter;
    if (Q.n == 0) return SVO_OK;
    HIP_TRY(hipSetDevice(t->device), SVO_EDEVICE);
    hipLaunchKernelGGL(k_hits_unpack, dim3((uint32_t)((Q.n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, Q);
    HIP_TRY(hipGetLastError(), SVO_EDEVICE);
    return SVO_OK;
}

extern "C" int svo_hits_unpack(const svo_tree* t, const svo_cast_desc* d, const void* wire, const svo_hits* hits, void* stream) {
    return wire_decode(t, d, wire, nullptr, hits, stream, 0, "svo_hits_unpack");
}

extern "C" int svo_wire_scatter(const svo_tree* t, const svo_cast_desc* d, const void* wire, const uint8_t* ao, const svo_hits* frames,
                                void* stream) {
    return wire_decode(t, d, wire, ao, frames, stream, 1, "svo_wire_scatter");
}
