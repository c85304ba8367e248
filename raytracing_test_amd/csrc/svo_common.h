// svo_common.h — definitions shared by the host builder (svo_world.cpp) and the gfx950 kernels
// (svo_cast.hip).  Everything arithmetic here is compiled with -ffp-contract=off on both sides and
// rounds identically on x86-64 and gfx950: float divisions and square roots go through double
// precision and are rounded once to float (double rounding is innocuous for +,-,*,/,sqrt when the
// wide format has >= 2p+2 bits: 53 >= 50), so no result depends on a compiler's fp32 div/sqrt mode.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define SVO_HD __host__ __device__ __forceinline__
#define SVO_HOST __host__ static inline
#else
#define SVO_HD static inline
#define SVO_HOST static inline
#endif

namespace svo {

// ------------------------------------------------------------------------------------------------
// Linearised tree node, 16 B (the reference's node is 16 B too: src/voxel_data/types.hpp:29-47, but
// its children live in 256 B pointer arrays; here children are contiguous in breadth-first order
// and addressed by popcount of a 64-bit child mask — the variant the reference sketches at
// tetrahexa_tree.cpp:144-145).
//   kind INTERIOR: mask bit i = child i (index z<<4 | y<<2 | x) holds a solid voxel;
//                  ref = node index of the first child; child i = ref + popcount(mask & (2^i - 1))
//   kind BRICK   : a 4^3 region at depth levels-1; mask bit v = voxel v is solid;
//                  info & UNIFORM -> every solid voxel has material info>>16,
//                  else material of voxel v = mats[ref + popcount(mask & (2^v - 1))]
//   kind SOLID   : the whole region is solid with material info>>16 (mask = ~0)
// The root is node 0; an empty world is an INTERIOR root with mask 0.
// ------------------------------------------------------------------------------------------------
struct alignas(16) Node {
    uint64_t mask;
    uint32_t ref;
    uint32_t info;
};
static_assert(sizeof(Node) == 16, "node must be 16 B");

enum : uint32_t { K_INTERIOR = 0u, K_BRICK = 1u, K_SOLID = 2u, K_KIND_MASK = 3u, K_UNIFORM = 4u };

SVO_HD uint32_t node_kind(uint32_t info) { return info & K_KIND_MASK; }
SVO_HD uint32_t node_material(uint32_t info) { return info >> 16; }

// child slot of wrapped voxel coordinates at bit offset `sh` (tetrahexa_tree.cpp:127-129)
SVO_HD uint32_t child_slot(uint32_t x, uint32_t y, uint32_t z, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
    // three bit-field extracts and two shift-ors (v_lshl_or_b32); the or-of-shifts form compiles to
    // two shifts and an or3
    uint32_t r;
    asm("v_lshl_or_b32 %0, %1, 2, %2" : "=v"(r) : "v"(__builtin_amdgcn_ubfe(z, sh, 2u)), "v"(__builtin_amdgcn_ubfe(y, sh, 2u)));
    asm("v_lshl_or_b32 %0, %1, 2, %2" : "=v"(r) : "v"(r), "v"(__builtin_amdgcn_ubfe(x, sh, 2u)));
    return r;
#else
    return (((z >> sh) & 3u) << 4) | (((y >> sh) & 3u) << 2) | ((x >> sh) & 3u);
#endif
}

// Frame mode: log2 of a wavefront's pixel rows (3: 8x8, 2: 16x4 — the default —, 1: 32x2) from
// svo_cast_desc.flags (SVO_CAST_TILE_8X8 = 256, SVO_CAST_TILE_32X2 = 512), and wavefronts per
// 8-pixel tile row
SVO_HD int32_t frame_wave_lh(int32_t flags) { return (flags & 512) ? 1 : ((flags & 256) ? 3 : 2); }
SVO_HD int32_t frame_wave_cols(int32_t width, int32_t lh) { return ((width + (1 << (6 - lh)) - 1) >> (6 - lh)) << (3 - lh); }
// Small launches (a strong-scaling shard: a few thousand waves, fewer than the GPU's wave slots) are bound by their
// longest waves, the far field's: their first-dispatched (top) tile rows are cast by half footprints, 32 rays per
// wavefront (lanes 32-63 idle), which serialise fewer diverging paths per wave.  As many rows as keep the launch within
// kHalfWaves wavefronts; a launch already above it (a whole frame: 32400 at 1080p) keeps whole footprints, which share
// their node reads (half footprints made full frames 3-12 % slower).  Measured, one GPU, the slowest 1/8 shard
// (tools/shard_curve.py): C3 128.6 -> 114.2 us, C5 125.2 -> 113.6 us (ranks within 1.12x), 1/4 C3 128.3 -> 112.4
// (profiles/r05/shard_half_footprints.json).  None bottom-first.
constexpr int32_t kHalfWaves = 20480;
SVO_HD int32_t frame_half_rows(int32_t rows, int32_t flags, int32_t lh, int32_t cols, int32_t frames) {
    if ((flags & 4) || lh < 1 || rows <= 0 || cols <= 0) return 0;  // (4: SVO_CAST_BOTTOM_FIRST)
    const int64_t k = (int64_t)kHalfWaves / ((int64_t)cols * (frames > 1 ? frames : 1)) - rows;
    return k <= 0 ? 0 : (int32_t)(k < rows ? k : rows);
}

// hit-record info word (see include/svo_rt.h)
enum : uint32_t { HIT_BIT = 1u << 31, AXIS_SHIFT = 16, NEG_BIT = 1u << 18, MAT_MASK = 0xFFFFu };
constexpr uint32_t kNoHit = 0xFFFFFFFFu;  // trace: material id while no voxel was hit

// ------------------------------------------------------------------------------------------------
// Correctly rounded f32 division / sqrt via f64 (see header note)
// ------------------------------------------------------------------------------------------------
SVO_HD float div_rn(float a, float b) { return (float)((double)a / (double)b); }
#if defined(__HIP_DEVICE_COMPILE__)
// HIP's f32 square root is correctly rounded (v_sqrt_f32 and an FMA residual check of the two
// neighbouring floats), so it equals the double square root rounded once, at f32 cost
SVO_HD float sqrt_rn(float a) { return __builtin_sqrtf(a); }
#else
SVO_HD float sqrt_rn(float a) { return (float)__builtin_sqrt((double)a); }
#endif

// 1/x correctly rounded.  Device: for |x| in [2^-126, 2^126) (x and 1/x normal), v_rcp_f32 and
// one FMA Newton step give exactly div_rn(1, x) — checked for every such float, both signs
// (tools/micro/rcp_check.hip); other x (zero, subnormal, huge, inf, NaN) take the division.
#if defined(__HIP_DEVICE_COMPILE__)
SVO_HD float rcp_rn(float x) {
    const float ax = __builtin_fabsf(x);
    if (ax >= 0x1p-126f && ax < 0x1p126f) {
        const float r0 = __builtin_amdgcn_rcpf(x);
        return __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
    }
    return div_rn(1.0f, x);
}
#else
SVO_HD float rcp_rn(float x) { return div_rn(1.0f, x); }
#endif

// sin of a float through double precision, rounded once to float (the shading pass's liquid wobble,
// low_res.frag:226): Cody-Waite reduction by pi/2 (k * PIO2_HI is exact for |k| < 2^20), Taylor
// polynomials of sin / cos on [-pi/4, pi/4] (truncation < 3e-14), the quadrant's sign and function.
// The same double operations on host and device (no contraction), so both round alike; far cheaper
// in registers than a libm sin.
SVO_HD float sin_f32(float xf) {
    // (beyond the exact reduction range the argument is first taken modulo fl(2 pi) — an exact remainder
    // on host and device alike — so the value stays a bounded sine of an equal argument on both)
    const double x0 = (double)xf;
    const double x = __builtin_fabs(x0) < 524288.0 ? x0 : __builtin_fmod(x0, 6.283185307179586);
    const double k = __builtin_rint(x * 0.63661977236758134308);
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
    const double kq = k - 4.0 * __builtin_floor(k * 0.25);
    const int q = (kq >= 0.0 && kq < 4.0) ? (int)kq : 0;
    const double v = (q & 1) ? cs : sn;
    return (float)((q & 2) ? -v : v);
}

// glm::cross (x.y*y.z - y.y*x.z, x.z*y.x - y.z*x.x, x.x*y.y - y.x*x.y)
SVO_HD void cross3(const float a[3], const float b[3], float o[3]) {
    o[0] = a[1] * b[2] - b[1] * a[2];
    o[1] = a[2] * b[0] - b[2] * a[0];
    o[2] = a[0] * b[1] - b[0] * a[1];
}

// glm::normalize: v * (1 / sqrt((x*x + y*y) + z*z))
SVO_HD void normalize3(const float v[3], float o[3]) {
    float d = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
    float r = rcp_rn(sqrt_rn(d));
    o[0] = v[0] * r;
    o[1] = v[1] * r;
    o[2] = v[2] * r;
}

// Per-pixel primary ray (src/shaders/low_res.frag:264-288): FragCoord = gl_FragCoord.xy * (1/res)
// with the pixel centre at +0.5 and rows counted from the bottom; `left` is cross(dir, up)
// unnormalised (the shader's projection_plane_left), `up' = cross(dir, left)`;
// d = normalize((dir + left * -(ppx * (fx - 0.5))) + (up' * (-fy + 0.5)) * ppy).
struct RayGen {
    float c[3], l[3], u[3];
    float ppx, ppy, rw, rh;
};

SVO_HD void raygen_init(RayGen& g, const float cam[3], float ppx, float ppy, int32_t w, int32_t h) {
    const float up[3] = {0.0f, 1.0f, 0.0f};
    g.c[0] = cam[0];
    g.c[1] = cam[1];
    g.c[2] = cam[2];
    cross3(g.c, up, g.l);
    cross3(g.c, g.l, g.u);
    g.ppx = ppx;
    g.ppy = ppy;
    g.rw = div_rn(1.0f, (float)w);
    g.rh = div_rn(1.0f, (float)h);
}

SVO_HD void raygen_pixel(const RayGen& g, int32_t px, int32_t py, float d[3]) {
    float fx = ((float)px + 0.5f) * g.rw;
    float fy = ((float)py + 0.5f) * g.rh;
    float sl = -(g.ppx * (fx - 0.5f));
    float su = -fy + 0.5f;
    float v[3];
    for (int a = 0; a < 3; a++) {
        float lt = g.l[a] * sl;
        float ut = (g.u[a] * su) * g.ppy;
        v[a] = (g.c[a] + lt) + ut;
    }
    normalize3(v, d);
}

// ------------------------------------------------------------------------------------------------
// DDA set-up of RAY_CASTER::buildRay + castRayFromCam (src/ray_caster.cpp:19-66): step = sign with
// -0.0 / NaN -> +1; delta = 1/dir as a FLOAT division widened to double; absDelta = glm::abs;
// round = trunc(origin); exact = origin - 1 on negative-step axes;
// deltaPos = absDelta - (exact - round) * delta  (the product is exact in double).
// ------------------------------------------------------------------------------------------------
struct Dda1 {
    int32_t step;
    int32_t cell;
    double adelta;
    double dpos;
};

SVO_HD Dda1 dda_axis(float o, float d) {
    Dda1 r;
    r.step = d < 0.0f ? -1 : 1;
    double delta = (double)rcp_rn(d);
    r.adelta = delta >= 0.0 ? delta : -delta;
    r.cell = (int32_t)__builtin_truncf(o);
    double exact = (double)o;
    if (r.step < 0) exact -= 1.0;
    r.dpos = r.adelta - (exact - (double)r.cell) * delta;
    return r;
}

// gen_hemisphare_distrib.py:4-13 — Fibonacci-spiral hemisphere, polar span 0.85, evaluated in
// double and rounded to float; (x, y, pole).  Host only (libm).
SVO_HOST void hemisphere_table(int32_t n, float* out) {
    const double pi = 3.141592653589793;
    for (int32_t i = 0; i < n; i++) {
        const double idx = (double)i + 0.5;
        const double phi = __builtin_acos(1.0 - idx * 0.85 / (double)n);
        const double theta = pi * (1.0 + __builtin_sqrt(5.0)) * idx;
        out[3 * i + 0] = (float)(__builtin_cos(theta) * __builtin_sin(phi));
        out[3 * i + 1] = (float)(__builtin_sin(theta) * __builtin_sin(phi));
        out[3 * i + 2] = (float)__builtin_cos(phi);
    }
}

// AO direction: the table entry's pole turned to axis `ax` (sign sg), its first two components to
// the next two axes cyclically.  Exact (a permutation and a sign).
SVO_HD void ao_dir(const float h[3], uint32_t ax, int32_t sg, float d[3]) {
    const float p = sg > 0 ? h[2] : -h[2];
    d[0] = ax == 0u ? p : (ax == 1u ? h[1] : h[0]);
    d[1] = ax == 1u ? p : (ax == 2u ? h[1] : h[0]);
    d[2] = ax == 2u ? p : (ax == 0u ? h[1] : h[0]);
}

}  // namespace svo
