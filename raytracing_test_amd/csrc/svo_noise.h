// svo_noise.h — 2D OpenSimplex noise and the genWorld column model, host + device.
//
// Algorithm: KdotJPG's OpenSimplex (2014) 2D, as vendored by the reference in
// include/OpenSimplexNoise.cpp:52-208,2518-2523 (a 2019 C++ port), used by src/world_gen.cpp:15-22
// with seeds 42 / 64 / 100.  Restated here as "four lattice-vertex contributions": the two fixed
// vertices (1,0) and (0,1), the near corner ((0,0) or (1,1)) and one extra vertex chosen by the
// region test.  Each contribution rounds exactly as the reference's expression does, so heights
// are bit-identical (tests pin this against the reference's own compiled noise, oracle/_ref).
#pragma once

#include <math.h>
#include <stdint.h>

#include "svo_common.h"

namespace svo {

struct Simplex2 {
    uint8_t perm[256];
};

// Noise(int64_t seed): three LCG warm-up steps, then a Fisher-Yates shuffle of 0..255 driven by
// the same LCG (multiplier 6364136223846793005, increment 1442695040888963407).
static inline void simplex2_seed(Simplex2& s, int64_t seed) {
    uint8_t pool[256];
    for (int i = 0; i < 256; i++) pool[i] = (uint8_t)i;
    const uint64_t mul = 6364136223846793005ull, inc = 1442695040888963407ull;
    uint64_t st = (uint64_t)seed;
    for (int k = 0; k < 3; k++) st = st * mul + inc;
    for (int i = 255; i >= 0; i--) {
        st = st * mul + inc;
        int64_t q = (int64_t)(st + 31u) % (int64_t)(i + 1);
        int r = (int)(q < 0 ? q + (i + 1) : q);
        s.perm[i] = pool[r];
        pool[r] = pool[i];
    }
}

// 8 gradient directions (the reference's 16-entry table read as pairs)
SVO_HD double simplex2_grad(const uint8_t* perm, int32_t xv, int32_t yv, double dx, double dy) {
    const int8_t gx[8] = {5, 2, -5, -2, 5, 2, -5, -2};
    const int8_t gy[8] = {2, 5, 2, 5, -2, -5, -2, -5};
    uint32_t h = (uint32_t)perm[((int32_t)perm[xv & 0xFF] + yv) & 0xFF] & 0x0Eu;
    return (double)gx[h >> 1] * dx + (double)gy[h >> 1] * dy;
}

// contribution of lattice vertex (xsb+i, ysb+j): offsets (dx0 - i) - (i+j)*SQUISH, attenuation
// (2 - dx^2) - dy^2, weight attn^4
SVO_HD double simplex2_vertex(const uint8_t* perm, int32_t xsb, int32_t ysb, int32_t i, int32_t j, double dx0, double dy0) {
    const double SQUISH = 0.366025403784439;
    double k = (double)(i + j) * SQUISH;
    double dx = (dx0 - (double)i) - k;
    double dy = (dy0 - (double)j) - k;
    double a = (2.0 - dx * dx) - dy * dy;
    if (!(a > 0.0)) return 0.0;
    a = a * a;
    return (a * a) * simplex2_grad(perm, xsb + i, ysb + j, dx, dy);
}

SVO_HD double simplex2_eval(const uint8_t* perm, double x, double y) {
    const double STRETCH = -0.211324865405187, SQUISH = 0.366025403784439;
    double so = (x + y) * STRETCH;
    double xs = x + so, ys = y + so;
    int32_t xsb = (int32_t)floor(xs), ysb = (int32_t)floor(ys);
    double sq = (double)(xsb + ysb) * SQUISH;
    double xin = xs - (double)xsb, yin = ys - (double)ysb;
    double dx0 = x - ((double)xsb + sq), dy0 = y - ((double)ysb + sq);
    double s = xin + yin;
    // near corner (c, c) and extra vertex (ei, ej)
    int32_t c, ei, ej;
    if (s <= 1.0) {
        c = 0;
        double z = 1.0 - s;
        if (z > xin || z > yin) {
            ei = xin > yin ? 1 : -1;
            ej = -ei;
        } else {
            ei = 1;
            ej = 1;
        }
    } else {
        c = 1;
        double z = 2.0 - s;
        if (z < xin || z < yin) {
            ei = xin > yin ? 2 : 0;
            ej = 2 - ei;
        } else {
            ei = 0;
            ej = 0;
        }
    }
    // summation order of the reference: (1,0), (0,1), near corner, extra vertex; a vertex whose
    // attenuation is <= 0 adds +0.0, which leaves every partial sum unchanged (it starts at +0)
    double v = 0.0;
    v += simplex2_vertex(perm, xsb, ysb, 1, 0, dx0, dy0);
    v += simplex2_vertex(perm, xsb, ysb, 0, 1, dx0, dy0);
    v += simplex2_vertex(perm, xsb, ysb, c, c, dx0, dy0);
    v += simplex2_vertex(perm, xsb, ysb, ei, ej, dx0, dy0);
    return v / 47.0;
}

// genWorld's column top (world_gen.cpp:22)
SVO_HD int32_t terrain_height(const uint8_t* p42, const uint8_t* p64, const uint8_t* p100, int32_t x, int32_t z) {
    double a = round(simplex2_eval(p42, x * 0.005, z * 0.005) * 30);
    double b = round(simplex2_eval(p64, x * 0.05, z * 0.05) * 5);
    double c = round(simplex2_eval(p100, x * 0.1, z * 0.1) * 3);
    return (int32_t)(a + b + c + 32);
}

// Column materials for top h (world_gen.cpp:24-39): water (h, 20] when h < 20; the top voxel dirt
// under water, grass otherwise; three dirt voxels below while y > 0; stone down to y = 1.
enum : uint32_t { TM_AIR = 0, TM_WATER = 1, TM_GRASS = 2, TM_DIRT = 3, TM_STONE = 4 };

SVO_HD uint32_t terrain_material(int32_t h, int32_t y) {
    if (y == h) return h < 20 ? TM_DIRT : TM_GRASS;
    if (y > h) return (h < 20 && y <= 20) ? TM_WATER : TM_AIR;
    if (y <= 0) return TM_AIR;
    return y >= h - 3 ? TM_DIRT : TM_STONE;
}

// Tree views (include/svo_rt.h SVO_VIEW_*): the solid view stores what castRayFromCam hits (water is
// empty, ray_caster.cpp:82); the full view stores every block genWorld puts, water included.
// Stored top of a column: its top voxel, or the water surface (y = 20) over a top below 20.
SVO_HD int32_t terrain_top(int32_t h, int32_t view) { return (view && h < 20) ? 20 : h; }

// Class of an aligned region of rows y0..y1 over a full footprint of columns whose tops span
// [hmin, hmax]: `empty`, a uniform material id_of[terrain material], or `mixed`.  Emptiness comes
// first (callers treat a non-empty region over a partial footprint as mixed).
SVO_HD bool terrain_region_empty(int32_t view, int32_t hmax, int32_t y0, int32_t y1) {
    return y1 < 1 || y0 > terrain_top(hmax, view);
}
SVO_HD uint32_t terrain_region_class(const uint32_t id_of[5], int32_t view, int32_t hmin, int32_t hmax, int32_t y0, int32_t y1,
                                     uint32_t empty, uint32_t mixed) {
    if (terrain_region_empty(view, hmax, y0, y1)) return empty;
    if (y0 >= 1 && y1 <= hmin - 4) return id_of[TM_STONE];
    if (view && y0 > hmax && y1 <= 20) return id_of[TM_WATER];  // above every top, below the surface
    if (hmin != hmax) return mixed;  // dirt / grass runs are < 4 voxels unless all columns agree
    const int32_t h = hmin;
    const uint32_t c0 = id_of[terrain_material(h, y0)];
    const int32_t cand[5] = {1, h - 3, h, h + 1, 21};  // where a column's material can change
    for (int i = 0; i < 5; i++) {
        const int32_t b = cand[i];
        if (b > y0 && b <= y1 && id_of[terrain_material(h, b)] != id_of[terrain_material(h, b - 1)]) return mixed;
    }
    return c0;
}

}  // namespace svo
