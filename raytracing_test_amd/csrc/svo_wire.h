// svo_wire.h — the wire formats of hit records (include/svo_rt.h) for the tile-row gather: encoding (the
// cast kernel's fused output, svo_hits_pack) and decoding (svo_hits_unpack, svo_wire_scatter, the
// exchange's receive side), shared by svo_cast.hip and svo_exchange.hip.
//
//   12 B (any desc):  int16 dx, dy, dz = pos - trunc(origin) | u16 hit << 15 | axis << 13 | (step < 0) << 12 |
//                     material (12 bits) | f32 t
//   8 B (compact):    u64 n_x | n_y << 15 | n_z << 30 | hit << 45 | axis << 46 | material << 48, where n_k is
//                     the number of DDA steps the ray took on axis k (15 bits each).
//
// The compact form is used for frame descs whose every camera position is integral or half-integral
// (|o| < 2^30), with budgets up to 32767 and at most 4096 palette entries.  The receiver knows each
// record's pixel, so it regenerates the ray (raygen_pixel, dda_axis, the same code the kernel runs) and
// recovers the step signs, the position (cell + s n), the steps left (a hit: steps - n_x - n_y - n_z) and
// t.  From such origins deltaPos starts at a, 0, a/2, 3a/2 or -a/2 and every crossing sum the DDA takes is
// exact (svo_cast.hip, lin_origin), so after n steps on the last axis its deltaPos is fma(n, a, T0) —
// the double the kernel holds — and t = that - a (an infinite absDelta keeps it as is: inf or NaN, as
// the kernel's recovery does).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/svo_rt.h"
#include "svo_common.h"

namespace svo {

struct WireParams {
    int64_t n;              // records
    int64_t frame_records;  // records of one frame of the source shard
    int32_t compact;        // 8-B records (else 12 B)
    int32_t explicit_mode, steps;
    RayGen rg;              // compact records: the frame's ray generation
    int32_t width, tile_row_start, tile_row_step;  // the source shard's tile rows
    int32_t scatter;        // decode into whole frames at pixel positions (frame k at k * frame_pixels)
    int64_t frame_pixels;   // width * height
    float frame_org[3 * SVO_MAX_FRAMES];
    const float* rorg;      // explicit rays: per-ray origins (or null: frame_org[0..2])
    int32_t* pos;
    float* t;
    uint32_t* info;
    uint32_t* wire;
    const uint8_t* ao_in;   // decode: AO counts in record order, copied alongside (or null)
    uint8_t* ao_out;
};

// the frame of frame record i: 32-bit division (a launch holds fewer than 2^32 records: wire_params; a 64-bit
// division is a long instruction sequence on the GPU, and the decode ran two of them per record)
__device__ __forceinline__ uint32_t wire_frame(const WireParams& Q, int64_t i) {
    return (uint32_t)i / (uint32_t)Q.frame_records;
}

// the origin record i's ray started from
__device__ __forceinline__ void wire_origin(const WireParams& Q, int64_t i, float o[3]) {
    if (Q.explicit_mode && Q.rorg) {
#pragma unroll
        for (int k = 0; k < 3; k++) o[k] = Q.rorg[3 * i + k];
    } else {
        const uint32_t f = Q.explicit_mode ? 0u : wire_frame(Q, i);
#pragma unroll
        for (int k = 0; k < 3; k++) o[k] = Q.frame_org[3 * f + k];
    }
}

// frame and pixel of frame record i (svo_cast_rays' record order over the shard's tile rows)
__device__ __forceinline__ void wire_pixel(const WireParams& Q, int64_t i, int64_t& f, int32_t& px, int32_t& py) {
    const uint32_t fu = wire_frame(Q, i);
    f = fu;
    const uint32_t j = (uint32_t)i - fu * (uint32_t)Q.frame_records;
    const uint32_t lr = j / (uint32_t)Q.width;
    px = (int32_t)(j - lr * (uint32_t)Q.width);
    py = (int32_t)(((int64_t)Q.tile_row_start + (int64_t)(lr >> 3) * Q.tile_row_step) * 8 + (lr & 7u));
}

// one record from a ray's result (its origin o): 8 or 12 B at wire record i
__device__ __forceinline__ void wire_put(uint32_t* wire, bool compact, int64_t i, const float o[3], int32_t x, int32_t y, int32_t z,
                                         float t, uint32_t inf) {
    const int32_t cx = (int32_t)__builtin_truncf(o[0]), cy = (int32_t)__builtin_truncf(o[1]), cz = (int32_t)__builtin_truncf(o[2]);
    if (compact) {
        const uint32_t nx = (uint32_t)abs(x - cx), ny = (uint32_t)abs(y - cy), nz = (uint32_t)abs(z - cz);
        uint2 w;
        w.x = nx | (ny << 15) | (nz << 30);
        w.y = (nz >> 2) | ((inf >> 31) << 13) | (((inf >> AXIS_SHIFT) & 3u) << 14) | ((inf & 0xFFFu) << 16);
        reinterpret_cast<uint2*>(wire)[i] = w;
    } else {
        const uint32_t i16 = ((inf >> 31) << 15) | (((inf >> AXIS_SHIFT) & 3u) << 13) | (((inf & NEG_BIT) ? 1u : 0u) << 12) | (inf & 0xFFFu);
        const uint32_t dx = (uint32_t)(x - cx) & 0xFFFFu, dy = (uint32_t)(y - cy) & 0xFFFFu, dz = (uint32_t)(z - cz) & 0xFFFFu;
        uint32_t* w = wire + 3 * i;
        w[0] = dx | (dy << 16);
        w[1] = dz | (i16 << 16);
        w[2] = __float_as_uint(t);
    }
}

// record i back into a hit record (at record i, or at its pixel of the whole frames with Q.scatter)
__device__ __forceinline__ void wire_get(const WireParams& Q, int64_t i) {
    float o[3];
    int64_t out = i;
    int32_t px = 0, py = 0;
    if (!Q.explicit_mode) {
        int64_t f;
        wire_pixel(Q, i, f, px, py);
#pragma unroll
        for (int k = 0; k < 3; k++) o[k] = Q.frame_org[3 * f + k];
        if (Q.scatter) out = f * Q.frame_pixels + (int64_t)py * Q.width + px;
    } else {
        wire_origin(Q, i, o);
    }
    int4 ps;
    float t;
    uint32_t info;
    if (Q.compact) {
        const uint2 w = reinterpret_cast<const uint2*>(Q.wire)[i];
        const uint32_t n[3] = {w.x & 0x7FFFu, (w.x >> 15) & 0x7FFFu, (w.x >> 30) | ((w.y & 0x1FFFu) << 2)};
        const bool hit = ((w.y >> 13) & 1u) != 0u;
        const uint32_t axis = (w.y >> 14) & 3u;
        float d[3];
        raygen_pixel(Q.rg, px, py, d);
        int32_t p[3];
        double tl = 0.0;
        bool neg = false;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const Dda1 ax = dda_axis(o[k], d[k]);
            p[k] = ax.cell + ax.step * (int32_t)n[k];
            if (axis == (uint32_t)k) {
                const double T = __builtin_fma((double)n[k], ax.adelta, ax.dpos);  // deltaPos after the n steps (exact sums)
                tl = __builtin_isinf(ax.adelta) ? T : T - ax.adelta;
                neg = ax.step < 0;
            }
        }
        ps = make_int4(p[0], p[1], p[2], hit ? Q.steps - (int32_t)(n[0] + n[1] + n[2]) : 0);
        t = (float)tl;
        info = (hit ? HIT_BIT : 0u) | (axis << AXIS_SHIFT) | (neg ? NEG_BIT : 0u) | (w.y >> 16);
    } else {
        const uint32_t* w = Q.wire + 3 * i;
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
        const int32_t dx = (int32_t)(int16_t)(w0 & 0xFFFFu), dy = (int32_t)(int16_t)(w0 >> 16), dz = (int32_t)(int16_t)(w1 & 0xFFFFu);
        const uint32_t i16 = w1 >> 16;
        const bool hit = (i16 >> 15) != 0u;
        // one voxel per DDA step on one axis: a hit used |dx| + |dy| + |dz| steps, a miss all of them
        const int32_t left = hit ? Q.steps - (abs(dx) + abs(dy) + abs(dz)) : 0;
        ps = make_int4((int32_t)__builtin_truncf(o[0]) + dx, (int32_t)__builtin_truncf(o[1]) + dy, (int32_t)__builtin_truncf(o[2]) + dz, left);
        t = __uint_as_float(w2);
        info = (hit ? HIT_BIT : 0u) | (((i16 >> 13) & 3u) << AXIS_SHIFT) | (((i16 >> 12) & 1u) ? NEG_BIT : 0u) | (i16 & 0xFFFu);
    }
    reinterpret_cast<int4*>(Q.pos)[out] = ps;
    Q.t[out] = t;
    Q.info[out] = info;
    if (Q.ao_out) Q.ao_out[out] = Q.ao_in[i];
}

// host: the wire record size of a desc's records (8: compact, 12) and the decode / encode parameters
int32_t wire_bytes_for(const svo_tree* t, const svo_cast_desc* d);
int wire_params(const svo_tree* t, const svo_cast_desc* d, const char* fn, WireParams& Q);

}  // namespace svo
