// svo_exchange.hip — the multi-GPU frame exchange of libsvo_rt: frames are sharded by
// interleaved 8-pixel tile rows (row r -> rank r mod N), every rank casts its rows of every frame, and
// each frame's shards are gathered over RCCL (xGMI) to the rank that displays it, where they are
// unpacked into a whole frame.  The reference is single-GPU (src/main.cpp:107, one fullscreen draw);
// this is the north_star's "RCCL gather of the per-tile hit buffers".
//
// Transport: RCCL point-to-point inside one group (ncclGroupStart / ncclSend / ncclRecv /
// ncclGroupEnd) — one frame to one rank is a gather, N frames to N ranks an all-to-all, and either is
// one group call whose traffic spreads over every rank's links (xGMI is point to point: a gather of
// N frames into rank 0 would put all of it on rank 0's links).  Records travel in the 12-B wire format
// of svo_hits_pack (+1 B of AO count).  The local shard goes through RCCL as well (a send to self), so
// a single-rank exchange runs the whole path.
//
// RCCL is bound at run time (dlopen "librccl.so.1"): inside a process that already holds an RCCL
// (e.g. torch's), that library instance is reused, so communicators the caller made there can be
// wrapped; libsvo_rt itself does not depend on RCCL until an exchange is created.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/svo_rt.h"
#include "svo_hip.h"
#include "svo_internal.h"

using namespace svo;

namespace {

struct Rccl {
    bool ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*CommUserRank)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            R.err = std::string("cannot load librccl.so.1: ") + dlerror();
            return;
        }
        bool all = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn) {
                all = false;
                R.err = std::string("librccl.so.1 lacks ") + name;
            }
        };
        sym(R.GetUniqueId, "ncclGetUniqueId");
        sym(R.CommInitRank, "ncclCommInitRank");
        sym(R.CommDestroy, "ncclCommDestroy");
        sym(R.CommCount, "ncclCommCount");
        sym(R.CommUserRank, "ncclCommUserRank");
        sym(R.GroupStart, "ncclGroupStart");
        sym(R.GroupEnd, "ncclGroupEnd");
        sym(R.Send, "ncclSend");
        sym(R.Recv, "ncclRecv");
        sym(R.GetErrorString, "ncclGetErrorString");
        R.ok = all;
    });
    return R;
}

#define NCCL_TRY(expr)                                                                                         \
    do {                                                                                                       \
        ncclResult_t r_ = (expr);                                                                              \
        if (r_ != ncclSuccess) SVO_FAIL(SVO_EDEVICE, std::string(#expr " failed: ") + rccl().GetErrorString(r_)); \
    } while (0)

// One shard's wire records (and AO counts) -> their pixels of a whole frame.  Shard record i (rank r
// of N, local row lr = i / W, column px = i % W) is pixel row (r + (lr / 8) * N) * 8 + lr % 8.
struct ScatterParams {
    const uint32_t* wire;
    const uint8_t* ao_in;
    int64_t n;
    int32_t width, rank, nranks, steps;
    int32_t cell[3];  // trunc(frame origin)
    int32_t* pos;
    float* t;
    uint32_t* info;
    uint8_t* ao_out;
};

__global__ __launch_bounds__(256) void k_scatter_unpack(const ScatterParams Q) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= Q.n) return;
    const int64_t lr = i / Q.width, px = i - lr * Q.width;
    const int64_t py = ((int64_t)Q.rank + (lr >> 3) * Q.nranks) * 8 + (lr & 7);
    const int64_t o = py * Q.width + px;
    const uint32_t* w = Q.wire + 3 * i;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    const int32_t dx = (int32_t)(int16_t)(w0 & 0xFFFFu), dy = (int32_t)(int16_t)(w0 >> 16), dz = (int32_t)(int16_t)(w1 & 0xFFFFu);
    const uint32_t i16 = w1 >> 16;
    const bool hit = (i16 >> 15) != 0u;
    // (svo_hits_unpack's reconstruction: one voxel per DDA step on one axis)
    const int32_t left = hit ? Q.steps - (abs(dx) + abs(dy) + abs(dz)) : 0;
    reinterpret_cast<int4*>(Q.pos)[o] = make_int4(Q.cell[0] + dx, Q.cell[1] + dy, Q.cell[2] + dz, left);
    Q.t[o] = __uint_as_float(w2);
    Q.info[o] = (hit ? HIT_BIT : 0u) | (((i16 >> 13) & 3u) << AXIS_SHIFT) | (((i16 >> 12) & 1u) ? NEG_BIT : 0u) | (i16 & 0xFFFu);
    if (Q.ao_out) Q.ao_out[o] = Q.ao_in[i];
}

// records of one frame in the shard of `rank` (svo_cast_count's rows x width)
int64_t shard_records(int32_t width, int32_t height, int32_t rank, int32_t nranks) {
    const int32_t tile_rows = (height + 7) / 8;
    int64_t rows = 0;
    for (int32_t r = rank; r < tile_rows; r += nranks) rows += std::min(8, height - r * 8);
    return rows * width;
}

}  // namespace

struct svo_exchange {
    ncclComm_t comm = nullptr;
    bool owns_comm = false;
    int32_t rank = 0, nranks = 1, device = 0;
    void* send = nullptr;
    size_t send_bytes = 0;
    void* recv = nullptr;
    size_t recv_bytes = 0;
};

static int grow(void** p, size_t* cap, size_t need) {
    if (need <= *cap) return SVO_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc(p, need), SVO_ENOMEM);
    *cap = need;
    return SVO_OK;
}

extern "C" int svo_nccl_unique_id(void* out) {
    if (!out) SVO_FAIL(SVO_EINVAL, "svo_nccl_unique_id: NULL argument");
    Rccl& R = rccl();
    if (!R.ok) SVO_FAIL(SVO_EDEVICE, "svo_nccl_unique_id: " + R.err);
    ncclUniqueId id;
    NCCL_TRY(R.GetUniqueId(&id));
    memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return SVO_OK;
}

extern "C" int svo_exchange_create(int32_t nranks, int32_t rank, const void* unique_id, int32_t device, svo_exchange** out) {
    if (!out || !unique_id) SVO_FAIL(SVO_EINVAL, "svo_exchange_create: NULL argument");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) SVO_FAIL(SVO_EINVAL, "svo_exchange_create: rank outside [0, nranks)");
    Rccl& R = rccl();
    if (!R.ok) SVO_FAIL(SVO_EDEVICE, "svo_exchange_create: " + R.err);
    HIP_TRY(hipSetDevice(device), SVO_EDEVICE);
    ncclUniqueId id;
    memcpy(id.internal, unique_id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t comm = nullptr;
    NCCL_TRY(R.CommInitRank(&comm, nranks, id, rank));
    svo_exchange* x = new (std::nothrow) svo_exchange();
    if (!x) {
        (void)R.CommDestroy(comm);
        SVO_FAIL(SVO_ENOMEM, "svo_exchange_create: out of memory");
    }
    x->comm = comm;
    x->owns_comm = true;
    x->rank = rank;
    x->nranks = nranks;
    x->device = device;
    *out = x;
    return SVO_OK;
}

extern "C" int svo_exchange_wrap(void* nccl_comm, int32_t device, svo_exchange** out) {
    if (!out || !nccl_comm) SVO_FAIL(SVO_EINVAL, "svo_exchange_wrap: NULL argument");
    *out = nullptr;
    Rccl& R = rccl();
    if (!R.ok) SVO_FAIL(SVO_EDEVICE, "svo_exchange_wrap: " + R.err);
    int n = 0, r = 0;
    NCCL_TRY(R.CommCount((ncclComm_t)nccl_comm, &n));
    NCCL_TRY(R.CommUserRank((ncclComm_t)nccl_comm, &r));
    svo_exchange* x = new (std::nothrow) svo_exchange();
    if (!x) SVO_FAIL(SVO_ENOMEM, "svo_exchange_wrap: out of memory");
    x->comm = (ncclComm_t)nccl_comm;
    x->rank = r;
    x->nranks = n;
    x->device = device;
    *out = x;
    return SVO_OK;
}

extern "C" void svo_exchange_destroy(svo_exchange* x) {
    if (!x) return;
    (void)hipSetDevice(x->device);
    if (x->send) (void)hipFree(x->send);
    if (x->recv) (void)hipFree(x->recv);
    if (x->owns_comm && x->comm && rccl().ok) (void)rccl().CommDestroy(x->comm);
    delete x;
}

extern "C" int svo_exchange_info(const svo_exchange* x, int32_t* rank, int32_t* nranks) {
    if (!x) SVO_FAIL(SVO_EINVAL, "svo_exchange_info: NULL exchange");
    if (rank) *rank = x->rank;
    if (nranks) *nranks = x->nranks;
    return SVO_OK;
}

extern "C" int svo_exchange_frames(svo_exchange* x, const svo_tree* t, const svo_cast_desc* d, const svo_hits* mine,
                                   const svo_hits* frames_out, void* stream) {
    if (!x || !t || !d || !mine) SVO_FAIL(SVO_EINVAL, "svo_exchange_frames: NULL argument");
    if (d->ray_dirs) SVO_FAIL(SVO_EINVAL, "svo_exchange_frames: frame-mode descs only");
    if (d->tile_row_start != x->rank || d->tile_row_step != x->nranks)
        SVO_FAIL(SVO_EINVAL, "svo_exchange_frames: desc is not this rank's shard (tile_row_start = rank, tile_row_step = nranks)");
    const int32_t nf = d->n_frames > 1 ? d->n_frames : 1;
    const int32_t N = x->nranks, me = x->rank;
    const bool ao = d->ao_samples > 0;
    if (ao && !mine->ao) SVO_FAIL(SVO_EINVAL, "svo_exchange_frames: AO counts requested without an ao buffer");
    const int32_t n_own = nf > me ? (nf - me + N - 1) / N : 0;  // frames me, me + N, ...
    if (n_own > 0 && (!frames_out || !frames_out->pos_steps || !frames_out->t || !frames_out->info || (ao && !frames_out->ao)))
        SVO_FAIL(SVO_EINVAL, "svo_exchange_frames: this rank displays frames but frames_out is incomplete");
    const int64_t frame = (int64_t)d->width * d->height;
    std::vector<int64_t> cnt(N), off(N + 1, 0);
    for (int32_t r = 0; r < N; r++) {
        cnt[r] = shard_records(d->width, d->height, r, N);
        off[r + 1] = off[r] + cnt[r];
    }
    const int64_t n_mine = cnt[me];
    HIP_TRY(hipSetDevice(x->device), SVO_EDEVICE);
    hipStream_t st = (hipStream_t)stream;
    // my records of every frame, packed: frame f's at f * n_mine
    int rc = grow(&x->send, &x->send_bytes, std::max<size_t>(16, (size_t)(n_mine * nf) * SVO_WIRE_BYTES));
    if (!rc) rc = grow(&x->recv, &x->recv_bytes, std::max<size_t>(16, (size_t)(n_own * frame) * (SVO_WIRE_BYTES + (ao ? 1 : 0))));
    if (rc) return rc;
    rc = svo_hits_pack(t, d, mine, x->send, stream);
    if (rc) return rc;
    uint8_t* sw = reinterpret_cast<uint8_t*>(x->send);
    uint8_t* rw = reinterpret_cast<uint8_t*>(x->recv);
    uint8_t* rao = rw + (size_t)(n_own * frame) * SVO_WIRE_BYTES;  // AO counts after the records
    Rccl& R = rccl();
    NCCL_TRY(R.GroupStart());
    for (int32_t f = 0; f < nf && n_mine > 0; f++) {
        const int32_t owner = f % N;
        NCCL_TRY(R.Send(sw + (size_t)(f * n_mine) * SVO_WIRE_BYTES, (size_t)n_mine * SVO_WIRE_BYTES, ncclUint8, owner, x->comm, st));
        if (ao) NCCL_TRY(R.Send(mine->ao + (size_t)(f * n_mine), (size_t)n_mine, ncclUint8, owner, x->comm, st));
    }
    for (int32_t k = 0; k < n_own; k++)
        for (int32_t r = 0; r < N; r++) {
            if (cnt[r] == 0) continue;
            const size_t base = (size_t)(k * frame + off[r]);
            NCCL_TRY(R.Recv(rw + base * SVO_WIRE_BYTES, (size_t)cnt[r] * SVO_WIRE_BYTES, ncclUint8, r, x->comm, st));
            if (ao) NCCL_TRY(R.Recv(rao + base, (size_t)cnt[r], ncclUint8, r, x->comm, st));
        }
    NCCL_TRY(R.GroupEnd());
    // unpack every received shard into its pixels of the frame
    for (int32_t k = 0; k < n_own; k++) {
        const int32_t f = me + k * N;
        const float* org = nf > 1 ? d->frame_origins + 3 * f : d->origin;
        for (int32_t r = 0; r < N; r++) {
            if (cnt[r] == 0) continue;
            ScatterParams Q;
            memset(&Q, 0, sizeof(Q));
            const size_t base = (size_t)(k * frame + off[r]);
            Q.wire = reinterpret_cast<const uint32_t*>(rw + base * SVO_WIRE_BYTES);
            Q.ao_in = ao ? rao + base : nullptr;
            Q.n = cnt[r];
            Q.width = d->width;
            Q.rank = r;
            Q.nranks = N;
            Q.steps = d->steps;
            for (int a = 0; a < 3; a++) Q.cell[a] = (int32_t)truncf(org[a]);
            Q.pos = frames_out->pos_steps + 4 * (size_t)(k * frame);
            Q.t = frames_out->t + (size_t)(k * frame);
            Q.info = frames_out->info + (size_t)(k * frame);
            Q.ao_out = ao ? frames_out->ao + (size_t)(k * frame) : nullptr;
            hipLaunchKernelGGL(k_scatter_unpack, dim3((uint32_t)((Q.n + 255) / 256)), dim3(256), 0, st, Q);
            HIP_TRY(hipGetLastError(), SVO_EDEVICE);
        }
    }
    return SVO_OK;
}
