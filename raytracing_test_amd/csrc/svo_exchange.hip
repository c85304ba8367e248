// svo_exchange.hip — the multi-GPU frame exchange of libsvo_rt: frames are sharded by
// interleaved 8-pixel tile rows (row r -> rank r mod N), every rank casts its rows of every frame, and
// each frame's shards are gathered over RCCL (xGMI) to the rank that displays it, where they are
// unpacked into a whole frame.  The reference is single-GPU (src/main.cpp:107, one fullscreen draw);
// this is the north_star's "RCCL gather of the per-tile hit buffers".
//
// Transport: RCCL point-to-point inside one group (ncclGroupStart / ncclSend / ncclRecv /
// ncclGroupEnd) — one frame to one rank is a gather, N frames to N ranks an all-to-all, and either is
// one group call whose traffic spreads over every rank's links (xGMI is point to point: a gather of
// N frames into rank 0 would put all of it on rank 0's links).  Records travel in the wire formats of
// svo_wire.h — 8 B for frames from integral / half-integral camera positions, else 12 B — (+1 B of AO
// count).  The local shard never travels: the display rank decodes it straight from its own wire buffer.
// svo_exchange_wire takes the wire records the cast kernel wrote itself (svo_cast_wire: no hit records,
// no pack pass); svo_exchange_frames packs given hit records first.
//
// RCCL is bound at run time (dlopen "librccl.so.1"): inside a process that already holds an RCCL
// (e.g. torch's), that library instance is reused, so communicators the caller made there can be
// wrapped; libsvo_rt itself does not depend on RCCL until an exchange is created.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/svo_rt.h"
#include "svo_hip.h"
#include "svo_internal.h"
#include "svo_wire.h"

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
    ncclResult_t (*CommCuDevice)(const ncclComm_t, int*) = nullptr;
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
        // SVO_RCCL_LIB: another library with RCCL's entry points instead (tests/standin/rccl_standin.cpp, the test-only
        // stand-in that runs the N > 1 pairing with several ranks on one GPU), loaded locally so it shadows nothing
        // — only with the second, explicit opt-in SVO_RCCL_STANDIN=1, so a stray SVO_RCCL_LIB cannot turn a measurement
        // into a stand-in run; bench.py reports such runs as "transport": "standin"
        const char* over = getenv("SVO_RCCL_LIB");
        const char* opt = getenv("SVO_RCCL_STANDIN");
        const bool o = over && *over && opt && strcmp(opt, "1") == 0;
        if (over && *over && !o) {
            R.err = "SVO_RCCL_LIB is set without SVO_RCCL_STANDIN=1 (the test-only RCCL stand-in needs both)";
            return;
        }
        const std::string name = o ? over : "librccl.so.1";
        void* h = dlopen(name.c_str(), o ? (RTLD_NOW | RTLD_LOCAL) : (RTLD_NOW | RTLD_GLOBAL));
        if (!h) {
            R.err = "cannot load " + name + ": " + dlerror();
            return;
        }
        bool all = true;
        auto sym = [&](auto& fn, const char* sname) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, sname));
            if (!fn) {
                all = false;
                R.err = name + " lacks " + sname;
            }
        };
        sym(R.GetUniqueId, "ncclGetUniqueId");
        sym(R.CommInitRank, "ncclCommInitRank");
        sym(R.CommDestroy, "ncclCommDestroy");
        sym(R.CommCount, "ncclCommCount");
        sym(R.CommUserRank, "ncclCommUserRank");
        sym(R.CommCuDevice, "ncclCommCuDevice");
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

// One source shard's wire records (and AO counts) -> their pixels of the whole frames (svo_wire.h).  1024-thread blocks:
// the decode runs beside the next step's cast, whose one-wave blocks hold every wave slot until its tail; a 16-wave block
// starts only where a CU has emptied, i.e. in that tail (forced 1-rank exchange at C3: 0.1844 -> 0.1822 ms per step
// against 256-thread blocks; 64-thread blocks, which take slots as soon as single cast waves retire: 0.1900)
__global__ __launch_bounds__(1024) void k_wire_scatter(const WireParams Q) {
    const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    if (i >= Q.n) return;
    wire_get(Q, i);
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
    int cdev = -1;
    NCCL_TRY(R.CommCuDevice((ncclComm_t)nccl_comm, &cdev));
    if (cdev != device) SVO_FAIL(SVO_EINVAL, "svo_exchange_wrap: the communicator is on another device");
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

// one step's exchange from `wire` (this rank's records of every frame of d, frame-major, in d's wire format;
// frame f's at f * n_mine records)
static int exchange_wire(svo_exchange* x, const svo_tree* t, const svo_cast_desc* d, const void* wire, const uint8_t* ao_mine,
                         const svo_hits* frames_out, hipStream_t st, const char* fn) {
    const int32_t nf = d->n_frames > 1 ? d->n_frames : 1;
    const int32_t N = x->nranks, me = x->rank;
    const bool ao = d->ao_samples > 0;
    const int32_t n_own = nf > me ? (nf - me + N - 1) / N : 0;  // frames me, me + N, ...
    if (n_own > 0 && (!frames_out || !frames_out->pos_steps || !frames_out->t || !frames_out->info || (ao && !frames_out->ao)))
        SVO_FAIL(SVO_EINVAL, std::string(fn) + ": this rank displays frames but frames_out is incomplete");
    const int64_t frame = (int64_t)d->width * d->height;
    std::vector<int64_t> cnt(N), off(N + 1, 0);
    for (int32_t r = 0; r < N; r++) {
        cnt[r] = shard_records(d->width, d->height, r, N);
        off[r + 1] = off[r] + cnt[r];
    }
    const int64_t n_mine = cnt[me];
    WireParams Q0;
    int rc = wire_params(t, d, fn, Q0);
    if (rc) return rc;
    const size_t wb = Q0.compact ? 8 : 12;
    // the records of my frames from every other rank (their shard of frame k at k * frame + off[r])
    rc = grow(&x->recv, &x->recv_bytes, std::max<size_t>(16, (size_t)(n_own * frame) * (wb + (ao ? 1 : 0))));
    if (rc) return rc;
    const uint8_t* sw = reinterpret_cast<const uint8_t*>(wire);
    uint8_t* rw = reinterpret_cast<uint8_t*>(x->recv);
    uint8_t* rao = rw + (size_t)(n_own * frame) * wb;  // AO counts after the records
    if (N > 1) {
        Rccl& R = rccl();
        NCCL_TRY(R.GroupStart());
        for (int32_t f = 0; f < nf && n_mine > 0; f++) {
            const int32_t owner = f % N;
            if (owner == me) continue;  // (decoded from the wire buffer below)
            NCCL_TRY(R.Send(sw + (size_t)(f * n_mine) * wb, (size_t)n_mine * wb, ncclUint8, owner, x->comm, st));
            if (ao) NCCL_TRY(R.Send(ao_mine + (size_t)(f * n_mine), (size_t)n_mine, ncclUint8, owner, x->comm, st));
        }
        for (int32_t k = 0; k < n_own; k++)
            for (int32_t r = 0; r < N; r++) {
                if (cnt[r] == 0 || r == me) continue;
                const size_t base = (size_t)(k * frame + off[r]);
                NCCL_TRY(R.Recv(rw + base * wb, (size_t)cnt[r] * wb, ncclUint8, r, x->comm, st));
                if (ao) NCCL_TRY(R.Recv(rao + base, (size_t)cnt[r], ncclUint8, r, x->comm, st));
            }
        NCCL_TRY(R.GroupEnd());
    }
    // decode every shard of my frames into its pixels (my own shard straight from the wire buffer)
    for (int32_t k = 0; k < n_own; k++) {
        const int32_t f = me + k * N;
        const float* org = nf > 1 ? d->frame_origins + 3 * f : d->origin;
        for (int32_t r = 0; r < N; r++) {
            if (cnt[r] == 0) continue;
            WireParams Q = Q0;
            const size_t base = (size_t)(k * frame + off[r]);
            if (r == me) {
                Q.wire = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(sw + (size_t)(f * n_mine) * wb));
                Q.ao_in = ao ? ao_mine + (size_t)(f * n_mine) : nullptr;
            } else {
                Q.wire = reinterpret_cast<uint32_t*>(rw + base * wb);
                Q.ao_in = ao ? rao + base : nullptr;
            }
            Q.n = cnt[r];
            Q.frame_records = cnt[r];
            Q.tile_row_start = r;
            Q.tile_row_step = N;
            Q.scatter = 1;
            Q.frame_pixels = frame;
            for (int a = 0; a < 3; a++) Q.frame_org[a] = org[a];
            Q.pos = frames_out->pos_steps + 4 * (size_t)(k * frame);
            Q.t = frames_out->t + (size_t)(k * frame);
            Q.info = frames_out->info + (size_t)(k * frame);
            Q.ao_out = ao ? frames_out->ao + (size_t)(k * frame) : nullptr;
            hipLaunchKernelGGL(k_wire_scatter, dim3((uint32_t)((Q.n + 1024 - 1) / 1024)), dim3(1024), 0, st, Q);
            HIP_TRY(hipGetLastError(), SVO_EDEVICE);
        }
    }
    return SVO_OK;
}

static int exchange_check(svo_exchange* x, const svo_tree* t, const svo_cast_desc* d, const char* fn) {
    if (!x || !t || !d) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": NULL argument");
    if (d->ray_dirs) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": frame-mode descs only");
    if (d->tile_row_start != x->rank || d->tile_row_step != x->nranks)
        SVO_FAIL(SVO_EINVAL, std::string(fn) + ": desc is not this rank's shard (tile_row_start = rank, tile_row_step = nranks)");
    if (t->device != x->device) SVO_FAIL(SVO_EINVAL, std::string(fn) + ": the tree lives on another device than the exchange");
    HIP_TRY(hipSetDevice(x->device), SVO_EDEVICE);
    return SVO_OK;
}

extern "C" int svo_exchange_wire(svo_exchange* x, const svo_tree* t, const svo_cast_desc* d, const void* wire, const uint8_t* ao,
                                 const svo_hits* frames_out, void* stream) {
    int rc = exchange_check(x, t, d, "svo_exchange_wire");
    if (rc) return rc;
    if (!wire) SVO_FAIL(SVO_EINVAL, "svo_exchange_wire: NULL wire buffer");
    if (d->ao_samples > 0 && !ao) SVO_FAIL(SVO_EINVAL, "svo_exchange_wire: AO counts requested without an ao buffer");
    return exchange_wire(x, t, d, wire, ao, frames_out, (hipStream_t)stream, "svo_exchange_wire");
}

extern "C" int svo_exchange_frames(svo_exchange* x, const svo_tree* t, const svo_cast_desc* d, const svo_hits* mine,
                                   const svo_hits* frames_out, void* stream) {
    int rc = exchange_check(x, t, d, "svo_exchange_frames");
    if (rc) return rc;
    if (!mine) SVO_FAIL(SVO_EINVAL, "svo_exchange_frames: NULL argument");
    if (d->ao_samples > 0 && !mine->ao) SVO_FAIL(SVO_EINVAL, "svo_exchange_frames: AO counts requested without an ao buffer");
    const int32_t nf = d->n_frames > 1 ? d->n_frames : 1;
    const int64_t n_mine = shard_records(d->width, d->height, x->rank, x->nranks);
    // my records of every frame, packed (frame f's at f * n_mine)
    rc = grow(&x->send, &x->send_bytes, std::max<size_t>(16, (size_t)(n_mine * nf) * 12));
    if (rc) return rc;
    rc = svo_hits_pack(t, d, mine, x->send, stream);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(x->device), SVO_EDEVICE);  // (svo_hits_pack selected the tree's device: the same one)
    return exchange_wire(x, t, d, x->send, mine->ao, frames_out, (hipStream_t)stream, "svo_exchange_frames");
}
