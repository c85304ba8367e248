// rccl_standin.cpp — TEST-ONLY stand-in for librccl.so.1, so that libsvo_rt's N > 1 exchange code
// (raytracing_test_amd/csrc/svo_exchange.hip: the ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd
// pairing of exchange_wire) runs with several ranks on ONE GPU, where a real RCCL communicator cannot
// be formed (two ranks of an RCCL communicator need two devices).  libsvo_rt loads it instead of RCCL
// when SVO_RCCL_LIB names it (svo_exchange.hip rccl()).  It is never part of the product: the driver's
// multi-GPU run uses the real RCCL.
//
// It implements exactly the 11 entry points libsvo_rt binds, with NCCL's matching rules:
//   * point-to-point operations between a pair of ranks match in issue order (the k-th send from a to
//     b is the k-th receive of b from a), inside or outside a group;
//   * a group (ncclGroupStart ... ncclGroupEnd) executes as a whole at ncclGroupEnd.
// Transport: host memory.  At ncclGroupEnd every stream the group names is synchronised (the data the
// sends read is complete), each send's bytes are copied device -> host into a message file of the
// communicator's directory (<dir>/<src>_<dst>_<seq>.msg, written under a temporary name, then renamed,
// so a receiver never sees a partial message), and then each receive waits for its message and copies
// it host -> device on its stream, synchronously.  Sends never wait, so a group cannot deadlock on
// ordering as long as every rank reaches its ncclGroupEnd; a receive that waits longer than
// SVO_STANDIN_TIMEOUT_S (default 120 s) fails with ncclSystemError instead of hanging.  A received
// message whose size differs from the receive's is ncclInvalidUsage (a mismatched pairing is an error,
// not a silent truncation).  ncclCommInitRank is a barrier over the communicator's ranks (each
// announces itself with a file, then waits for all).  The directory is /dev/shm (SVO_STANDIN_DIR
// overrides), named from the unique id.
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

#define STANDIN_API extern "C" __attribute__((visibility("default")))

struct ncclComm {
    std::string dir;
    int nranks = 0, rank = 0, device = 0;
    bool host_only = false;  // SVO_STANDIN_HOST_ONLY=1: buffers are host memory (the CPU test of the pairing rules)
    std::vector<unsigned long long> send_seq, recv_seq;  // per peer
};

namespace {

struct Op {
    bool send;
    void* buf;
    size_t bytes;
    int peer;
    ncclComm* comm;
    hipStream_t stream;
};

thread_local int g_depth = 0;
thread_local std::vector<Op> g_ops;

const char kMagic[] = "svo-rccl-standin:";

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8:
        case ncclUint8:
            return 1;
        case ncclFloat16:
        case ncclBfloat16:
            return 2;
        case ncclInt32:
        case ncclUint32:
        case ncclFloat32:
            return 4;
        case ncclInt64:
        case ncclUint64:
        case ncclFloat64:
            return 8;
        default:
            return 0;
    }
}

double timeout_s() {
    const char* e = getenv("SVO_STANDIN_TIMEOUT_S");
    const double v = e && *e ? atof(e) : 120.0;
    return v > 0 ? v : 120.0;
}

std::string base_dir() {
    const char* e = getenv("SVO_STANDIN_DIR");
    if (e && *e) return e;
    struct stat st;
    if (stat("/dev/shm", &st) == 0 && S_ISDIR(st.st_mode) && access("/dev/shm", W_OK) == 0) return "/dev/shm";
    const char* t = getenv("TMPDIR");
    return t && *t ? t : "/tmp";
}

bool write_all(int fd, const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n) {
        const ssize_t w = write(fd, c, n);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        c += w;
        n -= (size_t)w;
    }
    return true;
}

bool read_all(int fd, void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n) {
        const ssize_t r = read(fd, c, n);
        if (r < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        if (r == 0) return false;
        c += r;
        n -= (size_t)r;
    }
    return true;
}

std::string msg_path(const ncclComm* c, int src, int dst, unsigned long long seq) {
    return c->dir + "/" + std::to_string(src) + "_" + std::to_string(dst) + "_" + std::to_string(seq) + ".msg";
}

// polls `pred` with a growing sleep (20 us .. 1 ms) until it holds or the timeout passes
template <class F>
bool wait_for(F pred) {
    const auto t0 = std::chrono::steady_clock::now();
    const double lim = timeout_s();
    int us = 20;
    while (!pred()) {
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(us));
        us = us < 1000 ? us * 2 : 1000;
    }
    return true;
}

// TEST HOOK (tests/test_gpu_bench_gather.py: the bench watchdog): SVO_STANDIN_WITHHOLD=<rank>:<k> drops that rank's k-th
// send (counted over the process from 0) without a word: its receiver waits for a message that never comes, as a rank
// stuck inside a real RCCL group would
bool withheld(const ncclComm* c) {
    static unsigned long long n_sends = 0;
    const unsigned long long k = n_sends++;
    const char* e = getenv("SVO_STANDIN_WITHHOLD");
    int r = -1;
    unsigned long long kk = 0;
    return e && sscanf(e, "%d:%llu", &r, &kk) == 2 && r == c->rank && kk == k;
}

ncclResult_t do_send(const Op& op) {
    ncclComm* c = op.comm;
    if (withheld(c)) {
        c->send_seq[op.peer]++;
        fprintf(stderr, "rccl_standin: rank %d: TEST HOOK withholds its send to rank %d\n", c->rank, op.peer);
        return ncclSuccess;
    }
    std::vector<char> host(op.bytes);
    if (c->host_only) {
        if (op.bytes) memcpy(host.data(), op.buf, op.bytes);
    } else if (op.bytes && hipMemcpy(host.data(), op.buf, op.bytes, hipMemcpyDeviceToHost) != hipSuccess) {
        return ncclUnhandledCudaError;
    }
    const unsigned long long seq = c->send_seq[op.peer]++;
    const std::string path = msg_path(c, c->rank, op.peer, seq);
    const std::string tmp = path + ".tmp";
    const int fd = open(tmp.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0600);
    if (fd < 0) return ncclSystemError;
    const unsigned long long n = op.bytes;
    const bool ok = write_all(fd, &n, sizeof n) && write_all(fd, host.data(), op.bytes);
    close(fd);
    if (!ok || rename(tmp.c_str(), path.c_str()) != 0) {
        unlink(tmp.c_str());
        return ncclSystemError;
    }
    return ncclSuccess;
}

ncclResult_t do_recv(const Op& op) {
    ncclComm* c = op.comm;
    const unsigned long long seq = c->recv_seq[op.peer]++;
    const std::string path = msg_path(c, op.peer, c->rank, seq);
    if (!wait_for([&] { return access(path.c_str(), R_OK) == 0; })) {
        fprintf(stderr, "rccl_standin: rank %d: no message %s within %.0f s\n", c->rank, path.c_str(), timeout_s());
        return ncclSystemError;
    }
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return ncclSystemError;
    unsigned long long n = 0;
    std::vector<char> host;
    bool ok = read_all(fd, &n, sizeof n);
    if (ok && n == op.bytes) {
        host.resize(n);
        ok = read_all(fd, host.data(), n);
    }
    close(fd);
    unlink(path.c_str());
    if (!ok) return ncclSystemError;
    if (n != op.bytes) {
        fprintf(stderr, "rccl_standin: rank %d: message from rank %d has %llu bytes, the receive expects %zu\n", c->rank, op.peer, n,
                op.bytes);
        return ncclInvalidUsage;
    }
    if (c->host_only) {
        if (n) memcpy(op.buf, host.data(), n);
        return ncclSuccess;
    }
    if (n && (hipMemcpyAsync(op.buf, host.data(), n, hipMemcpyHostToDevice, op.stream) != hipSuccess ||
              hipStreamSynchronize(op.stream) != hipSuccess))
        return ncclUnhandledCudaError;
    return ncclSuccess;
}

ncclResult_t run_group(std::vector<Op>& ops) {
    // every send buffer complete: the streams the group names (stream-ordered semantics of ncclSend)
    std::vector<hipStream_t> seen;
    for (const Op& op : ops) {
        bool dup = false;
        for (hipStream_t s : seen) dup |= s == op.stream;
        if (dup) continue;
        seen.push_back(op.stream);
        if (!op.comm->host_only && hipStreamSynchronize(op.stream) != hipSuccess) return ncclUnhandledCudaError;
    }
    ncclResult_t rc = ncclSuccess;
    for (const Op& op : ops)
        if (op.send && rc == ncclSuccess) rc = do_send(op);
    for (const Op& op : ops)
        if (!op.send && rc == ncclSuccess) rc = do_recv(op);
    ops.clear();
    return rc;
}

ncclResult_t enqueue(const Op& op) {
    if (!op.comm) return ncclInvalidArgument;
    if (op.peer < 0 || op.peer >= op.comm->nranks || op.peer == op.comm->rank) return ncclInvalidArgument;
    if (op.bytes && !op.buf) return ncclInvalidArgument;
    if (g_depth > 0) {
        g_ops.push_back(op);
        return ncclSuccess;
    }
    std::vector<Op> one{op};
    return run_group(one);
}

}  // namespace

STANDIN_API ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    memset(id->internal, 0, sizeof id->internal);
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    snprintf(id->internal, sizeof id->internal, "%s%d_%lld_%ld", kMagic, (int)getpid(), (long long)ts.tv_sec, ts.tv_nsec);
    return ncclSuccess;
}

STANDIN_API ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    *out = nullptr;
    if (strncmp(id.internal, kMagic, sizeof kMagic - 1) != 0) return ncclInvalidArgument;  // not this stand-in's id
    char name[NCCL_UNIQUE_ID_BYTES + 1];
    memcpy(name, id.internal + sizeof kMagic - 1, NCCL_UNIQUE_ID_BYTES - (sizeof kMagic - 1));
    name[NCCL_UNIQUE_ID_BYTES - (sizeof kMagic - 1)] = 0;
    ncclComm* c = new ncclComm();
    c->dir = base_dir() + "/svo_rccl_standin_" + name;
    c->nranks = nranks;
    c->rank = rank;
    c->send_seq.assign(nranks, 0);
    c->recv_seq.assign(nranks, 0);
    const char* ho = getenv("SVO_STANDIN_HOST_ONLY");
    c->host_only = ho && *ho == '1';
    if (!c->host_only && hipGetDevice(&c->device) != hipSuccess) {
        delete c;
        return ncclUnhandledCudaError;
    }
    if (mkdir(c->dir.c_str(), 0700) != 0 && errno != EEXIST) {
        delete c;
        return ncclSystemError;
    }
    // barrier: announce, then wait for every rank's announcement
    const std::string me = c->dir + "/rank" + std::to_string(rank);
    const int fd = open(me.c_str(), O_CREAT | O_WRONLY, 0600);
    if (fd < 0) {
        delete c;
        return ncclSystemError;
    }
    close(fd);
    const bool all = wait_for([&] {
        for (int r = 0; r < nranks; r++)
            if (access((c->dir + "/rank" + std::to_string(r)).c_str(), F_OK) != 0) return false;
        return true;
    });
    if (!all) {
        fprintf(stderr, "rccl_standin: rank %d of %d: not every rank joined %s within %.0f s\n", rank, nranks, c->dir.c_str(), timeout_s());
        unlink(me.c_str());
        delete c;
        return ncclSystemError;
    }
    *out = c;
    return ncclSuccess;
}

STANDIN_API ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    // any message addressed to this rank that nobody received; then it marks itself gone (its announcement stays: a rank
    // still in ncclCommInitRank's barrier must find it — ranks with nothing to exchange may finish before a slow one has
    // joined), and the last rank out removes the announcements and the directory
    if (DIR* d = opendir(c->dir.c_str())) {
        while (struct dirent* e = readdir(d)) {
            int src = -1, dst = -1;
            unsigned long long seq = 0;
            if (sscanf(e->d_name, "%d_%d_%llu.msg", &src, &dst, &seq) == 3 && dst == c->rank) unlink((c->dir + "/" + e->d_name).c_str());
        }
        closedir(d);
    }
    const int fd = open((c->dir + "/left" + std::to_string(c->rank)).c_str(), O_CREAT | O_WRONLY, 0600);
    if (fd >= 0) close(fd);
    bool last = true;
    for (int r = 0; r < c->nranks && last; r++) last = access((c->dir + "/left" + std::to_string(r)).c_str(), F_OK) == 0;
    if (last) {
        for (int r = 0; r < c->nranks; r++) {
            unlink((c->dir + "/rank" + std::to_string(r)).c_str());
            unlink((c->dir + "/left" + std::to_string(r)).c_str());
        }
        rmdir(c->dir.c_str());
    }
    delete c;
    return ncclSuccess;
}

STANDIN_API ncclResult_t ncclCommCount(const ncclComm_t c, int* n) {
    if (!c || !n) return ncclInvalidArgument;
    *n = c->nranks;
    return ncclSuccess;
}

STANDIN_API ncclResult_t ncclCommUserRank(const ncclComm_t c, int* r) {
    if (!c || !r) return ncclInvalidArgument;
    *r = c->rank;
    return ncclSuccess;
}

STANDIN_API ncclResult_t ncclCommCuDevice(const ncclComm_t c, int* dev) {
    if (!c || !dev) return ncclInvalidArgument;
    *dev = c->device;
    return ncclSuccess;
}

STANDIN_API ncclResult_t ncclGroupStart() {
    g_depth++;
    return ncclSuccess;
}

STANDIN_API ncclResult_t ncclGroupEnd() {
    if (g_depth <= 0) return ncclInvalidUsage;
    if (--g_depth > 0) return ncclSuccess;
    return run_group(g_ops);
}

STANDIN_API ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
    const size_t tb = type_bytes(t);
    if (!tb) return ncclInvalidArgument;
    return enqueue(Op{true, const_cast<void*>(buf), count * tb, peer, c, s});
}

STANDIN_API ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
    const size_t tb = type_bytes(t);
    if (!tb) return ncclInvalidArgument;
    return enqueue(Op{false, buf, count * tb, peer, c, s});
}

STANDIN_API const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess:
            return "no error (rccl stand-in)";
        case ncclUnhandledCudaError:
            return "HIP call failed (rccl stand-in)";
        case ncclSystemError:
            return "system error or timeout (rccl stand-in)";
        case ncclInvalidArgument:
            return "invalid argument (rccl stand-in)";
        case ncclInvalidUsage:
            return "invalid usage: mismatched send / receive (rccl stand-in)";
        default:
            return "error (rccl stand-in)";
    }
}
