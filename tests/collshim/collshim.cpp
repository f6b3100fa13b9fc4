// Test-only collective library with the NCCL API (the entry points libmcpt_hip.so binds in
// monte_carlo_path_tracing_amd/csrc/comm.cpp), reducing over host shared memory instead of xGMI.
//
// Why: RCCL refuses two ranks on one GPU ("duplicate GPU"), and the test box has ONE MI355X, so the
// library's multi-rank protocol -- render_rank's in-place ncclReduce from a non-root rank, the
// status slot that tells rank 0 a peer failed, comm_all_reduce_sum's group over several
// communicators, bench.py --gpus N -- would otherwise first run on the driver's 8-GPU node.  With
// mcpt_debug_set_collective_lib(<this .so>) the library's calls land here, and 2-8 processes (or the
// ranks of one ncclCommInitAll) share the one GPU.  The reference has no collective at all
// (README.md:418, single-threaded main.cpp:557-588); this only stands in for RCCL in tests.
//
// Semantics (the subset the library uses):
//  * ncclGetUniqueId: a magic + 16 random bytes naming a POSIX shared-memory header;
//  * ncclCommInitRank: maps the header, waits until all nranks have joined (a barrier);
//  * ncclReduce(float64, sum, root): synchronises the stream, a non-root rank copies its device buffer
//    into a shared-memory segment named by (id, call sequence, rank); the root waits for the
//    nranks - 1 segments of that call, sums them in rank order onto its own buffer's host copy and
//    writes the result to recvbuff.  Non-root receive buffers are never written (NCCL's contract);
//  * ncclCommInitAll: one in-process clique (a device may repeat); its ncclReduce calls must come in a
//    ncclGroupStart/End pair and are executed together at ncclGroupEnd;
//  * waits time out after MCPT_COLLSHIM_TIMEOUT seconds (default 120) with ncclSystemError, so a
//    protocol bug fails a test instead of hanging it.
// Host code only; the device work is hipMemcpy.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr char kMagic[8] = {'M', 'C', 'P', 'T', 'S', 'H', 'I', 'M'};

constexpr int kMaxRanks = 64;
struct Hdr {  // in shared memory, zero-filled by ftruncate
    std::atomic<uint32_t> joined;
    std::atomic<uint32_t> left;
    // posted[r]: the last reduce call whose contribution rank r has posted.  Per rank, not one shared
    // count: a non-root rank returns from its reduce at once and may post call s + 1 before a slower
    // peer posts call s, so a total would let the root proceed without the slow peer's segment
    std::atomic<uint64_t> posted[kMaxRanks];
};
static_assert(std::atomic<uint32_t>::is_always_lock_free && std::atomic<uint64_t>::is_always_lock_free,
              "shared-memory atomics must be lock-free");

struct Clique;
struct Comm {
    int nranks = 1, rank = 0, device = 0;
    std::string name;  // shared-memory header (ncclCommInitRank)
    Hdr* hdr = nullptr;
    uint64_t seq = 0;  // reduce calls so far (every rank calls them in the same order)
    Clique* clq = nullptr;  // ncclCommInitAll
};
struct Clique {
    int n = 0;
    int alive = 0;
};
struct Op {
    const void* send;
    void* recv;
    size_t count;
    int root;
    Comm* comm;
    hipStream_t stream;
};
thread_local int g_group = 0;
thread_local std::vector<Op> g_ops;

double timeout_s() {
    const char* e = std::getenv("MCPT_COLLSHIM_TIMEOUT");
    const double v = e ? std::atof(e) : 0.0;
    return v > 0 ? v : 120.0;
}

template <class F>
bool wait_for(F ready) {
    const auto t0 = std::chrono::steady_clock::now();
    const double lim = timeout_s();
    while (!ready()) {
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    return true;
}

std::string hex(const unsigned char* b, int n) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (int i = 0; i < n; i++) s += d[b[i] >> 4], s += d[b[i] & 15];
    return s;
}

std::string seg_name(const Comm* c, uint64_t seq, int rank) {
    return c->name + "_" + std::to_string(seq) + "_" + std::to_string(rank);
}

ncclResult_t check_args(size_t count, ncclDataType_t dt, ncclRedOp_t op, int root, const Comm* c) {
    if (!c || dt != ncclFloat64 || op != ncclSum || root < 0 || root >= c->nranks) return ncclInvalidArgument;
    if (count > (size_t(1) << 40)) return ncclInvalidArgument;
    return ncclSuccess;
}

// one multi-process reduce (ncclCommInitRank communicator)
ncclResult_t reduce_rank(const Op& o) {
    Comm* c = o.comm;
    const size_t bytes = o.count * sizeof(double);
    if (hipStreamSynchronize(o.stream) != hipSuccess) return ncclUnhandledCudaError;
    const uint64_t seq = ++c->seq;
    if (c->nranks == 1) {
        if (o.recv != o.send && hipMemcpy(o.recv, o.send, bytes, hipMemcpyDeviceToDevice) != hipSuccess)
            return ncclUnhandledCudaError;
        return ncclSuccess;
    }
    if (c->rank != o.root) {
        const std::string nm = seg_name(c, seq, c->rank);
        const int fd = shm_open(nm.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0) return ncclSystemError;
        if (ftruncate(fd, (off_t)std::max<size_t>(bytes, 8)) != 0) {
            close(fd);
            return ncclSystemError;
        }
        void* p = mmap(nullptr, std::max<size_t>(bytes, 8), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) return ncclSystemError;
        const hipError_t e = bytes ? hipMemcpy(p, o.send, bytes, hipMemcpyDeviceToHost) : hipSuccess;
        munmap(p, std::max<size_t>(bytes, 8));
        if (e != hipSuccess) return ncclUnhandledCudaError;
        c->hdr->posted[c->rank].store(seq);
        return ncclSuccess;
    }
    auto all_posted = [&] {
        for (int r = 0; r < c->nranks; r++)
            if (r != o.root && c->hdr->posted[r].load() < seq) return false;
        return true;
    };
    if (!wait_for(all_posted)) {
        std::fprintf(stderr, "collshim: rank %d timed out waiting for reduce %llu\n", c->rank, (unsigned long long)seq);
        return ncclSystemError;
    }
    std::vector<double> acc(o.count);
    if (bytes && hipMemcpy(acc.data(), o.send, bytes, hipMemcpyDeviceToHost) != hipSuccess) return ncclUnhandledCudaError;
    for (int r = 0; r < c->nranks; r++) {
        if (r == o.root) continue;
        const std::string nm = seg_name(c, seq, r);
        const int fd = shm_open(nm.c_str(), O_RDONLY, 0600);
        if (fd < 0) return ncclSystemError;
        void* p = mmap(nullptr, std::max<size_t>(bytes, 8), PROT_READ, MAP_SHARED, fd, 0);
        close(fd);
        shm_unlink(nm.c_str());
        if (p == MAP_FAILED) return ncclSystemError;
        const double* v = static_cast<const double*>(p);
        for (size_t i = 0; i < o.count; i++) acc[i] += v[i];
        munmap(p, std::max<size_t>(bytes, 8));
    }
    if (bytes && hipMemcpy(o.recv, acc.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return ncclUnhandledCudaError;
    return ncclSuccess;
}

// the reduces of one ncclCommInitAll clique, issued inside one group
ncclResult_t reduce_clique(std::vector<Op>& ops) {
    if (ops.empty()) return ncclSuccess;
    Clique* q = ops[0].comm->clq;
    if ((int)ops.size() != q->n) return ncclInvalidUsage;  // every rank of the clique, once
    std::vector<const Op*> by_rank(q->n, nullptr);
    for (const Op& o : ops) {
        if (o.comm->clq != q || by_rank[o.comm->rank] || o.root != ops[0].root || o.count != ops[0].count)
            return ncclInvalidUsage;
        by_rank[o.comm->rank] = &o;
    }
    const int root = ops[0].root;
    const size_t count = ops[0].count, bytes = count * sizeof(double);
    std::vector<double> acc(count), tmp(count);
    for (int r = 0; r < q->n; r++) {  // root first, then the others in rank order
        const int rr = r == 0 ? root : (r <= root ? r - 1 : r);
        const Op& o = *by_rank[rr];
        if (hipSetDevice(o.comm->device) != hipSuccess || hipStreamSynchronize(o.stream) != hipSuccess)
            return ncclUnhandledCudaError;
        if (bytes && hipMemcpy(r == 0 ? acc.data() : tmp.data(), o.send, bytes, hipMemcpyDeviceToHost) != hipSuccess)
            return ncclUnhandledCudaError;
        if (r > 0)
            for (size_t i = 0; i < count; i++) acc[i] += tmp[i];
    }
    const Op& ro = *by_rank[root];
    if (hipSetDevice(ro.comm->device) != hipSuccess) return ncclUnhandledCudaError;
    if (bytes && hipMemcpy(ro.recv, acc.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return ncclUnhandledCudaError;
    return ncclSuccess;
}

ncclResult_t run(std::vector<Op>& ops) {
    std::vector<Op> clq;
    for (const Op& o : ops) {
        if (o.comm->clq) {
            clq.push_back(o);
        } else {
            const ncclResult_t r = reduce_rank(o);
            if (r != ncclSuccess) return r;
        }
    }
    // one clique per group (the library issues one group per device-list reduce)
    if (!clq.empty()) {
        for (const Op& o : clq)
            if (o.comm->clq != clq[0].comm->clq) return ncclInvalidUsage;
        return reduce_clique(clq);
    }
    return ncclSuccess;
}

void release(Comm* c) {
    if (!c) return;
    if (c->hdr) {
        if (c->hdr->left.fetch_add(1) + 1 == (uint32_t)c->nranks) shm_unlink(c->name.c_str());
        munmap(c->hdr, sizeof(Hdr));
    }
    if (c->clq && --c->clq->alive == 0) delete c->clq;
    delete c;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id->internal, 0, sizeof id->internal);
    std::memcpy(id->internal, kMagic, sizeof kMagic);
    const int fd = open("/dev/urandom", O_RDONLY);
    if (fd < 0) return ncclSystemError;
    const ssize_t n = read(fd, id->internal + 8, 16);
    close(fd);
    return n == 16 ? ncclSuccess : ncclSystemError;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks ||
        std::memcmp(id.internal, kMagic, sizeof kMagic) != 0)
        return ncclInvalidArgument;
    auto* c = new Comm();
    c->nranks = nranks;
    c->rank = rank;
    if (hipGetDevice(&c->device) != hipSuccess) {
        delete c;
        return ncclUnhandledCudaError;
    }
    c->name = "/mcptshim_" + hex(reinterpret_cast<const unsigned char*>(id.internal) + 8, 16);
    const int fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, sizeof(Hdr)) != 0) {
        if (fd >= 0) close(fd);
        delete c;
        return ncclSystemError;
    }
    void* p = mmap(nullptr, sizeof(Hdr), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        delete c;
        return ncclSystemError;
    }
    c->hdr = static_cast<Hdr*>(p);
    c->hdr->joined.fetch_add(1);
    if (!wait_for([&] { return c->hdr->joined.load() >= (uint32_t)nranks; })) {
        std::fprintf(stderr, "collshim: rank %d of %d timed out waiting for the others to join\n", rank, nranks);
        munmap(c->hdr, sizeof(Hdr));
        delete c;
        return ncclSystemError;
    }
    *comm = reinterpret_cast<ncclComm_t>(c);
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
    if (!comms || ndev < 1) return ncclInvalidArgument;
    auto* q = new Clique();
    q->n = ndev;
    q->alive = ndev;
    for (int i = 0; i < ndev; i++) {
        auto* c = new Comm();
        c->nranks = ndev;
        c->rank = i;
        c->device = devlist ? devlist[i] : i;
        c->clq = q;
        comms[i] = reinterpret_cast<ncclComm_t>(c);
    }
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    release(reinterpret_cast<Comm*>(comm));
    return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
    release(reinterpret_cast<Comm*>(comm));
    return ncclSuccess;
}

ncclResult_t ncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, ncclRedOp_t op,
                        int root, ncclComm_t comm, hipStream_t stream) {
    Comm* c = reinterpret_cast<Comm*>(comm);
    const ncclResult_t a = check_args(count, datatype, op, root, c);
    if (a != ncclSuccess) return a;
    Op o{sendbuff, recvbuff, count, root, c, stream};
    if (g_group > 0) {
        g_ops.push_back(o);
        return ncclSuccess;
    }
    if (c->clq) {
        if (c->clq->n != 1) return ncclInvalidUsage;  // a multi-rank clique needs a group
        std::vector<Op> one{o};
        return reduce_clique(one);
    }
    return reduce_rank(o);
}

ncclResult_t ncclGroupStart() {
    ++g_group;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (g_group <= 0) return ncclInvalidUsage;
    if (--g_group > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(g_ops);
    return run(ops);
}

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (collshim)";
        case ncclUnhandledCudaError: return "HIP call failed (collshim)";
        case ncclSystemError: return "system error or timeout (collshim)";
        case ncclInvalidArgument: return "invalid argument (collshim)";
        case ncclInvalidUsage: return "invalid usage (collshim)";
        default: return "error (collshim)";
    }
}

}  // extern "C"
