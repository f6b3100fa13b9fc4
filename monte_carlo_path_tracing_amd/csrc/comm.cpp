// RCCL (NCCL API on ROCm) for the multi-GPU frame reduce (BASELINE north star:
// "a single RCCL reduce over xGMI to sum per-tile sample buffers into the final framebuffer").
//
// The reference is single-threaded (README.md:418 "Multi-thread: To be continued"); its frame loop
// main.cpp:557-588 shards by camera sample with no exchange, so the only collective is ONE
// ncclReduce(sum) of the fp64 framebuffers at the end of a render call.  The library owns the
// communicators:
//   * one process, several devices (mcpt_render_opts.devices): ncclCommInitAll over the distinct
//     devices, cached per scene handle (comm_all_*);
//   * one process per device (torchrun-style): mcpt_comm_unique_id on rank 0, broadcast by the
//     caller, mcpt_comm_init_rank on every rank (the mcpt_comm handle of include/mcpt.h).
//
// RCCL is resolved with dlopen at first use, not linked: a process that already holds an RCCL
// (torch's bundled librccl.so.1, same soname) shares it, and single-device renders never load it.
// mcpt_debug_set_collective_lib (include/mcpt_debug.h) points that dlopen at another library with the
// same NCCL entry points before the first use -- the test-only host-memory collective of
// tests/collshim, which lets 2-8 ranks share the one GPU of a test box (RCCL refuses two ranks on one
// device), so the multi-rank protocol below (the shard split, the buffers, the calls and their order, the
// failure flag) runs in CI as the 8-GPU run issues it.  The shim differs from RCCL in its transport and in
// one failure mode: it is synchronous and times out (MCPT_COLLSHIM_TIMEOUT) where an RCCL peer of an
// aborted rank blocks (include/mcpt.h, mcpt_render_opts.comm).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "mcpt.h"
#include "comm.h"
#include "mcpt_internal.h"

static_assert(MCPT_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "mcpt_comm id size must match ncclUniqueId");

struct mcpt_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
};

namespace mcpt {
namespace {

std::mutex g_lib_mu;
std::string g_lib_path;  // mcpt_debug_set_collective_lib; empty: librccl.so.1
bool g_lib_resolved = false;

struct RcclApi {
    ncclResult_t (*GetUniqueId)(ncclUniqueId*);
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*);
    ncclResult_t (*CommDestroy)(ncclComm_t);
    ncclResult_t (*Reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*GroupStart)();
    ncclResult_t (*GroupEnd)();
    const char* (*GetErrorString)(ncclResult_t);
    ncclResult_t (*CommAbort)(ncclComm_t);
};

const RcclApi* rccl() {
    static std::once_flag once;
    static RcclApi api;
    static bool ok = false;
    static char why[256] = "";
    std::call_once(once, [] {
        std::string path;
        {
            std::lock_guard<std::mutex> lk(g_lib_mu);
            g_lib_resolved = true;
            path = g_lib_path;
        }
        void* h = nullptr;
        if (!path.empty()) {
            h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
            if (!h) {
                std::snprintf(why, sizeof why, "cannot load the collective library %s: %s", path.c_str(), dlerror());
                return;
            }
        } else {
            h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
            if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        }
        if (!h) {
            std::snprintf(why, sizeof why, "cannot load RCCL (librccl.so.1): %s", dlerror());
            return;
        }
        bool all = true;
        auto sym = [&](const char* name) {
            void* p = dlsym(h, name);
            if (!p) all = false;
            return p;
        };
        api.GetUniqueId = (decltype(api.GetUniqueId))sym("ncclGetUniqueId");
        api.CommInitRank = (decltype(api.CommInitRank))sym("ncclCommInitRank");
        api.CommInitAll = (decltype(api.CommInitAll))sym("ncclCommInitAll");
        api.CommDestroy = (decltype(api.CommDestroy))sym("ncclCommDestroy");
        api.Reduce = (decltype(api.Reduce))sym("ncclReduce");
        api.GroupStart = (decltype(api.GroupStart))sym("ncclGroupStart");
        api.GroupEnd = (decltype(api.GroupEnd))sym("ncclGroupEnd");
        api.GetErrorString = (decltype(api.GetErrorString))sym("ncclGetErrorString");
        api.CommAbort = (decltype(api.CommAbort))sym("ncclCommAbort");
        if (!all) {
            std::snprintf(why, sizeof why, "RCCL library lacks an NCCL entry point");
            return;
        }
        ok = true;
    });
    if (!ok) {
        set_error("%s", why);
        return nullptr;
    }
    return &api;
}

#define RCCL_OK(A, x)                                                                           \
    do {                                                                                        \
        ncclResult_t r_ = (x);                                                                  \
        if (r_ != ncclSuccess) {                                                                \
            set_error("%s failed: %s (%s:%d)", #x, (A)->GetErrorString(r_), __FILE__, __LINE__); \
            return MCPT_E_DEVICE;                                                               \
        }                                                                                       \
    } while (0)

}  // namespace

int comm_all_init(const std::vector<int>& devices, std::vector<void*>& comms) {
    const RcclApi* A = rccl();
    if (!A) return MCPT_E_DEVICE;
    std::vector<ncclComm_t> c(devices.size(), nullptr);
    RCCL_OK(A, A->CommInitAll(c.data(), (int)devices.size(), devices.data()));
    comms.assign(c.begin(), c.end());
    return MCPT_OK;
}

void comm_all_destroy(std::vector<void*>& comms) {
    const RcclApi* A = rccl();
    if (A)
        for (void* c : comms)
            if (c) (void)A->CommDestroy((ncclComm_t)c);
    comms.clear();
}

// in-place sum of bufs[i] (n doubles on devices[i], stream streams[i]) into bufs[0] (rank 0 =
// devices[0]); non-root buffers are left as they are.  Enqueued only: the caller synchronises.
int comm_all_reduce_sum(const std::vector<void*>& comms, const std::vector<int>& devices, const std::vector<double*>& bufs,
                        const std::vector<hipStream_t>& streams, size_t n) {
    const RcclApi* A = rccl();
    if (!A) return MCPT_E_DEVICE;
    RCCL_OK(A, A->GroupStart());
    for (size_t i = 0; i < comms.size(); i++) {
        if (hipSetDevice(devices[i]) != hipSuccess) {
            (void)A->GroupEnd();
            set_error("hipSetDevice(%d) failed", devices[i]);
            return MCPT_E_DEVICE;
        }
        const ncclResult_t r = A->Reduce(bufs[i], bufs[i], n, ncclFloat64, ncclSum, 0, (ncclComm_t)comms[i], streams[i]);
        if (r != ncclSuccess) {
            (void)A->GroupEnd();
            set_error("ncclReduce failed: %s", A->GetErrorString(r));
            return MCPT_E_DEVICE;
        }
    }
    RCCL_OK(A, A->GroupEnd());
    return MCPT_OK;
}

int comm_rank_reduce_sum(mcpt_comm* c, double* buf, size_t n, hipStream_t st) {
    const RcclApi* A = rccl();
    if (!A) return MCPT_E_DEVICE;
    if (!c->comm) {
        set_error("the communicator was aborted after an earlier failure; create a new one");
        return MCPT_E_DEVICE;
    }
    RCCL_OK(A, A->Reduce(buf, buf, n, ncclFloat64, ncclSum, 0, c->comm, st));
    return MCPT_OK;
}

// after a failure that leaves this rank unable to join a collective (the enqueue itself failed): abort
// the communicator so that RCCL frees its resources; the handle stays allocated (mcpt_comm_destroy)
void comm_rank_abort(mcpt_comm* c) {
    const RcclApi* A = rccl();
    if (A && c && c->comm) {
        (void)A->CommAbort(c->comm);
        c->comm = nullptr;
    }
}

int comm_rank_info(const mcpt_comm* c, int* nranks, int* rank, int* device) {
    if (!c) return MCPT_E_INVALID;
    *nranks = c->nranks;
    *rank = c->rank;
    *device = c->device;
    return MCPT_OK;
}

}  // namespace mcpt

using namespace mcpt;

extern "C" {

int mcpt_debug_set_collective_lib(const char* path) {
    std::lock_guard<std::mutex> lk(g_lib_mu);
    if (g_lib_resolved) {
        set_error("the collective library is already resolved (set it before the first communicator)");
        return MCPT_E_INVALID;
    }
    g_lib_path = path ? path : "";
    return MCPT_OK;
}

int mcpt_comm_unique_id(uint8_t id[MCPT_COMM_ID_BYTES]) {
    if (!id) {
        set_error("null argument");
        return MCPT_E_INVALID;
    }
    const RcclApi* A = rccl();
    if (!A) return MCPT_E_DEVICE;
    ncclUniqueId u;
    RCCL_OK(A, A->GetUniqueId(&u));
    std::memcpy(id, u.internal, MCPT_COMM_ID_BYTES);
    return MCPT_OK;
}

int mcpt_comm_init_rank(int32_t nranks, int32_t rank, const uint8_t id[MCPT_COMM_ID_BYTES], int32_t device,
                        mcpt_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) {
        set_error("invalid argument (nranks %d, rank %d)", nranks, rank);
        return MCPT_E_INVALID;
    }
    const RcclApi* A = rccl();
    if (!A) return MCPT_E_DEVICE;
    if (device < 0 && hipGetDevice(&device) != hipSuccess) {
        set_error("hipGetDevice failed");
        return MCPT_E_DEVICE;
    }
    if (hipSetDevice(device) != hipSuccess) {
        set_error("hipSetDevice(%d) failed", device);
        return MCPT_E_DEVICE;
    }
    ncclUniqueId u;
    std::memcpy(u.internal, id, MCPT_COMM_ID_BYTES);
    auto* c = new mcpt_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    const ncclResult_t r = A->CommInitRank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        set_error("ncclCommInitRank(%d ranks, rank %d, device %d) failed: %s", nranks, rank, device, A->GetErrorString(r));
        delete c;
        return MCPT_E_DEVICE;
    }
    *out = c;
    return MCPT_OK;
}

void mcpt_comm_destroy(mcpt_comm* c) {
    if (!c) return;
    const RcclApi* A = rccl();
    if (A && c->comm) (void)A->CommDestroy(c->comm);
    delete c;
}

}  // extern "C"
