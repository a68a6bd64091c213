// The RCCL stats all-reduce helper of the drop-in boundary (SURVEY §8b "Collectives"): one
// communicator per process, SUM of a small fp64 vector, enqueued on a caller's HIP stream.
//
// Why not torch.distributed alone: ProcessGroupNCCL runs every collective on its own stream
// and joins it to the caller's with default HIP events; on MI355X each such event record is a
// system-scope release that idles the compute queue ~20 us (measured: two 24-B all-reduces
// per PPO step cost 50 us at world size 1, profiles/r02_rccl_world1.log).  Here the
// all-reduce is enqueued straight on the stream that runs the step (no join at all), or on a
// side stream the caller joins with fence-free events.
//
// RCCL itself is the library the process already runs (PyTorch's librccl.so): the caller
// passes its path and it is dlopen'ed — the same loaded instance, no second RCCL in the
// process — and the five entry points used are bound by name.  Their C signatures are the
// stable NCCL API; the handful of types they need are declared here rather than taken from
// a header of a possibly different RCCL build.
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>

#include <hip/hip_runtime.h>

#include "common.h"

namespace {

constexpr int kUniqueIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES
struct UniqueId {
    char internal[kUniqueIdBytes];
};
typedef void* Comm;
enum { kNcclSuccess = 0, kNcclFloat64 = 8, kNcclSum = 0 };

struct Api {
    void* lib = nullptr;
    int (*get_unique_id)(UniqueId*) = nullptr;
    int (*comm_init_rank)(Comm*, int, UniqueId, int) = nullptr;
    int (*all_reduce)(const void*, void*, size_t, int, int, Comm, hipStream_t) = nullptr;
    int (*comm_destroy)(Comm) = nullptr;
    const char* (*error_string)(int) = nullptr;
};
Api g_api;

int nccl_status(int r, const char* what) {
    if (r == kNcclSuccess) return TRLX_OK;
    trlx::set_error("%s failed: %s (%d)", what, g_api.error_string ? g_api.error_string(r) : "?", r);
    return TRLX_ERR_LAUNCH;
}

}  // namespace

extern "C" int trlx_comm_load(const char* librccl_path) {
    TRLX_REQUIRE(librccl_path && *librccl_path, TRLX_ERR_ARG, "trlx_comm_load: empty library path");
    if (g_api.lib) return TRLX_OK;
    void* h = dlopen(librccl_path, RTLD_NOW | RTLD_LOCAL);
    TRLX_REQUIRE(h, TRLX_ERR_ARG, "dlopen(%s) failed: %s", librccl_path, dlerror());
    Api a;
    a.lib = h;
    a.get_unique_id = reinterpret_cast<int (*)(UniqueId*)>(dlsym(h, "ncclGetUniqueId"));
    a.comm_init_rank = reinterpret_cast<int (*)(Comm*, int, UniqueId, int)>(dlsym(h, "ncclCommInitRank"));
    a.all_reduce = reinterpret_cast<int (*)(const void*, void*, size_t, int, int, Comm, hipStream_t)>(
        dlsym(h, "ncclAllReduce"));
    a.comm_destroy = reinterpret_cast<int (*)(Comm)>(dlsym(h, "ncclCommDestroy"));
    a.error_string = reinterpret_cast<const char* (*)(int)>(dlsym(h, "ncclGetErrorString"));
    TRLX_REQUIRE(a.get_unique_id && a.comm_init_rank && a.all_reduce && a.comm_destroy && a.error_string,
                 TRLX_ERR_ARG, "%s does not export the NCCL API (ncclAllReduce, ...)", librccl_path);
    g_api = a;
    return TRLX_OK;
}

extern "C" int64_t trlx_comm_unique_id_bytes(void) { return kUniqueIdBytes; }

extern "C" int trlx_comm_unique_id(void* id_out, int64_t nbytes) {
    TRLX_REQUIRE(g_api.lib, TRLX_ERR_ARG, "trlx_comm_load first");
    TRLX_REQUIRE(id_out && nbytes == kUniqueIdBytes, TRLX_ERR_ARG, "unique id buffer must be %d bytes",
                 kUniqueIdBytes);
    UniqueId id;
    const int rc = nccl_status(g_api.get_unique_id(&id), "ncclGetUniqueId");
    if (rc) return rc;
    memcpy(id_out, id.internal, kUniqueIdBytes);
    return TRLX_OK;
}

extern "C" int trlx_comm_init(void** comm_out, const void* id, int64_t nbytes, int nranks, int rank) {
    TRLX_REQUIRE(g_api.lib, TRLX_ERR_ARG, "trlx_comm_load first");
    TRLX_REQUIRE(comm_out && id && nbytes == kUniqueIdBytes, TRLX_ERR_ARG, "bad unique id");
    TRLX_REQUIRE(nranks > 0 && rank >= 0 && rank < nranks, TRLX_ERR_ARG, "bad rank %d of %d", rank, nranks);
    UniqueId uid;
    memcpy(uid.internal, id, kUniqueIdBytes);
    Comm c = nullptr;
    const int rc = nccl_status(g_api.comm_init_rank(&c, nranks, uid, rank), "ncclCommInitRank");
    if (rc) return rc;
    *comm_out = c;
    return TRLX_OK;
}

extern "C" int trlx_comm_allreduce_sum_f64(void* comm, double* buf, int64_t n, void* stream) {
    TRLX_REQUIRE(g_api.lib && comm, TRLX_ERR_ARG, "no communicator");
    TRLX_REQUIRE(buf && n > 0, TRLX_ERR_ARG, "empty all-reduce");
    return nccl_status(g_api.all_reduce(buf, buf, size_t(n), kNcclFloat64, kNcclSum, comm, (hipStream_t)stream),
                       "ncclAllReduce");
}

extern "C" int trlx_comm_destroy(void* comm) {
    TRLX_REQUIRE(g_api.lib, TRLX_ERR_ARG, "trlx_comm_load first");
    if (!comm) return TRLX_OK;
    return nccl_status(g_api.comm_destroy(comm), "ncclCommDestroy");
}
