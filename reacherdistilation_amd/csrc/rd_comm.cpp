// RCCL all-reduce on the trainer's stream (include/reacher_comm.h).
//
// RCCL is bound at run time: dlopen("librccl.so.1") first with RTLD_NOLOAD, which returns
// the copy torch already loaded (same SONAME), else loads it from the library path.  Only
// types come from <rccl/rccl.h>; nothing links against RCCL, so libreacher.so still loads
// (and its other entry points work) where RCCL is absent.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <chrono>
#include <mutex>
#include <new>
#include <thread>

#include "../../include/reacher.h"
#include "../../include/reacher_comm.h"
#include "rd_comm_impl.h"
#include "rd_common.h"

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRankConfig) init_rank_config = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommCount) count = nullptr;
    decltype(&ncclCommUserRank) user_rank = nullptr;
    decltype(&ncclCommCuDevice) cu_device = nullptr;
    bool ok = false;
    char why[256] = "";
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            snprintf(r.why, sizeof r.why, "librccl.so.1 not loadable: %s", dlerror());
            return;
        }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.init_rank_config = (decltype(r.init_rank_config))dlsym(h, "ncclCommInitRankConfig");
        r.async_error = (decltype(r.async_error))dlsym(h, "ncclCommGetAsyncError");
        r.abort = (decltype(r.abort))dlsym(h, "ncclCommAbort");
        r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
        r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        r.count = (decltype(r.count))dlsym(h, "ncclCommCount");
        r.user_rank = (decltype(r.user_rank))dlsym(h, "ncclCommUserRank");
        r.cu_device = (decltype(r.cu_device))dlsym(h, "ncclCommCuDevice");
        r.ok = r.get_unique_id && r.init_rank_config && r.async_error && r.abort && r.all_reduce && r.destroy &&
               r.error_string && r.count && r.user_rank && r.cu_device;
        if (!r.ok) snprintf(r.why, sizeof r.why, "librccl.so.1 lacks an nccl* entry point");
    });
    return r;
}

int nccl_fail(ncclResult_t e, const char* what) {
    return rd::set_error(RD_EINVAL, "%s: RCCL error %d (%s)", what, (int)e, rccl().error_string(e));
}

}  // namespace

namespace {

// The communicator is non-blocking (ncclConfig_t.blocking = 0): its creation, and a
// collective that still has connections to set up, return ncclInProgress and complete in
// the background.  Wait for that with a deadline; past it the communicator is aborted, so a
// rank whose peers never arrive fails with a message instead of hanging in RCCL.
int wait_ready(rd_comm* c, const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        ncclResult_t st = ncclInProgress;
        if (ncclResult_t e = rccl().async_error(c->comm, &st); e != ncclSuccess) return nccl_fail(e, what);
        if (st == ncclSuccess) return RD_OK;
        if (st != ncclInProgress) return nccl_fail(st, what);
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt > c->timeout_s)
            return rd::set_error(RD_EINVAL, "%s: rank %d of %d: the other ranks did not join within %.0f s", what,
                                 c->rank, c->nranks, c->timeout_s);
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

}  // namespace

extern "C" {

int rd_comm_unique_id(uint8_t* id) {
    if (!id) return rd::set_error(RD_EINVAL, "rd_comm_unique_id: null argument");
    const Rccl& r = rccl();
    if (!r.ok) return rd::set_error(RD_EINVAL, "rd_comm_unique_id: %s", r.why);
    ncclUniqueId u;
    if (ncclResult_t e = r.get_unique_id(&u); e != ncclSuccess) return nccl_fail(e, "ncclGetUniqueId");
    static_assert(sizeof(u) == RD_COMM_ID_BYTES, "RCCL unique id size");
    memcpy(id, &u, sizeof(u));
    return RD_OK;
}

int rd_comm_probe(int device) {
    const Rccl& r = rccl();
    if (!r.ok) return rd::set_error(RD_EINVAL, "rd_comm_probe: %s", r.why);
    int n = 0;
    RD_HIP(hipGetDeviceCount(&n), "rd_comm_probe: hipGetDeviceCount");
    if (device < 0 || device >= n) return rd::set_error(RD_EINVAL, "rd_comm_probe: no HIP device %d (%d visible)", device, n);
    rd::DeviceGuard g(device);
    RD_HIP(g.err, "rd_comm_probe: hipSetDevice");
    return RD_OK;
}

int rd_comm_create(rd_comm** out, const uint8_t* id, int nranks, int rank, int device, double timeout_s) {
    if (!out || !id || nranks <= 0 || rank < 0 || rank >= nranks || !(timeout_s > 0))
        return rd::set_error(RD_EINVAL, "rd_comm_create: bad argument");
    const Rccl& r = rccl();
    if (!r.ok) return rd::set_error(RD_EINVAL, "rd_comm_create: %s", r.why);
    rd::DeviceGuard g(device);
    RD_HIP(g.err, "rd_comm_create: hipSetDevice");
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    rd_comm* c = new (std::nothrow) rd_comm();
    if (!c) return rd::set_error(RD_EINVAL, "rd_comm_create: out of host memory");
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    c->timeout_s = timeout_s;
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t e = r.init_rank_config(&c->comm, nranks, u, rank, &cfg);
    int rc = (e == ncclSuccess || e == ncclInProgress) ? wait_ready(c, "ncclCommInitRankConfig")
                                                       : nccl_fail(e, "ncclCommInitRankConfig");
    if (rc != RD_OK) {
        if (c->comm) (void)r.abort(c->comm);
        delete c;
        return rc;
    }
    *out = c;
    return RD_OK;
}

int rd_comm_allreduce_f32(rd_comm* c, float* buf, int64_t n, void* hip_stream) {
    if (!c || !buf || n <= 0) return rd::set_error(RD_EINVAL, "rd_comm_allreduce_f32: bad argument");
    rd::DeviceGuard g(c->device);
    RD_HIP(g.err, "rd_comm_allreduce_f32: hipSetDevice");
    if (c->xgmi) return xgmi_allreduce(c, buf, n, (hipStream_t)hip_stream);
    ncclResult_t e = rccl().all_reduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, c->comm, (hipStream_t)hip_stream);
    if (e == ncclInProgress) return wait_ready(c, "ncclAllReduce");   // first use: connection setup
    if (e != ncclSuccess) return nccl_fail(e, "ncclAllReduce");
    return RD_OK;
}

int rd_comm_nranks(const rd_comm* c) { return c ? c->nranks : 0; }

int rd_comm_query(rd_comm* c, int* count, int* user_rank, int* device, int* from_rccl) {
    if (!c || !count || !user_rank || !device || !from_rccl) return rd::set_error(RD_EINVAL, "rd_comm_query: bad argument");
    if (c->xgmi || !c->comm) {   // the xGMI push has no RCCL communicator: what it was created with
        *count = c->nranks;
        *user_rank = c->rank;
        *device = c->device;
        *from_rccl = 0;
        return RD_OK;
    }
    if (int rc = wait_ready(c, "rd_comm_query")) return rc;
    const Rccl& r = rccl();
    if (ncclResult_t e = r.count(c->comm, count); e != ncclSuccess) return nccl_fail(e, "ncclCommCount");
    if (ncclResult_t e = r.user_rank(c->comm, user_rank); e != ncclSuccess) return nccl_fail(e, "ncclCommUserRank");
    if (ncclResult_t e = r.cu_device(c->comm, device); e != ncclSuccess) return nccl_fail(e, "ncclCommCuDevice");
    *from_rccl = 1;
    return RD_OK;
}

int rd_comm_destroy(rd_comm* c) {
    if (!c) return RD_OK;
    rd::DeviceGuard g(c->device);
    if (c->xgmi) xgmi_release(c);
    if (c->comm) {
        if (wait_ready(c, "rd_comm_destroy") == RD_OK) (void)rccl().destroy(c->comm);
        else (void)rccl().abort(c->comm);
    }
    delete c;
    return RD_OK;
}

}  // extern "C"
