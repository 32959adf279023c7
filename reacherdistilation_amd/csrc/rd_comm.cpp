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

#include <mutex>
#include <new>

#include "../../include/reacher.h"
#include "../../include/reacher_comm.h"
#include "rd_common.h"

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
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
        r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
        r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
        r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        r.ok = r.get_unique_id && r.init_rank && r.all_reduce && r.destroy && r.error_string;
        if (!r.ok) snprintf(r.why, sizeof r.why, "librccl.so.1 lacks an nccl* entry point");
    });
    return r;
}

int nccl_fail(ncclResult_t e, const char* what) {
    return rd::set_error(RD_EINVAL, "%s: RCCL error %d (%s)", what, (int)e, rccl().error_string(e));
}

}  // namespace

struct rd_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
};

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

int rd_comm_create(rd_comm** out, const uint8_t* id, int nranks, int rank, int device) {
    if (!out || !id || nranks <= 0 || rank < 0 || rank >= nranks)
        return rd::set_error(RD_EINVAL, "rd_comm_create: bad argument");
    const Rccl& r = rccl();
    if (!r.ok) return rd::set_error(RD_EINVAL, "rd_comm_create: %s", r.why);
    rd::DeviceGuard g(device);
    RD_HIP(g.err, "rd_comm_create: hipSetDevice");
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    rd_comm* c = new (std::nothrow) rd_comm();
    if (!c) return rd::set_error(RD_EINVAL, "rd_comm_create: out of host memory");
    if (ncclResult_t e = r.init_rank(&c->comm, nranks, u, rank); e != ncclSuccess) {
        delete c;
        return nccl_fail(e, "ncclCommInitRank");
    }
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    *out = c;
    return RD_OK;
}

int rd_comm_allreduce_f32(rd_comm* c, float* buf, int64_t n, void* hip_stream) {
    if (!c || !buf || n <= 0) return rd::set_error(RD_EINVAL, "rd_comm_allreduce_f32: bad argument");
    rd::DeviceGuard g(c->device);
    RD_HIP(g.err, "rd_comm_allreduce_f32: hipSetDevice");
    if (ncclResult_t e = rccl().all_reduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, c->comm, (hipStream_t)hip_stream);
        e != ncclSuccess)
        return nccl_fail(e, "ncclAllReduce");
    return RD_OK;
}

int rd_comm_nranks(const rd_comm* c) { return c ? c->nranks : 0; }

int rd_comm_destroy(rd_comm* c) {
    if (!c) return RD_OK;
    rd::DeviceGuard g(c->device);
    if (c->comm) (void)rccl().destroy(c->comm);
    delete c;
    return RD_OK;
}

}  // extern "C"
