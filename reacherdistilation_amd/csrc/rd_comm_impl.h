// The communicator behind include/reacher_comm.h: an RCCL communicator (rd_comm.cpp) or the
// xGMI one-shot push exchange (rd_xgmi.hip).  Internal to libreacher.so.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>

constexpr int RD_XG_MAX = 8;   // ranks of one node

struct rd_comm {
    ncclComm_t comm = nullptr;   // RCCL (kind 0)
    int nranks = 0, rank = 0, device = 0;
    double timeout_s = 60.0;
    // xGMI push exchange (kind 1): every rank's exchange buffer mapped into this process
    int xgmi = 0;
    int64_t cap = 0;                  // floats per slot
    char* mine = nullptr;             // this rank's buffer (uncached device memory)
    char* peer[RD_XG_MAX] = {};       // every rank's buffer (peer[rank] = mine)
    uint32_t epoch = 0;               // exchanges issued so far
    uint32_t* err = nullptr;          // device words: [0] an exchange failed, [1] blocks that pushed
    volatile uint32_t* herr = nullptr;   // host-visible copy of err[0] (pinned): read without a sync
};

// Device word that is nonzero once an exchange of `c` failed (the trainer's Adam kernel skips
// its update when it is set), or null for a communicator that cannot fail that way (RCCL).
inline const uint32_t* rd_comm_device_err(const rd_comm* c) { return c && c->xgmi ? c->err : nullptr; }
// Nonzero once an exchange of `c` failed (host read, no synchronisation).
inline int rd_comm_failed(const rd_comm* c) { return c && c->herr && *c->herr ? 1 : 0; }

// rd_xgmi.hip
int xgmi_allreduce(rd_comm* c, float* buf, int64_t n, hipStream_t stream);
void xgmi_release(rd_comm* c);
