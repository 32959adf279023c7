// The gradient all-reduce as ONE kernel that pushes over xGMI (include/reacher_comm.h,
// rd_xcomm_*): every rank owns an exchange buffer in uncached device memory, exported with
// hipIpcGetMemHandle and mapped by every other rank of the node.  Per exchange each rank
//   1. writes its n floats into slot[rank] of EVERY rank's buffer (block b -> rank b, so the
//      writes leave on all of the GPU's xGMI links at once; a 20 KB gradient is one burst),
//   2. fences (system scope) and raises flag[rank] = epoch in that rank's buffer,
//   3. waits until every flag in its own buffer shows the epoch, then
//   4. sums the nranks slots in rank order 0 .. nranks-1 into the gradient.
// Every rank adds the same numbers in the same order, so the replicas stay bitwise identical.
// The sums overwrite the gradient in place, so they wait until every block of the kernel has
// pushed it (a device counter): a block that reached its sums early would otherwise feed a
// slower block's push (found as diverging replicas after ~3,000 two-rank steps).
// One launch, no host round trip, no ring: for a latency-bound 20 KB message on a
// point-to-point xGMI mesh the one-shot push is the shortest path (RCCL's ring/tree pays
// 2(N-1) hops).  Slots and flags are double-buffered by epoch parity: a rank can only start
// exchange e+2 (same parity) after every rank raised its flag of e+1, which each raises only
// after it finished summing e, so no slot is overwritten while it is read.  A wait that does
// does not see a peer before its deadline (rd_xcomm_create's timeout_s, wall clock) FAILS
// the communicator: it raises the error words (device + host-visible), POISONS every rank's
// buffer (so a peer that arrives late fails its exchange too instead of completing it alone),
// and leaves the gradient as it was.  The blocks of one exchange kernel agree on ONE outcome
// before any in-place sum: each posts its verdict on a device counter after
// raising the failure word if it failed, and every block reads the failure word only once all
// verdicts are in, so the gradient is either fully summed or untouched.  The trainer's Adam
// kernel reads the device word and skips its update; rdd_step / rd_comm_check report it.
// Across ranks the outcome can still differ (a peer whose last flag lands just before this
// rank's deadline sums and steps while this rank skips): after RD_ECOMM the replicas must be
// re-synchronised from one rank before training goes on (reacher_comm.h;
// DistillTrainer.step checks and reports it).  A poisoned communicator fails every later
// exchange at once (destroy it, make a new one).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <new>

#include "../../include/reacher.h"
#include "../../include/reacher_comm.h"
#include "rd_comm_impl.h"
#include "rd_common.h"

namespace {

constexpr int XG_BLOCK = 256;
constexpr int XG_FLAGS_BYTES = 256;                 // flags[2][RD_XG_MAX] (uint32), the poison word, padded
constexpr int XG_POISON = 2 * RD_XG_MAX;            // uint32 index of the poison word in the flags area
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int XG_UNROLL = 8;                        // float4 per thread issued at once: n <= 8,192

struct XgArgs {
    char* buf[RD_XG_MAX];     // every rank's exchange buffer (mapped here)
    const char* mine;         // this rank's
    float* grad;              // in/out: this rank's n floats
    int64_t n, cap;
    int nranks, rank;
    int vec;                  // n >= 4 and grad 16-B aligned: the float4 push
    uint32_t epoch;
    uint64_t deadline_ticks;  // wall-clock limit of each wait, in s_memrealtime ticks (100 MHz)
    uint32_t* err;            // [0] this communicator failed, [1] blocks that finished pushing, [2] blocks
                              // that posted their verdict (both counted over all epochs)
    volatile uint32_t* herr;  // host-visible copy of err[0]
};

__device__ __forceinline__ uint32_t* flags_of(char* b, uint32_t parity) {
    return reinterpret_cast<uint32_t*>(b) + parity * RD_XG_MAX;
}
__device__ __forceinline__ uint32_t* poison_of(char* b) { return reinterpret_cast<uint32_t*>(b) + XG_POISON; }
__device__ __forceinline__ float* slot_of(char* b, int64_t cap, uint32_t parity, int r) {
    return reinterpret_cast<float*>(b + XG_FLAGS_BYTES) + ((int64_t)parity * RD_XG_MAX + r) * cap;
}

__device__ __forceinline__ bool poisoned(const XgArgs& a) {
    return __hip_atomic_load(poison_of(const_cast<char*>(a.mine)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
}

// this rank gives up: error words, and the poison word in every rank's buffer
__device__ void fail(const XgArgs& a) {
    __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    *a.herr = 1u;
    for (int r = 0; r < a.nranks; ++r)
        __hip_atomic_store(poison_of(a.buf[r]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
}

__global__ __launch_bounds__(XG_BLOCK) void xgmi_allreduce_kernel(XgArgs a) {
    const uint32_t par = a.epoch & 1u;
    const int dst = blockIdx.x;                       // one block per destination rank
    __shared__ int bad;
    if (threadIdx.x == 0) bad = poisoned(a) || __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (bad) {   // a peer (or this rank) failed an earlier exchange: fail this one, touch nothing
        if (threadIdx.x == 0) {
            fail(a);
            __hip_atomic_fetch_add(a.err + 2, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);   // verdict
        }
        return;
    }
    // 1. push: this rank's gradient -> slot[rank] of rank dst's buffer
    float* to = slot_of(a.buf[dst], a.cap, par, a.rank);
    if (a.vec) {   // every load is issued before the first store (clamped indices, no branch
        // around a load): a load -> store loop waited one memory latency per iteration
        const int n4 = (int)(a.n / 4);
        const f32x4* s4 = reinterpret_cast<const f32x4*>(a.grad);
        f32x4* t4 = reinterpret_cast<f32x4*>(to);
        f32x4 v[XG_UNROLL];   // a native vector type: HIP's float4 (a union) kept the array in scratch
#pragma unroll
        for (int u = 0; u < XG_UNROLL; ++u) {
            const int i = threadIdx.x + u * XG_BLOCK;
            v[u] = s4[i < n4 ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < XG_UNROLL; ++u) {   // no branch around a store either: on gfx9 the
            const int i = threadIdx.x + u * XG_BLOCK;   // store counter is vmcnt, and a store in a
            t4[i < n4 ? i : 0] = v[u];   // branch waited for every earlier one (one xGMI round
        }                                // trip each); past n4 a lane rewrites t4[0] = s4[0]
        for (int i = threadIdx.x + XG_UNROLL * XG_BLOCK; i < n4; i += XG_BLOCK) t4[i] = s4[i];   // n > 8,192
        for (int64_t i = 4 * (int64_t)n4 + threadIdx.x; i < a.n; i += XG_BLOCK) to[i] = a.grad[i];
    } else {       // n < 4 or a gradient that is not 16-B aligned
        for (int64_t i = threadIdx.x; i < a.n; i += XG_BLOCK) to[i] = a.grad[i];
    }
    __threadfence_system();   // every thread's stores have landed (acknowledged) ...
    __syncthreads();
    if (threadIdx.x == 0) {   // ... before the flag that publishes them
        __hip_atomic_store(flags_of(a.buf[dst], par) + a.rank, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        // and this block no longer reads the gradient: count it (the sums overwrite it in place)
        __hip_atomic_fetch_add(a.err + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    // 3. wait (a) until every block of this kernel has pushed (the in-place sums must not
    // reach a block's source) and (b) for every rank's slot in this rank's buffer; every wait
    // ends at the wall-clock deadline, or early once the buffer is poisoned
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == a.nranks) {
        const uint32_t want = a.epoch * (uint32_t)a.nranks;
        for (;;) {
            if ((int32_t)(__hip_atomic_load(a.err + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - want) >= 0)
                break;   // wrap-safe: the count passes 2^32 after ~5e8 exchanges
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.deadline_ticks || poisoned(a)) {
                bad = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (threadIdx.x < a.nranks) {
        const uint32_t* f = flags_of(const_cast<char*>(a.mine), par) + threadIdx.x;
        for (;;) {
            if (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == a.epoch) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.deadline_ticks || poisoned(a)) {
                bad = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // this block's verdict: its waits, or a peer that gave up on this exchange meanwhile;
        // a failing block raises the failure word BEFORE posting, then every block waits for
        // all verdicts and decides on the failure word alone -- one outcome per rank
        if (bad || poisoned(a)) fail(a);
        __hip_atomic_fetch_add(a.err + 2, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t want = a.epoch * (uint32_t)gridDim.x;
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        while ((int32_t)(__hip_atomic_load(a.err + 2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
            if (__builtin_amdgcn_s_memrealtime() - t1 > a.deadline_ticks) {   // (cannot happen: every
                fail(a);                                                      // block posts; bounded anyway)
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        bad = __hip_atomic_load(a.err, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    }
    __syncthreads();
    if (bad) return;   // the gradient keeps its input; the Adam kernel sees err[0] and skips
    __threadfence_system();
    // 4. this block's share of the columns: the sum over ranks in rank order
    const int64_t per = (a.n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = per * blockIdx.x, hi = lo + per < a.n ? lo + per : a.n;
    char* me = const_cast<char*>(a.mine);
    for (int64_t i = lo + threadIdx.x; i < hi; i += XG_BLOCK) {
        float v[RD_XG_MAX];   // all ranks' values in flight at once (uncached: HBM latency each)
#pragma unroll
        for (int r = 0; r < RD_XG_MAX; ++r) v[r] = slot_of(me, a.cap, par, r < a.nranks ? r : 0)[i];
        float s = v[0];
#pragma unroll
        for (int r = 1; r < RD_XG_MAX; ++r) s = r < a.nranks ? s + v[r] : s;   // rank order
        a.grad[i] = s;
    }
}

}  // namespace

int xgmi_allreduce(rd_comm* c, float* buf, int64_t n, hipStream_t stream) {
    if (rd_comm_failed(c))
        return rd::set_error(RD_ECOMM, "rd_comm_allreduce_f32: rank %d: the exchange failed earlier (a peer did not "
                                       "arrive within %.1f s); destroy the communicator", c->rank, c->timeout_s);
    if (n > c->cap) return rd::set_error(RD_EINVAL, "rd_comm_allreduce_f32: %lld floats > the exchange slots' %lld",
                                         (long long)n, (long long)c->cap);
    for (int r = 0; r < c->nranks; ++r)
        if (!c->peer[r]) return rd::set_error(RD_EINVAL, "rd_comm_allreduce_f32: rd_xcomm_connect has not run");
    XgArgs a;
    for (int r = 0; r < RD_XG_MAX; ++r) a.buf[r] = r < c->nranks ? c->peer[r] : nullptr;
    a.mine = c->mine;
    a.grad = buf;
    a.n = n;
    a.cap = c->cap;
    a.nranks = c->nranks;
    a.rank = c->rank;
    a.vec = n >= 4 && ((uintptr_t)buf & 15u) == 0;
    a.epoch = ++c->epoch;
    a.deadline_ticks = (uint64_t)(c->timeout_s * 1e8);   // s_memrealtime: 100 MHz
    a.err = c->err;
    a.herr = c->herr;
    hipLaunchKernelGGL(xgmi_allreduce_kernel, dim3(c->nranks), dim3(XG_BLOCK), 0, stream, a);
    RD_HIP(hipGetLastError(), "xgmi_allreduce_kernel launch");
    return RD_OK;
}

void xgmi_release(rd_comm* c) {
    for (int r = 0; r < RD_XG_MAX; ++r) {
        if (c->peer[r] && c->peer[r] != c->mine) (void)hipIpcCloseMemHandle(c->peer[r]);
        c->peer[r] = nullptr;
    }
    if (c->mine) (void)hipFree(c->mine);
    if (c->err) (void)hipFree(c->err);
    if (c->herr) (void)hipHostFree((void*)c->herr);
    c->mine = nullptr;
    c->err = nullptr;
    c->herr = nullptr;
}

extern "C" {

int rd_xcomm_create(rd_comm** out, int nranks, int rank, int device, int64_t cap, double timeout_s, uint8_t* handle) {
    if (!out || !handle || nranks <= 0 || nranks > RD_XG_MAX || rank < 0 || rank >= nranks || cap <= 0 ||
        !(timeout_s > 0 && timeout_s < 1e6))
        return rd::set_error(RD_EINVAL, "rd_xcomm_create: bad argument (at most %d ranks)", RD_XG_MAX);
    rd::DeviceGuard g(device);
    RD_HIP(g.err, "rd_xcomm_create: hipSetDevice");
    rd_comm* c = new (std::nothrow) rd_comm();
    if (!c) return rd::set_error(RD_EINVAL, "rd_xcomm_create: out of host memory");
    c->xgmi = 1;
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    c->timeout_s = timeout_s;
    c->cap = (cap + 3) / 4 * 4;   // 16-B aligned slots
    const size_t bytes = XG_FLAGS_BYTES + sizeof(float) * 2 * RD_XG_MAX * (size_t)c->cap;
    static_assert((XG_POISON + 1) * sizeof(uint32_t) <= XG_FLAGS_BYTES, "flag words");
    hipError_t e = hipExtMallocWithFlags((void**)&c->mine, bytes, hipDeviceMallocUncached);
    if (e == hipSuccess) e = hipMemset(c->mine, 0, bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&c->err, 4 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(c->err, 0, 4 * sizeof(uint32_t));
    void* hp = nullptr;   // pinned, coherent host word the kernel raises on failure
    if (e == hipSuccess) e = hipHostMalloc(&hp, sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) {
        c->herr = (volatile uint32_t*)hp;
        *c->herr = 0u;
    }
    hipIpcMemHandle_t h;
    if (e == hipSuccess) e = hipIpcGetMemHandle(&h, c->mine);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        xgmi_release(c);
        delete c;
        return rd::hip_fail(e, "rd_xcomm_create");
    }
    static_assert(sizeof(h) == RD_XCOMM_HANDLE_BYTES, "IPC handle size");
    memcpy(handle, &h, sizeof(h));
    c->peer[rank] = c->mine;
    *out = c;
    return RD_OK;
}

int rd_xcomm_connect(rd_comm* c, const uint8_t* handles) {
    if (!c || !c->xgmi || !handles) return rd::set_error(RD_EINVAL, "rd_xcomm_connect: bad argument");
    rd::DeviceGuard g(c->device);
    RD_HIP(g.err, "rd_xcomm_connect: hipSetDevice");
    for (int r = 0; r < c->nranks; ++r) {
        if (r == c->rank || c->peer[r]) continue;
        hipIpcMemHandle_t h;
        memcpy(&h, handles + (size_t)r * RD_XCOMM_HANDLE_BYTES, sizeof(h));
        void* p = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) return rd::set_error(-(int)e, "rd_xcomm_connect: rank %d cannot map rank %d's buffer: %s",
                                                  c->rank, r, hipGetErrorString(e));
        c->peer[r] = (char*)p;
    }
    return RD_OK;
}

int rd_comm_check(rd_comm* c) {
    if (!c) return rd::set_error(RD_EINVAL, "rd_comm_check: null handle");
    if (!c->xgmi) return RD_OK;
    if (rd_comm_failed(c))
        return rd::set_error(RD_ECOMM, "rd_comm_check: rank %d: an exchange failed (a peer did not arrive within "
                                       "%.1f s, or a peer failed first); its optimiser step was skipped", c->rank,
                             c->timeout_s);
    return RD_OK;
}

}  // extern "C"
