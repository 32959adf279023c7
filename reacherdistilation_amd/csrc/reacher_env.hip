// Batched Reacher-v2 env kernels for gfx950 + the rd_* C ABI (include/reacher.h).
//
// Drop-in for the reference's env object (gym ReacherEnv + TimeLimit(50), MuJoCo 1.50):
//   env.reset()  reference mlp_train.py:112,138,200   -> rd_reset
//   env.step(a)  reference mlp_train.py:135,196       -> rd_step
// HBM layout: state SoA [8][N] f32 (one row per field, env on the fastest axis) so one
// lane = one env and every state load/store is a fully coalesced dword stream.  obs
// [N][11] (gym layout) is written through an LDS transpose as 16-B stores.
// Algorithmic bytes per env-step (rd_step): read act 8 + q,v 16 + target 8 + held
// fingertip offset 8 = 40; write q,v 16 + offset 8 + obs 44 + rew 4 + done 1 = 73
// -> 113 B.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <new>

#include "../../include/reacher.h"
#include "rd_common.h"
#include "rd_physics.h"

namespace {

constexpr int kBlock = 256;

// The step's outputs (state, obs, rew, done) are written once per step and read by a later
// kernel, so they are stored non-temporal: +1 % at 16.8M envs, +3.5 % at 4.2M, +4.5 % at 1M
// against plain stores (profiles/r03n_env_nt.txt; same bits).
template <class T> __device__ __forceinline__ void ost(T* p, T v) { __builtin_nontemporal_store(v, p); }
template <class T> __device__ __forceinline__ T ild(const T* p) { return *p; }

struct ResetSrc {
    int mode;              // RD_RESET_PHILOX / RD_RESET_TABLE
    const float* table;    // [n_episodes][N][6]
    int32_t n_episodes;
    uint64_t seed;
    int64_t env_base;
};

__device__ __forceinline__ void draw_reset(const ResetSrc& src, int64_t n, int64_t i, int32_t episode,
                                           float d[6]) {
    if (src.mode == RD_RESET_TABLE) {
        const float* p = src.table + ((int64_t)episode * n + i) * 6;
#pragma unroll
        for (int k = 0; k < 6; ++k) d[k] = p[k];
    } else {
        rd::philox_draw(src.seed, (uint64_t)(src.env_base + i), (uint32_t)episode, d);
    }
}

__device__ __forceinline__ rd::State load_state(const float* __restrict__ s, int64_t n, int64_t i) {
    rd::State st;
    st.q0 = ild(s + 0 * n + i); st.q1 = ild(s + 1 * n + i); st.v0 = ild(s + 2 * n + i); st.v1 = ild(s + 3 * n + i);
    st.tx = ild(s + 4 * n + i); st.ty = ild(s + 5 * n + i); st.dx = ild(s + 6 * n + i); st.dy = ild(s + 7 * n + i);
    return st;
}

__device__ __forceinline__ void store_state(float* __restrict__ s, int64_t n, int64_t i, const rd::State& st,
                                            bool target_too) {
    ost(s + 0 * n + i, st.q0); ost(s + 1 * n + i, st.q1); ost(s + 2 * n + i, st.v0); ost(s + 3 * n + i, st.v1);
    if (target_too) { ost(s + 4 * n + i, st.tx); ost(s + 5 * n + i, st.ty); }
    ost(s + 6 * n + i, st.dx); ost(s + 7 * n + i, st.dy);
}

// Write this block's obs rows [base, base+cnt) x 11 via an LDS transpose: lane-strided
// 44-B rows become contiguous 16-B stores (the block's rows start 16-B aligned because
// base is a multiple of 256).
__device__ __forceinline__ void write_obs(float* __restrict__ obs, int64_t base, int cnt, const float ob[11],
                                          float* lds) {
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 11; ++k) lds[t * 11 + k] = ob[k];   // stride 11: conflict-free
    __syncthreads();
    float* dst = obs + base * 11;
    if (cnt == kBlock) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        const v4f* src4 = reinterpret_cast<const v4f*>(lds);
        v4f* dst4 = reinterpret_cast<v4f*>(dst);
        for (int j = t; j < kBlock * 11 / 4; j += kBlock) ost(dst4 + j, src4[j]);
    } else {
        for (int j = t; j < cnt * 11; j += kBlock) ost(dst + j, lds[j]);
    }
}

__global__ __launch_bounds__(kBlock) void rd_reset_kernel(int64_t n, float* __restrict__ state,
                                                          float* __restrict__ obs, ResetSrc src,
                                                          int32_t episode) {
    __shared__ float lds[kBlock * 11];
    const int64_t base = (int64_t)blockIdx.x * kBlock;
    const int64_t i = base + threadIdx.x;
    const int cnt = (int)min((int64_t)kBlock, n - base);
    float ob[11];
    if (i < n) {
        float d[6];
        draw_reset(src, n, i, episode, d);
        rd::State st;
        rd::env_reset(st, d);
        store_state(state, n, i, st, true);
        rd::observe(st, ob);
    }
    write_obs(obs, base, cnt, ob, lds);
}

// One lockstep env.step.  done_step: this step ends the episode (TimeLimit 50) -> the
// env auto-resets from reset draw `next_episode` and obs holds the reset observation.
__global__ __launch_bounds__(kBlock) void rd_step_kernel(int64_t n, float* __restrict__ state,
                                                         const float* __restrict__ act,
                                                         float* __restrict__ obs, float* __restrict__ rew,
                                                         uint8_t* __restrict__ done, int done_step,
                                                         ResetSrc src, int32_t next_episode) {
    __shared__ float lds[kBlock * 11];
    const int64_t base = (int64_t)blockIdx.x * kBlock;
    const int64_t i = base + threadIdx.x;
    const int cnt = (int)min((int64_t)kBlock, n - base);
    float ob[11];
    if (i < n) {
        rd::State st = load_state(state, n, i);
        typedef float v2f __attribute__((ext_vector_type(2)));
        const v2f a = ild(reinterpret_cast<const v2f*>(act) + i);
        const float r = rd::env_step(st, a[0], a[1]);
        if (done_step) {
            float d[6];
            draw_reset(src, n, i, next_episode, d);
            rd::env_reset(st, d);
        }
        store_state(state, n, i, st, done_step != 0);
        rd::observe(st, ob);
        ost(rew + i, r);
        ost(done + i, (uint8_t)(done_step != 0));
    }
    write_obs(obs, base, cnt, ob, lds);
}

}  // namespace

struct rd_env {
    int64_t n = 0, env_base = 0;
    uint64_t seed = 0;
    int device = 0;
    hipStream_t stream = nullptr;
    float* state = nullptr;          // [8][n]
    int32_t step = 0;                // steps taken in the current episode
    int32_t episode = -1;            // index of the current episode's reset draw
    int reset_mode = RD_RESET_PHILOX;
    const float* table = nullptr;
    int32_t n_table = 0;
};

static ResetSrc make_src(const rd_env* e) {
    ResetSrc s;
    s.mode = e->reset_mode;
    s.table = e->table;
    s.n_episodes = e->n_table;
    s.seed = e->seed;
    s.env_base = e->env_base;
    return s;
}

static unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

extern "C" {

const char* rd_last_error(void) { return rd::last_error_buf(); }

const char* rd_version(void) { return "libreacher gfx950 env v1 (rk4 f32, philox/gym resets)"; }

int rd_create(rd_env** out, int64_t n_envs, int64_t env_base, uint64_t seed, int device, void* hip_stream) {
    if (!out || n_envs <= 0 || env_base < 0) return rd::set_error(RD_EINVAL, "rd_create: bad argument");
    if (n_envs > ((int64_t)1 << 31)) return rd::set_error(RD_EINVAL, "rd_create: n_envs too large");
    rd::DeviceGuard g(device);
    RD_HIP(g.err, "rd_create: hipSetDevice");
    rd_env* e = new (std::nothrow) rd_env();
    if (!e) return rd::set_error(RD_EINVAL, "rd_create: out of host memory");
    e->n = n_envs;
    e->env_base = env_base;
    e->seed = seed;
    e->device = device;
    e->stream = (hipStream_t)hip_stream;
    hipError_t err = hipMalloc(&e->state, sizeof(float) * rd::kStateDim * n_envs);
    if (err != hipSuccess) {
        delete e;
        return rd::hip_fail(err, "rd_create: hipMalloc(state)");
    }
    *out = e;
    return RD_OK;
}

int rd_set_stream(rd_env* e, void* hip_stream) {
    if (!e) return rd::set_error(RD_EINVAL, "rd_set_stream: null handle");
    e->stream = (hipStream_t)hip_stream;
    return RD_OK;
}

int rd_destroy(rd_env* e) {
    if (!e) return RD_OK;
    rd::DeviceGuard g(e->device);
    if (e->state) (void)hipFree(e->state);
    delete e;
    return RD_OK;
}

static int check_table(const rd_env* e, int32_t episode) {
    if (e->reset_mode == RD_RESET_TABLE && (episode < 0 || episode >= e->n_table))
        return rd::set_error(RD_EINVAL, "reset table exhausted: episode %d of %d draws", episode, e->n_table);
    return RD_OK;
}

int rd_reset(rd_env* e, float* obs) {
    if (!e || !obs) return rd::set_error(RD_EINVAL, "rd_reset: null argument");
    const int32_t ep = e->episode + 1;
    if (int rc = check_table(e, ep)) return rc;
    rd::DeviceGuard g(e->device);
    RD_HIP(g.err, "rd_reset: hipSetDevice");
    hipLaunchKernelGGL(rd_reset_kernel, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->n, e->state,
                       obs, make_src(e), ep);
    RD_HIP(hipGetLastError(), "rd_reset: launch");
    e->episode = ep;
    e->step = 0;
    return RD_OK;
}

int rd_step(rd_env* e, const float* act, float* obs, float* rew, uint8_t* done) {
    if (!e || !act || !obs || !rew || !done) return rd::set_error(RD_EINVAL, "rd_step: null argument");
    if (e->episode < 0) return rd::set_error(RD_EINVAL, "rd_step: env needs reset before step");
    const int done_step = (e->step + 1 >= rd::kEpisodeSteps) ? 1 : 0;
    const int32_t next_ep = e->episode + 1;
    if (done_step)
        if (int rc = check_table(e, next_ep)) return rc;
    rd::DeviceGuard g(e->device);
    RD_HIP(g.err, "rd_step: hipSetDevice");
    hipLaunchKernelGGL(rd_step_kernel, dim3(grid_for(e->n)), dim3(kBlock), 0, e->stream, e->n, e->state, act,
                       obs, rew, done, done_step, make_src(e), next_ep);
    RD_HIP(hipGetLastError(), "rd_step: launch");
    if (done_step) {
        e->episode = next_ep;
        e->step = 0;
    } else {
        e->step += 1;
    }
    return RD_OK;
}

int rd_set_state(rd_env* e, const float* state, int32_t step, int32_t episode) {
    if (!e || !state || step < 0 || step >= rd::kEpisodeSteps || episode < 0)
        return rd::set_error(RD_EINVAL, "rd_set_state: bad argument");
    rd::DeviceGuard g(e->device);
    RD_HIP(g.err, "rd_set_state: hipSetDevice");
    RD_HIP(hipMemcpyAsync(e->state, state, sizeof(float) * rd::kStateDim * e->n, hipMemcpyDeviceToDevice,
                          e->stream),
           "rd_set_state: copy");
    e->step = step;
    e->episode = episode;
    return RD_OK;
}

int rd_get_state(rd_env* e, float* state, int32_t* step, int32_t* episode) {
    if (!e || !state) return rd::set_error(RD_EINVAL, "rd_get_state: null argument");
    rd::DeviceGuard g(e->device);
    RD_HIP(g.err, "rd_get_state: hipSetDevice");
    RD_HIP(hipMemcpyAsync(state, e->state, sizeof(float) * rd::kStateDim * e->n, hipMemcpyDeviceToDevice,
                          e->stream),
           "rd_get_state: copy");
    if (step) *step = e->step;
    if (episode) *episode = e->episode;
    return RD_OK;
}

int rd_set_reset_mode(rd_env* e, int mode, const float* draws, int32_t n_episodes) {
    if (!e) return rd::set_error(RD_EINVAL, "rd_set_reset_mode: null handle");
    if (mode == RD_RESET_PHILOX) {
        e->reset_mode = mode;
        e->table = nullptr;
        e->n_table = 0;
        return RD_OK;
    }
    if (mode == RD_RESET_TABLE && draws && n_episodes > 0) {
        e->reset_mode = mode;
        e->table = draws;
        e->n_table = n_episodes;
        return RD_OK;
    }
    return rd::set_error(RD_EINVAL, "rd_set_reset_mode: bad mode/table");
}

}  // extern "C"
