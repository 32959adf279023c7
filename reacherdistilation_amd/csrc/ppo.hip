// PPO training of the teacher on batched Reacher-v2 (include/reacher_ppo.h), for gfx950:
// the reference's baselines ppo1 pposgd_simple.learn (teacher.py:23-37) over n_envs
// parallel envs.
//
// MI355X mapping:
//  * rollout: 32 envs per workgroup for the whole horizon, one per lane of wave 0 (the
//    shared Reacher physics of rd_physics.h, noise, episode clocks); the 32 envs' policy and
//    value MLPs (2 x 64 tanh each) run on f32 MFMA by all four waves with the weights in LDS;
//    the actor batch (ob, ac, vpred, rew, new) is written t-major so every later pass is
//    coalesced;
//  * GAE: one env per lane, backward over its horizon; the advantage moments and the
//    observation filter's sums are deterministic two-level f64 reductions;
//  * minibatch step, two launches: minibatch_kernel gathers a 32-row tile (filter applied)
//    and runs both MLPs forward, the clipped surrogate + value loss per row and both
//    backward passes with the weights in LDS, each workgroup keeping its weight-gradient
//    sums in registers over its tiles; reduce_adam_kernel sums the per-workgroup partial rows
//    in a fixed order and runs TF1/MpiAdam over the concatenated [pol | vf] vector.  No
//    atomics: deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <new>
#include <random>
#include <vector>

#include "../../include/reacher_ppo.h"
#include "rd_common.h"
#include "rd_physics.h"

namespace {

constexpr int OBD = 11, HID = 64, ZLD = 16;
// LDS row strides of the minibatch tiles: inputs z [row][ZLD] with column OBD = 1 (the bias
// input of dW1) and columns 12-15 = 0 (the MFMA's 16-row dW1 block), activations [row][HLD]
constexpr int HLD = HID + 4;
// policy (MlpPolicy layout of reacher_distill.h)
constexpr int PW1 = 0, PB1 = PW1 + OBD * HID, PW2 = PB1 + HID, PB2 = PW2 + HID * HID, PW3 = PB2 + HID,
              PB3 = PW3 + HID * 2, PLS = PB3 + 2, P_POL = PLS + 2;
// value net, after the policy in the combined vector
constexpr int VB = P_POL;
constexpr int VW1 = 0, VC1 = VW1 + OBD * HID, VW2 = VC1 + HID, VC2 = VW2 + HID * HID, VW3 = VC2 + HID,
              VC3 = VW3 + HID, P_VF = VC3 + 1;
constexpr int P_ALL = P_POL + P_VF;
static_assert(P_POL == RDP_POLICY_PARAMS && P_VF == RDP_VALUE_PARAMS, "layouts");
static_assert(VB % 4 == 0 && PW2 % 4 == 0 && PW3 % 4 == 0 && (VB + VW2) % 4 == 0 && (VB + VW3) % 4 == 0,
              "16-B aligned weight matrices");
constexpr int N_MET = RDP_METRICS;
constexpr int RB = 256;                 // reduction block
constexpr float LOG2PI = 1.8378770664093453f;

__device__ __forceinline__ float clip5(float x) { return fminf(fmaxf(x, -5.0f), 5.0f); }

// filter statistics as the policy graph uses them (mpi_running_mean_std: float32 mean/std)
__global__ void rms_finalize_kernel(const double* s, float* rms) {
    const int k = threadIdx.x;
    if (k >= OBD) return;
    const double cnt = s[2 * OBD];
    const float mean = (float)(s[k] / cnt);
    const float var = (float)(s[OBD + k] / cnt) - mean * mean;
    rms[k] = mean;
    rms[OBD + k] = sqrtf(fmaxf(var, 1e-2f));
}

struct RolloutArgs {
    int64_t n, env_base;
    int T;
    uint64_t seed;
    uint32_t iter;
    const float* params;   // [P_ALL]
    const float* rms;      // [22]
    float* state;          // [8][n]
    int* ep_step;
    int* ep_idx;
    float* ep_ret;
    float* new_next;       // [n] 1 if the env's next observation starts an episode
    float* it_ret;         // [n] returns of episodes completed this iteration
    float* it_eps;         // [n]
    float *ob, *ac, *vpred, *rew, *newf, *nextv;
};

// block sums of up to 4 per-thread f64 values into part[blockIdx][4] (fixed-order tree)
__device__ __forceinline__ void block_sum4(double v0, double v1, double v2, double v3, double* part) {
    __shared__ double s[4][RB];
    s[0][threadIdx.x] = v0; s[1][threadIdx.x] = v1; s[2][threadIdx.x] = v2; s[3][threadIdx.x] = v3;
    __syncthreads();
    for (int w = RB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
#pragma unroll
            for (int q = 0; q < 4; ++q) s[q][threadIdx.x] += s[q][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < 4) part[blockIdx.x * 4 + threadIdx.x] = s[threadIdx.x][0];
}

// GAE(lambda) per env (add_vtarg_and_adv), + per-block sums of adv, adv^2, episode returns
__global__ __launch_bounds__(RB) void gae_kernel(int64_t n, int T, float gamma, float lam, const float* rew,
                                                 const float* vpred, const float* newf, const float* nextv,
                                                 const float* it_ret, const float* it_eps, float* adv, float* ret,
                                                 double* part) {
    const int64_t e = (int64_t)blockIdx.x * RB + threadIdx.x;
    double sa = 0.0, sq = 0.0, er = 0.0, ec = 0.0;
    if (e < n) {
        float last = 0.0f, vnext = nextv[e], nonterm = 1.0f;   // new[T] := 0 (baselines)
        for (int t = T - 1; t >= 0; --t) {
            const int64_t r = (int64_t)t * n + e;
            const float delta = rew[r] + gamma * vnext * nonterm - vpred[r];
            last = delta + gamma * lam * nonterm * last;
            adv[r] = last;
            ret[r] = last + vpred[r];
            sa += last;
            sq += (double)last * last;
            vnext = vpred[r];
            nonterm = 1.0f - newf[r];
        }
        er = it_ret[e];
        ec = it_eps[e];
    }
    block_sum4(sa, sq, er, ec, part);
}

// fixed-order sum of `nblk` x 4 partials -> out[0..3]
__global__ void sum_parts_kernel(const double* part, int nblk, double* out) {
    __shared__ double s[4][RB];
    double a[4] = {0, 0, 0, 0};
    for (int b = threadIdx.x; b < nblk; b += RB)
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] += part[b * 4 + q];
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q][threadIdx.x] = a[q];
    __syncthreads();
    for (int w = RB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
#pragma unroll
            for (int q = 0; q < 4; ++q) s[q][threadIdx.x] += s[q][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < 4) out[threadIdx.x] = s[threadIdx.x][0];
}

// atarg = (adv - mean) / std (population std)
__global__ __launch_bounds__(256) void standardize_kernel(const float* adv, int64_t S, const double* stats,
                                                          float* atarg) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= S) return;
    const double mean = stats[0] / (double)S;
    const double var = stats[1] / (double)S - mean * mean;
    atarg[r] = (float)((adv[r] - mean) / sqrt(var > 0 ? var : 0.0));
}

// observation-filter sums of the batch: per block f64 sums of ob[k], ob[k]^2 (k < 11)
__global__ __launch_bounds__(RB) void ob_sums_kernel(const float* ob, int64_t S, double* part) {
    __shared__ double s[2 * OBD][RB];
    const int64_t r0 = (int64_t)blockIdx.x * RB * 8;
    double a[2 * OBD];
#pragma unroll
    for (int k = 0; k < 2 * OBD; ++k) a[k] = 0.0;
    for (int q = 0; q < 8; ++q) {
        const int64_t r = r0 + q * RB + threadIdx.x;
        if (r < S)
#pragma unroll
            for (int k = 0; k < OBD; ++k) {
                const double x = ob[r * OBD + k];
                a[k] += x;
                a[OBD + k] += x * x;
            }
    }
#pragma unroll
    for (int k = 0; k < 2 * OBD; ++k) s[k][threadIdx.x] = a[k];
    __syncthreads();
    for (int w = RB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
#pragma unroll
            for (int k = 0; k < 2 * OBD; ++k) s[k][threadIdx.x] += s[k][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < 2 * OBD) part[blockIdx.x * 2 * OBD + threadIdx.x] = s[threadIdx.x][0];
}

// RunningMeanStd.update: sums += fixed-order sum of the partials, count += S
__global__ void rms_update_kernel(const double* part, int nblk, int64_t S, double* sums) {
    const int k = threadIdx.x;
    if (k < 2 * OBD) {
        double a = 0.0;
        for (int b = 0; b < nblk; ++b) a += part[b * 2 * OBD + k];
        sums[k] += a;
    }
    if (k == 0) sums[2 * OBD] += (double)S;
}

// old policy's log-probabilities (pi frozen, filter already updated: pposgd_simple order)

// ---- the minibatch step: two launches --------------------------------------------------
// minibatch_kernel: workgroup b owns the row tiles b, b + G, b + 2G, ... of MB_R rows: it
// gathers a tile (filter applied), runs both MLPs forward, the clipped surrogate + value
// loss per row and both backward passes with the weights in LDS, and keeps its share of the
// weight-gradient sums in registers across its tiles; at the end it writes one partial
// gradient row in the flat [pol | vf] layout, plus its loss sums in f64.
// reduce_adam_kernel: fixed-order column sums of the G partial rows -> grad, then Adam.
// The old path (gather, 11 grouped GEMMs, loss, loss sums, Adam: 15 dependent launches per
// minibatch) was latency-bound.  The GEMM-shaped parts of a tile (layers 1-2 forward, the
// layer-2 data gradient, dW2, dW1) run on v_mfma_f32_16x16x4_f32 (exact f32 products; a
// VALU form with broadcast LDS operands measured 10 + 13 us per tile for layer 2 alone).
constexpr int MB_R = 32;                   // rows per tile
constexpr int MB_H = MB_R / 2;             // rows per wave in the forward / data-gradient phases
constexpr int MB_G = 256;                  // at most this many workgroups (= partial rows)
constexpr int W2LD = HID + 4;              // LDS row stride of W2 (B operands read both ways)
constexpr int PSTR = (P_ALL + 3) & ~3;     // partial row stride (floats)
constexpr int NSTAT = 8;                   // f64 per workgroup: pol_surr, vf_loss, clipfrac, dlogstd0, dlogstd1
constexpr int RA_COLS = 16, RA_SLICES = 16;   // reduce_adam: 16 columns x 16 row slices per block (32 x 8: +4 %, 64 x 4: +19 %)
static_assert(RA_COLS * RA_SLICES == 256 && (RA_SLICES & (RA_SLICES - 1)) == 0, "256 threads, power-of-two slices");
static_assert(MB_R == 32 && HID == 64 && PB1 == OBD * HID && VC1 == OBD * HID,
              "two 16-row MFMA blocks per tile; b1 follows W1");

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// tanh as 1 - 2 / (e^{2|x|} + 1) with the sign of x: v_exp + v_rcp (|error| < 3e-7)
__device__ __forceinline__ float tanh_fast(float x) {
    const float t = 1.0f - __fdividef(2.0f, __expf(2.0f * fabsf(x)) + 1.0f);
    return copysignf(t, x);
}

struct MbArgs {
    const int* perm;                        // the minibatch's rows of the actor batch
    int mb;
    const float *params, *rms, *ob, *ac, *lpo, *atarg, *ret;
    float clip_eps;
    float* part;                            // [G][PSTR]
    double* stat;                           // [G][NSTAT]
    uint32_t* ctl;
};

struct MbLds {
    alignas(16) float w1[2][(OBD + 1) * HID];   // W1 rows, then b1 as row OBD (the ones column of z)
    alignas(16) float w2[2][HID * W2LD];
    alignas(16) float b2[2][HID];
    alignas(16) float w3p[HID * 2];
    alignas(16) float w3v[HID];
    float b3[4];                            // policy b3[0..1], value c3, -
    float ls[2];                            // logstd
    float rm[2 * OBD];                      // filter mean | std
    alignas(16) float z[MB_R][ZLD];         // column OBD = 1: the bias input of dW1
    alignas(16) float h1[2][MB_R][HLD];
    alignas(16) float h2[2][MB_R][HLD];
    alignas(16) float d2[2][MB_R][HLD];
    alignas(16) float d1[2][MB_R][HLD];
    float dm[MB_R][2];
    float dv[MB_R];
    float v[MB_R];                          // rollout: the value head's output
    double red[5][64];
};

// parameter i of the flat [pol | vf] vector -> its LDS slot (W2 rows padded to W2LD)
__device__ __forceinline__ float* mb_slot(MbLds& L, int i) {
    if (i < VB) {
        if (i < PW2) return &L.w1[0][i];        // W1 | b1 (PB1 = 11 x 64)
        if (i < PB2) return &L.w2[0][((i - PW2) >> 6) * W2LD + ((i - PW2) & 63)];
        if (i < PW3) return &L.b2[0][i - PB2];
        if (i < PB3) return &L.w3p[i - PW3];
        if (i < PLS) return &L.b3[i - PB3];
        return &L.ls[i - PLS];
    }
    const int o = i - VB;
    if (o < VW2) return &L.w1[1][o];
    if (o < VC2) return &L.w2[1][((o - VW2) >> 6) * W2LD + ((o - VW2) & 63)];
    if (o < VW3) return &L.b2[1][o - VC2];
    if (o < VC3) return &L.w3v[o - VW3];
    return &L.b3[2];
}

// all parameters into LDS, all loads in flight before the first LDS store (a load-store loop
// serialises ~37 L2 round trips); the filter statistics
__device__ __forceinline__ void mb_load_params(MbLds& L, const float* params, const float* rms, int tid) {
    constexpr int NQ = (P_ALL + 255) / 256;
    float pv[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) pv[q] = tid + q * 256 < P_ALL ? params[tid + q * 256] : 0.0f;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
        if (tid + q * 256 < P_ALL) *mb_slot(L, tid + q * 256) = pv[q];
    if (tid < 2 * OBD) L.rm[tid] = rms[tid];
}

// layers 1-2 of both nets over the 32 rows of L.z: wave (net, half) computes rows r0 .. r0 + 15
// as four 16 x 16 MFMA blocks (layer 1 over k = 0..11: b1 rides in as row 11 of W1 against z's
// ones column; layer 2 starts C at b2); h1 then h2 written, one barrier in between
__device__ __forceinline__ void mb_forward(MbLds& L, int net, int r0, int lr, int lk) {
    f32x4 c[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
        c[cb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < 3; ++s)
            c[cb] = mfma4(L.z[r0 + lr][4 * s + lk], L.w1[net][(4 * s + lk) * HID + 16 * cb + lr], c[cb]);
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i) L.h1[net][r0 + 4 * lk + i][16 * cb + lr] = tanh_fast(c[cb][i]);
    __syncthreads();
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
        const float b = L.b2[net][16 * cb + lr];
        c[cb] = f32x4{b, b, b, b};
    }
#pragma unroll
    for (int s = 0; s < HID / 4; ++s) {
        const float av = L.h1[net][r0 + lr][4 * s + lk];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) c[cb] = mfma4(av, L.w2[net][(4 * s + lk) * W2LD + 16 * cb + lr], c[cb]);
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i) L.h2[net][r0 + 4 * lk + i][16 * cb + lr] = tanh_fast(c[cb][i]);
}

// the heads of row r (after the barrier that follows mb_forward)
__device__ __forceinline__ void policy_head(const MbLds& L, int r, float& m0, float& m1) {
    m0 = L.b3[0];
    m1 = L.b3[1];
#pragma unroll 4
    for (int k = 0; k < HID; k += 4) {
        const float4 h = *(const float4*)&L.h2[0][r][k];
        m0 = fmaf(h.x, L.w3p[2 * k], m0);         m1 = fmaf(h.x, L.w3p[2 * k + 1], m1);
        m0 = fmaf(h.y, L.w3p[2 * k + 2], m0);     m1 = fmaf(h.y, L.w3p[2 * k + 3], m1);
        m0 = fmaf(h.z, L.w3p[2 * k + 4], m0);     m1 = fmaf(h.z, L.w3p[2 * k + 5], m1);
        m0 = fmaf(h.w, L.w3p[2 * k + 6], m0);     m1 = fmaf(h.w, L.w3p[2 * k + 7], m1);
    }
}

__device__ __forceinline__ float value_head(const MbLds& L, int r) {
    float v = L.b3[2];
#pragma unroll 4
    for (int k = 0; k < HID; k += 4) {
        const float4 h = *(const float4*)&L.h2[1][r][k];
        v = fmaf(h.w, L.w3v[k + 3], fmaf(h.z, L.w3v[k + 2], fmaf(h.y, L.w3v[k + 1], fmaf(h.x, L.w3v[k], v))));
    }
    return v;
}

// z row r of an observation (filter applied; 0 for a padded row), the ones column, zero pad
__device__ __forceinline__ float z_entry(const MbLds& L, float ob, int k, bool valid) {
    return k == OBD ? 1.0f : k > OBD ? 0.0f : valid ? clip5((ob - L.rm[k]) / L.rm[OBD + k]) : 0.0f;
}

// rollout (traj_segment_generator): 32 envs per workgroup, one per lane of wave 0 (physics,
// noise, episode clocks, records); the policy and value MLPs of the 32 envs run as the
// minibatch tile's forward (MFMA layers 1-2 by all four waves, heads by waves 0 / 1); one more
// value forward after the segment bootstraps nextvpred
constexpr int RO_E = MB_R;
__global__ __launch_bounds__(256) void rollout_kernel(RolloutArgs a) {
    __shared__ MbLds L;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int net = w >> 1, r0 = (w & 1) * 16, lr = lane & 15, lk = lane >> 4;
    mb_load_params(L, a.params, a.rms, tid);
    const int64_t n = a.n, e = (int64_t)blockIdx.x * RO_E + lane;
    const bool envl = w == 0 && lane < RO_E && e < n;
    rd::State st{};
    int step = 0, epi = 0;
    float ret = 0.f, newf = 0.f, it_ret = 0.f, it_eps = 0.f;
    if (envl) {
        st.q0 = a.state[e]; st.q1 = a.state[n + e]; st.v0 = a.state[2 * n + e]; st.v1 = a.state[3 * n + e];
        st.tx = a.state[4 * n + e]; st.ty = a.state[5 * n + e]; st.dx = a.state[6 * n + e]; st.dy = a.state[7 * n + e];
        step = a.ep_step[e]; epi = a.ep_idx[e]; ret = a.ep_ret[e]; newf = a.new_next[e];
    }
    const uint64_t gid = (uint64_t)(a.env_base + e);
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32) ^ 0xA5A5A5A5u;
    __syncthreads();
    const float s0 = expf(L.ls[0]), s1 = expf(L.ls[1]);
    for (int t = 0;; ++t) {
        float ob[OBD];
        if (w == 0 && lane < RO_E) {
            rd::observe(st, ob);
#pragma unroll
            for (int k = 0; k < ZLD; ++k) L.z[lane][k] = z_entry(L, k < OBD ? ob[k] : 0.0f, k, envl);
        }
        __syncthreads();
        mb_forward(L, net, r0, lr, lk);
        __syncthreads();
        float m0 = 0.f, m1 = 0.f;
        if (w == 1 && lane < RO_E) L.v[lane] = value_head(L, lane);
        else if (w == 0 && lane < RO_E && t < a.T) policy_head(L, lane, m0, m1);
        __syncthreads();
        if (t == a.T) {   // bootstrap value of the observation after the segment (0 if it starts an episode)
            if (envl) a.nextv[e] = newf > 0.5f ? 0.0f : L.v[lane];
            break;
        }
        if (envl) {
            const int64_t r = (int64_t)t * n + e;
            uint32_t wd[4];
            rd::philox((uint32_t)gid, (uint32_t)(gid >> 32), a.iter, (uint32_t)t, k0, k1, wd);
            const float u1 = (float)((wd[0] >> 8) + 1u) * (1.0f / 16777216.0f);   // (0, 1]
            const float u2 = (float)(wd[1] >> 8) * (1.0f / 16777216.0f);
            const float rad = sqrtf(-2.0f * logf(u1));
            const float ang = 6.283185307179586f * u2;
            const float a0 = fmaf(s0, rad * cosf(ang), m0), a1 = fmaf(s1, rad * sinf(ang), m1);
#pragma unroll
            for (int k = 0; k < OBD; ++k) a.ob[r * OBD + k] = ob[k];
            a.ac[2 * r] = a0;
            a.ac[2 * r + 1] = a1;
            a.vpred[r] = L.v[lane];
            a.newf[r] = newf;
            const float rw = rd::env_step(st, a0, a1);
            a.rew[r] = rw;
            ret += rw;
            newf = 0.0f;
            if (++step == rd::kEpisodeSteps) {   // TimeLimit(50): episode ends, env resets
                it_ret += ret;
                it_eps += 1.0f;
                ret = 0.0f;
                step = 0;
                ++epi;
                float d[6];
                rd::philox_draw(a.seed, gid, (uint32_t)epi, d);
                rd::env_reset(st, d);
                newf = 1.0f;
            }
        }
    }
    if (envl) {
        a.state[e] = st.q0; a.state[n + e] = st.q1; a.state[2 * n + e] = st.v0; a.state[3 * n + e] = st.v1;
        a.state[4 * n + e] = st.tx; a.state[5 * n + e] = st.ty; a.state[6 * n + e] = st.dx; a.state[7 * n + e] = st.dy;
        a.ep_step[e] = step;
        a.ep_idx[e] = epi;
        a.ep_ret[e] = ret;
        a.new_next[e] = newf;
        a.it_ret[e] = it_ret;
        a.it_eps[e] = it_eps;
    }
}

// oldpi's log-probs of the whole actor batch under the updated filter: minibatch_kernel's tile
// forward (same products in the same order), so the first minibatch of an epoch sees ratio 1
constexpr int LP_GRID = 1024;
__global__ __launch_bounds__(256) void logp_old_kernel(const float* params, const float* rms, const float* ob,
                                                       const float* ac, int64_t S, float* lpo) {
    __shared__ MbLds L;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int net = w >> 1, r0 = (w & 1) * 16, lr = lane & 15, lk = lane >> 4;
    mb_load_params(L, params, rms, tid);
    __syncthreads();
    const float ls0 = L.ls[0], ls1 = L.ls[1], sd0 = expf(ls0), sd1 = expf(ls1);
    const int64_t ntiles = (S + MB_R - 1) / MB_R;
    for (int64_t tl = blockIdx.x; tl < ntiles; tl += gridDim.x) {
        const int64_t i0 = tl * MB_R;
        constexpr int NZ = (MB_R * ZLD + 255) / 256;
#pragma unroll
        for (int q = 0; q < NZ; ++q) {
            const int e = tid + q * 256, r = e / ZLD, k = e % ZLD;
            const int64_t i = i0 + r;
            if (e < MB_R * ZLD) L.z[r][k] = z_entry(L, k < OBD && i < S ? ob[i * OBD + k] : 0.0f, k, i < S);
        }
        __syncthreads();
        mb_forward(L, net, r0, lr, lk);
        __syncthreads();
        const int64_t i = i0 + lane;
        if (w == 0 && lane < MB_R && i < S) {
            float m0, m1;
            policy_head(L, lane, m0, m1);
            const float x0 = (ac[2 * i] - m0) / sd0, x1 = (ac[2 * i + 1] - m1) / sd1;
            lpo[i] = -0.5f * (x0 * x0 + x1 * x1) - (ls0 + ls1) - LOG2PI;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void minibatch_kernel(MbArgs a) {
    __shared__ MbLds L;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int net = w >> 1, half = w & 1, r0 = half * MB_H;
    mb_load_params(L, a.params, a.rms, tid);
    if (blockIdx.x == 0 && tid < 4) a.ctl[4 + tid] = a.ctl[tid];   // Adam words for reduce_adam_kernel
    const float inv = 1.0f / (float)a.mb;
    // this wave's weight-gradient blocks: dW2 rows 32 half + 16 kb.., columns 16 jb..; dW1 | db1
    // columns 32 half + 16 jj..; plus db2 (half 0) and one head-gradient slot
    const int lr = lane & 15, lk = lane >> 4;
    f32x4 a2[2][4], a1[2];
    float ab = 0.0f, a3 = 0.0f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        a1[kb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) a2[kb][jb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    double ps = 0, vl = 0, cf = 0, g0 = 0, g1 = 0;
    const int ntiles = (a.mb + MB_R - 1) / MB_R;
    __syncthreads();
    for (int tl = blockIdx.x; tl < ntiles; tl += gridDim.x) {
        const int i0 = tl * MB_R;
        // 1. gather: filtered observations into z; the loss lanes keep their row's scalars
        constexpr int NZ = (MB_R * ZLD + 255) / 256;
        float zo[NZ];
#pragma unroll
        for (int q = 0; q < NZ; ++q) {
            const int e = tid + q * 256, r = e / ZLD, k = e % ZLD, i = i0 + r;
            zo[q] = e < MB_R * ZLD && k < OBD && i < a.mb ? a.ob[(int64_t)a.perm[i] * OBD + k] : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < NZ; ++q) {
            const int e = tid + q * 256, r = e / ZLD, k = e % ZLD, i = i0 + r;
            if (e < MB_R * ZLD) L.z[r][k] = z_entry(L, zo[q], k, i < a.mb);
        }
        const int li = i0 + lane;
        const bool lrow = w < 2 && lane < MB_R && li < a.mb;
        float ac0 = 0, ac1 = 0, lpo = 0, atg = 0, ret = 0;
        if (lrow) {
            const int64_t p = a.perm[li];
            if (w == 0) {
                ac0 = a.ac[2 * p]; ac1 = a.ac[2 * p + 1]; lpo = a.lpo[p]; atg = a.atarg[p];
            } else {
                ret = a.ret[p];
            }
        }
        __syncthreads();
        // 2-3. layers 1-2 of both nets
        mb_forward(L, net, r0, lr, lk);
        __syncthreads();
        // 4. heads and the loss, one lane per row: wave 0 the policy, wave 1 the value net
        if (w == 0 && lane < MB_R) {
            float m0, m1;
            policy_head(L, lane, m0, m1);
            float dm0 = 0.0f, dm1 = 0.0f;
            if (lrow) {
                // TF's min / clip gradient conventions (see oracle/ppo_np.py loss_and_grads)
                const float ls0 = L.ls[0], ls1 = L.ls[1];
                const float sd0 = expf(ls0), sd1 = expf(ls1);
                const float x0 = (ac0 - m0) / sd0, x1 = (ac1 - m1) / sd1;
                const float lp = -0.5f * (x0 * x0 + x1 * x1) - (ls0 + ls1) - LOG2PI;
                const float ratio = expf(lp - lpo);
                const float s1 = ratio * atg;
                const float rc = fminf(fmaxf(ratio, 1.0f - a.clip_eps), 1.0f + a.clip_eps);
                const float s2 = rc * atg;
                const bool take1 = s1 <= s2;                       // tf.minimum: ties to the first
                const bool inside = ratio >= 1.0f - a.clip_eps && ratio <= 1.0f + a.clip_eps;
                const float dlp = (take1 || inside) ? -atg * inv * ratio : 0.0f;
                dm0 = dlp * x0 / sd0;
                dm1 = dlp * x1 / sd1;
                ps += -(double)(take1 ? s1 : s2) * inv;
                cf += fabsf(ratio - 1.0f) > a.clip_eps ? (double)inv : 0.0;
                g0 += (double)dlp * (x0 * x0 - 1.0f);
                g1 += (double)dlp * (x1 * x1 - 1.0f);
            }
            L.dm[lane][0] = dm0;
            L.dm[lane][1] = dm1;
        } else if (w == 1 && lane < MB_R) {
            const float v = value_head(L, lane);
            float dvr = 0.0f;
            if (lrow) {
                const float d = v - ret;
                dvr = 2.0f * d * inv;
                vl += (double)d * d * inv;
            }
            L.dv[lane] = dvr;
        }
        __syncthreads();
        // 5. head backward: D2 = (dY W3^T) * tanh'; the head weight / bias gradients
#pragma unroll
        for (int i = 0; i < MB_H; ++i) {
            const int r = r0 + i;
            const float h = L.h2[net][r][lane];
            const float gy = net == 0 ? fmaf(L.dm[r][1], L.w3p[2 * lane + 1], L.dm[r][0] * L.w3p[2 * lane])
                                      : L.dv[r] * L.w3v[lane];
            L.d2[net][r][lane] = gy * (1.0f - h * h);
        }
        if (w < 3) {
#pragma unroll 8
            for (int r = 0; r < MB_R; ++r)
                a3 = fmaf(L.h2[net][r][lane], w == 2 ? L.dv[r] : L.dm[r][w], a3);
        } else if (lane < 3) {
#pragma unroll 8
            for (int r = 0; r < MB_R; ++r) a3 += lane < 2 ? L.dm[r][lane] : L.dv[r];
        }
        __syncthreads();
        // 6. layer 2 backward: D1 = (D2 W2^T) * tanh' for rows r0.. (B = W2 read transposed),
        //    then dW2 += H1^T D2 over the tile's 32 rows (k = 32 half ..), and db2 (half 0)
        f32x4 c[4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) c[cb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < HID / 4; ++s) {
            const float av = L.d2[net][r0 + lr][4 * s + lk];
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) c[cb] = mfma4(av, L.w2[net][(16 * cb + lr) * W2LD + 4 * s + lk], c[cb]);
        }
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = r0 + 4 * lk + i;
                const float h = L.h1[net][r][16 * cb + lr];
                L.d1[net][r][16 * cb + lr] = c[cb][i] * (1.0f - h * h);
            }
#pragma unroll
        for (int s = 0; s < MB_R / 4; ++s) {
            const float h0 = L.h1[net][4 * s + lk][32 * half + lr], h1 = L.h1[net][4 * s + lk][32 * half + 16 + lr];
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) {
                const float d = L.d2[net][4 * s + lk][16 * jb + lr];
                a2[0][jb] = mfma4(h0, d, a2[0][jb]);
                a2[1][jb] = mfma4(h1, d, a2[1][jb]);
            }
        }
        if (half == 0) {
#pragma unroll 8
            for (int r = 0; r < MB_R; ++r) ab += L.d2[net][r][lane];
        }
        __syncthreads();
        // 7. dW1 | db1 += z^T D1: one 16-row block (k = 0..11 used, 12-15 zero), columns 32 half ..
#pragma unroll
        for (int s = 0; s < MB_R / 4; ++s) {
            const float zv = L.z[4 * s + lk][lr];
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) a1[jj] = mfma4(zv, L.d1[net][4 * s + lk][32 * half + 16 * jj + lr], a1[jj]);
        }
        __syncthreads();
    }
    // partial gradient row of this workgroup (every slot written by exactly one thread)
    float* pr = a.part + (int64_t)blockIdx.x * PSTR;
    const int nb = net ? VB : 0;
    const int ow2 = nb + (net ? VW2 : PW2), ow1 = nb + (net ? VW1 : PW1);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int i = 0; i < 4; ++i) pr[ow2 + (32 * half + 16 * kb + 4 * lk + i) * HID + 16 * jb + lr] = a2[kb][jb][i];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (4 * lk + i <= OBD) pr[ow1 + (4 * lk + i) * HID + 32 * half + 16 * jj + lr] = a1[jj][i];   // row OBD = db1
    if (half == 0) pr[nb + (net ? VC2 : PB2) + lane] = ab;
    if (w == 0) pr[PW3 + 2 * lane] = a3;
    else if (w == 1) pr[PW3 + 2 * lane + 1] = a3;
    else if (w == 2) pr[VB + VW3 + lane] = a3;
    else if (lane < 2) pr[PB3 + lane] = a3;
    else if (lane == 2) pr[VB + VC3] = a3;
    if (w == 0) {
        L.red[0][lane] = ps; L.red[2][lane] = cf; L.red[3][lane] = g0; L.red[4][lane] = g1;
    } else if (w == 1) {
        L.red[1][lane] = vl;
    }
    __syncthreads();
    if (tid < 5) {
        double s = 0.0;
        for (int l = 0; l < 64; ++l) s += L.red[tid][l];
        a.stat[(int64_t)blockIdx.x * NSTAT + tid] = s;
    }
}

struct RaArgs {
    const float* part;
    const double* stat;
    int G;
    float* grad;
    float* params;
    float* m;
    float* v;
    uint32_t* ctl;
    double* acc;
    int accumulate;
    float lr, b1, b2, eps;
};

// grad[p] = fixed-order sum of the G partial rows (logstd: of the f64 sums), then MpiAdam.update
// (= TF1 form) over [pol | vf]; t counts minibatch steps.  Block 0 also folds the loss sums into
// the epoch accumulators (acc: pol_surr, vf_loss, clipfrac, minibatches).
__global__ __launch_bounds__(256) void reduce_adam_kernel(RaArgs a) {
    __shared__ float rs[RA_SLICES][RA_COLS];
    __shared__ double rq[RA_SLICES][RA_COLS];
    const int c = threadIdx.x % RA_COLS, s = threadIdx.x / RA_COLS, p = blockIdx.x * RA_COLS + c;
    const bool lsc = p == PLS || p == PLS + 1;
    // Adam's operands in flight before the column sums
    const bool own = s == 0 && p < P_ALL;
    const float m0 = own ? a.m[p] : 0.0f, v0 = own ? a.v[p] : 0.0f, x0 = own ? a.params[p] : 0.0f;
    float sum = 0.0f;
    double q = 0.0;
    if (p < P_ALL && !lsc) {
#pragma unroll 8
        for (int b = s; b < a.G; b += RA_SLICES) sum += a.part[(int64_t)b * PSTR + p];
    } else if (lsc) {
        for (int b = s; b < a.G; b += RA_SLICES) q += a.stat[(int64_t)b * NSTAT + 3 + (p - PLS)];
    }
    if (blockIdx.x == 0 && c < 3)
        for (int b = s; b < a.G; b += RA_SLICES) q += a.stat[(int64_t)b * NSTAT + c];
    rs[s][c] = sum;
    rq[s][c] = q;
    __syncthreads();
    if (s != 0) return;
    float fs[RA_SLICES];   // adjacent-pair tree over the slices: ((0 + 1) + (2 + 3)) + ...
    double ds[RA_SLICES];
#pragma unroll
    for (int q = 0; q < RA_SLICES; ++q) {
        fs[q] = rs[q][c];
        ds[q] = rq[q][c];
    }
#pragma unroll
    for (int w = RA_SLICES / 2; w >= 1; w /= 2)
#pragma unroll
        for (int q = 0; q < w; ++q) {
            fs[q] = fs[2 * q] + fs[2 * q + 1];
            ds[q] = ds[2 * q] + ds[2 * q + 1];
        }
    const float g0 = fs[0];
    const double d0 = ds[0];
    const uint32_t S = a.ctl[4];
    const float b1p = __uint_as_float(a.ctl[5]), b2p = __uint_as_float(a.ctl[6]);
    if (p < P_ALL) {
        const float g = lsc ? (float)d0 : g0;
        a.grad[p] = g;
        const float alpha = a.lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
        float m = m0, v = v0;
        m += (g - m) * (1.0f - a.b1);
        v += (g * g - v) * (1.0f - a.b2);
        a.m[p] = m;
        a.v[p] = v;
        a.params[p] = x0 - (m * alpha) / (sqrtf(v) + a.eps);
    }
    if (blockIdx.x == 0) {
        if (a.accumulate && c < 3) a.acc[c] += d0;
        if (a.accumulate && c == 3) a.acc[3] += 1.0;
        if (c == 0) {
            a.ctl[0] = S + 1u;
            a.ctl[1] = __float_as_uint(b1p * a.b1);
            a.ctl[2] = __float_as_uint(b2p * a.b2);
        }
    }
}

__global__ void metrics_kernel(const double* ep, const double* acc, const float* params, float lrmult, double ts,
                               float* hist) {
    if (threadIdx.x != 0) return;
    const double nb = acc[3] > 0 ? acc[3] : 1.0;
    hist[0] = ep[3] > 0 ? (float)(ep[2] / ep[3]) : 0.0f;   // mean return of episodes completed
    hist[1] = (float)ep[3];
    hist[2] = (float)(acc[0] / nb);
    hist[3] = (float)(acc[1] / nb);
    hist[4] = params[PLS] + params[PLS + 1] + 2.0f * 0.5f * (LOG2PI + 1.0f);   // entropy of the Gaussian
    hist[5] = (float)(acc[2] / nb);
    hist[6] = lrmult;
    hist[7] = (float)ts;
}

__global__ void reset_envs_kernel(int64_t n, int64_t env_base, uint64_t seed, float* state, int* ep_step, int* ep_idx,
                                  float* ep_ret, float* new_next) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    float d[6];
    rd::philox_draw(seed, (uint64_t)(env_base + e), 0u, d);
    rd::State st;
    rd::env_reset(st, d);
    state[e] = st.q0; state[n + e] = st.q1; state[2 * n + e] = st.v0; state[3 * n + e] = st.v1;
    state[4 * n + e] = st.tx; state[5 * n + e] = st.ty; state[6 * n + e] = st.dx; state[7 * n + e] = st.dy;
    ep_step[e] = 0;
    ep_idx[e] = 0;
    ep_ret[e] = 0.0f;
    new_next[e] = 1.0f;
}

__global__ void reset_misc_kernel(double* sums, uint32_t* ctl, float b1, float b2) {
    const int k = threadIdx.x;
    if (k < OBD) sums[k] = 0.0;
    if (k < OBD) sums[OBD + k] = 1e-2;   // RunningMeanStd(epsilon = 1e-2): sumsq and count start at eps
    if (k == 0) sums[2 * OBD] = 1e-2;
    if (k < 2) {
        const int o = 4 * k;
        ctl[o] = 0u; ctl[o + 1] = __float_as_uint(b1); ctl[o + 2] = __float_as_uint(b2); ctl[o + 3] = 0u;
    }
}

}  // namespace

struct rdp_trainer {
    rdp_config cfg{};
    int device = 0, cus = 256;
    hipStream_t stream = nullptr;
    int64_t n = 0, S = 0;
    int mb = 0;
    uint32_t iter = 0;
    double timesteps = 0.0;
    float lrmult = 1.0f;
    float *params = nullptr, *m = nullptr, *v = nullptr, *grad = nullptr, *own_grad = nullptr;
    float *state = nullptr, *ep_ret = nullptr, *new_next = nullptr, *it_ret = nullptr, *it_eps = nullptr;
    int *ep_step = nullptr, *ep_idx = nullptr;
    float *ob = nullptr, *ac = nullptr, *vpred = nullptr, *rew = nullptr, *newf = nullptr, *nextv = nullptr;
    float *adv = nullptr, *ret = nullptr, *atarg = nullptr, *lpo = nullptr;
    double *rms_sums = nullptr, *part = nullptr, *stats = nullptr, *acc = nullptr;
    float* rms = nullptr;
    int* perm = nullptr;
    std::vector<int> host_perm[2];   // double-buffered: the next iteration's shuffles are drawn
    int perm_buf = 0;                 //   while the GPU runs this iteration's minibatches
    uint32_t perm_for = UINT32_MAX;   // iteration whose shuffles host_perm[perm_buf] holds
    // minibatch step: per-workgroup partial gradient rows and loss sums
    float* mbpart = nullptr;
    double* mbstat = nullptr;
    float* hist = nullptr;
    uint32_t* ctl = nullptr;
    int64_t part_doubles = 0;
};

namespace {

#define RDP_CK(call, what) RD_HIP((call), what)

int run_rollout(rdp_trainer* t) {
    const int64_t n = t->n, S = t->S;
    const int T = t->cfg.horizon;
    hipLaunchKernelGGL(rms_finalize_kernel, dim3(1), dim3(64), 0, t->stream, (const double*)t->rms_sums, t->rms);
    RolloutArgs a;
    a.n = n; a.env_base = t->cfg.env_base; a.T = T; a.seed = t->cfg.seed; a.iter = t->iter;
    a.params = t->params; a.rms = t->rms; a.state = t->state; a.ep_step = t->ep_step; a.ep_idx = t->ep_idx;
    a.ep_ret = t->ep_ret; a.new_next = t->new_next; a.it_ret = t->it_ret; a.it_eps = t->it_eps;
    a.ob = t->ob; a.ac = t->ac; a.vpred = t->vpred; a.rew = t->rew; a.newf = t->newf; a.nextv = t->nextv;
    hipLaunchKernelGGL(rollout_kernel, dim3((unsigned)((n + RO_E - 1) / RO_E)), dim3(256), 0, t->stream, a);
    RDP_CK(hipGetLastError(), "rdp rollout_kernel");
    const int gblk = (int)((n + RB - 1) / RB);
    hipLaunchKernelGGL(gae_kernel, dim3(gblk), dim3(RB), 0, t->stream, n, T, t->cfg.gamma, t->cfg.lam,
                       (const float*)t->rew, (const float*)t->vpred, (const float*)t->newf, (const float*)t->nextv,
                       (const float*)t->it_ret, (const float*)t->it_eps, t->adv, t->ret, t->part);
    hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(RB), 0, t->stream, (const double*)t->part, gblk, t->stats);
    hipLaunchKernelGGL(standardize_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, t->stream,
                       (const float*)t->adv, S, (const double*)t->stats, t->atarg);
    RDP_CK(hipGetLastError(), "rdp gae");
    const int oblk = (int)((S + RB * 8 - 1) / (RB * 8));
    hipLaunchKernelGGL(ob_sums_kernel, dim3(oblk), dim3(RB), 0, t->stream, (const float*)t->ob, S, t->part);
    hipLaunchKernelGGL(rms_update_kernel, dim3(1), dim3(64), 0, t->stream, (const double*)t->part, oblk, S,
                       t->rms_sums);
    hipLaunchKernelGGL(rms_finalize_kernel, dim3(1), dim3(64), 0, t->stream, (const double*)t->rms_sums, t->rms);
    hipLaunchKernelGGL(logp_old_kernel, dim3((unsigned)std::min<int64_t>((S + MB_R - 1) / MB_R, LP_GRID)), dim3(256), 0,
                       t->stream,
                       (const float*)t->params, (const float*)t->rms, (const float*)t->ob, (const float*)t->ac, S,
                       t->lpo);
    RDP_CK(hipGetLastError(), "rdp filter / logp_old");
    return RD_OK;
}

// MpiAdam's epsilon: pposgd_simple.learn(..., adam_epsilon=1e-5) (baselines ppo1; the reference's
// teacher.py:30-36 call leaves it at that default), not tf.train.AdamOptimizer's 1e-8
constexpr float kAdamEps = 1e-5f;

int minibatch(rdp_trainer* t, const int* perm, bool last_epoch) {
    const int mb = t->mb;
    const int ntiles = (mb + MB_R - 1) / MB_R, G = ntiles < MB_G ? ntiles : MB_G;
    MbArgs a{perm, mb, t->params, t->rms, t->ob, t->ac, t->lpo, t->atarg, t->ret,
             t->cfg.clip_param * t->lrmult, t->mbpart, t->mbstat, t->ctl};
    hipLaunchKernelGGL(minibatch_kernel, dim3((unsigned)G), dim3(256), 0, t->stream, a);
    RDP_CK(hipGetLastError(), "rdp minibatch_kernel");
    RaArgs r{t->mbpart, t->mbstat, G, t->grad, t->params, t->m, t->v, t->ctl, t->acc, last_epoch ? 1 : 0,
             t->cfg.optim_stepsize * t->lrmult, 0.9f, 0.999f, kAdamEps};
    hipLaunchKernelGGL(reduce_adam_kernel, dim3((P_ALL + RA_COLS - 1) / RA_COLS), dim3(RA_SLICES * RA_COLS), 0,
                       t->stream, r);
    RDP_CK(hipGetLastError(), "rdp reduce_adam_kernel");
    return RD_OK;
}

// the optim_epochs shuffles of iteration `iter` (host Fisher-Yates, seeded by seed and iter)
void draw_perms(const rdp_trainer* t, uint32_t iter, int* out) {
    const int64_t S = t->S;
    std::mt19937_64 rng(t->cfg.seed * 0x9E3779B97F4A7C15ull + iter + 1);
    for (int e = 0; e < t->cfg.optim_epochs; ++e) {
        int* p = out + (int64_t)e * S;
        for (int64_t i = 0; i < S; ++i) p[i] = (int)i;
        for (int64_t i = S - 1; i > 0; --i) {   // Fisher-Yates
            const int64_t j = (int64_t)(rng() % (uint64_t)(i + 1));
            const int tmp = p[i];
            p[i] = p[j];
            p[j] = tmp;
        }
    }
}

int run_optimize(rdp_trainer* t) {
    const int64_t S = t->S;
    const int E = t->cfg.optim_epochs;
    const int nmb = (int)(S / t->mb);   // baselines iterate_once: full minibatches only
    const int cur = t->perm_buf;
    if (t->perm_for != t->iter) draw_perms(t, t->iter, t->host_perm[cur].data());
    RDP_CK(hipMemcpyAsync(t->perm, t->host_perm[cur].data(), sizeof(int) * (size_t)E * S, hipMemcpyHostToDevice,
                          t->stream),
           "rdp perm");
    RDP_CK(hipMemsetAsync(t->acc, 0, sizeof(double) * 4, t->stream), "rdp acc");
    for (int e = 0; e < E; ++e)
        for (int b = 0; b < nmb; ++b)
            if (int rc = minibatch(t, t->perm + (int64_t)e * S + (int64_t)b * t->mb, e == E - 1)) return rc;
    t->timesteps += (double)S;
    hipLaunchKernelGGL(metrics_kernel, dim3(1), dim3(64), 0, t->stream, (const double*)t->stats,
                       (const double*)t->acc, (const float*)t->params, t->lrmult, t->timesteps,
                       t->hist + (int64_t)(t->iter % (uint32_t)t->cfg.metrics_len) * N_MET);
    RDP_CK(hipGetLastError(), "rdp metrics");
    draw_perms(t, t->iter + 1, t->host_perm[cur ^ 1].data());   // overlaps the minibatches on the GPU
    t->perm_buf = cur ^ 1;
    t->perm_for = t->iter + 1;
    RDP_CK(hipStreamSynchronize(t->stream), "rdp optimize");
    ++t->iter;
    t->lrmult = t->cfg.schedule_linear
                    ? (float)fmax(1.0 - t->timesteps / (double)t->cfg.max_timesteps, 0.0)
                    : 1.0f;
    return RD_OK;
}

}  // namespace

extern "C" {

int rdp_param_counts(int32_t* policy, int32_t* value) {
    if (policy) *policy = P_POL;
    if (value) *value = P_VF;
    return RD_OK;
}

int rdp_create(rdp_trainer** out, const rdp_config* cfg, int device, void* hip_stream) {
    if (!out || !cfg) return rd::set_error(RD_EINVAL, "rdp_create: null argument");
    const int64_t S = cfg->n_envs * (int64_t)cfg->horizon;
    if (cfg->n_envs <= 0 || cfg->horizon <= 0 || S > ((int64_t)1 << 24) || cfg->env_base < 0 ||
        !(cfg->clip_param > 0) || cfg->entcoeff != 0.0f || cfg->optim_epochs <= 0 || !(cfg->optim_stepsize > 0) ||
        cfg->optim_batchsize < 0 || cfg->optim_batchsize > S || cfg->max_timesteps <= 0 || cfg->metrics_len < 0)
        return rd::set_error(RD_EINVAL, "rdp_create: bad config (entcoeff must be 0)");
    rd::DeviceGuard dg(device);
    RD_HIP(dg.err, "rdp_create: hipSetDevice");
    rdp_trainer* t = new (std::nothrow) rdp_trainer();
    if (!t) return rd::set_error(RD_EINVAL, "rdp_create: out of host memory");
    t->cfg = *cfg;
    if (t->cfg.metrics_len == 0) t->cfg.metrics_len = 1024;
    t->device = device;
    hipDeviceProp_t prop;
    t->cus = hipGetDeviceProperties(&prop, device) == hipSuccess ? prop.multiProcessorCount : 256;
    t->stream = (hipStream_t)hip_stream;
    t->n = cfg->n_envs;
    t->S = S;
    t->mb = cfg->optim_batchsize > 0 ? cfg->optim_batchsize : (int)S;
    for (auto& h : t->host_perm) h.resize((size_t)cfg->optim_epochs * S);
    const int64_t n = t->n;
    hipError_t e = hipSuccess;
    auto af = [&](float** p, int64_t cnt) {
        if (e == hipSuccess) e = hipMalloc((void**)p, sizeof(float) * (size_t)(cnt > 0 ? cnt : 1));
        if (e == hipSuccess) e = hipMemsetAsync(*p, 0, sizeof(float) * (size_t)(cnt > 0 ? cnt : 1), t->stream);
    };
    auto ai = [&](int** p, int64_t cnt) {
        if (e == hipSuccess) e = hipMalloc((void**)p, sizeof(int) * (size_t)cnt);
    };
    auto ad = [&](double** p, int64_t cnt) {
        if (e == hipSuccess) e = hipMalloc((void**)p, sizeof(double) * (size_t)cnt);
        if (e == hipSuccess) e = hipMemsetAsync(*p, 0, sizeof(double) * (size_t)cnt, t->stream);
    };
    af(&t->params, P_ALL); af(&t->m, P_ALL); af(&t->v, P_ALL); af(&t->own_grad, P_ALL);
    t->grad = t->own_grad;
    af(&t->state, 8 * n); af(&t->ep_ret, n); af(&t->new_next, n); af(&t->it_ret, n); af(&t->it_eps, n);
    ai(&t->ep_step, n); ai(&t->ep_idx, n);
    af(&t->ob, S * OBD); af(&t->ac, 2 * S); af(&t->vpred, S); af(&t->rew, S); af(&t->newf, S); af(&t->nextv, n);
    af(&t->adv, S); af(&t->ret, S); af(&t->atarg, S); af(&t->lpo, S);
    ad(&t->rms_sums, 2 * OBD + 1);
    t->part_doubles = 2 * OBD * ((S + RB * 8 - 1) / (RB * 8) + 1) + 5 * ((S + RB - 1) / RB + 1) + 4 * ((n + RB - 1) / RB + 1);
    ad(&t->part, t->part_doubles);
    ad(&t->stats, 4);
    ad(&t->acc, 4);
    af(&t->rms, 2 * OBD);
    ai(&t->perm, (int64_t)cfg->optim_epochs * S);
    af(&t->mbpart, (int64_t)MB_G * PSTR);
    ad(&t->mbstat, (int64_t)MB_G * NSTAT);
    af(&t->hist, (int64_t)t->cfg.metrics_len * N_MET);
    if (e == hipSuccess) e = hipMalloc((void**)&t->ctl, sizeof(uint32_t) * 8);
    if (e != hipSuccess) {
        rdp_destroy(t);
        return rd::hip_fail(e, "rdp_create: allocation");
    }
    if (int rc = rdp_reset(t)) {
        rdp_destroy(t);
        return rc;
    }
    *out = t;
    return RD_OK;
}

int rdp_destroy(rdp_trainer* t) {
    if (!t) return RD_OK;
    rd::DeviceGuard dg(t->device);
    void* bufs[] = {t->params, t->m, t->v, t->own_grad, t->state, t->ep_ret, t->new_next, t->it_ret, t->it_eps,
                    t->ep_step, t->ep_idx, t->ob, t->ac, t->vpred, t->rew, t->newf, t->nextv, t->adv, t->ret,
                    t->atarg, t->lpo, t->rms_sums, t->part, t->stats, t->acc, t->rms, t->perm, t->mbpart,
                    t->mbstat, t->hist, t->ctl};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    delete t;
    return RD_OK;
}

int rdp_set_stream(rdp_trainer* t, void* hip_stream) {
    if (!t) return rd::set_error(RD_EINVAL, "rdp_set_stream: null handle");
    t->stream = (hipStream_t)hip_stream;
    return RD_OK;
}

static int copy_params(rdp_trainer* t, float* dst, const float* src, int count, const char* what) {
    if (!t || !src || !dst) return rd::set_error(RD_EINVAL, "%s: null argument", what);
    rd::DeviceGuard dg(t->device);
    RD_HIP(hipMemcpyAsync(dst, src, sizeof(float) * count, hipMemcpyDeviceToDevice, t->stream), what);
    return RD_OK;
}

int rdp_set_policy(rdp_trainer* t, const float* p) {
    return copy_params(t, t ? t->params : nullptr, p, P_POL, "rdp_set_policy");
}
int rdp_get_policy(rdp_trainer* t, float* p) { return copy_params(t, p, t ? t->params : nullptr, P_POL, "rdp_get_policy"); }
int rdp_set_value(rdp_trainer* t, const float* p) {
    return copy_params(t, t ? t->params + VB : nullptr, p, P_VF, "rdp_set_value");
}
int rdp_get_value(rdp_trainer* t, float* p) {
    return copy_params(t, p, t ? t->params + VB : nullptr, P_VF, "rdp_get_value");
}

int rdp_get_obfilter(rdp_trainer* t, float* mean, float* std) {
    if (!t || !mean || !std) return rd::set_error(RD_EINVAL, "rdp_get_obfilter: null argument");
    rd::DeviceGuard dg(t->device);
    hipLaunchKernelGGL(rms_finalize_kernel, dim3(1), dim3(64), 0, t->stream, (const double*)t->rms_sums, t->rms);
    RD_HIP(hipMemcpyAsync(mean, t->rms, sizeof(float) * OBD, hipMemcpyDeviceToDevice, t->stream), "rdp_get_obfilter");
    RD_HIP(hipMemcpyAsync(std, t->rms + OBD, sizeof(float) * OBD, hipMemcpyDeviceToDevice, t->stream),
           "rdp_get_obfilter");
    return RD_OK;
}

int rdp_reset(rdp_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdp_reset: null handle");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdp_reset");
    hipLaunchKernelGGL(reset_envs_kernel, dim3((unsigned)((t->n + 255) / 256)), dim3(256), 0, t->stream, t->n,
                       t->cfg.env_base, t->cfg.seed, t->state, t->ep_step, t->ep_idx, t->ep_ret, t->new_next);
    hipLaunchKernelGGL(reset_misc_kernel, dim3(1), dim3(64), 0, t->stream, t->rms_sums, t->ctl, 0.9f, 0.999f);
    RD_HIP(hipMemsetAsync(t->m, 0, sizeof(float) * P_ALL, t->stream), "rdp_reset");
    RD_HIP(hipMemsetAsync(t->v, 0, sizeof(float) * P_ALL, t->stream), "rdp_reset");
    RD_HIP(hipGetLastError(), "rdp_reset");
    t->iter = 0;
    t->perm_for = UINT32_MAX;
    t->timesteps = 0.0;
    t->lrmult = 1.0f;
    return RD_OK;
}

int rdp_rollout(rdp_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdp_rollout: null handle");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdp_rollout");
    return run_rollout(t);
}

int rdp_optimize(rdp_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdp_optimize: null handle");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdp_optimize");
    return run_optimize(t);
}

int rdp_iterate(rdp_trainer* t) {
    if (int rc = rdp_rollout(t)) return rc;
    return rdp_optimize(t);
}

int rdp_get_batch(rdp_trainer* t, float* ob, float* ac, float* vpred, float* rew, float* newf, float* nextvpred,
                  float* adv, float* ret) {
    if (!t) return rd::set_error(RD_EINVAL, "rdp_get_batch: null handle");
    rd::DeviceGuard dg(t->device);
    const int64_t S = t->S;
    struct {
        float* dst;
        const float* src;
        int64_t cnt;
    } cp[] = {{ob, t->ob, S * OBD}, {ac, t->ac, 2 * S}, {vpred, t->vpred, S}, {rew, t->rew, S},
              {newf, t->newf, S},  {nextvpred, t->nextv, t->n}, {adv, t->adv, S}, {ret, t->ret, S}};
    for (auto& c : cp)
        if (c.dst)
            RD_HIP(hipMemcpyAsync(c.dst, c.src, sizeof(float) * c.cnt, hipMemcpyDeviceToDevice, t->stream),
                   "rdp_get_batch");
    return RD_OK;
}

float* rdp_grad_buffer(rdp_trainer* t) { return t ? t->grad : nullptr; }

int rdp_bind_grad_buffer(rdp_trainer* t, float* grad) {
    if (!t) return rd::set_error(RD_EINVAL, "rdp_bind_grad_buffer: null handle");
    t->grad = grad ? grad : t->own_grad;
    return RD_OK;
}

int rdp_get_counter(rdp_trainer* t, int64_t* iterations) {
    if (!t || !iterations) return rd::set_error(RD_EINVAL, "rdp_get_counter: null argument");
    *iterations = t->iter;
    return RD_OK;
}

int rdp_read_metrics(rdp_trainer* t, int64_t count, double* out) {
    if (!t || !out || count < 0) return rd::set_error(RD_EINVAL, "rdp_read_metrics: bad argument");
    const int64_t H = t->cfg.metrics_len, it = t->iter;
    if (count > it || count > H)
        return rd::set_error(RD_EINVAL, "rdp_read_metrics: only %lld iterations kept", (long long)(it < H ? it : H));
    rd::DeviceGuard dg(t->device);
    std::vector<float> host((size_t)H * N_MET);
    RD_HIP(hipStreamSynchronize(t->stream), "rdp_read_metrics");
    RD_HIP(hipMemcpy(host.data(), t->hist, sizeof(float) * H * N_MET, hipMemcpyDeviceToHost), "rdp_read_metrics");
    for (int64_t k = 0; k < count; ++k) {
        const int64_t s = (it - count + k) % H;
        for (int j = 0; j < N_MET; ++j) out[k * N_MET + j] = host[s * N_MET + j];
    }
    return RD_OK;
}

}  // extern "C"
