// PPO training of the teacher on batched Reacher-v2 (include/reacher_ppo.h), for gfx950:
// the reference's baselines ppo1 pposgd_simple.learn (teacher.py:23-37) over n_envs
// parallel envs.
//
// MI355X mapping:
//  * rollout: one env per lane for the whole horizon; the policy and value MLPs (2 x 64
//    tanh each) run per lane as unrolled f32 FMA chains over weights broadcast from LDS
//    (40 KB), the env step is the shared Reacher physics (rd_physics.h); the actor batch
//    (ob, ac, vpred, rew, new) is written t-major so every later pass is coalesced;
//  * GAE: one env per lane, backward over its horizon; the advantage moments and the
//    observation filter's sums are deterministic two-level f64 reductions;
//  * minibatch step: gather (with the filter applied), the two MLPs' forward and backward
//    as MFMA GEMMs with fused bias / tanh / tanh' epilogues (rd_gemm.h), the clipped
//    surrogate + value loss per row, fixed-order column sums for the biases and logstd,
//    and TF1/MpiAdam over the concatenated [pol | vf] vector.  No atomics: deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <new>
#include <random>
#include <vector>

#include "../../include/reacher_ppo.h"
#include "rd_common.h"
#include "rd_gemm.h"
#include "rd_physics.h"

namespace {

constexpr int OBD = 11, HID = 64, ZLD = 12;
// Hidden activations are stored [row][HLD] with column HID = 1: a weight-gradient GEMM over
// HID + 1 rows of A^T then yields dW (rows 0..HID-1) AND the bias gradient db (row HID) in
// one launch, written straight into the flat [W | b] parameter layout (the input batch Z
// carries the same 1 in column OBD).
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

// 2 x 64 tanh hidden stack of one lane: weights broadcast from LDS (L = W1 | b1 | W2 | b2),
// the lane's input z and first hidden layer in per-lane LDS columns (zs [11][64], h1s
// [64][64], lane-contiguous) so the k loops stay rolled and only the 64 accumulators of
// the current layer live in registers.
__device__ __forceinline__ void hidden(const float* L, const float* zs, float* h1s, int lane, float (&h2)[HID]) {
    float acc[HID];
#pragma unroll
    for (int j = 0; j < HID; ++j) acc[j] = L[PB1 + j];
#pragma unroll 1
    for (int k = 0; k < OBD; ++k) {
        const float zk = zs[k * 64 + lane];
#pragma unroll
        for (int j = 0; j < HID; ++j) acc[j] = fmaf(zk, L[PW1 + k * HID + j], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < HID; ++j) h1s[j * 64 + lane] = tanhf(acc[j]);
#pragma unroll
    for (int j = 0; j < HID; ++j) h2[j] = L[PB2 + j];
#pragma unroll 2
    for (int k = 0; k < HID; ++k) {
        const float hk = h1s[k * 64 + lane];
#pragma unroll
        for (int j = 0; j < HID; ++j) h2[j] = fmaf(hk, L[PW2 + k * HID + j], h2[j]);
    }
#pragma unroll
    for (int j = 0; j < HID; ++j) h2[j] = tanhf(h2[j]);
}

__device__ __forceinline__ void policy_mean(const float* L, const float* zs, float* h1s, int lane, float& m0,
                                            float& m1) {
    float h2[HID];
    hidden(L, zs, h1s, lane, h2);
    m0 = L[PB3];
    m1 = L[PB3 + 1];
#pragma unroll
    for (int k = 0; k < HID; ++k) {
        m0 = fmaf(h2[k], L[PW3 + 2 * k], m0);
        m1 = fmaf(h2[k], L[PW3 + 2 * k + 1], m1);
    }
}

__device__ __forceinline__ float value(const float* V, const float* zs, float* h1s, int lane) {
    float h2[HID];
    hidden(V, zs, h1s, lane, h2);   // the value net has the same W1 b1 W2 b2 offsets
    float v = V[VC3];
#pragma unroll
    for (int k = 0; k < HID; ++k) v = fmaf(h2[k], V[VW3 + k], v);
    return v;
}

// z = clip((ob - mean) / std, -5, 5) into the lane's LDS column
__device__ __forceinline__ void normalize(const float* ob, const float* rms, float* zs, int lane) {
#pragma unroll
    for (int k = 0; k < OBD; ++k) zs[k * 64 + lane] = clip5((ob[k] - rms[k]) / rms[OBD + k]);
}

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

__global__ __launch_bounds__(64) void rollout_kernel(RolloutArgs a) {
    __shared__ float L[P_ALL + 2 * OBD];
    __shared__ float zs[OBD * 64], h1s[HID * 64];
    const int lane = threadIdx.x;
    for (int i = threadIdx.x; i < P_ALL; i += 64) L[i] = a.params[i];
    if (threadIdx.x < 2 * OBD) L[P_ALL + threadIdx.x] = a.rms[threadIdx.x];
    __syncthreads();
    const int64_t e = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (e >= a.n) return;
    const float* Lp = L;
    const float* Lv = L + VB;
    const float* rms = L + P_ALL;
    const int64_t n = a.n;
    rd::State st;
    st.q0 = a.state[e]; st.q1 = a.state[n + e]; st.v0 = a.state[2 * n + e]; st.v1 = a.state[3 * n + e];
    st.tx = a.state[4 * n + e]; st.ty = a.state[5 * n + e]; st.dx = a.state[6 * n + e]; st.dy = a.state[7 * n + e];
    int step = a.ep_step[e], epi = a.ep_idx[e];
    float ret = a.ep_ret[e], newf = a.new_next[e], it_ret = 0.f, it_eps = 0.f;
    const float s0 = expf(Lp[PLS]), s1 = expf(Lp[PLS + 1]);
    const uint64_t gid = (uint64_t)(a.env_base + e);
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32) ^ 0xA5A5A5A5u;
    for (int t = 0; t < a.T; ++t) {
        const int64_t r = (int64_t)t * n + e;
        float ob[OBD];
        rd::observe(st, ob);
        normalize(ob, rms, zs, lane);
        float m0, m1;
        policy_mean(Lp, zs, h1s, lane, m0, m1);
        const float v = value(Lv, zs, h1s, lane);
        uint32_t w[4];
        rd::philox((uint32_t)gid, (uint32_t)(gid >> 32), a.iter, (uint32_t)t, k0, k1, w);
        const float u1 = (float)((w[0] >> 8) + 1u) * (1.0f / 16777216.0f);   // (0, 1]
        const float u2 = (float)(w[1] >> 8) * (1.0f / 16777216.0f);
        const float rad = sqrtf(-2.0f * logf(u1));
        const float ang = 6.283185307179586f * u2;
        const float a0 = fmaf(s0, rad * cosf(ang), m0), a1 = fmaf(s1, rad * sinf(ang), m1);
#pragma unroll
        for (int k = 0; k < OBD; ++k) a.ob[r * OBD + k] = ob[k];
        a.ac[2 * r] = a0;
        a.ac[2 * r + 1] = a1;
        a.vpred[r] = v;
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
    {   // bootstrap value of the observation after the segment (0 if it starts an episode)
        float ob[OBD];
        rd::observe(st, ob);
        normalize(ob, rms, zs, lane);
        a.nextv[e] = newf > 0.5f ? 0.0f : value(Lv, zs, h1s, lane);
    }
    a.state[e] = st.q0; a.state[n + e] = st.q1; a.state[2 * n + e] = st.v0; a.state[3 * n + e] = st.v1;
    a.state[4 * n + e] = st.tx; a.state[5 * n + e] = st.ty; a.state[6 * n + e] = st.dx; a.state[7 * n + e] = st.dy;
    a.ep_step[e] = step;
    a.ep_idx[e] = epi;
    a.ep_ret[e] = ret;
    a.new_next[e] = newf;
    a.it_ret[e] = it_ret;
    a.it_eps[e] = it_eps;
}

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
__global__ __launch_bounds__(64) void logp_old_kernel(const float* params, const float* rms, const float* ob,
                                                      const float* ac, int64_t S, float* lpo) {
    __shared__ float L[P_POL + 2 * OBD];
    __shared__ float zs[OBD * 64], h1s[HID * 64];
    const int lane = threadIdx.x;
    for (int i = threadIdx.x; i < P_POL; i += 64) L[i] = params[i];
    if (threadIdx.x < 2 * OBD) L[P_POL + threadIdx.x] = rms[threadIdx.x];
    __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (r >= S) return;
    float m0, m1;
    normalize(ob + r * OBD, L + P_POL, zs, lane);
    policy_mean(L, zs, h1s, lane, m0, m1);
    const float ls0 = L[PLS], ls1 = L[PLS + 1];
    const float d0 = (ac[2 * r] - m0) / expf(ls0), d1 = (ac[2 * r + 1] - m1) / expf(ls1);
    lpo[r] = -0.5f * (d0 * d0 + d1 * d1) - (ls0 + ls1) - LOG2PI;
}

// minibatch rows perm[i] -> Z (filtered obs, 12-wide), A, LPO, ATG, RET.  16 lanes per row,
// one gathered value each (one lane per row left the random-row loads of a 4,096-row
// minibatch on 16 workgroups: a chain of load latencies)
constexpr int GATHER_LANES = 16;
__global__ __launch_bounds__(256) void gather_kernel(const int* perm, int mb, const float* rms, const float* ob,
                                                     const float* ac, const float* lpo, const float* atarg,
                                                     const float* ret, float* Z, float* A, float* LPO, float* ATG,
                                                     float* RET) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int i = (int)(t / GATHER_LANES), j = (int)(t % GATHER_LANES);
    if (i >= mb) return;
    const int64_t r = perm[i];
    if (j < OBD) Z[i * ZLD + j] = clip5((ob[r * OBD + j] - rms[j]) / rms[OBD + j]);
    else if (j == OBD) Z[i * ZLD + OBD] = 1.0f;   // the bias input of the layer-1 gradient GEMM
    else if (j == 12) A[2 * i] = ac[2 * r];
    else if (j == 13) A[2 * i + 1] = ac[2 * r + 1];
    else if (j == 14) LPO[i] = lpo[r];
    else {
        ATG[i] = atarg[r];
        RET[i] = ret[r];
    }
}

// clipped surrogate + value loss per row: dMEAN, dV, and per-block sums of
// (pol_surr, vf_loss, clipfrac, dlogstd0, dlogstd1)
__global__ __launch_bounds__(RB) void ppo_loss_kernel(int mb, const float* params, const float* MEAN, const float* V,
                                                      const float* A, const float* LPO, const float* ATG,
                                                      const float* RET, float clip_eps, float* dMEAN, float* dV,
                                                      double* part) {
    __shared__ double s[5][RB];
    const int i = blockIdx.x * RB + threadIdx.x;
    double ps = 0, vl = 0, cf = 0, g0 = 0, g1 = 0;
    if (i < mb) {
        const float ls0 = params[PLS], ls1 = params[PLS + 1];
        const float sd0 = expf(ls0), sd1 = expf(ls1);
        const float m0 = MEAN[2 * i], m1 = MEAN[2 * i + 1];
        const float x0 = (A[2 * i] - m0) / sd0, x1 = (A[2 * i + 1] - m1) / sd1;
        const float lp = -0.5f * (x0 * x0 + x1 * x1) - (ls0 + ls1) - LOG2PI;
        const float ratio = expf(lp - LPO[i]);
        const float at = ATG[i];
        const float s1 = ratio * at;
        const float rc = fminf(fmaxf(ratio, 1.0f - clip_eps), 1.0f + clip_eps);
        const float s2 = rc * at;
        const bool take1 = s1 <= s2;                       // tf.minimum: ties to the first
        const bool inside = ratio >= 1.0f - clip_eps && ratio <= 1.0f + clip_eps;
        const float inv = 1.0f / (float)mb;
        const float dlp = (take1 || inside) ? -at * inv * ratio : 0.0f;
        dMEAN[2 * i] = dlp * x0 / sd0;
        dMEAN[2 * i + 1] = dlp * x1 / sd1;
        const float dv = V[i] - RET[i];
        dV[i] = 2.0f * dv * inv;
        ps = -(double)(take1 ? s1 : s2) * inv;
        vl = (double)dv * dv * inv;
        cf = fabsf(ratio - 1.0f) > clip_eps ? (double)inv : 0.0;
        g0 = (double)dlp * (x0 * x0 - 1.0f);
        g1 = (double)dlp * (x1 * x1 - 1.0f);
    }
    s[0][threadIdx.x] = ps; s[1][threadIdx.x] = vl; s[2][threadIdx.x] = cf; s[3][threadIdx.x] = g0; s[4][threadIdx.x] = g1;
    __syncthreads();
    for (int w = RB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
#pragma unroll
            for (int q = 0; q < 5; ++q) s[q][threadIdx.x] += s[q][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < 5) part[blockIdx.x * 5 + threadIdx.x] = s[threadIdx.x][0];
}

// sum the loss partials: dlogstd into the gradient, losses into the epoch accumulators
// (acc: pol_surr, vf_loss, clipfrac, minibatches); snapshot of the Adam words
__global__ void loss_final_kernel(const double* part, int nblk, float* grad, double* acc, int accumulate,
                                  uint32_t* ctl) {
    if (threadIdx.x != 0) return;
    double q[5] = {0, 0, 0, 0, 0};
    for (int b = 0; b < nblk; ++b)
        for (int k = 0; k < 5; ++k) q[k] += part[b * 5 + k];
    grad[PLS] = (float)q[3];
    grad[PLS + 1] = (float)q[4];
    if (accumulate) {
        acc[0] += q[0];
        acc[1] += q[1];
        acc[2] += q[2];
        acc[3] += 1.0;
    }
    for (int k = 0; k < 4; ++k) ctl[4 + k] = ctl[k];
}

// column HID of a [rows][HLD] activation buffer = 1 (the bias input of the next layer's
// weight-gradient GEMM); the forward GEMMs write columns 0..HID-1 only
__global__ __launch_bounds__(256) void ones_column_kernel(float* H, int64_t rows) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r < rows) H[r * HLD + HID] = 1.0f;
}

struct AdamArgs {
    const float* grad;
    float* params;
    float* m;
    float* v;
    uint32_t* ctl;
    float lr, b1, b2, eps;
};

// MpiAdam.update (= TF1 form) over [pol | vf]; t counts minibatch steps
__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    const uint32_t S = a.ctl[4];
    const float b1p = __uint_as_float(a.ctl[5]), b2p = __uint_as_float(a.ctl[6]);
    if (p < P_ALL) {
        const float g = a.grad[p];
        const float alpha = a.lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
        float m = a.m[p], v = a.v[p];
        m += (g - m) * (1.0f - a.b1);
        v += (g * g - v) * (1.0f - a.b2);
        a.m[p] = m;
        a.v[p] = v;
        a.params[p] -= (m * alpha) / (sqrtf(v) + a.eps);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.ctl[0] = S + 1u;
        a.ctl[1] = __float_as_uint(b1p * a.b1);
        a.ctl[2] = __float_as_uint(b2p * a.b2);
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
    std::vector<int> host_perm;
    // minibatch buffers
    float *Z = nullptr, *A = nullptr, *LPO = nullptr, *ATG = nullptr, *RET = nullptr;
    float *H1 = nullptr, *H2 = nullptr, *MEAN = nullptr, *G1 = nullptr, *G2 = nullptr, *V = nullptr;
    float *dMEAN = nullptr, *dV = nullptr, *D2 = nullptr, *D1 = nullptr, *E2 = nullptr, *E1 = nullptr;
    float* split = nullptr;
    float* hist = nullptr;
    uint32_t* ctl = nullptr;
    int64_t part_doubles = 0;
};

namespace {

constexpr int64_t SPLIT_FLOATS = 4 << 20;

hipError_t mm(rdp_trainer* t, int M, int N, int K, const float* A, int64_t lda, int ta, const float* B, int64_t ldb,
              int tb, float* C, int64_t ldc, const float* bias = nullptr, int epi = rdg::EPI_NONE,
              const float* aux = nullptr, int64_t ldaux = 0) {
    rdg::GemmArgs g{};
    g.M = M; g.N = N; g.K = K;
    g.A = A; g.lda = lda; g.ta = ta;
    g.B = B; g.ldb = ldb; g.tb = tb;
    g.C = C; g.ldc = ldc;
    g.bias = bias; g.epi = epi; g.aux = aux; g.ldaux = ldaux;
    return rdg::gemm(t->stream, g, t->split, SPLIT_FLOATS, t->cus);
}

rdg::GemmArgs gm(int M, int N, int K, const float* A, int64_t lda, int ta, const float* B, int64_t ldb, int tb,
                 float* C, int64_t ldc, const float* bias = nullptr, int epi = rdg::EPI_NONE,
                 const float* aux = nullptr, int64_t ldaux = 0) {
    rdg::GemmArgs g{};
    g.M = M; g.N = N; g.K = K;
    g.A = A; g.lda = lda; g.ta = ta;
    g.B = B; g.ldb = ldb; g.tb = tb;
    g.C = C; g.ldc = ldc;
    g.bias = bias; g.epi = epi; g.aux = aux; g.ldaux = ldaux;
    return g;
}

// the policy's and the value net's GEMM of one layer as one grouped launch (rdg::gemm2)
hipError_t mm2(rdp_trainer* t, const rdg::GemmArgs& pol, const rdg::GemmArgs& vf) {
    return rdg::gemm2(t->stream, pol, vf, t->split, SPLIT_FLOATS, t->cus);
}


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
    hipLaunchKernelGGL(rollout_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, t->stream, a);
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
    hipLaunchKernelGGL(logp_old_kernel, dim3((unsigned)((S + 63) / 64)), dim3(64), 0, t->stream,
                       (const float*)t->params, (const float*)t->rms, (const float*)t->ob, (const float*)t->ac, S,
                       t->lpo);
    RDP_CK(hipGetLastError(), "rdp filter / logp_old");
    return RD_OK;
}

int minibatch(rdp_trainer* t, const int* perm, bool last_epoch) {
    const int mb = t->mb;
    const float* P = t->params;
    float* g = t->grad;
    const float* Pv = P + VB;
    float* gv = g + VB;
    const float eps = t->cfg.clip_param * t->lrmult;
    hipLaunchKernelGGL(gather_kernel, dim3((unsigned)(((int64_t)mb * GATHER_LANES + 255) / 256)), dim3(256), 0,
                       t->stream, perm, mb,
                       (const float*)t->rms, (const float*)t->ob, (const float*)t->ac, (const float*)t->lpo,
                       (const float*)t->atarg, (const float*)t->ret, t->Z, t->A, t->LPO, t->ATG, t->RET);
    RDP_CK(hipGetLastError(), "rdp gather");
    // forward: layer k of the policy and of the value net in one launch
    RDP_CK(mm2(t, gm(mb, HID, OBD, t->Z, ZLD, 0, P + PW1, HID, 0, t->H1, HLD, P + PB1, rdg::EPI_TANH),
               gm(mb, HID, OBD, t->Z, ZLD, 0, Pv + VW1, HID, 0, t->G1, HLD, Pv + VC1, rdg::EPI_TANH)),
           "rdp pol1 vf1");
    RDP_CK(mm2(t, gm(mb, HID, HID, t->H1, HLD, 0, P + PW2, HID, 0, t->H2, HLD, P + PB2, rdg::EPI_TANH),
               gm(mb, HID, HID, t->G1, HLD, 0, Pv + VW2, HID, 0, t->G2, HLD, Pv + VC2, rdg::EPI_TANH)),
           "rdp pol2 vf2");
    RDP_CK(mm2(t, gm(mb, 2, HID, t->H2, HLD, 0, P + PW3, 2, 0, t->MEAN, 2, P + PB3),
               gm(mb, 1, HID, t->G2, HLD, 0, Pv + VW3, 1, 0, t->V, 1, Pv + VC3)),
           "rdp pol3 vf3");
    const int lblk = (mb + RB - 1) / RB;
    hipLaunchKernelGGL(ppo_loss_kernel, dim3(lblk), dim3(RB), 0, t->stream, mb, P, (const float*)t->MEAN,
                       (const float*)t->V, (const float*)t->A, (const float*)t->LPO, (const float*)t->ATG,
                       (const float*)t->RET, eps, t->dMEAN, t->dV, t->part);
    hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(64), 0, t->stream, (const double*)t->part, lblk, g, t->acc,
                       last_epoch ? 1 : 0, t->ctl);
    RDP_CK(hipGetLastError(), "rdp loss");
    // backward, policy and value side by side: [dW; db] of a layer in one GEMM (the ones
    // column of its input), then the data gradient with tanh' fused
    RDP_CK(mm2(t, gm(HID + 1, 2, mb, t->H2, HLD, 1, t->dMEAN, 2, 0, g + PW3, 2),
               gm(HID + 1, 1, mb, t->G2, HLD, 1, t->dV, 1, 0, gv + VW3, 1)),
           "rdp gW3 gV3");
    RDP_CK(mm2(t, gm(mb, HID, 2, t->dMEAN, 2, 0, P + PW3, 2, 1, t->D2, HID, nullptr, rdg::EPI_DTANH, t->H2, HLD),
               gm(mb, HID, 1, t->dV, 1, 0, Pv + VW3, 1, 1, t->E2, HID, nullptr, rdg::EPI_DTANH, t->G2, HLD)),
           "rdp d2 e2");
    RDP_CK(mm2(t, gm(HID + 1, HID, mb, t->H1, HLD, 1, t->D2, HID, 0, g + PW2, HID),
               gm(HID + 1, HID, mb, t->G1, HLD, 1, t->E2, HID, 0, gv + VW2, HID)),
           "rdp gW2 gV2");
    RDP_CK(mm2(t, gm(mb, HID, HID, t->D2, HID, 0, P + PW2, HID, 1, t->D1, HID, nullptr, rdg::EPI_DTANH, t->H1, HLD),
               gm(mb, HID, HID, t->E2, HID, 0, Pv + VW2, HID, 1, t->E1, HID, nullptr, rdg::EPI_DTANH, t->G1, HLD)),
           "rdp d1 e1");
    RDP_CK(mm2(t, gm(OBD + 1, HID, mb, t->Z, ZLD, 1, t->D1, HID, 0, g + PW1, HID),
               gm(OBD + 1, HID, mb, t->Z, ZLD, 1, t->E1, HID, 0, gv + VW1, HID)),
           "rdp gW1 gV1");
    AdamArgs aa{t->grad, t->params, t->m, t->v, t->ctl, t->cfg.optim_stepsize * t->lrmult, 0.9f, 0.999f, 1e-8f};
    hipLaunchKernelGGL(adam_kernel, dim3((P_ALL + 255) / 256), dim3(256), 0, t->stream, aa);
    RDP_CK(hipGetLastError(), "rdp adam");
    return RD_OK;
}

int run_optimize(rdp_trainer* t) {
    const int64_t S = t->S;
    const int E = t->cfg.optim_epochs;
    const int nmb = (int)(S / t->mb);   // baselines iterate_once: full minibatches only
    std::mt19937_64 rng(t->cfg.seed * 0x9E3779B97F4A7C15ull + t->iter + 1);
    for (int e = 0; e < E; ++e) {
        int* p = t->host_perm.data() + (int64_t)e * S;
        for (int64_t i = 0; i < S; ++i) p[i] = (int)i;
        for (int64_t i = S - 1; i > 0; --i) {   // Fisher-Yates
            const int64_t j = (int64_t)(rng() % (uint64_t)(i + 1));
            const int tmp = p[i];
            p[i] = p[j];
            p[j] = tmp;
        }
    }
    RDP_CK(hipMemcpyAsync(t->perm, t->host_perm.data(), sizeof(int) * (size_t)E * S, hipMemcpyHostToDevice, t->stream),
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
    RDP_CK(hipStreamSynchronize(t->stream), "rdp optimize");   // host_perm is reused next iteration
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
    t->host_perm.resize((size_t)cfg->optim_epochs * S);
    const int64_t n = t->n, mb = t->mb;
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
    af(&t->Z, mb * ZLD); af(&t->A, 2 * mb); af(&t->LPO, mb); af(&t->ATG, mb); af(&t->RET, mb);
    af(&t->H1, mb * HLD); af(&t->H2, mb * HLD); af(&t->MEAN, 2 * mb); af(&t->G1, mb * HLD); af(&t->G2, mb * HLD);
    af(&t->V, mb); af(&t->dMEAN, 2 * mb); af(&t->dV, mb); af(&t->D2, mb * HID); af(&t->D1, mb * HID);
    af(&t->E2, mb * HID); af(&t->E1, mb * HID);
    af(&t->split, SPLIT_FLOATS);
    af(&t->hist, (int64_t)t->cfg.metrics_len * N_MET);
    if (e == hipSuccess) e = hipMalloc((void**)&t->ctl, sizeof(uint32_t) * 8);
    if (e != hipSuccess) {
        rdp_destroy(t);
        return rd::hip_fail(e, "rdp_create: allocation");
    }
    for (float* h : {t->H1, t->H2, t->G1, t->G2})
        hipLaunchKernelGGL(ones_column_kernel, dim3((unsigned)((mb + 255) / 256)), dim3(256), 0, t->stream, h,
                           (int64_t)mb);
    if ((e = hipGetLastError()) != hipSuccess) {
        rdp_destroy(t);
        return rd::hip_fail(e, "rdp_create: ones columns");
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
                    t->atarg, t->lpo, t->rms_sums, t->part, t->stats, t->acc, t->rms, t->perm, t->Z, t->A, t->LPO,
                    t->ATG, t->RET, t->H1, t->H2, t->MEAN, t->G1, t->G2, t->V, t->dMEAN, t->dV, t->D2, t->D1,
                    t->E2, t->E1, t->split, t->hist, t->ctl};
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
