// Fused rollout + distillation step for gfx950 (include/reacher_distill.h).
//
// One launch of rollout_kernel runs, for every env, one iteration of the reference's hot
// loop (mlp_train.py:143-204): observation -> teacher MlpPolicy (teacher.py:14-16) ->
// student MlpPolicy -> loss (loss.py:3-13 KL, or action-MSE) -> student backward ->
// env.step(action) with auto-reset; per-workgroup gradient partials go to a workspace.
// reduce_adam_kernel then sums the partials and applies TF1 Adam (mlp_train.py:73-80).
//
// MI355X mapping:
//  * a wave owns a 32-env tile; lane l = (env c = l&31, half h = l>>5).  Both halves
//    integrate the env's physics (so every lane holds the full observation) and the
//    networks run on v_mfma_f32_32x32x2_f32 in the transposed orientation
//    Z^T[feature x env] = W^T[feature x in] . X^T[in x env]:  the accumulator of one
//    layer (feature rows in registers, env on the lane) IS the B operand of the next
//    layer, so activations never leave registers in the forward/backward chain.
//  * weights of both nets live in LDS (W2 padded to 65 columns: the same copy is read
//    row-wise for W^T.X and column-wise for W.dZ without bank conflicts).
//  * weight gradients (sums over envs) are MFMAs with the env as K: H1 and dZ are
//    transposed through a per-wave LDS scratch; accumulators persist across the tiles a
//    wave processes and are reduced once per workgroup at the end.
//  * exact f32 arithmetic throughout (f32-input MFMA = k-ordered fmaf chain).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <new>

#include "../../include/reacher_distill.h"
#include "rd_common.h"
#include "rd_physics.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int OBD = 11, HID = 64, ACD = 2;
constexpr int P_W1 = 0;
constexpr int P_B1 = P_W1 + OBD * HID;   // 704
constexpr int P_W2 = P_B1 + HID;         // 768
constexpr int P_B2 = P_W2 + HID * HID;   // 4864
constexpr int P_W3 = P_B2 + HID;         // 4928
constexpr int P_B3 = P_W3 + HID * ACD;   // 5056
constexpr int P_LS = P_B3 + ACD;         // 5058
constexpr int P_TOT = P_LS + ACD;        // 5060
constexpr int P_PAD = P_TOT + 4;         // + metrics: reward, loss, sq err, envs
constexpr int N_MET = 4;

constexpr int WAVES = 4, BLOCK = 64 * WAVES;
constexpr int LDW = 65;   // padded row length of W2 and of the scratch tiles

// per-network LDS image (floats)
constexpr int N_W1 = 0;                  // [12][64], row 11 = 0 (K padded to 12)
constexpr int N_B1 = N_W1 + 12 * HID;
constexpr int N_W2 = N_B1 + HID;         // [64][65]
constexpr int N_B2 = N_W2 + HID * LDW;
constexpr int N_W3 = N_B2 + HID;         // [64][2]
constexpr int N_B3 = N_W3 + HID * ACD;
constexpr int N_LS = N_B3 + ACD;
constexpr int N_MU = N_LS + ACD;         // [12]
constexpr int N_RS = N_MU + 12;          // [12] 1/std (0 in the pad)
constexpr int NET = ((N_RS + 12) + 3) & ~3;
// per-wave scratch (floats)
constexpr int S_TILE = 32 * LDW;
constexpr int S_B0 = 0, S_B1 = S_TILE, S_B2 = 2 * S_TILE, S_DM = 3 * S_TILE;
constexpr int SCR = 3 * S_TILE + 64;
constexpr int LDS_FLOATS = 2 * NET + WAVES * SCR;
static_assert(WAVES * P_PAD <= WAVES * SCR, "final reduction must fit in the scratch");
static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");

struct RolloutArgs {
    int64_t n, env_base;
    uint64_t seed;
    float* state;                          // [8][n]
    const float* tnet;                     // teacher: params[P], mu[11], sd[11] (contiguous)
    const float* snet;                     // student
    uint32_t* ctl;                         // [0] completed steps, [4..7] snapshot
    float* ws;                             // [gridDim.x][P_PAD]
    int loss, act_student, stagger;
    float inv_n_global;
};

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// accumulator register r of lane-half h holds feature row featD(r, h) (+32 per block)
__device__ __forceinline__ int featD(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ float tanh_f(float x) {
    // 1 - 2/(exp(2x)+1): one v_exp_f32 + one v_rcp_f32; saturates correctly at +-inf
    const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);
    return 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
}

// The per-wave scratch is private to its wave: LDS instructions of one wave execute in
// issue order, so staging needs only a compiler-level barrier, not s_barrier.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// global net = params[P] | mu[11] | sd[11]  ->  LDS image
__device__ void load_net(float* L, const float* g) {
    const float* mu = g + P_TOT;
    const float* sd = g + P_TOT + OBD;
    for (int i = threadIdx.x; i < 12 * HID; i += BLOCK) {
        const int k = i >> 6;
        L[N_W1 + i] = k < OBD ? g[P_W1 + i] : 0.0f;
    }
    for (int i = threadIdx.x; i < HID * HID; i += BLOCK) L[N_W2 + (i >> 6) * LDW + (i & 63)] = g[P_W2 + i];
    for (int i = threadIdx.x; i < HID; i += BLOCK) {
        L[N_B1 + i] = g[P_B1 + i];
        L[N_B2 + i] = g[P_B2 + i];
    }
    for (int i = threadIdx.x; i < HID * ACD; i += BLOCK) L[N_W3 + i] = g[P_W3 + i];
    if (threadIdx.x < ACD) {
        L[N_B3 + threadIdx.x] = g[P_B3 + threadIdx.x];
        L[N_LS + threadIdx.x] = g[P_LS + threadIdx.x];
    }
    if (threadIdx.x < 12) {
        const int k = threadIdx.x;
        L[N_MU + k] = k < OBD ? mu[k] : 0.0f;
        L[N_RS + k] = k < OBD ? 1.0f / sd[k] : 0.0f;
    }
}

// MlpPolicy forward for the lane's env (obs in registers): H1, H2 in accumulator layout,
// z = filtered observation, (m0, m1) = action mean (identical in both halves).
__device__ __forceinline__ void mlp_forward(const float* L, const float ob[OBD], int lane, f32x16 (&H1)[2],
                                            f32x16 (&H2)[2], float (&z)[12], float& m0, float& m1) {
    const int h = lane >> 5, c = lane & 31;
#pragma unroll
    for (int k = 0; k < OBD; ++k) z[k] = fminf(fmaxf((ob[k] - L[N_MU + k]) * L[N_RS + k], -5.0f), 5.0f);
    z[11] = 0.0f;
    f32x16 a0, a1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        a0[r] = L[N_B1 + featD(r, h)];
        a1[r] = L[N_B1 + 32 + featD(r, h)];
    }
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const float b = h ? z[2 * s + 1] : z[2 * s];
        const float* w = L + N_W1 + (2 * s + h) * HID + c;
        a0 = mfma(w[0], b, a0);
        a1 = mfma(w[32], b, a1);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        H1[0][r] = tanh_f(a0[r]);
        H1[1][r] = tanh_f(a1[r]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        a0[r] = L[N_B2 + featD(r, h)];
        a1[r] = L[N_B2 + 32 + featD(r, h)];
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float b = H1[kb][r];
            const float* w = L + N_W2 + (32 * kb + featD(r, h)) * LDW + c;
            a0 = mfma(w[0], b, a0);
            a1 = mfma(w[32], b, a1);
        }
    float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        H2[0][r] = tanh_f(a0[r]);
        H2[1][r] = tanh_f(a1[r]);
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = 32 * kb + featD(r, h);
            p0 = fmaf(H2[kb][r], L[N_W3 + 2 * f], p0);
            p1 = fmaf(H2[kb][r], L[N_W3 + 2 * f + 1], p1);
        }
    p0 += __shfl_xor(p0, 32);
    p1 += __shfl_xor(p1, 32);
    m0 = p0 + L[N_B3];
    m1 = p1 + L[N_B3 + 1];
}

__global__ __launch_bounds__(BLOCK, 1) void rollout_kernel(RolloutArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
    float* LT = lds;
    float* LS = lds + NET;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane >> 5, c = lane & 31;
    float* S = lds + 2 * NET + wave * SCR;

    load_net(LT, a.tnet);
    load_net(LS, a.snet);

    const uint32_t C = a.ctl[0];
    // snapshot of the step words for reduce_adam_kernel, which rewrites ctl[0..3]
    if (blockIdx.x == 0 && threadIdx.x < 4) a.ctl[4 + threadIdx.x] = a.ctl[threadIdx.x];

    // teacher / student log-std (state independent)
    const float tl0 = a.tnet[P_LS], tl1 = a.tnet[P_LS + 1];
    const float sl0 = a.snet[P_LS], sl1 = a.snet[P_LS + 1];
    const float tv0 = __expf(2.0f * tl0), tv1 = __expf(2.0f * tl1);
    const float sv0 = __expf(2.0f * sl0), sv1 = __expf(2.0f * sl1);

    f32x16 gW2[2][2], gW1[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        gW2[0][0][r] = gW2[0][1][r] = gW2[1][0][r] = gW2[1][1][r] = 0.0f;
        gW1[0][r] = gW1[1][r] = 0.0f;
    }
    float gb1 = 0, gb2 = 0, gw3a = 0, gw3b = 0, gb3a = 0, gb3b = 0, gls0 = 0, gls1 = 0;
    float met_r = 0, met_l = 0, met_m = 0, met_n = 0;
    __syncthreads();

    const int64_t ntiles = (a.n + 31) / 32;
    for (int64_t t0 = (int64_t)blockIdx.x * WAVES; t0 < ntiles; t0 += (int64_t)gridDim.x * WAVES) {
        const int64_t i = (t0 + wave) * 32 + c;
        const bool valid = i < a.n;
        // ---------------------------------------------------------------- observe
        rd::State st{};
        if (valid) {
            const float* s = a.state;
            const int64_t n = a.n;
            st.q0 = s[i]; st.q1 = s[n + i]; st.v0 = s[2 * n + i]; st.v1 = s[3 * n + i];
            st.tx = s[4 * n + i]; st.ty = s[5 * n + i]; st.dx = s[6 * n + i]; st.dy = s[7 * n + i];
        }
        float ob[OBD];
        rd::observe(st, ob);
        // ---------------------------------------------------------------- teacher
        float mt0, mt1, ms0, ms1;
        f32x16 H1[2], H2[2];
        float z[12];
        mlp_forward(LT, ob, lane, H1, H2, z, mt0, mt1);
        // ---------------------------------------------------------------- student
        mlp_forward(LS, ob, lane, H1, H2, z, ms0, ms1);
        // ---------------------------------------------------------------- loss
        const float d0 = ms0 - mt0, d1 = ms1 - mt1;
        float dm0, dm1, dl0 = 0.0f, dl1 = 0.0f, lossv;
        if (a.loss == RDD_LOSS_MSE) {
            dm0 = d0 * a.inv_n_global;
            dm1 = d1 * a.inv_n_global;
            lossv = (d0 * d0 + d1 * d1) * (0.5f * a.inv_n_global);
        } else {
            dm0 = d0 / tv0;
            dm1 = d1 / tv1;
            dl0 = sv0 / tv0 - 1.0f;
            dl1 = sv1 / tv1 - 1.0f;
            lossv = (tl0 - sl0 + (sv0 + d0 * d0) / (2.0f * tv0) - 0.5f) +
                    (tl1 - sl1 + (sv1 + d1 * d1) / (2.0f * tv1) - 0.5f);
        }
        if (!valid) { dm0 = dm1 = dl0 = dl1 = 0.0f; }
        // ---------------------------------------------------------------- env.step
        const float ac0 = a.act_student ? ms0 : mt0;
        const float ac1 = a.act_student ? ms1 : mt1;
        const float rew = rd::env_step(st, ac0, ac1);
        // episode clock of this env (RDD_STAGGER_GROUP envs share an offset: wave-uniform
        // unless a tile straddles a group boundary)
        const int64_t g = a.env_base + i;
        const uint32_t u = C + (a.stagger ? (uint32_t)((g / RDD_STAGGER_GROUP) % rd::kEpisodeSteps) : 0u);
        const bool done_step = (u % rd::kEpisodeSteps) == rd::kEpisodeSteps - 1;
        if (done_step) {
            float dr[6];
            rd::philox_draw(a.seed, (uint64_t)g, u / rd::kEpisodeSteps + 1, dr);
            rd::env_reset(st, dr);
        }
        if (valid && h == 0) {
            float* s = a.state;
            const int64_t n = a.n;
            s[i] = st.q0; s[n + i] = st.q1; s[2 * n + i] = st.v0; s[3 * n + i] = st.v1;
            if (done_step) { s[4 * n + i] = st.tx; s[5 * n + i] = st.ty; }
            s[6 * n + i] = st.dx; s[7 * n + i] = st.dy;
            met_r += rew;
            met_l += lossv;
            met_m += d0 * d0 + d1 * d1;
            met_n += 1.0f;
            gb3a += dm0; gb3b += dm1; gls0 += dl0; gls1 += dl1;
        }
        // ---------------------------------------------------------------- backward
        // dZ2 = (W3 . dmean) * (1 - H2^2)   (registers, accumulator layout)
        f32x16 dZ[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * kb + featD(r, h);
                const float dh = fmaf(LS[N_W3 + 2 * f], dm0, LS[N_W3 + 2 * f + 1] * dm1);
                dZ[kb][r] = dh * (1.0f - H2[kb][r] * H2[kb][r]);
            }
        // stage H1 | dZ2 | H2 | dmean (env-major rows) for the env-summed products
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = 32 * kb + featD(r, h);
                S[S_B0 + c * LDW + f] = H1[kb][r];
                S[S_B1 + c * LDW + f] = dZ[kb][r];
                S[S_B2 + c * LDW + f] = H2[kb][r];
            }
        if (h == 0) {
            S[S_DM + 2 * c] = dm0;
            S[S_DM + 2 * c + 1] = dm1;
        }
        wave_sync();
        // dW2 += H1^T dZ2 over the tile's 32 envs (K = env pairs)
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const float* r0 = S + S_B0 + (2 * s + h) * LDW + c;
            const float* r1 = S + S_B1 + (2 * s + h) * LDW + c;
            const float x0 = r0[0], x1 = r0[32], y0 = r1[0], y1 = r1[32];
            gW2[0][0] = mfma(x0, y0, gW2[0][0]);
            gW2[0][1] = mfma(x0, y1, gW2[0][1]);
            gW2[1][0] = mfma(x1, y0, gW2[1][0]);
            gW2[1][1] = mfma(x1, y1, gW2[1][1]);
        }
        // db2, dW3: lane = feature, loop over envs
#pragma unroll 8
        for (int e = 0; e < 32; ++e) {
            gb2 += S[S_B1 + e * LDW + lane];
            const float hv = S[S_B2 + e * LDW + lane];
            gw3a = fmaf(hv, S[S_DM + 2 * e], gw3a);
            gw3b = fmaf(hv, S[S_DM + 2 * e + 1], gw3b);
        }
        // dH1 = W2 . dZ2  (A = W2 read column-wise from the padded image)
        f32x16 acc0, acc1;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.0f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = 32 * kb + featD(r, h);
                const float b = dZ[kb][r];
                acc0 = mfma(LS[N_W2 + c * LDW + k], b, acc0);
                acc1 = mfma(LS[N_W2 + (32 + c) * LDW + k], b, acc1);
            }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            dZ[0][r] = acc0[r] * (1.0f - H1[0][r] * H1[0][r]);
            dZ[1][r] = acc1[r] * (1.0f - H1[1][r] * H1[1][r]);
        }
        wave_sync();
        // stage dZ1 and the student's filtered observation z (cols 0..31, zero-padded)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) S[S_B1 + c * LDW + 32 * kb + featD(r, h)] = dZ[kb][r];
#pragma unroll
        for (int k = 0; k < 16; ++k) S[S_B0 + c * LDW + 16 * h + k] = (h == 0 && k < 12) ? z[k] : 0.0f;
        wave_sync();
        // dW1 += z^T dZ1  (rows = input feature, only 0..10 meaningful)
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const float x = S[S_B0 + (2 * s + h) * LDW + c];
            const float* r1 = S + S_B1 + (2 * s + h) * LDW + c;
            gW1[0] = mfma(x, r1[0], gW1[0]);
            gW1[1] = mfma(x, r1[32], gW1[1]);
        }
#pragma unroll 8
        for (int e = 0; e < 32; ++e) gb1 += S[S_B1 + e * LDW + lane];
        wave_sync();
    }

    __syncthreads();   // the reduction below reuses every wave's scratch
    // ---------------------------------------------------------------- workgroup reduction
    float* R = lds + 2 * NET + wave * P_PAD;   // reuses the scratch (all tiles done)
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                R[P_W2 + (32 * mb + featD(r, h)) * HID + 32 * nb + c] = gW2[mb][nb][r];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = featD(r, h);
            if (k < OBD) R[P_W1 + k * HID + 32 * nb + c] = gW1[nb][r];
        }
    R[P_B1 + lane] = gb1;
    R[P_B2 + lane] = gb2;
    R[P_W3 + 2 * lane] = gw3a;
    R[P_W3 + 2 * lane + 1] = gw3b;
    gb3a = wave_sum(gb3a); gb3b = wave_sum(gb3b);
    gls0 = wave_sum(gls0); gls1 = wave_sum(gls1);
    met_r = wave_sum(met_r); met_l = wave_sum(met_l); met_m = wave_sum(met_m); met_n = wave_sum(met_n);
    if (lane == 0) {
        R[P_B3] = gb3a; R[P_B3 + 1] = gb3b; R[P_LS] = gls0; R[P_LS + 1] = gls1;
        R[P_TOT] = met_r; R[P_TOT + 1] = met_l; R[P_TOT + 2] = met_m; R[P_TOT + 3] = met_n;
    }
    __syncthreads();
    const float* R0 = lds + 2 * NET;
    float* out = a.ws + (int64_t)blockIdx.x * P_PAD;
    for (int p = threadIdx.x; p < P_PAD; p += BLOCK) {
        float s = R0[p];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) s += R0[w * P_PAD + p];
        out[p] = s;
    }
}

// ctl words: [0] completed steps C, [2] beta1^t, [3] beta2^t (f32 bits); [4..7] the
// rollout's snapshot of [0..3], which this kernel reads so that block 0 may rewrite
// [0..3] without racing the other blocks (no atomics, no fences: stream order suffices).
struct ReduceArgs {
    const float* ws;
    int nblk;
    float* grad;       // [P]
    float* params;     // student params [P] (in the student net buffer)
    float* m;
    float* v;
    uint32_t* ctl;
    float* hist;       // [hist_len][4]
    int hist_len;
    int reduce, adam, bump;
    float lr, b1, b2, eps;
};

constexpr int RED_COLS = 64;                        // params per reduce block
constexpr int RED_ROWS = 16;                        // partial rows summed in parallel
constexpr int RED_BLOCK = RED_COLS * RED_ROWS;
constexpr int RED_GRID = (P_PAD + RED_COLS - 1) / RED_COLS;

// Sum the rollout's per-workgroup partials (fixed order: deterministic), then TF1 Adam.
__global__ __launch_bounds__(RED_BLOCK) void reduce_adam_kernel(ReduceArgs a) {
    __shared__ float part[RED_ROWS][RED_COLS];
    const uint32_t C = a.ctl[4];
    const float b1p = __uint_as_float(a.ctl[6]), b2p = __uint_as_float(a.ctl[7]);
    const int col = threadIdx.x & (RED_COLS - 1), row = threadIdx.x / RED_COLS;
    const int p = blockIdx.x * RED_COLS + col;
    if (a.reduce) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        if (p < P_PAD) {
            const float* w = a.ws + p;
            int b = row;
#pragma unroll 4
            for (; b + 3 * RED_ROWS < a.nblk; b += 4 * RED_ROWS) {
                s0 += w[(int64_t)b * P_PAD];
                s1 += w[(int64_t)(b + RED_ROWS) * P_PAD];
                s2 += w[(int64_t)(b + 2 * RED_ROWS) * P_PAD];
                s3 += w[(int64_t)(b + 3 * RED_ROWS) * P_PAD];
            }
            for (; b < a.nblk; b += RED_ROWS) s0 += w[(int64_t)b * P_PAD];
        }
        part[row][col] = (s0 + s1) + (s2 + s3);
    }
    __syncthreads();
    if (row == 0 && p < P_PAD) {
        float g;
        if (a.reduce) {
            float q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < RED_ROWS; ++r) q[r & 3] += part[r][col];
            g = (q[0] + q[1]) + (q[2] + q[3]);
            if (p < P_TOT) a.grad[p] = g;
            else a.hist[(int64_t)(C % (uint32_t)a.hist_len) * N_MET + (p - P_TOT)] = g;
        } else {
            g = p < P_TOT ? a.grad[p] : 0.f;
        }
        if (a.adam && p < P_TOT) {
            // TF1 ApplyAdam functor (training_ops.cc)
            const float alpha = a.lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
            float m = a.m[p], v = a.v[p];
            m += (g - m) * (1.0f - a.b1);
            v += (g * g - v) * (1.0f - a.b2);
            a.m[p] = m;
            a.v[p] = v;
            a.params[p] -= (m * alpha) / (sqrtf(v) + a.eps);
        }
    }
    if (a.bump && blockIdx.x == 0 && threadIdx.x == 0) {
        a.ctl[0] = C + 1u;
        a.ctl[2] = __float_as_uint(b1p * a.b1);
        a.ctl[3] = __float_as_uint(b2p * a.b2);
    }
}

__global__ __launch_bounds__(256) void reset_state_kernel(int64_t n, int64_t env_base, uint64_t seed, float* state) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float d[6];
    rd::philox_draw(seed, (uint64_t)(env_base + i), 0u, d);
    rd::State st;
    rd::env_reset(st, d);
    state[i] = st.q0; state[n + i] = st.q1; state[2 * n + i] = st.v0; state[3 * n + i] = st.v1;
    state[4 * n + i] = st.tx; state[5 * n + i] = st.ty; state[6 * n + i] = st.dx; state[7 * n + i] = st.dy;
}

__global__ __launch_bounds__(256) void init_ctl_kernel(uint32_t* ctl, float b1, float b2) {
    if (threadIdx.x < 2) {
        const int o = 4 * threadIdx.x;   // live words and their snapshot
        ctl[o] = 0u; ctl[o + 1] = 0u; ctl[o + 2] = __float_as_uint(b1); ctl[o + 3] = __float_as_uint(b2);
    }
}

// policy query: obs rows -> pdflat of teacher and/or student (one 32-env tile per wave)
__global__ __launch_bounds__(BLOCK, 1) void forward_kernel(const float* tnet, const float* snet, const float* obs,
                                                           int64_t n, float* tflat, float* sflat) {
    __shared__ __attribute__((aligned(16))) float lds[2 * NET];
    load_net(lds, tnet);
    load_net(lds + NET, snet);
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31;
    const int64_t ntiles = (n + 31) / 32;
    for (int64_t t0 = (int64_t)blockIdx.x * WAVES + wave; t0 < ntiles; t0 += (int64_t)gridDim.x * WAVES) {
        const int64_t i = t0 * 32 + c;
        float ob[OBD];
#pragma unroll
        for (int k = 0; k < OBD; ++k) ob[k] = i < n ? obs[i * OBD + k] : 0.0f;
        f32x16 H1[2], H2[2];
        float z[12], m0, m1;
        for (int net = 0; net < 2; ++net) {
            float* out = net ? sflat : tflat;
            if (!out) continue;   // wave-uniform
            const float* L = lds + net * NET;
            mlp_forward(L, ob, lane, H1, H2, z, m0, m1);
            if (i < n && lane < 32) {
                out[i * 4 + 0] = m0;
                out[i * 4 + 1] = m1;
                out[i * 4 + 2] = L[N_LS];
                out[i * 4 + 3] = L[N_LS + 1];
            }
        }
    }
}

int num_cus(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 256;
    return prop.multiProcessorCount;
}

}  // namespace

struct rdd_trainer {
    rdd_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    int grid = 0;
    float* state = nullptr;    // [8][n]
    float* tnet = nullptr;     // [P + 22]
    float* snet = nullptr;     // [P + 22]
    float* m = nullptr;
    float* v = nullptr;
    float* grad = nullptr;     // [P] (own or bound)
    float* own_grad = nullptr;
    float* ws = nullptr;       // [grid][P_PAD]
    float* hist = nullptr;     // [hist_len][4]
    uint32_t* ctl = nullptr;   // [8]: step words + snapshot
};

namespace {

int launch_rollout(rdd_trainer* t) {
    RolloutArgs a;
    a.n = t->cfg.n_envs;
    a.env_base = t->cfg.env_base;
    a.seed = t->cfg.seed;
    a.state = t->state;
    a.tnet = t->tnet;
    a.snet = t->snet;
    a.ctl = t->ctl;
    a.ws = t->ws;
    a.loss = t->cfg.loss;
    a.act_student = t->cfg.act_with == RDD_ACT_STUDENT;
    a.stagger = t->cfg.stagger;
    a.inv_n_global = 1.0f / (float)t->cfg.n_envs_global;
    hipLaunchKernelGGL(rollout_kernel, dim3(t->grid), dim3(BLOCK), 0, t->stream, a);
    RD_HIP(hipGetLastError(), "rollout_kernel launch");
    return RD_OK;
}

int launch_reduce(rdd_trainer* t, int reduce, int adam, int bump) {
    ReduceArgs a;
    a.ws = t->ws;
    a.nblk = t->grid;
    a.grad = t->grad;
    a.params = t->snet;
    a.m = t->m;
    a.v = t->v;
    a.ctl = t->ctl;
    a.hist = t->hist;
    a.hist_len = t->cfg.metrics_len;
    a.reduce = reduce;
    a.adam = adam;
    a.bump = bump;
    a.lr = t->cfg.lr;
    a.b1 = t->cfg.beta1;
    a.b2 = t->cfg.beta2;
    a.eps = t->cfg.eps;
    hipLaunchKernelGGL(reduce_adam_kernel, dim3(RED_GRID), dim3(RED_BLOCK), 0, t->stream, a);
    RD_HIP(hipGetLastError(), "reduce_adam_kernel launch");
    return RD_OK;
}

}  // namespace

extern "C" {

int rdd_param_count(void) { return P_TOT; }

int rdd_set_stream(rdd_trainer* t, void* hip_stream) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_set_stream: null handle");
    t->stream = (hipStream_t)hip_stream;
    return RD_OK;
}

int rdd_create(rdd_trainer** out, const rdd_config* cfg, int device, void* hip_stream) {
    if (!out || !cfg) return rd::set_error(RD_EINVAL, "rdd_create: null argument");
    if (cfg->n_envs <= 0 || cfg->n_envs_global < cfg->n_envs || cfg->env_base < 0 ||
        cfg->n_envs > ((int64_t)1 << 31) || (cfg->loss != RDD_LOSS_MSE && cfg->loss != RDD_LOSS_KL) ||
        (cfg->act_with != RDD_ACT_TEACHER && cfg->act_with != RDD_ACT_STUDENT) || !(cfg->lr > 0) ||
        cfg->grid < 0 || cfg->metrics_len < 0 || (cfg->stagger != 0 && cfg->stagger != 1))
        return rd::set_error(RD_EINVAL, "rdd_create: bad config");
    rd::DeviceGuard g(device);
    RD_HIP(g.err, "rdd_create: hipSetDevice");
    rdd_trainer* t = new (std::nothrow) rdd_trainer();
    if (!t) return rd::set_error(RD_EINVAL, "rdd_create: out of host memory");
    t->cfg = *cfg;
    if (t->cfg.metrics_len == 0) t->cfg.metrics_len = 4096;
    t->device = device;
    t->stream = (hipStream_t)hip_stream;
    const int64_t ntiles = (cfg->n_envs + 31) / 32;
    const int64_t want = (ntiles + WAVES - 1) / WAVES;
    const int cap = cfg->grid > 0 ? cfg->grid : num_cus(device);
    t->grid = (int)(want < cap ? want : cap);
    const size_t netf = P_TOT + 2 * OBD;
    hipError_t e = hipSuccess;
    auto alloc = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(p, bytes);
        if (e == hipSuccess) e = hipMemsetAsync(*p, 0, bytes, t->stream);
    };
    alloc((void**)&t->state, sizeof(float) * 8 * cfg->n_envs);
    alloc((void**)&t->tnet, sizeof(float) * netf);
    alloc((void**)&t->snet, sizeof(float) * netf);
    alloc((void**)&t->m, sizeof(float) * P_TOT);
    alloc((void**)&t->v, sizeof(float) * P_TOT);
    alloc((void**)&t->own_grad, sizeof(float) * P_TOT);
    t->grad = t->own_grad;
    alloc((void**)&t->ws, sizeof(float) * (size_t)t->grid * P_PAD);
    alloc((void**)&t->hist, sizeof(float) * (size_t)t->cfg.metrics_len * N_MET);
    alloc((void**)&t->ctl, sizeof(uint32_t) * 8);
    if (e != hipSuccess) {
        rdd_destroy(t);
        return rd::hip_fail(e, "rdd_create: allocation");
    }
    *out = t;
    return RD_OK;
}

int rdd_destroy(rdd_trainer* t) {
    if (!t) return RD_OK;
    rd::DeviceGuard g(t->device);
    for (void* p : {(void*)t->state, (void*)t->tnet, (void*)t->snet, (void*)t->m, (void*)t->v, (void*)t->own_grad,
                    (void*)t->ws, (void*)t->hist, (void*)t->ctl})
        if (p) (void)hipFree(p);
    delete t;
    return RD_OK;
}

static int set_net(rdd_trainer* t, float* dst, const float* params, const float* mu, const float* sd,
                   const char* what) {
    if (!t || !params || !mu || !sd) return rd::set_error(RD_EINVAL, "%s: null argument", what);
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, what);
    RD_HIP(hipMemcpyAsync(dst, params, sizeof(float) * P_TOT, hipMemcpyDeviceToDevice, t->stream), what);
    RD_HIP(hipMemcpyAsync(dst + P_TOT, mu, sizeof(float) * OBD, hipMemcpyDeviceToDevice, t->stream), what);
    RD_HIP(hipMemcpyAsync(dst + P_TOT + OBD, sd, sizeof(float) * OBD, hipMemcpyDeviceToDevice, t->stream), what);
    return RD_OK;
}

int rdd_set_teacher(rdd_trainer* t, const float* p, const float* mu, const float* sd) {
    return set_net(t, t ? t->tnet : nullptr, p, mu, sd, "rdd_set_teacher");
}

int rdd_set_student(rdd_trainer* t, const float* p, const float* mu, const float* sd) {
    return set_net(t, t ? t->snet : nullptr, p, mu, sd, "rdd_set_student");
}

int rdd_get_student(rdd_trainer* t, float* params) {
    if (!t || !params) return rd::set_error(RD_EINVAL, "rdd_get_student: null argument");
    rd::DeviceGuard g(t->device);
    RD_HIP(hipMemcpyAsync(params, t->snet, sizeof(float) * P_TOT, hipMemcpyDeviceToDevice, t->stream),
           "rdd_get_student");
    return RD_OK;
}

int rdd_reset(rdd_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_reset: null handle");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_reset: hipSetDevice");
    const int64_t n = t->cfg.n_envs;
    hipLaunchKernelGGL(reset_state_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, t->stream, n,
                       t->cfg.env_base, t->cfg.seed, t->state);
    hipLaunchKernelGGL(init_ctl_kernel, dim3(1), dim3(64), 0, t->stream, t->ctl, t->cfg.beta1, t->cfg.beta2);
    RD_HIP(hipMemsetAsync(t->m, 0, sizeof(float) * P_TOT, t->stream), "rdd_reset");
    RD_HIP(hipMemsetAsync(t->v, 0, sizeof(float) * P_TOT, t->stream), "rdd_reset");
    RD_HIP(hipGetLastError(), "rdd_reset: launch");
    return RD_OK;
}

int rdd_rollout(rdd_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_rollout: null handle");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_rollout: hipSetDevice");
    if (int rc = launch_rollout(t)) return rc;
    return launch_reduce(t, 1, 0, 0);
}

int rdd_apply(rdd_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_apply: null handle");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_apply: hipSetDevice");
    return launch_reduce(t, 0, 1, 1);
}

int rdd_step(rdd_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_step: null handle");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_step: hipSetDevice");
    if (int rc = launch_rollout(t)) return rc;
    return launch_reduce(t, 1, 1, 1);
}

int rdd_launch_stage(rdd_trainer* t, int stage) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_launch_stage: null handle");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_launch_stage: hipSetDevice");
    switch (stage) {
        case RDD_STAGE_ROLLOUT: return launch_rollout(t);
        case RDD_STAGE_REDUCE: return launch_reduce(t, 1, 0, 0);
        case RDD_STAGE_APPLY: return launch_reduce(t, 0, 1, 1);
        case RDD_STAGE_REDUCE_APPLY: return launch_reduce(t, 1, 1, 1);
        default: return rd::set_error(RD_EINVAL, "rdd_launch_stage: bad stage %d", stage);
    }
}

float* rdd_grad_buffer(rdd_trainer* t) { return t ? t->grad : nullptr; }

int rdd_bind_grad_buffer(rdd_trainer* t, float* grad) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_bind_grad_buffer: null handle");
    t->grad = grad ? grad : t->own_grad;
    return RD_OK;
}

int rdd_forward(rdd_trainer* t, const float* obs, int64_t n, float* tflat, float* sflat) {
    if (!t || !obs || n <= 0) return rd::set_error(RD_EINVAL, "rdd_forward: bad argument");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_forward: hipSetDevice");
    const int64_t ntiles = (n + 31) / 32;
    int64_t blocks = (ntiles + WAVES - 1) / WAVES;
    if (blocks > 4 * num_cus(t->device)) blocks = 4 * num_cus(t->device);
    hipLaunchKernelGGL(forward_kernel, dim3((unsigned)blocks), dim3(BLOCK), 0, t->stream, t->tnet, t->snet, obs,
                       n, tflat, sflat);
    RD_HIP(hipGetLastError(), "forward_kernel launch");
    return RD_OK;
}

int rdd_get_env_state(rdd_trainer* t, float* state) {
    if (!t || !state) return rd::set_error(RD_EINVAL, "rdd_get_env_state: null argument");
    rd::DeviceGuard g(t->device);
    RD_HIP(hipMemcpyAsync(state, t->state, sizeof(float) * 8 * t->cfg.n_envs, hipMemcpyDeviceToDevice, t->stream),
           "rdd_get_env_state");
    return RD_OK;
}

int rdd_set_env_state(rdd_trainer* t, const float* state) {
    if (!t || !state) return rd::set_error(RD_EINVAL, "rdd_set_env_state: null argument");
    rd::DeviceGuard g(t->device);
    RD_HIP(hipMemcpyAsync(t->state, state, sizeof(float) * 8 * t->cfg.n_envs, hipMemcpyDeviceToDevice, t->stream),
           "rdd_set_env_state");
    return RD_OK;
}

int rdd_get_counter(rdd_trainer* t, int64_t* steps) {
    if (!t || !steps) return rd::set_error(RD_EINVAL, "rdd_get_counter: null argument");
    rd::DeviceGuard g(t->device);
    uint32_t c = 0;
    RD_HIP(hipMemcpyAsync(&c, t->ctl, sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream), "rdd_get_counter");
    RD_HIP(hipStreamSynchronize(t->stream), "rdd_get_counter");
    *steps = c;
    return RD_OK;
}

int rdd_read_metrics(rdd_trainer* t, int64_t count, double* out) {
    if (!t || !out || count < 0) return rd::set_error(RD_EINVAL, "rdd_read_metrics: bad argument");
    int64_t steps = 0;
    if (int rc = rdd_get_counter(t, &steps)) return rc;
    const int64_t H = t->cfg.metrics_len;
    if (count > steps || count > H) return rd::set_error(RD_EINVAL, "rdd_read_metrics: only %lld steps kept",
                                                         (long long)(steps < H ? steps : H));
    float* host = new (std::nothrow) float[(size_t)H * N_MET];
    if (!host) return rd::set_error(RD_EINVAL, "rdd_read_metrics: out of host memory");
    hipError_t e = hipMemcpy(host, t->hist, sizeof(float) * H * N_MET, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        delete[] host;
        return rd::hip_fail(e, "rdd_read_metrics");
    }
    for (int64_t k = 0; k < count; ++k) {
        const int64_t s = (steps - count + k) % H;
        for (int j = 0; j < N_MET; ++j) out[k * N_MET + j] = host[s * N_MET + j];
    }
    delete[] host;
    return RD_OK;
}

}  // extern "C"
