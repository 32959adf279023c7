// The reference's own MLP student (include/reacher_student_mlp.h): forward and one
// distillation training step over a batch of rows, for gfx950.
//
// Graph (reference student_nn.py:51-57): 16 -> 24 tanh -> 128 tanh -> 128 -> 32 tanh -> 4.
// Unlike the 2x64 MlpPolicy path (distill.hip), a 16-row tile cannot keep the whole chain
// plus its 24,380 weight gradients in one wave's registers, so a workgroup of 8 waves
// cooperates on 64-row blocks (16-row blocks for small batches, where 64-row blocks would
// leave CUs idle):
//  * every layer is a small GEMM over the block, v_mfma_f32_16x16x4_f32 in the natural
//    orientation (rows x features): A = the block's activations in LDS ([row][feature],
//    row stride = width + 4 so the 16 rows x 4 k of one A operand hit 64 distinct banks),
//    B = the layer's weights, a padded [in][out] image read through L1/L2 (98 KB, shared
//    by every workgroup on the chip);
//  * all activations of the block stay in LDS (139 KB) between the forward and the
//    backward; the backward reuses dead buffers (dZ1 overwrites H3 after dW3 is taken);
//  * weight gradients dW_l = H_{l-1}^T dZ_l are MFMAs with the 64 rows as K; each wave
//    owns a fixed subset of the 100 16x16 gradient blocks and accumulates them in
//    registers across the workgroup's row blocks; bias gradients are per-thread column
//    sums.  One workspace row per workgroup, summed in a fixed order by the Adam kernel
//    (deterministic, no atomics);
//  * exact f32 products (f32-input MFMA); tanh = 1 - 2 / (2^(2 log2(e) z) + 1).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <new>

#include "../../include/reacher_student_mlp.h"
#include "rd_common.h"
#include "rd_physics.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace sm {

constexpr int NL = 5;
constexpr int IN[NL] = {16, 24, 128, 128, 32};
constexpr int OUT[NL] = {24, 128, 128, 32, 4};
constexpr int KP[NL] = {16, 32, 128, 128, 32};   // padded fan-in  (multiple of 16)
constexpr int MP[NL] = {32, 128, 128, 32, 16};   // padded fan-out (multiple of 16)
constexpr bool TANH[NL] = {true, true, false, true, false};

// flat parameter vector: per layer W[in][out] then b[out] (tf.layers.dense order)
constexpr int pw(int l) { return l == 0 ? 0 : pw(l - 1) + IN[l - 1] * OUT[l - 1] + OUT[l - 1]; }
constexpr int P_REF = pw(NL);
static_assert(P_REF == RDM_PARAMS, "flat layout");
// gradient workspace: per layer dW[KP][MP] (row-major) then db[MP]
constexpr int gw(int l) { return l == 0 ? 0 : gw(l - 1) + KP[l - 1] * MP[l - 1] + MP[l - 1]; }
constexpr int gb(int l) { return gw(l) + KP[l] * MP[l]; }
constexpr int GIMG = gw(NL);                    // 25,936
// weight image (zero padding that stays zero): per layer
//   forward  FW[L]: W[k][c] at ((k/16) MP + c) 16 + 4 (k%4) + (k/4)%4
//   backward BW[L]: W[k][c] at ((c/16) KP + k) 16 + 4 (c%4) + (c/4)%4
//   bias     BB[L]: b[c] at c
// so the B operand of 4 consecutive k-steps (k = 16 S + 4 sub + g, sub = 0..3) is one 16-B
// load per lane, in both the forward (K = fan-in) and the backward (K = fan-out) GEMMs.
constexpr int fw(int l) { return l == 0 ? 0 : fw(l - 1) + 2 * KP[l - 1] * MP[l - 1] + MP[l - 1]; }
constexpr int IMG = fw(NL);                     // 51,808
constexpr int PW[NL + 1] = {pw(0), pw(1), pw(2), pw(3), pw(4), pw(5)};
constexpr int GW[NL] = {gw(0), gw(1), gw(2), gw(3), gw(4)};
constexpr int GB[NL] = {gb(0), gb(1), gb(2), gb(3), gb(4)};
constexpr int FW[NL] = {fw(0), fw(1), fw(2), fw(3), fw(4)};
constexpr int BW[NL] = {fw(0) + KP[0] * MP[0], fw(1) + KP[1] * MP[1], fw(2) + KP[2] * MP[2], fw(3) + KP[3] * MP[3],
                        fw(4) + KP[4] * MP[4]};
constexpr int BB[NL] = {BW[0] + KP[0] * MP[0], BW[1] + KP[1] * MP[1], BW[2] + KP[2] * MP[2], BW[3] + KP[3] * MP[3],
                        BW[4] + KP[4] * MP[4]};
constexpr int N_MET = 4;                        // loss, sq err, rows, 0
constexpr int WS_ROW = GIMG + N_MET;

// Activations are stored with the columns of every 16-group permuted, k -> pk(k), so that
// the A operand of 4 consecutive k-steps (k = 16 S + 4 sub + g) is one ds_read_b128.
__host__ __device__ constexpr int pk(int k) { return (k & ~15) | ((k & 3) << 2) | ((k >> 2) & 3); }

constexpr int WAVES = 8, BLOCK = 64 * WAVES;

// LDS buffers [row][pk(feature)], stride = width + 4
constexpr int S_X0 = 20, S_X1 = 36, S_X2 = 132, S_X3 = 132, S_X4 = 36, S_D5 = 20, S_D4 = 36, S_DA = 132;
// Row block of ROWS rows per workgroup pass: 64 (the throughput kernel) or 16 (small
// batches, e.g. the reference's 200-row step: 13 workgroups in parallel instead of 4).
template <int ROWS>
struct Lay {
    static constexpr int RB = ROWS / 16;                   // 16-row MFMA blocks of a row block
    static constexpr int O_X0 = 0;
    static constexpr int O_X1 = O_X0 + ROWS * S_X0;
    static constexpr int O_X2 = O_X1 + ROWS * S_X1;
    static constexpr int O_X3 = O_X2 + ROWS * S_X2;
    static constexpr int O_X4 = O_X3 + ROWS * S_X3;
    static constexpr int O_D5 = O_X4 + ROWS * S_X4;        // layer-5 outputs, then dZ5
    static constexpr int O_D4 = O_D5 + ROWS * S_D5;        // dZ4
    static constexpr int O_DA = O_D4 + ROWS * S_D4;        // dZ3, later dZ1
    static constexpr int LDS_FLOATS = O_DA + ROWS * S_DA;  // 34,816 floats = 136 KiB at 64 rows
    static_assert(ROWS % 16 == 0 && ROWS * 4 <= BLOCK && LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
};
static_assert(S_X0 == KP[0] + 4 && S_X1 == KP[1] + 4 && S_X2 == KP[2] + 4 && S_X3 == KP[3] + 4 &&
                  S_X4 == KP[4] + 4 && S_D5 == MP[4] + 4 && S_D4 == MP[3] + 4 && S_DA == MP[2] + 4,
              "buffer strides");

}  // namespace sm

using namespace sm;

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float tanh_fast(float z) {
    return fmaf(-2.0f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z * 2.8853900817779268f) + 1.0f), 1.0f);
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Output blocks of a [ROWS x 16*NCB] result (RB = ROWS / 16), split over the 8 waves: for
// NCB >= 8 a wave owns NCB/8 column blocks x all RB row blocks (the B operand is shared by
// its row blocks); for NCB < 8 a wave owns at most one block.
template <int NCB, int RB>
struct Part {
    static constexpr int CPW = NCB >= WAVES ? NCB / WAVES : 1;
    static constexpr int RPW = NCB >= WAVES ? RB : 1;
    static_assert(NCB < WAVES || NCB % WAVES == 0, "partition");
    __device__ static bool active(int wave) { return NCB >= WAVES || wave < RB * NCB; }
    __device__ static int rb(int wave, int r) { return NCB >= WAVES ? r : wave % RB; }
    __device__ static int cb(int wave, int c) { return NCB >= WAVES ? wave * CPW + c : wave / RB; }
};

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// Forward of layer L: Y[row][pk(c)] = act(b[c] + sum_k X[row][k] W[k][c]), c = 16 cb + i.
template <int RB, int L, int SI, int SO>
__device__ __forceinline__ void fwd_layer(const float* X, float* Y, const float* img, int wave, int i, int g) {
    constexpr int NCB = MP[L] / 16, KG = (IN[L] + 15) / 16;
    using PT = Part<NCB, RB>;
    if (!PT::active(wave)) return;
    const float* W = img + FW[L];
    const float* bias = img + BB[L];
    f32x4 acc[PT::CPW][PT::RPW];
#pragma unroll
    for (int c = 0; c < PT::CPW; ++c) {
        const float b = bias[16 * PT::cb(wave, c) + i];
#pragma unroll
        for (int r = 0; r < PT::RPW; ++r) acc[c][r] = f32x4{b, b, b, b};
    }
#pragma unroll 2
    for (int S = 0; S < KG; ++S) {   // 4 k-steps per iteration: k = 16 S + 4 sub + g
        f32x4 a[PT::RPW];
#pragma unroll
        for (int r = 0; r < PT::RPW; ++r) a[r] = ld4(X + (16 * PT::rb(wave, r) + i) * SI + 16 * S + 4 * g);
#pragma unroll
        for (int c = 0; c < PT::CPW; ++c) {
            const f32x4 w = ld4(W + ((S * MP[L] + 16 * PT::cb(wave, c) + i) << 4) + 4 * g);
#pragma unroll
            for (int sub = 0; sub < 4; ++sub)
#pragma unroll
                for (int r = 0; r < PT::RPW; ++r) acc[c][r] = mfma(a[r][sub], w[sub], acc[c][r]);
        }
    }
#pragma unroll
    for (int c = 0; c < PT::CPW; ++c)
#pragma unroll
        for (int r = 0; r < PT::RPW; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float v = acc[c][r][q];
                Y[(16 * PT::rb(wave, r) + 4 * g + q) * SO + pk(16 * PT::cb(wave, c) + i)] = TANH[L] ? tanh_fast(v) : v;
            }
}

// Backward data of layer L: out[row][pk(c)] = (sum_m D[row][m] W[c][m]) * act'(H[row][c]),
// c = 16 cb + i an input feature of layer L; act' = 1 - H^2 when layer L-1 ends in tanh
// (H = X_L, the layer's input).
template <int RB, int L, int SD, int SH, int SO>
__device__ __forceinline__ void dgrad_layer(const float* D, const float* H, float* out, const float* img, int wave,
                                            int i, int g) {
    constexpr int NCB = KP[L] / 16, MG = (OUT[L] + 15) / 16;
    using PT = Part<NCB, RB>;
    if (!PT::active(wave)) return;
    const float* W = img + BW[L];
    f32x4 acc[PT::CPW][PT::RPW];
#pragma unroll
    for (int c = 0; c < PT::CPW; ++c)
#pragma unroll
        for (int r = 0; r < PT::RPW; ++r) acc[c][r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int S = 0; S < MG; ++S) {
        f32x4 a[PT::RPW];
#pragma unroll
        for (int r = 0; r < PT::RPW; ++r) a[r] = ld4(D + (16 * PT::rb(wave, r) + i) * SD + 16 * S + 4 * g);
#pragma unroll
        for (int c = 0; c < PT::CPW; ++c) {
            const f32x4 w = ld4(W + ((S * KP[L] + 16 * PT::cb(wave, c) + i) << 4) + 4 * g);
#pragma unroll
            for (int sub = 0; sub < 4; ++sub)
#pragma unroll
                for (int r = 0; r < PT::RPW; ++r) acc[c][r] = mfma(a[r][sub], w[sub], acc[c][r]);
        }
    }
#pragma unroll
    for (int c = 0; c < PT::CPW; ++c)
#pragma unroll
        for (int r = 0; r < PT::RPW; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 16 * PT::rb(wave, r) + 4 * g + q, pos = pk(16 * PT::cb(wave, c) + i);
                float v = acc[c][r][q];
                if (TANH[L - 1]) {
                    const float h = H[row * SH + pos];
                    v *= fmaf(-h, h, 1.0f);
                }
                out[row * SO + pos] = v;
            }
}

// Weight gradient of layer L over the block: G[16kb + 4g + q][16cb + i] += sum_row
// H[row][16kb + 4g + q] D[row][16cb + i].  A wave owns one column block cb = wave % NCB
// (its B operand is loaded once per k-step) and the row blocks kb = wave / NCB + (8/NCB) t.
template <int L>
struct WG {
    static constexpr int NCB = MP[L] / 16, KBN = KP[L] / 16, STEP = WAVES / NCB;
    static constexpr int Q = (KBN + STEP - 1) / STEP;
    static_assert(WAVES % NCB == 0, "wgrad partition");
    __device__ static int kb(int wave, int t) { return wave / NCB + STEP * t; }
    __device__ static bool ok(int wave, int t) { return KBN % STEP == 0 || kb(wave, t) < KBN; }
};

// SrcC fence around one k-step's MFMAs (as distill.hip's fence_begin/fence_end): the
// accumulators pass through an empty asm (memory clobber) before and after them, and each is
// read by a VALU before the closing asm, so no LDS load issues while one of these 8-pass f32
// MFMAs is in flight.  Without it hipcc rotates the accumulators (D = v[20:23], C = v[22:25])
// and issues the next k-step's operand loads into registers an in-flight MFMA still reads as
// SrcC, 0-9 wait states after it (scripts/isa/hazards.py class LDSRC; such a load is lost for
// lanes 48-63 when the MFMA is held in the pipe).
template <int Q>
__device__ __forceinline__ void fence_begin(f32x4 (&G)[Q]) {
#pragma unroll
    for (int t = 0; t < Q; ++t) asm volatile("" : "+v"(G[t])::"memory");
}
template <int Q>
__device__ __forceinline__ void fence_end(f32x4 (&G)[Q]) {
#pragma unroll
    for (int t = 0; t < Q; ++t) G[t][3] = __builtin_amdgcn_fmed3f(G[t][3], G[t][3], G[t][3]);
#pragma unroll
    for (int t = 0; t < Q; ++t) asm volatile("" : "+v"(G[t])::"memory");
}

template <int ROWS, int L, int SH, int SD>
__device__ __forceinline__ void wgrad_layer(const float* H, const float* D, f32x4 (&G)[WG<L>::Q], int wave, int i,
                                            int g) {
    using W = WG<L>;
    const int cb = wave % W::NCB;
#pragma unroll 4
    for (int s = 0; s < ROWS / 4; ++s) {
        const int row = 4 * s + g;
        const float b = D[row * SD + pk(16 * cb + i)];
        float h[W::Q];
#pragma unroll
        for (int t = 0; t < W::Q; ++t) h[t] = W::ok(wave, t) ? H[row * SH + pk(16 * W::kb(wave, t) + i)] : 0.0f;
        fence_begin(G);
#pragma unroll
        for (int t = 0; t < W::Q; ++t)
            if (W::ok(wave, t)) G[t] = mfma(h[t], b, G[t]);
        fence_end(G);
    }
}

// partial-row stores (non-temporal measured no gain: profiles/r05_removed_diagnostic_variants.diff)
__device__ __forceinline__ void wst(float* p, float v) { *p = v; }

template <int L>
__device__ __forceinline__ void store_wgrad(float* ws, const f32x4 (&G)[WG<L>::Q], int wave, int i, int g) {
    using W = WG<L>;
    const int cb = wave % W::NCB;
#pragma unroll
    for (int t = 0; t < W::Q; ++t)
        if (W::ok(wave, t))
#pragma unroll
            for (int q = 0; q < 4; ++q)
                wst(ws + GW[L] + (16 * W::kb(wave, t) + 4 * g + q) * MP[L] + 16 * cb + i, G[t][q]);
}

// bias gradient: thread t < OUT[L] sums column t of dZ_L over the block's rows
template <int ROWS, int L, int SD>
__device__ __forceinline__ void bgrad_layer(const float* D, float& gb, int tid) {
    if (tid < OUT[L]) {
        const int col = pk(tid);
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll 4
        for (int r = 0; r < ROWS; r += 4) {
            s0 += D[(r + 0) * SD + col];
            s1 += D[(r + 1) * SD + col];
            s2 += D[(r + 2) * SD + col];
            s3 += D[(r + 3) * SD + col];
        }
        gb += (s0 + s1) + (s2 + s3);
    }
}

struct SmArgs {
    const float* x;        // [n][16]
    const float* tgt;      // [n][4] teacher pdflat (training)
    float* out;            // [n][4] pdflat (forward)
    int64_t n;
    const float* img;      // weight image [IMG]
    float* ws;             // [gridDim.x][WS_ROW] partials (training)
    uint32_t* ctl;
    int loss;
    float inv_n_global;
    float keep_prob;       // < 1: dropout on inputs 0..10 (training only)
    uint64_t seed;
    int64_t row_base;
};

template <bool TRAIN, int ROWS>
__global__ __launch_bounds__(BLOCK) void student_mlp_kernel(SmArgs a) {
    using LY = Lay<ROWS>;
    constexpr int RB = LY::RB;
    __shared__ __attribute__((aligned(16))) float lds[LY::LDS_FLOATS];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, g = lane >> 4;
    if (TRAIN && blockIdx.x == 0 && tid < 4) a.ctl[4 + tid] = a.ctl[tid];   // snapshot for the Adam kernel
    const uint32_t step = TRAIN ? a.ctl[0] : 0u;   // optimiser step (dropout counter); only Adam writes it
    f32x4 G0[WG<0>::Q], G1[WG<1>::Q], G2[WG<2>::Q], G3[WG<3>::Q], G4[WG<4>::Q];
    auto zero = [](auto& G) {
#pragma unroll
        for (auto& v : G) v = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    zero(G0); zero(G1); zero(G2); zero(G3); zero(G4);
    float gb0 = 0.f, gb1 = 0.f, gb2 = 0.f, gb3 = 0.f, gb4 = 0.f;
    float lsum = 0.f, ssum = 0.f, nrows = 0.f;
    float* X0 = lds + LY::O_X0;
    float* X1 = lds + LY::O_X1;
    float* X2 = lds + LY::O_X2;
    float* X3 = lds + LY::O_X3;
    float* X4 = lds + LY::O_X4;
    float* D5 = lds + LY::O_D5;
    float* D4 = lds + LY::O_D4;
    float* DA = lds + LY::O_DA;
    const int64_t nblk = (a.n + ROWS - 1) / ROWS;
    for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const int64_t row0 = blk * ROWS;
        if (tid < ROWS * 4) {   // ROWS rows x 16 inputs as 16-B vectors
            const int r = tid >> 2, c = tid & 3;
            f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
            if (row0 + r < a.n) v = *reinterpret_cast<const f32x4*>(a.x + (row0 + r) * RDM_IN + 4 * c);
            if (TRAIN && a.keep_prob < 1.0f && c < 3) {   // tf.nn.dropout on the observation
                const uint64_t grow = (uint64_t)(a.row_base + row0 + r);
                uint32_t w[4];
                rd::philox((uint32_t)grow, (uint32_t)(grow >> 32), step, (uint32_t)c, (uint32_t)a.seed,
                           (uint32_t)(a.seed >> 32), w);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (4 * c + k < 11) v[k] = rd::u01(w[k]) < a.keep_prob ? v[k] / a.keep_prob : 0.0f;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) X0[r * S_X0 + pk(4 * c + k)] = v[k];
        }
        __syncthreads();
        fwd_layer<RB, 0, S_X0, S_X1>(X0, X1, a.img, wave, i, g);
        __syncthreads();
        fwd_layer<RB, 1, S_X1, S_X2>(X1, X2, a.img, wave, i, g);
        __syncthreads();
        fwd_layer<RB, 2, S_X2, S_X3>(X2, X3, a.img, wave, i, g);
        __syncthreads();
        fwd_layer<RB, 3, S_X3, S_X4>(X3, X4, a.img, wave, i, g);
        __syncthreads();
        fwd_layer<RB, 4, S_X4, S_D5>(X4, D5, a.img, wave, i, g);
        __syncthreads();
        if constexpr (!TRAIN) {
            // the next block's first write (X0) is ordered after this block's F0 by the barriers above
            if (tid < ROWS * RDM_OUT) {
                const int r = tid >> 2, c = tid & 3;
                if (row0 + r < a.n) a.out[(row0 + r) * RDM_OUT + c] = D5[r * S_D5 + pk(c)];
            }
            continue;
        } else {
            // loss (reference loss.py:3-13 / action-MSE) and dZ5 = dL/dpdflat, one row per thread
            if (tid < ROWS) {
                const int64_t row = row0 + tid;
                float* o = D5 + tid * S_D5;
                float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
                if (row < a.n) {
                    const f32x4 t = *reinterpret_cast<const f32x4*>(a.tgt + row * RDM_OUT);
                    const float e0 = o[pk(0)] - t[0], e1 = o[pk(1)] - t[1];
                    ssum = fmaf(e0, e0, fmaf(e1, e1, ssum));
                    nrows += 1.0f;
                    if (a.loss == RDM_LOSS_MSE) {
                        d0 = e0 * a.inv_n_global;
                        d1 = e1 * a.inv_n_global;
                        lsum = fmaf(0.5f * a.inv_n_global, fmaf(e0, e0, e1 * e1), lsum);
                    } else {
                        const float ivt0 = expf(-2.0f * t[2]), ivt1 = expf(-2.0f * t[3]);
                        const float vs0 = expf(2.0f * o[pk(2)]), vs1 = expf(2.0f * o[pk(3)]);
                        lsum += (t[2] - o[pk(2)]) + 0.5f * (vs0 + e0 * e0) * ivt0 - 0.5f;
                        lsum += (t[3] - o[pk(3)]) + 0.5f * (vs1 + e1 * e1) * ivt1 - 0.5f;
                        d0 = e0 * ivt0;
                        d1 = e1 * ivt1;
                        d2 = fmaf(vs0, ivt0, -1.0f);
                        d3 = fmaf(vs1, ivt1, -1.0f);
                    }
                }
                o[pk(0)] = d0; o[pk(1)] = d1; o[pk(2)] = d2; o[pk(3)] = d3;   // columns 4..15 are exactly 0
            }
            __syncthreads();
            // layer 4 (32 -> 4): dW4, db4, dZ4 = (dZ5 W4^T) * (1 - H4^2)
            wgrad_layer<ROWS, 4, S_X4, S_D5>(X4, D5, G4, wave, i, g);
            bgrad_layer<ROWS, 4, S_D5>(D5, gb4, tid);
            dgrad_layer<RB, 4, S_D5, S_X4, S_D4>(D5, X4, D4, a.img, wave, i, g);
            __syncthreads();
            // layer 3 (128 -> 32): dZ3 = dZ4 W3^T (H3 is linear)
            wgrad_layer<ROWS, 3, S_X3, S_D4>(X3, D4, G3, wave, i, g);
            bgrad_layer<ROWS, 3, S_D4>(D4, gb3, tid);
            dgrad_layer<RB, 3, S_D4, S_X3, S_DA>(D4, X3, DA, a.img, wave, i, g);
            __syncthreads();
            // layer 2 (128 -> 128): dZ2 = (dZ3 W2^T) * (1 - H2^2) into X3's buffer (H3 is dead)
            wgrad_layer<ROWS, 2, S_X2, S_DA>(X2, DA, G2, wave, i, g);
            bgrad_layer<ROWS, 2, S_DA>(DA, gb2, tid);
            dgrad_layer<RB, 2, S_DA, S_X2, S_X3>(DA, X2, X3, a.img, wave, i, g);
            __syncthreads();
            // layer 1 (24 -> 128): dZ1 = (dZ2 W1^T) * (1 - H1^2) into DA
            wgrad_layer<ROWS, 1, S_X1, S_X3>(X1, X3, G1, wave, i, g);
            bgrad_layer<ROWS, 1, S_X3>(X3, gb1, tid);
            dgrad_layer<RB, 1, S_X3, S_X1, S_DA>(X3, X1, DA, a.img, wave, i, g);
            __syncthreads();
            // layer 0 (16 -> 24)
            wgrad_layer<ROWS, 0, S_X0, S_DA>(X0, DA, G0, wave, i, g);
            bgrad_layer<ROWS, 0, S_DA>(DA, gb0, tid);
            __syncthreads();
        }
    }
    if constexpr (TRAIN) {
        float* ws = a.ws + (int64_t)blockIdx.x * WS_ROW;
        store_wgrad<0>(ws, G0, wave, i, g);
        store_wgrad<1>(ws, G1, wave, i, g);
        store_wgrad<2>(ws, G2, wave, i, g);
        store_wgrad<3>(ws, G3, wave, i, g);
        store_wgrad<4>(ws, G4, wave, i, g);
        if (tid < OUT[0]) wst(ws + GB[0] + tid, gb0);
        if (tid < OUT[1]) wst(ws + GB[1] + tid, gb1);
        if (tid < OUT[2]) wst(ws + GB[2] + tid, gb2);
        if (tid < OUT[3]) wst(ws + GB[3] + tid, gb3);
        if (tid < OUT[4]) wst(ws + GB[4] + tid, gb4);
        if (wave == 0) {
            lsum = wave_sum(lsum);
            ssum = wave_sum(ssum);
            nrows = wave_sum(nrows);
            if (lane == 0) {
                ws[GIMG + 0] = lsum;
                ws[GIMG + 1] = ssum;
                ws[GIMG + 2] = nrows;
                ws[GIMG + 3] = 0.f;
            }
        }
    }
}

// flat parameter index -> (layer, k, c) -> positions in the gradient workspace and images
struct PIdx {
    int g;        // workspace (gradient) index
    int f, b;     // image positions (b < 0 for a bias)
};
__device__ __forceinline__ PIdx param_index(int p) {
    int L = 0;
#pragma unroll
    for (int k = 1; k < NL; ++k) L += p >= PW[k] ? 1 : 0;
    int base = 0, in = 0, out = 0, kp = 0, mp = 0, gwo = 0, gbo = 0, fwo = 0, bwo = 0, bbo = 0;
#pragma unroll
    for (int k = 0; k < NL; ++k)
        if (k == L) {
            base = PW[k]; in = IN[k]; out = OUT[k]; kp = KP[k]; mp = MP[k];
            gwo = GW[k]; gbo = GB[k]; fwo = FW[k]; bwo = BW[k]; bbo = BB[k];
        }
    const int o = p - base;
    PIdx r;
    if (o < in * out) {
        const int k = o / out, c = o % out;
        r.g = gwo + k * mp + c;
        r.f = fwo + ((((k >> 4) * mp + c)) << 4) + ((k & 3) << 2) + ((k >> 2) & 3);
        r.b = bwo + ((((c >> 4) * kp + k)) << 4) + ((c & 3) << 2) + ((c >> 2) & 3);
    } else {
        r.g = gbo + (o - in * out);
        r.f = bbo + (o - in * out);
        r.b = -1;
    }
    return r;
}

__device__ __forceinline__ void store_param(float* img, const PIdx& ix, float w) {
    img[ix.f] = w;
    if (ix.b >= 0) img[ix.b] = w;
}

__global__ __launch_bounds__(256) void pack_kernel(const float* params, float* img) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p < P_REF) store_param(img, param_index(p), params[p]);
}

// ctl: [0] optimiser steps S, [1] beta1^S, [2] beta2^S (f32 bits); [4..6] the training
// kernel's snapshot of them (block 0 of the Adam kernel rewrites [0..2]).
struct AdamArgs {
    const float* ws;
    int nblk;
    float* grad;
    float* params;
    float* img;
    float* m;
    float* v;
    uint32_t* ctl;
    float* hist;
    int hist_len;
    int reduce, adam;
    float lr, b1, b2, eps;
};

constexpr int ADAM_BLOCK = 256;
constexpr int ADAM_GRID = (P_REF + N_MET + ADAM_BLOCK - 1) / ADAM_BLOCK;

__global__ __launch_bounds__(ADAM_BLOCK) void reduce_adam_kernel(AdamArgs a) {
    const int p = blockIdx.x * ADAM_BLOCK + threadIdx.x;
    const uint32_t S = a.ctl[4];
    const float b1p = __uint_as_float(a.ctl[5]), b2p = __uint_as_float(a.ctl[6]);
    if (p < P_REF + N_MET) {
        const PIdx ix = p < P_REF ? param_index(p) : PIdx{GIMG + (p - P_REF), 0, -1};
        const int ip = ix.g;
        float gsum;
        if (a.reduce) {
            float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
            const float* w = a.ws + ip;
            int b = 0;
            for (; b + 3 < a.nblk; b += 4) {
                s0 += w[(int64_t)b * WS_ROW];
                s1 += w[(int64_t)(b + 1) * WS_ROW];
                s2 += w[(int64_t)(b + 2) * WS_ROW];
                s3 += w[(int64_t)(b + 3) * WS_ROW];
            }
            for (; b < a.nblk; ++b) s0 += w[(int64_t)b * WS_ROW];
            gsum = (s0 + s1) + (s2 + s3);
            if (p < P_REF) a.grad[p] = gsum;
            else a.hist[(int64_t)(S % (uint32_t)a.hist_len) * N_MET + (p - P_REF)] = gsum;
        } else {
            gsum = p < P_REF ? a.grad[p] : 0.f;
        }
        if (a.adam && p < P_REF) {   // TF1 ApplyAdam (mlp_train.py:75-80)
            const float alpha = a.lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
            float m = a.m[p], v = a.v[p];
            m += (gsum - m) * (1.0f - a.b1);
            v += (gsum * gsum - v) * (1.0f - a.b2);
            a.m[p] = m;
            a.v[p] = v;
            const float w = a.params[p] - (m * alpha) / (sqrtf(v) + a.eps);
            a.params[p] = w;
            store_param(a.img, ix, w);
        }
    }
    if (a.adam && blockIdx.x == 0 && threadIdx.x == 0) {
        a.ctl[0] = S + 1u;
        a.ctl[1] = __float_as_uint(b1p * a.b1);
        a.ctl[2] = __float_as_uint(b2p * a.b2);
    }
}

__global__ void init_ctl_kernel(uint32_t* ctl, float b1, float b2) {
    if (threadIdx.x < 2) {
        const int o = 4 * threadIdx.x;
        ctl[o] = 0u; ctl[o + 1] = __float_as_uint(b1); ctl[o + 2] = __float_as_uint(b2); ctl[o + 3] = 0u;
    }
}

int cu_count(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 256;
    return prop.multiProcessorCount;
}

}  // namespace

struct rdm_trainer {
    rdm_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    int grid = 0;               // workspace rows
    int last_grid = 0;          // workgroups of the last training launch
    float* params = nullptr;    // [P_REF] f32 master
    float* img = nullptr;       // [IMG] weight image (forward + backward layouts)
    float* m = nullptr;
    float* v = nullptr;
    float* grad = nullptr;
    float* own_grad = nullptr;
    float* ws = nullptr;        // [grid][WS_ROW]
    float* hist = nullptr;      // [metrics_len][4]
    uint32_t* ctl = nullptr;    // [8]
};

namespace {

// 16-row blocks for small batches: they are latency-bound, and four times the workgroups
// run the rows in parallel (measured, scripts/bench_student_mlp.py: the reference's 200-row
// step 21.8 us vs 35.8 us with 64-row blocks, 1,024 rows 27.2 vs 37.4 us).  Every workgroup
// writes a 104 KB partial row, so once the 16-row blocks would occupy more than half of the
// workgroups the 64-row kernel wins (4,096 rows: 51.2 vs 42.4 us).
bool use_small_rows(int64_t n, int grid) {
    return (n + 15) / 16 <= grid / 2;
}

int launch_train(rdm_trainer* t, const float* x, const float* tgt, int64_t n, int64_t n_global) {
    SmArgs a;
    a.x = x;
    a.tgt = tgt;
    a.out = nullptr;
    a.n = n;
    a.img = t->img;
    a.ws = t->ws;
    a.ctl = t->ctl;
    a.loss = t->cfg.loss;
    a.inv_n_global = 1.0f / (float)n_global;
    a.keep_prob = t->cfg.keep_prob;
    a.seed = t->cfg.seed;
    a.row_base = t->cfg.row_base;
    const bool small = use_small_rows(n, t->grid);
    const int rows = small ? 16 : 64;
    const int64_t nblk = (n + rows - 1) / rows;
    t->last_grid = (int)(nblk < t->grid ? nblk : t->grid);
    if (small)
        hipLaunchKernelGGL((student_mlp_kernel<true, 16>), dim3(t->last_grid), dim3(BLOCK), 0, t->stream, a);
    else
        hipLaunchKernelGGL((student_mlp_kernel<true, 64>), dim3(t->last_grid), dim3(BLOCK), 0, t->stream, a);
    RD_HIP(hipGetLastError(), "student_mlp_kernel launch");
    return RD_OK;
}

int launch_adam(rdm_trainer* t, int reduce, int adam) {
    AdamArgs a;
    a.ws = t->ws;
    a.nblk = t->last_grid;
    a.grad = t->grad;
    a.params = t->params;
    a.img = t->img;
    a.m = t->m;
    a.v = t->v;
    a.ctl = t->ctl;
    a.hist = t->hist;
    a.hist_len = t->cfg.metrics_len;
    a.reduce = reduce;
    a.adam = adam;
    a.lr = t->cfg.lr;
    a.b1 = t->cfg.beta1;
    a.b2 = t->cfg.beta2;
    a.eps = t->cfg.eps;
    hipLaunchKernelGGL(reduce_adam_kernel, dim3(ADAM_GRID), dim3(ADAM_BLOCK), 0, t->stream, a);
    RD_HIP(hipGetLastError(), "student_mlp reduce_adam_kernel launch");
    return RD_OK;
}

bool bad_rows(const float* x, int64_t n) {
    return !x || n <= 0 || n > ((int64_t)1 << 31) || ((uintptr_t)x & 15) != 0;
}

}  // namespace

extern "C" {

int rdm_param_count(void) { return P_REF; }

int rdm_create(rdm_trainer** out, const rdm_config* cfg, int device, void* hip_stream) {
    if (!out || !cfg) return rd::set_error(RD_EINVAL, "rdm_create: null argument");
    if ((cfg->loss != RDM_LOSS_MSE && cfg->loss != RDM_LOSS_KL) || !(cfg->lr > 0) || cfg->grid < 0 ||
        cfg->metrics_len < 0 || !(cfg->keep_prob > 0.0f && cfg->keep_prob <= 1.0f) || cfg->row_base < 0)
        return rd::set_error(RD_EINVAL, "rdm_create: bad config");
    rd::DeviceGuard dg(device);
    RD_HIP(dg.err, "rdm_create: hipSetDevice");
    rdm_trainer* t = new (std::nothrow) rdm_trainer();
    if (!t) return rd::set_error(RD_EINVAL, "rdm_create: out of host memory");
    t->cfg = *cfg;
    if (t->cfg.metrics_len == 0) t->cfg.metrics_len = 4096;
    t->device = device;
    t->stream = (hipStream_t)hip_stream;
    t->grid = cfg->grid > 0 ? cfg->grid : cu_count(device);
    t->last_grid = 0;
    hipError_t e = hipSuccess;
    auto alloc = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(p, bytes);
        if (e == hipSuccess) e = hipMemsetAsync(*p, 0, bytes, t->stream);
    };
    alloc((void**)&t->params, sizeof(float) * P_REF);
    alloc((void**)&t->img, sizeof(float) * IMG);
    alloc((void**)&t->m, sizeof(float) * P_REF);
    alloc((void**)&t->v, sizeof(float) * P_REF);
    alloc((void**)&t->own_grad, sizeof(float) * P_REF);
    alloc((void**)&t->ws, sizeof(float) * (size_t)t->grid * WS_ROW);
    alloc((void**)&t->hist, sizeof(float) * (size_t)t->cfg.metrics_len * N_MET);
    alloc((void**)&t->ctl, sizeof(uint32_t) * 8);
    t->grad = t->own_grad;
    if (e != hipSuccess) {
        rdm_destroy(t);
        return rd::hip_fail(e, "rdm_create: allocation");
    }
    if (int rc = rdm_reset(t)) {
        rdm_destroy(t);
        return rc;
    }
    *out = t;
    return RD_OK;
}

int rdm_destroy(rdm_trainer* t) {
    if (!t) return RD_OK;
    rd::DeviceGuard dg(t->device);
    for (void* p : {(void*)t->params, (void*)t->img, (void*)t->m, (void*)t->v, (void*)t->own_grad, (void*)t->ws,
                    (void*)t->hist, (void*)t->ctl})
        if (p) (void)hipFree(p);
    delete t;
    return RD_OK;
}

int rdm_set_stream(rdm_trainer* t, void* hip_stream) {
    if (!t) return rd::set_error(RD_EINVAL, "rdm_set_stream: null handle");
    t->stream = (hipStream_t)hip_stream;
    return RD_OK;
}

int rdm_set_params(rdm_trainer* t, const float* params) {
    if (!t || !params) return rd::set_error(RD_EINVAL, "rdm_set_params: null argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdm_set_params");
    RD_HIP(hipMemcpyAsync(t->params, params, sizeof(float) * P_REF, hipMemcpyDeviceToDevice, t->stream),
           "rdm_set_params");
    hipLaunchKernelGGL(pack_kernel, dim3((P_REF + 255) / 256), dim3(256), 0, t->stream, t->params, t->img);
    RD_HIP(hipGetLastError(), "rdm_set_params: pack");
    return RD_OK;
}

int rdm_get_params(rdm_trainer* t, float* params) {
    if (!t || !params) return rd::set_error(RD_EINVAL, "rdm_get_params: null argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(hipMemcpyAsync(params, t->params, sizeof(float) * P_REF, hipMemcpyDeviceToDevice, t->stream),
           "rdm_get_params");
    return RD_OK;
}

int rdm_reset(rdm_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdm_reset: null handle");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdm_reset");
    RD_HIP(hipMemsetAsync(t->m, 0, sizeof(float) * P_REF, t->stream), "rdm_reset");
    RD_HIP(hipMemsetAsync(t->v, 0, sizeof(float) * P_REF, t->stream), "rdm_reset");
    hipLaunchKernelGGL(init_ctl_kernel, dim3(1), dim3(64), 0, t->stream, t->ctl, t->cfg.beta1, t->cfg.beta2);
    RD_HIP(hipGetLastError(), "rdm_reset: launch");
    return RD_OK;
}

int rdm_forward(rdm_trainer* t, const float* x, int64_t n, float* pdflat) {
    if (!t || bad_rows(x, n) || !pdflat) return rd::set_error(RD_EINVAL, "rdm_forward: bad argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdm_forward");
    SmArgs a;
    a.x = x;
    a.tgt = nullptr;
    a.out = pdflat;
    a.n = n;
    a.img = t->img;
    a.ws = nullptr;
    a.ctl = nullptr;
    a.loss = 0;
    a.inv_n_global = 0.f;
    a.keep_prob = 1.0f;
    a.seed = 0;
    a.row_base = 0;
    const bool small = use_small_rows(n, t->grid);
    const int rows = small ? 16 : 64;
    const int64_t nblk = (n + rows - 1) / rows;
    const int grid = (int)(nblk < t->grid ? nblk : t->grid);
    if (small)
        hipLaunchKernelGGL((student_mlp_kernel<false, 16>), dim3(grid), dim3(BLOCK), 0, t->stream, a);
    else
        hipLaunchKernelGGL((student_mlp_kernel<false, 64>), dim3(grid), dim3(BLOCK), 0, t->stream, a);
    RD_HIP(hipGetLastError(), "student_mlp_kernel (forward) launch");
    return RD_OK;
}

int rdm_rollout(rdm_trainer* t, const float* x, const float* t_pdflat, int64_t n, int64_t n_global) {
    if (!t || bad_rows(x, n) || !t_pdflat || ((uintptr_t)t_pdflat & 15) != 0 || n_global < n)
        return rd::set_error(RD_EINVAL, "rdm_rollout: bad argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdm_rollout");
    if (int rc = launch_train(t, x, t_pdflat, n, n_global)) return rc;
    return launch_adam(t, 1, 0);
}

int rdm_apply(rdm_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdm_apply: null handle");
    if (t->last_grid == 0) return rd::set_error(RD_EINVAL, "rdm_apply: no rollout yet");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdm_apply");
    return launch_adam(t, 0, 1);
}

int rdm_step(rdm_trainer* t, const float* x, const float* t_pdflat, int64_t n) {
    if (!t || bad_rows(x, n) || !t_pdflat || ((uintptr_t)t_pdflat & 15) != 0)
        return rd::set_error(RD_EINVAL, "rdm_step: bad argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdm_step");
    if (int rc = launch_train(t, x, t_pdflat, n, n)) return rc;
    return launch_adam(t, 1, 1);
}

float* rdm_grad_buffer(rdm_trainer* t) { return t ? t->grad : nullptr; }

int rdm_bind_grad_buffer(rdm_trainer* t, float* grad) {
    if (!t) return rd::set_error(RD_EINVAL, "rdm_bind_grad_buffer: null handle");
    t->grad = grad ? grad : t->own_grad;
    return RD_OK;
}

int rdm_get_counter(rdm_trainer* t, int64_t* opt_steps) {
    if (!t || !opt_steps) return rd::set_error(RD_EINVAL, "rdm_get_counter: null argument");
    rd::DeviceGuard dg(t->device);
    uint32_t c[8];
    RD_HIP(hipMemcpyAsync(c, t->ctl, sizeof(c), hipMemcpyDeviceToHost, t->stream), "rdm_get_counter");
    RD_HIP(hipStreamSynchronize(t->stream), "rdm_get_counter");
    *opt_steps = c[0];
    return RD_OK;
}

int rdm_read_metrics(rdm_trainer* t, int64_t count, double* out) {
    if (!t || !out || count < 0) return rd::set_error(RD_EINVAL, "rdm_read_metrics: bad argument");
    int64_t steps = 0;
    if (int rc = rdm_get_counter(t, &steps)) return rc;
    const int64_t H = t->cfg.metrics_len;
    if (count > steps || count > H)
        return rd::set_error(RD_EINVAL, "rdm_read_metrics: only %lld steps kept", (long long)(steps < H ? steps : H));
    float* host = new (std::nothrow) float[(size_t)H * N_MET];
    if (!host) return rd::set_error(RD_EINVAL, "rdm_read_metrics: out of host memory");
    hipError_t e = hipMemcpy(host, t->hist, sizeof(float) * H * N_MET, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        delete[] host;
        return rd::hip_fail(e, "rdm_read_metrics");
    }
    for (int64_t k = 0; k < count; ++k) {
        const int64_t s = (steps - count + k) % H;
        for (int j = 0; j < N_MET; ++j) out[k * N_MET + j] = host[s * N_MET + j];
    }
    delete[] host;
    return RD_OK;
}

}  // extern "C"
