// f32 GEMM on gfx950 MFMA for the LSTM student and the PPO teacher (csrc/student_lstm.hip,
// csrc/ppo.hip):
//   C[M x N] (+)= epi( op(A)[M x K] . op(B)[K x N] + bias[N] )
// op(A) = A stored [M][lda] (ta = 0) or [K][lda] (ta = 1, A^T); likewise B [K][ldb] / [N][ldb].
// Epilogues: none, tanh, or x (1 - aux^2) (the tanh derivative of a stored activation);
// optional accumulate into C; or EPI_LSTM_BWD: the output (row, unit) is dh_{t-1} of the
// LSTM student's BPTT and the epilogue runs TF1 LSTMCell's backward for step t-1 instead of
// a store (csrc/student_lstm.hip).  Deterministic: fixed tiling, split-K partials summed in a
// fixed order by a second kernel (no atomics).
//
// Tiling: 256-thread workgroups own a 64 x 64 C tile (128 x 128 in diagnostic builds); 4
// waves in 2 x 2, each 2 x 2 (4 x 4) blocks of v_mfma_f32_16x16x4_f32 (exact f32 products).
// K advances 16 at a time through double-buffered LDS tiles stored [k][m] / [k][n] with row
// stride BT + 16 floats, so the 64 lanes of an MFMA operand read (16 consecutive m or n) x
// (4 k rows) hit 64 distinct banks; global loads (16-B when aligned) of the tile after next
// issue as soon as the next one is staged, so they span a barrier and an MFMA phase.
// gemm2() runs two independent problems (same or weight-/data-gradient orientations) as one
// launch over a 1-D grid, with one grouped split-K reduce.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rdg {

typedef float f32x4 __attribute__((ext_vector_type(4)));

enum { EPI_NONE = 0, EPI_TANH = 1, EPI_DTANH = 2, EPI_LSTM_BWD = 3 };

struct GemmArgs {
    int M, N, K;
    const float* A;
    int64_t lda;
    int ta;
    const float* B;
    int64_t ldb;
    int tb;
    float* C;
    int64_t ldc;
    const float* bias;    // [N] or null
    const float* aux;     // EPI_DTANH: [M][ldaux]
    int64_t ldaux;
    int epi;
    int accum;            // C += result
    float* part;          // split-K partials [splits][M][N] (splits > 1)
    int splits;
    int kchunk;           // K range per split (multiple of 32)
    // EPI_LSTM_BWD (N = units U): aux = dh from the head [M][ldaux]; gate activations
    // lg [M][4U] (i, j, f, o); c_t lct and c_{t-1} lcp [M][U]; dc carried in place lcc [M][U];
    // dz written to lz [M][4U]
    const float* lg;
    const float* lct;
    const float* lcp;
    float* lcc;
    float* lz;
};

// TF1 LSTMCell backward at one (row, unit) with dh = dh_head + dh_next: the arithmetic of
// the standalone cell kernel in csrc/student_lstm.hip, operation for operation (bitwise).
__device__ __forceinline__ void lstm_bwd_point(const GemmArgs& g, int64_t row, int u, float dh_next) {
    const int U = g.N;
    const int64_t idx = row * U + u;
    const float* gg = g.lg + row * 4 * U;
    const float gi = gg[u], gj = gg[U + u], gf = gg[2 * U + u], go = gg[3 * U + u];
    const float dh = g.aux[row * g.ldaux + u] + dh_next;
    const float tc = tanhf(g.lct[idx]);
    const float dcv = fmaf(dh * go, fmaf(-tc, tc, 1.0f), g.lcc[idx]);
    float* dz = g.lz + row * 4 * U;
    dz[u] = dcv * gj * gi * (1.0f - gi);
    dz[U + u] = dcv * gi * fmaf(-gj, gj, 1.0f);
    dz[2 * U + u] = dcv * g.lcp[idx] * gf * (1.0f - gf);
    dz[3 * U + u] = dh * tc * go * (1.0f - go);
    g.lcc[idx] = dcv * gf;
}

constexpr int TK = 16, GEMM_THREADS = 256;
// K tiles of global loads kept in flight by the 64/128-tile kernels (register ring).  1: tile
// t+2's loads issue right after tile t+1 is written to LDS, so they span a barrier and a whole
// MFMA phase.  Measured (LSTM 20 / 1,024 / 16,384 windows, PPO iteration): depth 1 0.467 /
// 0.679 / 4.31 ms, 63.1 ms; depth 3 0.474 / 0.691 / 4.37, 64.9; depth 5 0.472 / 0.693 / 4.41,
// 65.6; the previous loop (next tile loaded at the top of the step) 0.485 / 0.709 / 4.42, 70.0.
constexpr int PF = 1;

__device__ __forceinline__ float apply_epi(const GemmArgs& g, int row, int col, float v) {
    if (g.bias) v += g.bias[col];
    if (g.epi == EPI_TANH) {
        v = tanhf(v);
    } else if (g.epi == EPI_DTANH) {
        const float a = g.aux[(int64_t)row * g.ldaux + col];
        v *= fmaf(-a, a, 1.0f);
    }
    if (g.accum) v += g.C[(int64_t)row * g.ldc + col];
    return v;
}

// the epilogue on preloaded operands: bias b, stored activation a (EPI_DTANH), prior C c
__device__ __forceinline__ float epi_value(const GemmArgs& g, float v, float b, float a, float c) {
    v += b;
    if (g.epi == EPI_TANH) v = tanhf(v);
    else if (g.epi == EPI_DTANH) v *= fmaf(-a, a, 1.0f);
    if (g.accum) v += c;
    return v;
}

// 4 consecutive elements p[0..3] (along the contiguous dimension) of a tile row; `valid` of
// them are in range.  VEC: one 16-B load when all 4 are in range.
template <bool VEC>
__device__ __forceinline__ f32x4 load4(const float* p, int valid) {
    if (VEC && valid >= 4) return *reinterpret_cast<const f32x4*>(p);
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (e < valid) v[e] = p[e];
    return v;
}

template <int BT>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, f32x4 (&acc)[BT / 32][BT / 32], int m0, int n0,
                                              int wm, int wn, int i, int gq, int bz);

// BT x BT C tile per workgroup (BT = 64 or 128); 4 waves in 2 x 2, each (BT/2)^2 =
// (BT/32)^2 16x16 blocks.  LDS rows are BT + 16 floats: the 4 k-rows of one MFMA operand
// start 16 banks apart, so 16 consecutive m (or n) x 4 k hit 64 distinct banks.
// The tile (bx, by) of K split bz; gemm_kernel and the grouped kernels run it on the LDS
// staging buffers the kernel declares ([2][TK][BT + 16] floats each).
template <int BT>
struct TileLds {
    float A[2][TK][BT + 16];
    float B[2][TK][BT + 16];
};

template <int BT, bool TA, bool TB, bool VEC>
__device__ __forceinline__ void gemm_tile(const GemmArgs& g, int bx, int by, int bz, TileLds<BT>& lds) {
    constexpr int FB = BT / 32, NQ = BT / 64;   // blocks per wave dim, loads per thread
    auto& As = lds.A;
    auto& Bs = lds.B;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, gq = lane >> 4;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = by * BT, n0 = bx * BT;
    const int kbeg = bz * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);

    // quad q of a tile: [row][4 quads of k] (k-contiguous) or [k][BT/4 quads] (k-strided)
    auto load_a = [&](int k0, int q) -> f32x4 {
        if (!TA) {
            const int m = m0 + (q >> 2), k = k0 + 4 * (q & 3);
            const int valid = m < g.M ? min(4, kend - k) : 0;
            return load4<VEC>(g.A + (int64_t)m * g.lda + k, valid);
        } else {
            const int k = k0 + q / (BT / 4), m = m0 + 4 * (q % (BT / 4));
            const int valid = k < kend ? min(4, g.M - m) : 0;
            return load4<VEC>(g.A + (int64_t)k * g.lda + m, valid);
        }
    };
    auto load_b = [&](int k0, int q) -> f32x4 {
        if (!TB) {
            const int k = k0 + q / (BT / 4), n = n0 + 4 * (q % (BT / 4));
            const int valid = k < kend ? min(4, g.N - n) : 0;
            return load4<VEC>(g.B + (int64_t)k * g.ldb + n, valid);
        } else {
            const int n = n0 + (q >> 2), k = k0 + 4 * (q & 3);
            const int valid = n < g.N ? min(4, kend - k) : 0;
            return load4<VEC>(g.B + (int64_t)n * g.ldb + k, valid);
        }
    };
    auto store_a = [&](int buf, int q, f32x4 v) {
        if (!TA) {
#pragma unroll
            for (int e = 0; e < 4; ++e) As[buf][4 * (q & 3) + e][q >> 2] = v[e];
        } else {
            *reinterpret_cast<f32x4*>(&As[buf][q / (BT / 4)][4 * (q % (BT / 4))]) = v;
        }
    };
    auto store_b = [&](int buf, int q, f32x4 v) {
        if (!TB) {
            *reinterpret_cast<f32x4*>(&Bs[buf][q / (BT / 4)][4 * (q % (BT / 4))]) = v;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) Bs[buf][4 * (q & 3) + e][q >> 2] = v[e];
        }
    };

    f32x4 acc[FB][FB];
#pragma unroll
    for (int x = 0; x < FB; ++x)
#pragma unroll
        for (int y = 0; y < FB; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

    // K loop: tile kt is in LDS buffer kt & 1; the global loads of the next PF tiles are in
    // flight in a register ring (slot = tile % PF), so a step waits for a load issued PF
    // steps earlier rather than one (small-M GEMMs are a chain of load latencies otherwise)
    const int ntiles = kend > kbeg ? (kend - kbeg + TK - 1) / TK : 0;
    f32x4 ra[PF][NQ], rb[PF][NQ];
    if (ntiles > 0) {
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
            store_a(0, tid + GEMM_THREADS * u, load_a(kbeg, tid + GEMM_THREADS * u));
            store_b(0, tid + GEMM_THREADS * u, load_b(kbeg, tid + GEMM_THREADS * u));
        }
    }
#pragma unroll
    for (int p = 1; p <= PF; ++p)
        if (p < ntiles)
#pragma unroll
            for (int u = 0; u < NQ; ++u) {
                ra[p % PF][u] = load_a(kbeg + p * TK, tid + GEMM_THREADS * u);
                rb[p % PF][u] = load_b(kbeg + p * TK, tid + GEMM_THREADS * u);
            }
    __syncthreads();
    for (int kt0 = 0; kt0 < ntiles; kt0 += PF) {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            const int kt = kt0 + j;
            if (kt >= ntiles) break;
            const int buf = kt & 1;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int kk = 4 * s + gq;
                float a[FB], b[FB];
#pragma unroll
                for (int x = 0; x < FB; ++x) a[x] = As[buf][kk][(BT / 2) * wm + 16 * x + i];
#pragma unroll
                for (int y = 0; y < FB; ++y) b[y] = Bs[buf][kk][(BT / 2) * wn + 16 * y + i];
#pragma unroll
                for (int x = 0; x < FB; ++x)
#pragma unroll
                    for (int y = 0; y < FB; ++y)
                        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x], b[y], acc[x][y], 0, 0, 0);
            }
            const int SL = (j + 1) % PF;   // the slot of tile kt + 1 (kt0 is a multiple of PF; unrolled)
            if (kt + 1 < ntiles) {
#pragma unroll
                for (int u = 0; u < NQ; ++u) {
                    store_a(buf ^ 1, tid + GEMM_THREADS * u, ra[SL][u]);
                    store_b(buf ^ 1, tid + GEMM_THREADS * u, rb[SL][u]);
                }
                if (kt + 1 + PF < ntiles)   // refill the slot with tile kt + 1 + PF
#pragma unroll
                    for (int u = 0; u < NQ; ++u) {
                        ra[SL][u] = load_a(kbeg + (kt + 1 + PF) * TK, tid + GEMM_THREADS * u);
                        rb[SL][u] = load_b(kbeg + (kt + 1 + PF) * TK, tid + GEMM_THREADS * u);
                    }
            }
            __syncthreads();
        }
    }
    gemm_epilogue<BT>(g, acc, m0, n0, wm, wn, i, gq, bz);
}

template <int BT, bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(GEMM_THREADS) void gemm_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) TileLds<BT> lds;
    gemm_tile<BT, TA, TB, VEC>(g, blockIdx.x, blockIdx.y, blockIdx.z, lds);
}

// Two independent problems in one launch (the PPO policy and value nets' layers; a head
// layer's weight and data gradients): a 1-D grid, blocks [0, n0) = g0's tiles x K splits, the
// rest g1's, so two very different shapes cost no empty blocks.
struct Group2 {
    int tn0, tm0, n0, tn1, tm1;
};

__device__ __forceinline__ void group2_decode(const Group2& q, int bid, int& which, int& bx, int& by, int& bz) {
    which = bid >= q.n0;
    const int b = which ? bid - q.n0 : bid;
    const int tn = which ? q.tn1 : q.tn0, tm = which ? q.tm1 : q.tm0;
    bx = b % tn;
    by = (b / tn) % tm;
    bz = b / (tn * tm);
}

template <int BT, bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(GEMM_THREADS) void gemm_kernel_g2(GemmArgs g0, GemmArgs g1, Group2 q) {
    int which, bx, by, bz;
    group2_decode(q, blockIdx.x, which, bx, by, bz);
    __shared__ __attribute__((aligned(16))) TileLds<BT> lds;
    gemm_tile<BT, TA, TB, VEC>(which ? g1 : g0, bx, by, bz, lds);
}

// the same for two problems of DIFFERENT orientations (a weight gradient Hᵀ·dZ beside a data
// gradient dZ·Wᵀ): one LDS buffer set, the orientation chosen per block
template <bool TA0, bool TB0, bool TA1, bool TB1>
__global__ __launch_bounds__(GEMM_THREADS) void gemm_kernel_g2m(GemmArgs g0, GemmArgs g1, Group2 q) {
    int which, bx, by, bz;
    group2_decode(q, blockIdx.x, which, bx, by, bz);
    __shared__ __attribute__((aligned(16))) TileLds<64> lds;
    if (!which) gemm_tile<64, TA0, TB0, true>(g0, bx, by, bz, lds);
    else gemm_tile<64, TA1, TB1, true>(g1, bx, by, bz, lds);
}

// The C tile's epilogue (every kernel of this file): acc[x][y][r] = C[m0 + (BT/2) wm + 16x +
// 4gq + r][n0 + (BT/2) wn + 16y + i].
template <int BT>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, f32x4 (&acc)[BT / 32][BT / 32], int m0, int n0,
                                              int wm, int wn, int i, int gq, int bz) {
    constexpr int FB = BT / 32;
    if (g.epi == EPI_LSTM_BWD && g.splits <= 1) {   // (uniform) the cell backward per output
#pragma unroll
        for (int x = 0; x < FB; ++x)
#pragma unroll
            for (int y = 0; y < FB; ++y)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m0 + (BT / 2) * wm + 16 * x + 4 * gq + r, col = n0 + (BT / 2) * wn + 16 * y + i;
                    // + 0.0f: the value the unfused path stored (epi_value adds the zero bias)
                    if (row < g.M && col < g.N) lstm_bwd_point(g, row, col, acc[x][y][r] + 0.0f);
                }
        return;
    }
    // epilogue in two passes: every operand load (C when accumulating, the tanh' activation,
    // the bias) is issued before any result is formed, so their latencies overlap
    float in_c[FB][FB][4], in_a[FB][FB][4], in_b[FB][FB];
#pragma unroll
    for (int x = 0; x < FB; ++x)
#pragma unroll
        for (int y = 0; y < FB; ++y) {
            const int col = n0 + (BT / 2) * wn + 16 * y + i;
            in_b[x][y] = (g.splits <= 1 && g.bias && col < g.N) ? g.bias[col] : 0.0f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + (BT / 2) * wm + 16 * x + 4 * gq + r;
                const bool ok = g.splits <= 1 && row < g.M && col < g.N;
                in_c[x][y][r] = (ok && g.accum) ? g.C[(int64_t)row * g.ldc + col] : 0.0f;
                in_a[x][y][r] = (ok && g.epi == EPI_DTANH) ? g.aux[(int64_t)row * g.ldaux + col] : 0.0f;
            }
        }
#pragma unroll
    for (int x = 0; x < FB; ++x)
#pragma unroll
        for (int y = 0; y < FB; ++y)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + (BT / 2) * wm + 16 * x + 4 * gq + r, col = n0 + (BT / 2) * wn + 16 * y + i;
                if (row >= g.M || col >= g.N) continue;
                if (g.splits > 1)
                    g.part[((int64_t)bz * g.M + row) * g.N + col] = acc[x][y][r];
                else
                    g.C[(int64_t)row * g.ldc + col] = epi_value(g, acc[x][y][r], in_b[x][y], in_a[x][y][r],
                                                               in_c[x][y][r]);
            }
}

// 128 x 128 C tile, K advancing 32 at a time, on v_mfma_f32_32x32x2_f32: 4 waves in 2 x 2,
// each 64 x 64 = 2 x 2 blocks of 32 x 32 (64 accumulator registers).  Per k-step (K = 2) a
// wave reads 2 A + 2 B operands from LDS for 4 MFMAs of 64 cycles each, 4x the MFMA work per
// LDS read of the 64-tile kernel, and one barrier covers 64 MFMAs per wave.  LDS rows are
// 128 + 32 floats: the two k-rows of an operand (lanes 0-31 / 32-63) start 32 banks apart.
// Operand layouts (per lane l): A[i = l % 32][k = l / 32], B[k = l / 32][j = l % 32];
// D register r of lane l = C[8 (r / 4) + 4 (l / 32) + r % 4][l % 32].
template <bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(GEMM_THREADS) void gemm_kernel_big(GemmArgs g) {
    constexpr int BT = 128, BK = 32, LS = BT + 32, NQ = BT * BK / 4 / GEMM_THREADS;   // 4 quads per thread
    __shared__ __attribute__((aligned(16))) float As[2][BK][LS];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK][LS];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 31, kh = lane >> 5;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.y * BT, n0 = blockIdx.x * BT;
    const int kbeg = blockIdx.z * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);
    // quad q: k-contiguous operands are [row][8 quads], k-strided ones [k][32 quads]
    auto load_a = [&](int k0, int q) -> f32x4 {
        if (!TA) {
            const int m = m0 + (q >> 3), k = k0 + 4 * (q & 7);
            return load4<VEC>(g.A + (int64_t)m * g.lda + k, m < g.M ? min(4, kend - k) : 0);
        } else {
            const int k = k0 + (q >> 5), m = m0 + 4 * (q & 31);
            return load4<VEC>(g.A + (int64_t)k * g.lda + m, k < kend ? min(4, g.M - m) : 0);
        }
    };
    auto load_b = [&](int k0, int q) -> f32x4 {
        if (!TB) {
            const int k = k0 + (q >> 5), n = n0 + 4 * (q & 31);
            return load4<VEC>(g.B + (int64_t)k * g.ldb + n, k < kend ? min(4, g.N - n) : 0);
        } else {
            const int n = n0 + (q >> 3), k = k0 + 4 * (q & 7);
            return load4<VEC>(g.B + (int64_t)n * g.ldb + k, n < g.N ? min(4, kend - k) : 0);
        }
    };
    auto store_a = [&](int buf, int q, f32x4 v) {
        if (!TA) {
#pragma unroll
            for (int e = 0; e < 4; ++e) As[buf][4 * (q & 7) + e][q >> 3] = v[e];
        } else {
            *reinterpret_cast<f32x4*>(&As[buf][q >> 5][4 * (q & 31)]) = v;
        }
    };
    auto store_b = [&](int buf, int q, f32x4 v) {
        if (!TB) {
            *reinterpret_cast<f32x4*>(&Bs[buf][q >> 5][4 * (q & 31)]) = v;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) Bs[buf][4 * (q & 7) + e][q >> 3] = v[e];
        }
    };
    typedef float f32x16 __attribute__((ext_vector_type(16)));
    f32x16 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[x][y][r] = 0.0f;
    const int ntiles = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
    if (ntiles > 0) {
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
            store_a(0, tid + GEMM_THREADS * u, load_a(kbeg, tid + GEMM_THREADS * u));
            store_b(0, tid + GEMM_THREADS * u, load_b(kbeg, tid + GEMM_THREADS * u));
        }
    }
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
        const int buf = kt & 1;
        f32x4 na[NQ], nb[NQ];
        const bool more = kt + 1 < ntiles;
        if (more) {
#pragma unroll
            for (int u = 0; u < NQ; ++u) {
                na[u] = load_a(kbeg + (kt + 1) * BK, tid + GEMM_THREADS * u);
                nb[u] = load_b(kbeg + (kt + 1) * BK, tid + GEMM_THREADS * u);
            }
        }
#pragma unroll
        for (int s = 0; s < BK / 2; ++s) {
            const int kk = 2 * s + kh;
            const float a0 = As[buf][kk][64 * wm + i], a1 = As[buf][kk][64 * wm + 32 + i];
            const float b0 = Bs[buf][kk][64 * wn + i], b1 = Bs[buf][kk][64 * wn + 32 + i];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (more) {
#pragma unroll
            for (int u = 0; u < NQ; ++u) {
                store_a(buf ^ 1, tid + GEMM_THREADS * u, na[u]);
                store_b(buf ^ 1, tid + GEMM_THREADS * u, nb[u]);
            }
        }
        __syncthreads();
    }
    // two-pass epilogue (operand loads first, as in gemm_kernel), one 32 x 32 block at a time
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int col = n0 + 64 * wn + 32 * y + i;
            const float bv = (g.splits <= 1 && g.bias && col < g.N) ? g.bias[col] : 0.0f;
            float in_c[16], in_a[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + 64 * wm + 32 * x + 8 * (r >> 2) + 4 * kh + (r & 3);
                const bool ok = g.splits <= 1 && row < g.M && col < g.N;
                in_c[r] = (ok && g.accum) ? g.C[(int64_t)row * g.ldc + col] : 0.0f;
                in_a[r] = (ok && g.epi == EPI_DTANH) ? g.aux[(int64_t)row * g.ldaux + col] : 0.0f;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + 64 * wm + 32 * x + 8 * (r >> 2) + 4 * kh + (r & 3);
                if (row >= g.M || col >= g.N) continue;
                if (g.splits > 1)
                    g.part[((int64_t)blockIdx.z * g.M + row) * g.N + col] = acc[x][y][r];
                else
                    g.C[(int64_t)row * g.ldc + col] = epi_value(g, acc[x][y][r], bv, in_a[r], in_c[r]);
            }
        }
}

// split-K: C = epi(sum_z part[z]) in a fixed order.  64 outputs per block, 4 interleaved
// split phases per output (summed in a fixed order at the end).
__device__ __forceinline__ void splitk_reduce_block(const GemmArgs& g, int64_t blk) {
    __shared__ float s[4][64];
    const int64_t MN = (int64_t)g.M * g.N;
    const int64_t idx = blk * 64 + (threadIdx.x & 63);
    const int ph = threadIdx.x >> 6;
    float a = 0.f, b = 0.f;
    if (idx < MN) {
        int z = ph;
        for (; z + 4 < g.splits; z += 8) {
            a += g.part[z * MN + idx];
            b += g.part[(z + 4) * MN + idx];
        }
        if (z < g.splits) a += g.part[z * MN + idx];
    }
    s[ph][threadIdx.x & 63] = a + b;
    __syncthreads();
    if (ph == 0 && idx < MN) {
        const float v = (s[0][threadIdx.x] + s[1][threadIdx.x]) + (s[2][threadIdx.x] + s[3][threadIdx.x]);
        const int row = (int)(idx / g.N), col = (int)(idx % g.N);
        if (g.epi == EPI_LSTM_BWD)
            lstm_bwd_point(g, row, col, v);
        else
            g.C[(int64_t)row * g.ldc + col] = apply_epi(g, row, col, v);
    }
}

template <int = 0>   // a template: one definition per translation unit that includes this header
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs g) {
    splitk_reduce_block(g, blockIdx.x);
}

// grouped: blocks [0, nb0) reduce g0 (when it is split), the rest g1
template <int = 0>
__global__ __launch_bounds__(256) void splitk_reduce_g2(GemmArgs g0, GemmArgs g1, int nb0) {
    if ((int)blockIdx.x < nb0) splitk_reduce_block(g0, blockIdx.x);
    else splitk_reduce_block(g1, (int)blockIdx.x - nb0);
}

// Split K when the tile grid cannot fill the chip (`per_cu` resident workgroups per CU, so
// the loads of one tile's K-loop hide behind the others' MFMAs) and K is long.
inline void gemm_plan(GemmArgs& g, int tile, int per_cu, float* part, int64_t part_floats, int cus) {
    const int tiles = ((g.M + tile - 1) / tile) * ((g.N + tile - 1) / tile);
    int splits = 1;
    const int target = per_cu * cus;
    if (part && tiles < target && g.K >= 512) {
        splits = (target + tiles - 1) / tiles;
        // >= 16 k-tiles per split, <= 256 partials; a grid of a few tiles (small M and N: the
        // LSTM's dh GEMM at the reference's 20 windows) goes down to 4 k-tiles per split, since
        // each split's K loop is a chain of load latencies
        const int kmin = tiles <= 16 ? 64 : 256;
        const int maxs = g.K / kmin < 256 ? g.K / kmin : 256;
        if (splits > maxs) splits = maxs;
        while (splits > 1 && (int64_t)splits * g.M * g.N > part_floats) --splits;
    }
    g.splits = splits;
    g.part = part;
    g.kchunk = splits > 1 ? (((g.K + splits - 1) / splits + 31) / 32) * 32 : g.K;   // multiple of both K tiles
    if (splits > 1) g.splits = (g.K + g.kchunk - 1) / g.kchunk;
}

inline bool gemm_vec(const GemmArgs& g) {
    return ((uintptr_t)g.A % 16 == 0) && ((uintptr_t)g.B % 16 == 0) && g.lda % 4 == 0 && g.ldb % 4 == 0;
}

// Launch; `part`/`part_floats` = split-K workspace (may be null: no split).  Returns a hip error.
inline hipError_t gemm(hipStream_t st, GemmArgs g, float* part, int64_t part_floats, int cus) {
    if (g.M <= 0 || g.N <= 0) return hipSuccess;
    // 128 x 128 tiles (half the operand re-reads, 4x the MFMAs per LDS read) when both
    // dimensions fill them; 64 x 64 otherwise
    // the 16x16x4 64 x 64 kernel everywhere: on every LSTM / PPO shape it beats both the
    // 16x16x4 128-tile variant and the 32x32x2 128 x 128 x 32 kernel (BT 129), which are kept
    // for diagnostic builds (scripts/gemm_tile_compare.sh): the LSTM's GEMMs
    // are short-K (recurrent, K = 200) or weight gradients whose operands stream from HBM,
    // where 8 resident 64-tile workgroups per CU keep more loads in flight than 2 big ones.
    // Also measured slower: the 64 tile with k-contiguous LDS staging read by
    // ds_read_b128, 16 or 32 deep
    const int BT = 64;
    const int TILE = BT == 129 ? 128 : BT;
    const int tm = (g.M + TILE - 1) / TILE, tn = (g.N + TILE - 1) / TILE;
    gemm_plan(g, TILE, BT == 129 ? 2 : 8, part, part_floats, cus);   // the big kernel's 80 KB of LDS: 2 per CU
    const bool vec = gemm_vec(g);
    dim3 grid(tn, tm, g.splits);
#define RDG_LAUNCH(BT_, TA_, TB_, V_) \
    hipLaunchKernelGGL((gemm_kernel<BT_, TA_, TB_, V_>), grid, dim3(GEMM_THREADS), 0, st, g)
#define RDG_DISPATCH(BT_)                                                   \
    if (vec) {                                                              \
        if (!g.ta && !g.tb) RDG_LAUNCH(BT_, false, false, true);           \
        else if (!g.ta && g.tb) RDG_LAUNCH(BT_, false, true, true);        \
        else if (g.ta && !g.tb) RDG_LAUNCH(BT_, true, false, true);        \
        else RDG_LAUNCH(BT_, true, true, true);                             \
    } else {                                                                \
        if (!g.ta && !g.tb) RDG_LAUNCH(BT_, false, false, false);          \
        else if (!g.ta && g.tb) RDG_LAUNCH(BT_, false, true, false);       \
        else if (g.ta && !g.tb) RDG_LAUNCH(BT_, true, false, false);       \
        else RDG_LAUNCH(BT_, true, true, false);                            \
    }
#define RDG_LAUNCH_BIG(TA_, TB_, V_) \
    hipLaunchKernelGGL((gemm_kernel_big<TA_, TB_, V_>), grid, dim3(GEMM_THREADS), 0, st, g)
    if (BT == 129) {
        if (vec) {
            if (!g.ta && !g.tb) RDG_LAUNCH_BIG(false, false, true);
            else if (!g.ta && g.tb) RDG_LAUNCH_BIG(false, true, true);
            else if (g.ta && !g.tb) RDG_LAUNCH_BIG(true, false, true);
            else RDG_LAUNCH_BIG(true, true, true);
        } else {
            if (!g.ta && !g.tb) RDG_LAUNCH_BIG(false, false, false);
            else if (!g.ta && g.tb) RDG_LAUNCH_BIG(false, true, false);
            else if (g.ta && !g.tb) RDG_LAUNCH_BIG(true, false, false);
            else RDG_LAUNCH_BIG(true, true, false);
        }
    } else if (BT == 128) {
        RDG_DISPATCH(128)
    } else {
        RDG_DISPATCH(64)
    }
#undef RDG_LAUNCH_BIG
#undef RDG_DISPATCH
#undef RDG_LAUNCH
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || g.splits <= 1) return e;
    const int64_t MN = (int64_t)g.M * g.N;
    hipLaunchKernelGGL(splitk_reduce_kernel<0>, dim3((unsigned)((MN + 63) / 64)), dim3(256), 0, st, g);
    return hipGetLastError();
}

// Two independent problems of one orientation (same ta, tb) -- or a weight gradient (1, 0)
// beside a data gradient (0, 1) -- as ONE launch of the 64 tile, plus
// one grouped split-K reduce when either is split: the PPO policy and value nets run their
// layers side by side (half the dependent launches of a minibatch).  The split-K workspace is
// halved between them.  Problems that do not pair (orientation, 16-B alignment) and the
// diagnostic tile builds run as two gemm() calls.  Same tiles, splits and k order as gemm().
inline Group2 group2(const GemmArgs& g0, const GemmArgs& g1) {
    Group2 q;
    q.tn0 = (g0.N + 63) / 64;
    q.tm0 = (g0.M + 63) / 64;
    q.n0 = q.tn0 * q.tm0 * g0.splits;
    q.tn1 = (g1.N + 63) / 64;
    q.tm1 = (g1.M + 63) / 64;
    return q;
}

inline hipError_t gemm2(hipStream_t st, GemmArgs g0, GemmArgs g1, float* part, int64_t part_floats, int cus) {
    const bool pair = g0.M > 0 && g0.N > 0 && g1.M > 0 && g1.N > 0 && g0.ta == g1.ta && g0.tb == g1.tb &&
                      gemm_vec(g0) == gemm_vec(g1);
    if (pair) {
        const int64_t half = part_floats / 2;
        gemm_plan(g0, 64, 8, part, half, cus);
        gemm_plan(g1, 64, 8, part ? part + half : nullptr, half, cus);
        const Group2 q = group2(g0, g1);
        dim3 grid((unsigned)(q.n0 + q.tn1 * q.tm1 * g1.splits));
#define RDG_LAUNCH2(TA_, TB_, V_) \
    hipLaunchKernelGGL((gemm_kernel_g2<64, TA_, TB_, V_>), grid, dim3(GEMM_THREADS), 0, st, g0, g1, q)
        if (gemm_vec(g0)) {
            if (!g0.ta && !g0.tb) RDG_LAUNCH2(false, false, true);
            else if (!g0.ta && g0.tb) RDG_LAUNCH2(false, true, true);
            else if (g0.ta && !g0.tb) RDG_LAUNCH2(true, false, true);
            else RDG_LAUNCH2(true, true, true);
        } else {
            if (!g0.ta && !g0.tb) RDG_LAUNCH2(false, false, false);
            else if (!g0.ta && g0.tb) RDG_LAUNCH2(false, true, false);
            else if (g0.ta && !g0.tb) RDG_LAUNCH2(true, false, false);
            else RDG_LAUNCH2(true, true, false);
        }
#undef RDG_LAUNCH2
        hipError_t e = hipGetLastError();
        if (e != hipSuccess || (g0.splits <= 1 && g1.splits <= 1)) return e;
        const int nb0 = g0.splits > 1 ? (int)(((int64_t)g0.M * g0.N + 63) / 64) : 0;
        const int nb1 = g1.splits > 1 ? (int)(((int64_t)g1.M * g1.N + 63) / 64) : 0;
        // an unsplit problem contributes no reduce blocks: give the grouped kernel g1 first
        if (nb0 == 0)
            hipLaunchKernelGGL(splitk_reduce_g2<0>, dim3((unsigned)nb1), dim3(256), 0, st, g1, g1, nb1);
        else
            hipLaunchKernelGGL(splitk_reduce_g2<0>, dim3((unsigned)(nb0 + nb1)), dim3(256), 0, st, g0, g1, nb0);
        return hipGetLastError();
    }
    // a layer's weight gradient (ta, tb) = (1, 0) beside its data gradient (0, 1), both 16-B
    // aligned: one launch of the mixed kernel
    const bool mixed = g0.M > 0 && g0.N > 0 && g1.M > 0 && g1.N > 0 && g0.ta == 1 && g0.tb == 0 && g1.ta == 0 &&
                       g1.tb == 1 && gemm_vec(g0) && gemm_vec(g1);
    if (mixed) {
        const int64_t half = part_floats / 2;
        gemm_plan(g0, 64, 8, part, half, cus);
        gemm_plan(g1, 64, 8, part ? part + half : nullptr, half, cus);
        const Group2 q = group2(g0, g1);
        hipLaunchKernelGGL((gemm_kernel_g2m<true, false, false, true>), dim3((unsigned)(q.n0 + q.tn1 * q.tm1 * g1.splits)),
                           dim3(GEMM_THREADS), 0, st, g0, g1, q);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess || (g0.splits <= 1 && g1.splits <= 1)) return e;
        const int nb0 = g0.splits > 1 ? (int)(((int64_t)g0.M * g0.N + 63) / 64) : 0;
        const int nb1 = g1.splits > 1 ? (int)(((int64_t)g1.M * g1.N + 63) / 64) : 0;
        if (nb0 == 0)
            hipLaunchKernelGGL(splitk_reduce_g2<0>, dim3((unsigned)nb1), dim3(256), 0, st, g1, g1, nb1);
        else
            hipLaunchKernelGGL(splitk_reduce_g2<0>, dim3((unsigned)(nb0 + nb1)), dim3(256), 0, st, g0, g1, nb0);
        return hipGetLastError();
    }
    hipError_t e = gemm(st, g0, part, part_floats, cus);
    if (e != hipSuccess) return e;
    return gemm(st, g1, part, part_floats, cus);
}

}  // namespace rdg
