// f32 GEMM on gfx950 MFMA for the LSTM student (csrc/student_lstm.hip):
//   C[M x N] (+)= epi( op(A)[M x K] . op(B)[K x N] + bias[N] )
// op(A) = A stored [M][lda] (ta = 0) or [K][lda] (ta = 1, A^T); likewise B [K][ldb] / [N][ldb].
// Epilogues: none, tanh, or x (1 - aux^2) (the tanh derivative of a stored activation);
// optional accumulate into C.  Deterministic: fixed tiling, split-K partials summed in a
// fixed order by a second kernel (no atomics).
//
// Tiling: 256-thread workgroups own a 64 x 64 C tile; 4 waves each 32 x 32 = 2 x 2 blocks of
// v_mfma_f32_16x16x4_f32 (exact f32 products).  K advances 16 at a time through double-
// buffered LDS tiles stored [k][m] / [k][n] with row stride 80 floats, so the 64 lanes of an
// MFMA operand read (16 consecutive m or n) x (4 k rows) hit 64 distinct banks; the next
// tile's global loads (one 16-B load per thread per operand when aligned) are in flight
// while the current tile's 16 MFMAs per wave issue.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rdg {

typedef float f32x4 __attribute__((ext_vector_type(4)));

enum { EPI_NONE = 0, EPI_TANH = 1, EPI_DTANH = 2 };

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
    int kchunk;           // K range per split (multiple of 16)
};

constexpr int TM = 64, TN = 64, TK = 16, GEMM_THREADS = 256, LDS_STRIDE = 80;

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

template <bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(GEMM_THREADS) void gemm_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) float As[2][TK][LDS_STRIDE];
    __shared__ __attribute__((aligned(16))) float Bs[2][TK][LDS_STRIDE];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, gq = lane >> 4;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
    const int kbeg = blockIdx.z * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);
    // loader coordinates: [contiguous-dim quad][other dim]
    const int a_r = TA ? tid >> 4 : tid >> 2, a_q = TA ? tid & 15 : tid & 3;
    const int b_r = TB ? tid >> 2 : tid >> 4, b_q = TB ? tid & 3 : tid & 15;

    auto load_a = [&](int k0) -> f32x4 {
        if (!TA) {   // A[m][k]: row m0 + a_r, k = k0 + 4 a_q ..
            const int m = m0 + a_r, k = k0 + 4 * a_q;
            const int valid = m < g.M ? min(4, kend - k) : 0;
            return load4<VEC>(g.A + (int64_t)m * g.lda + k, valid);
        } else {     // A^T stored [k][m]: row k0 + a_r, m = m0 + 4 a_q ..
            const int k = k0 + a_r, m = m0 + 4 * a_q;
            const int valid = k < kend ? min(4, g.M - m) : 0;
            return load4<VEC>(g.A + (int64_t)k * g.lda + m, valid);
        }
    };
    auto load_b = [&](int k0) -> f32x4 {
        if (!TB) {   // B[k][n]
            const int k = k0 + b_r, n = n0 + 4 * b_q;
            const int valid = k < kend ? min(4, g.N - n) : 0;
            return load4<VEC>(g.B + (int64_t)k * g.ldb + n, valid);
        } else {     // B^T stored [n][k]
            const int n = n0 + b_r, k = k0 + 4 * b_q;
            const int valid = n < g.N ? min(4, kend - k) : 0;
            return load4<VEC>(g.B + (int64_t)n * g.ldb + k, valid);
        }
    };
    auto store_a = [&](int buf, f32x4 v) {
        if (!TA) {
#pragma unroll
            for (int e = 0; e < 4; ++e) As[buf][4 * a_q + e][a_r] = v[e];
        } else {
            *reinterpret_cast<f32x4*>(&As[buf][a_r][4 * a_q]) = v;
        }
    };
    auto store_b = [&](int buf, f32x4 v) {
        if (!TB) {
            *reinterpret_cast<f32x4*>(&Bs[buf][b_r][4 * b_q]) = v;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) Bs[buf][4 * b_q + e][b_r] = v[e];
        }
    };

    f32x4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int ntiles = kend > kbeg ? (kend - kbeg + TK - 1) / TK : 0;
    if (ntiles > 0) {
        store_a(0, load_a(kbeg));
        store_b(0, load_b(kbeg));
    }
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
        const int buf = kt & 1;
        f32x4 na, nb;
        const bool more = kt + 1 < ntiles;
        if (more) {
            na = load_a(kbeg + (kt + 1) * TK);
            nb = load_b(kbeg + (kt + 1) * TK);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int kk = 4 * s + gq;
            const float a0 = As[buf][kk][32 * wm + i], a1 = As[buf][kk][32 * wm + 16 + i];
            const float b0 = Bs[buf][kk][32 * wn + i], b1 = Bs[buf][kk][32 * wn + 16 + i];
            acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (more) {
            store_a(buf ^ 1, na);
            store_b(buf ^ 1, nb);
        }
        __syncthreads();
    }

#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + 32 * wm + 16 * x + 4 * gq + r, col = n0 + 32 * wn + 16 * y + i;
                if (row >= g.M || col >= g.N) continue;
                if (g.splits > 1)
                    g.part[((int64_t)blockIdx.z * g.M + row) * g.N + col] = acc[x][y][r];
                else
                    g.C[(int64_t)row * g.ldc + col] = apply_epi(g, row, col, acc[x][y][r]);
            }
}

// split-K: C = epi(sum_z part[z]) in a fixed order
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs g) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t MN = (int64_t)g.M * g.N;
    if (idx >= MN) return;
    float s = 0.f;
    for (int z = 0; z < g.splits; ++z) s += g.part[z * MN + idx];
    const int row = (int)(idx / g.N), col = (int)(idx % g.N);
    g.C[(int64_t)row * g.ldc + col] = apply_epi(g, row, col, s);
}

// Launch; `part`/`part_floats` = split-K workspace (may be null: no split).  Returns a hip error.
inline hipError_t gemm(hipStream_t st, GemmArgs g, float* part, int64_t part_floats, int cus) {
    if (g.M <= 0 || g.N <= 0) return hipSuccess;
    const int tm = (g.M + TM - 1) / TM, tn = (g.N + TN - 1) / TN;
    const int tiles = tm * tn;
    // split K when the tile grid cannot fill the chip and K is long
    int splits = 1;
    if (part && tiles < 2 * cus && g.K >= 512) {
        splits = (2 * cus + tiles - 1) / tiles;
        const int maxs = g.K / 256;
        if (splits > maxs) splits = maxs;
        while (splits > 1 && (int64_t)splits * g.M * g.N > part_floats) --splits;
    }
    g.splits = splits;
    g.part = part;
    g.kchunk = splits > 1 ? (((g.K + splits - 1) / splits + TK - 1) / TK) * TK : g.K;
    if (splits > 1) g.splits = (g.K + g.kchunk - 1) / g.kchunk;
    const bool vec = ((uintptr_t)g.A % 16 == 0) && ((uintptr_t)g.B % 16 == 0) && g.lda % 4 == 0 && g.ldb % 4 == 0;
    dim3 grid(tn, tm, g.splits);
#define RDG_LAUNCH(TA_, TB_, V_) hipLaunchKernelGGL((gemm_kernel<TA_, TB_, V_>), grid, dim3(GEMM_THREADS), 0, st, g)
    if (vec) {
        if (!g.ta && !g.tb) RDG_LAUNCH(false, false, true);
        else if (!g.ta && g.tb) RDG_LAUNCH(false, true, true);
        else if (g.ta && !g.tb) RDG_LAUNCH(true, false, true);
        else RDG_LAUNCH(true, true, true);
    } else {
        if (!g.ta && !g.tb) RDG_LAUNCH(false, false, false);
        else if (!g.ta && g.tb) RDG_LAUNCH(false, true, false);
        else if (g.ta && !g.tb) RDG_LAUNCH(true, false, false);
        else RDG_LAUNCH(true, true, false);
    }
#undef RDG_LAUNCH
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || g.splits <= 1) return e;
    const int64_t MN = (int64_t)g.M * g.N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, st, g);
    return hipGetLastError();
}

}  // namespace rdg
