// Microbenchmark: the rollout's hidden layer (K = 64, 64 outputs, 16 envs, teacher and
// student interleaved, tanh on the outputs) as exact f32 MFMAs (v_mfma_f32_16x16x4_f32)
// versus f32 emulated on bf16 MFMAs (v_mfma_f32_16x16x32_bf16): both operands split exactly
// into three bf16 pieces (x = x0 + x1 + x2, truncation split), six partial products
// (x0y0, x0y1, x1y0, x0y2, x1y1, x2y0), f32 accumulation.  Prints cycles per layer and the
// error of both forms against an f64 host reference.  Also: back-to-back issue rates of
// 16x16x16 / 16x16x32 bf16 and 16x16x4 f32.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr float kTS = 2.8853900817779268f;
__device__ __forceinline__ float tanh_pre(float y) {
    return fmaf(-2.0f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(y) + 1.0f), 1.0f);
}
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// exact three-way split of 8 floats into packed bf16 pieces
__device__ __forceinline__ void split8(f32x4 a, f32x4 b, bf16x8& p0, bf16x8& p1, bf16x8& p2) {
    float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    uint32_t u0[8], u1[8], u2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t u = __float_as_uint(x[i]);
        const float r = x[i] - __uint_as_float(u & 0xffff0000u);
        const uint32_t ur = __float_as_uint(r);
        const float l = r - __uint_as_float(ur & 0xffff0000u);
        u0[i] = u; u1[i] = ur; u2[i] = __float_as_uint(l);
    }
    u32x4 q0, q1, q2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        q0[i] = __builtin_amdgcn_perm(u0[2 * i + 1], u0[2 * i], 0x07060302u);
        q1[i] = __builtin_amdgcn_perm(u1[2 * i + 1], u1[2 * i], 0x07060302u);
        q2[i] = __builtin_amdgcn_perm(u2[2 * i + 1], u2[2 * i], 0x07060302u);
    }
    p0 = __builtin_bit_cast(bf16x8, q0);
    p1 = __builtin_bit_cast(bf16x8, q1);
    p2 = __builtin_bit_cast(bf16x8, q2);
}

__device__ __forceinline__ f32x4 mk32(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ bf16x8 ldb8(const unsigned short* p) { return *reinterpret_cast<const bf16x8*>(p); }

// LDS: f32 images (2 nets x [64][16][4]) or bf16 images (2 nets x 3 pieces x [2][4][4][16][8])
constexpr int F32_NET = 64 * 64;
constexpr int BF_PIECE = 2 * 4 * 4 * 16 * 8;   // bf16 elements
constexpr int BF_NET = 3 * BF_PIECE;

template <int MODE>   // 0 = f32 exact, 1 = split bf16 x6, 2 = split bf16 x3 (2 pieces, timing only)
__global__ __launch_bounds__(512, 1) void layer(const float* gimg, const float* hin, float* hout, int iters,
                                                unsigned long long* clk) {
    __shared__ __attribute__((aligned(16))) float L[2 * BF_NET / 2 > 2 * F32_NET ? 2 * BF_NET / 2 : 2 * F32_NET];
    constexpr int NF = MODE == 0 ? 2 * F32_NET : BF_NET;   // floats (bf16 pairs) for both nets
    for (int i = threadIdx.x; i < NF; i += blockDim.x) L[i] = gimg[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    f32x4 HT[4], HS[4];
    for (int fb = 0; fb < 4; ++fb)
        for (int r = 0; r < 4; ++r) {
            HT[fb][r] = hin[(16 * fb + 4 * g + r) * 16 + j];
            HS[fb][r] = -HT[fb][r];
        }
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    f32x4 at[4], as[4];
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) at[fb] = as[fb] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (MODE == 0) {
            const float* LT = L;
            const float* LS = L + F32_NET;
            f32x4 wtn = ld4(LT + (4 * g) * 64 + 4 * j), wsn = ld4(LS + (4 * g) * 64 + 4 * j);
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const f32x4 wt = wtn, ws = wsn;
                    if (kb * 4 + r < 15) {
                        const int kn = (r == 3) ? 16 * (kb + 1) + 4 * g : 16 * kb + 4 * g + r + 1;
                        wtn = ld4(LT + kn * 64 + 4 * j);
                        wsn = ld4(LS + kn * 64 + 4 * j);
                    }
#pragma unroll
                    for (int fb = 0; fb < 4; ++fb) {
                        at[fb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wt[fb], HT[kb][r], at[fb], 0, 0, 0);
                        as[fb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ws[fb], HS[kb][r], as[fb], 0, 0, 0);
                    }
                }
        } else {
            const unsigned short* LT = reinterpret_cast<const unsigned short*>(L);
            const unsigned short* LS = LT + BF_NET;   // second net: pieces follow
            auto net_layer = [&](const unsigned short* LW, const f32x4 (&Hn)[4], f32x4 (&acc)[4]) {
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    __builtin_amdgcn_sched_barrier(0);
                    bf16x8 h0, h1, h2, w0[4], w1[4], w2[4];
                    split8(Hn[2 * s], Hn[2 * s + 1], h0, h1, h2);
#pragma unroll
                    for (int fb = 0; fb < 4; ++fb) {
                        const int o = (((s * 4 + g) * 4 + fb) * 16 + j) * 8;
                        w0[fb] = ldb8(LW + o); w1[fb] = ldb8(LW + BF_PIECE + o);
                        if constexpr (MODE == 1) w2[fb] = ldb8(LW + 2 * BF_PIECE + o);
                    }
                    if constexpr (MODE == 1) {
#pragma unroll
                        for (int fb = 0; fb < 4; ++fb) acc[fb] = mk32(w2[fb], h0, acc[fb]);
#pragma unroll
                        for (int fb = 0; fb < 4; ++fb) acc[fb] = mk32(w1[fb], h1, acc[fb]);
#pragma unroll
                        for (int fb = 0; fb < 4; ++fb) acc[fb] = mk32(w0[fb], h2, acc[fb]);
                    }
#pragma unroll
                    for (int fb = 0; fb < 4; ++fb) acc[fb] = mk32(w1[fb], h0, acc[fb]);
#pragma unroll
                    for (int fb = 0; fb < 4; ++fb) acc[fb] = mk32(w0[fb], h1, acc[fb]);
#pragma unroll
                    for (int fb = 0; fb < 4; ++fb) acc[fb] = mk32(w0[fb], h0, acc[fb]);
                }
            };
            net_layer(LT, HT, at);
            net_layer(LS, HS, as);
        }
#pragma unroll
        for (int fb = 0; fb < 4; ++fb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                HT[fb][r] = tanh_pre(at[fb][r]);
                HS[fb][r] = tanh_pre(as[fb][r]);
            }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0 && blockIdx.x == 0) clk[threadIdx.x >> 6] = t1 - t0;
    if (iters == 1 && blockIdx.x == 0 && threadIdx.x < 64)   // one layer's outputs: accuracy
        for (int fb = 0; fb < 4; ++fb)
            for (int r = 0; r < 4; ++r) {
                hout[(16 * fb + 4 * g + r) * 16 + j] = at[fb][r];
                hout[1024 + (16 * fb + 4 * g + r) * 16 + j] = as[fb][r];
            }
    float sum = 0;
    for (int fb = 0; fb < 4; ++fb) sum += HT[fb][0] + HS[fb][1];
    if (sum == 12345.0f) hout[2048 + threadIdx.x] = sum;
}

template <int MODE, int SHAPE>   // back-to-back rates, 4 independent accumulators, 1 wave / SIMD
__global__ __launch_bounds__(256, 1) void rate(float* out, int iters, unsigned long long* clk) {
    const int lane = threadIdx.x & 63;
    f32x4 acc[4];
    for (int b = 0; b < 4; ++b) acc[b] = f32x4{0, 0, 0, 0};
    bf16x8 a8, b8; s16x4 a4, b4; float af = 1e-3f * lane, bf = 2e-3f * lane;
    for (int i = 0; i < 8; ++i) { a8[i] = (__bf16)(0.01f * (lane + i)); b8[i] = (__bf16)(0.02f * (lane - i)); }
    for (int i = 0; i < 4; ++i) { a4[i] = (short)(lane + i); b4[i] = (short)(lane * 3 + i); }
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                if (SHAPE == 0) acc[b] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[b], 0, 0, 0);
                if (SHAPE == 1) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[b], 0, 0, 0);
                if (SHAPE == 2) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af, bf, acc[b], 0, 0, 0);
            }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
    float s = 0;
    for (int b = 0; b < 4; ++b) s += acc[b][0] + acc[b][1] + acc[b][2] + acc[b][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static uint16_t trunc_bf(float x) { uint32_t u; std::memcpy(&u, &x, 4); return (uint16_t)(u >> 16); }
static float from_bf(uint16_t h) { uint32_t u = (uint32_t)h << 16; float x; std::memcpy(&x, &u, 4); return x; }
static void split3(float x, uint16_t p[3]) {
    p[0] = trunc_bf(x);
    float r = x - from_bf(p[0]);
    p[1] = trunc_bf(r);
    float l = r - from_bf(p[1]);
    p[2] = trunc_bf(l);
}
static int kperm(int s, int g, int jj) { return 32 * s + 4 * g + (jj & 3) + 16 * (jj >> 2); }

int main() {
    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.0f, 0.125f);
    std::uniform_real_distribution<float> ud(-1.0f, 1.0f);
    std::vector<float> W[2];   // W[net][k*64 + f], pre-scaled by kTS as the rollout's images
    for (int n = 0; n < 2; ++n) {
        W[n].resize(64 * 64);
        for (auto& w : W[n]) w = kTS * nd(rng);
    }
    std::vector<float> H(64 * 16);   // H[k][env]
    for (auto& h : H) h = ud(rng);
    // f32 image: [k][j][fb] per net
    std::vector<float> imgf(2 * F32_NET);
    for (int n = 0; n < 2; ++n)
        for (int k = 0; k < 64; ++k)
            for (int f = 0; f < 64; ++f) imgf[n * F32_NET + k * 64 + (f & 15) * 4 + (f >> 4)] = W[n][k * 64 + f];
    // bf16 image: per net 3 pieces of [s][g][fb][i][jj] = W[kperm][16fb+i]
    std::vector<uint16_t> imgb(2 * BF_NET);
    for (int n = 0; n < 2; ++n)
        for (int s = 0; s < 2; ++s)
            for (int g = 0; g < 4; ++g)
                for (int fb = 0; fb < 4; ++fb)
                    for (int i = 0; i < 16; ++i)
                        for (int jj = 0; jj < 8; ++jj) {
                            uint16_t p[3];
                            split3(W[n][kperm(s, g, jj) * 64 + 16 * fb + i], p);
                            const int o = (((s * 4 + g) * 4 + fb) * 16 + i) * 8 + jj;
                            for (int q = 0; q < 3; ++q) imgb[n * BF_NET + q * BF_PIECE + o] = p[q];
                        }
    float *dimgf, *dimgb, *dh, *dout, *dout2;
    unsigned long long* clk;
    hipMalloc(&dimgf, imgf.size() * 4);
    hipMalloc(&dimgb, imgb.size() * 2);
    hipMalloc(&dh, H.size() * 4);
    hipMalloc(&dout, 4096 * 4 * 4);
    hipMalloc(&dout2, 1 << 22);
    hipMalloc(&clk, 64 * 8);
    hipMemcpy(dimgf, imgf.data(), imgf.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dimgb, imgb.data(), imgb.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dh, H.data(), H.size() * 4, hipMemcpyHostToDevice);
    // f64 reference of the first layer: Z[f][env] = sum_k W[k][f] H[k][env] (student: -H)
    auto check = [&](const char* name) {
        std::vector<float> o(2048);
        hipMemcpy(o.data(), dout, 2048 * 4, hipMemcpyDeviceToHost);
        double emax = 0, rms = 0;
        for (int n = 0; n < 2; ++n)
            for (int f = 0; f < 64; ++f)
                for (int e = 0; e < 16; ++e) {
                    double z = 0, za = 0;
                    for (int k = 0; k < 64; ++k) {
                        const double t = (double)W[n][k * 64 + f] * (n ? -H[k * 16 + e] : H[k * 16 + e]);
                        z += t; za += fabs(t);
                    }
                    const double err = fabs(o[n * 1024 + f * 16 + e] - z) / za;
                    emax = fmax(emax, err); rms += err * err;
                }
        printf("  %s: max |err| / sum|terms| = %.3g (f32 eps %.3g), rms %.3g\n", name, emax, ldexp(1.0, -24),
               sqrt(rms / 2048));
    };
    const int blocks = 256, iters = 4000;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    auto run_layer = [&](auto kern, const float* img, const char* name) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(512), 0, 0, img, dh, dout, iters, clk);
        hipEventRecord(a);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(512), 0, 0, img, dh, dout, iters, clk);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        unsigned long long c[8]; hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
        const double flop = 2.0 * 2 * 64 * 64 * 16 * (double)iters * 8 * blocks;   // 2 nets, 8 waves
        hipLaunchKernelGGL(kern, dim3(1), dim3(512), 0, 0, img, dh, dout, 1, clk);
        hipDeviceSynchronize();
        printf("%s: %.3f ms, %.1f f32-TFLOP/s, wave0 %.0f cyc/layer (2 nets, 16 envs, +tanh), %.2f GHz\n", name, ms,
               flop / ms / 1e9, (double)c[0] / iters, c[0] / (ms * 1e6));
        check(name);
    };
    run_layer(layer<0>, dimgf, "f32 exact 16x16x4");
    run_layer(layer<1>, dimgb, "split bf16x6 16x16x32");
    run_layer(layer<2>, dimgb, "split bf16x3 (timing only)");
    auto run_rate = [&](auto kern, const char* name) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, dout2, 2000, clk);
        hipDeviceSynchronize();
        unsigned long long c; hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
        printf("%s: %.2f cyc per MFMA (one wave per SIMD, 4 accumulators)\n", name, (double)c / (2000.0 * 64));
    };
    run_rate(rate<0, 0>, "16x16x16 bf16_1k");
    run_rate(rate<0, 1>, "16x16x32 bf16");
    run_rate(rate<0, 2>, "16x16x4 f32");
    return 0;
}
