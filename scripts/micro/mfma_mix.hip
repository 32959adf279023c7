// Microbenchmark: how much VALU hides behind each MFMA kind the rollout kernel can use on
// gfx950.  One wave issues a chain of independent MFMAs (4 accumulators) with NV independent
// v_fma_f32 fillers after each; reported: shader cycles per MFMA (s_memtime) with 1 and 2
// waves per SIMD (both waves run the same mix).
//   f32   v_mfma_f32_16x16x4_f32    (exact f32; the kernel's layer 1, dW2, dW1 today)
//   k32   v_mfma_f32_16x16x32_bf16  (the split products of the K = 64 layers)
//   k16   v_mfma_f32_16x16x16_bf16  (K = 16: a tile's envs as K)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int KIND, int NV, int NA = 4>
__global__ __launch_bounds__(512, 1) void k(float* out, int iters, unsigned long long* clk) {
    const int lane = threadIdx.x & 63;
    f32x4 acc[NA] = {};
    float v[8];
    for (int r = 0; r < 8; ++r) v[r] = 1e-3f * (lane * 2 + r);
    const float h = 1e-3f * lane;
    s16x4 a4;
    bf16x8 a8;
    for (int r = 0; r < 4; ++r) a4[r] = (short)(0x3c00 + lane + r);
    for (int r = 0; r < 8; ++r) a8[r] = (__bf16)(1e-2f * (lane + r));
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int x = 0; x < 32 / NA; ++x)
#pragma unroll
            for (int b = 0; b < NA; ++b) {
                if constexpr (KIND == 0) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(h, h + b, acc[b], 0, 0, 0);
                if constexpr (KIND == 1) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, a8, acc[b], 0, 0, 0);
                if constexpr (KIND == 2) acc[b] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, a4, acc[b], 0, 0, 0);
#pragma unroll
                for (int q = 0; q < NV; ++q) v[q & 7] = __builtin_fmaf(v[q & 7], 0.999f, 1e-4f);
            }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0 && blockIdx.x == 0) clk[threadIdx.x >> 6] = t1 - t0;
    float s = 0;
    for (int b = 0; b < NA; ++b) s += acc[b][0] + acc[b][3];
    for (int r = 0; r < 8; ++r) s += v[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND, int NV, int NA = 4>
void run(int threads) {
    const int blocks = 256, iters = 2000;
    float* out;
    unsigned long long* clk;
    (void)hipMalloc(&out, sizeof(float) * blocks * 512);
    (void)hipMalloc(&clk, sizeof(unsigned long long) * 8);
    hipLaunchKernelGGL((k<KIND, NV, NA>), dim3(blocks), dim3(threads), 0, 0, out, iters, clk);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL((k<KIND, NV, NA>), dim3(blocks), dim3(threads), 0, 0, out, iters, clk);
    (void)hipDeviceSynchronize();
    unsigned long long c[8];
    (void)hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
    const char* name[] = {"f32 16x16x4 ", "bf16 16x16x32", "bf16 16x16x16"};
    printf("%s waves/SIMD %d  acc %2d valu/mfma %2d : %6.1f cycles per mfma\n", name[KIND], threads / 256, NA, NV,
           (double)c[0] / (32.0 * iters));
    (void)hipFree(out);
    (void)hipFree(clk);
}

template <int KIND>
void sweep() {
    for (int t : {256, 512}) {
        run<KIND, 0>(t); run<KIND, 1>(t); run<KIND, 2>(t); run<KIND, 4>(t); run<KIND, 8>(t);
    }
}

int main() {
    run<0, 0, 16>(256); run<1, 0, 16>(256); run<2, 0, 16>(256);
    run<1, 2, 16>(256); run<2, 2, 16>(256);
    run<0, 0, 4>(64); run<1, 0, 4>(64); run<2, 0, 4>(64);
    return 0;
}
