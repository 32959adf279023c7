// Microbenchmark: two waves per SIMD, each running our layer-2 MFMA pattern
// (16 k-steps x NCH dependent accumulator chains of v_mfma_f32_16x16x4_f32, A from LDS via
// ds_read_b128 one k-step ahead, B from registers), optionally with VALU "tanh" work
// (exp + rcp per accumulator element) after each 64-MFMA block, like a forward layer.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NCH, bool TANH>
__global__ __launch_bounds__(512, 1) void k(float* out, int iters, int waves_active) {
    __shared__ __attribute__((aligned(16))) float L[64 * 64];
    for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) L[i] = 1e-3f * (i % 7);
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    if (wave >= waves_active) return;
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    f32x4 acc[NCH];
    float h[16];
    for (int r = 0; r < 16; ++r) h[r] = 1e-3f * (lane + r);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int b = 0; b < NCH; ++b) acc[b] = f32x4{0, 0, 0, 0};
        f32x4 wn = *reinterpret_cast<const f32x4*>(L + (4 * g) * 64 + 4 * j);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const f32x4 w = wn;
            if (s < 15) wn = *reinterpret_cast<const f32x4*>(L + ((s + 1 + 4 * g) & 63) * 64 + 4 * j);
#pragma unroll
            for (int b = 0; b < NCH; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[b & 3], h[s], acc[b], 0, 0, 0);
        }
        if (TANH) {
#pragma unroll
            for (int b = 0; b < NCH && b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    h[b * 4 + r] = 1.0f - 2.0f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(acc[b][r]) + 1.0f);
        } else {
#pragma unroll
            for (int b = 0; b < NCH && b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) h[b * 4 + r] = acc[b][r];
        }
    }
    float sum = 0;
    for (int r = 0; r < 16; ++r) sum += h[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = sum;
}

template <int NCH, bool TANH>
void run(int waves, const char* name) {
    const int iters = 500;
    float* out;
    (void)hipMalloc(&out, sizeof(float) * 256 * 512);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    hipLaunchKernelGGL((k<NCH, TANH>), dim3(256), dim3(512), 0, 0, out, iters, waves);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((k<NCH, TANH>), dim3(256), dim3(512), 0, 0, out, iters, waves);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double mfma = (double)iters * 16 * NCH * waves * 256;
    const double ideal_ms = mfma / 4 / 256 * 32 / 2.3e9 * 1e3 * (waves > 4 ? 1 : 1);   // per-SIMD 32 cycles each
    printf("%-22s waves/CU=%d: %.3f ms  (MFMA-bound at 2.3 GHz: %.3f ms)\n", name, waves, ms,
           mfma / (256.0 * 4) * 32 / 2.3e9 * 1e3);
    (void)hipFree(out);
}

int main() {
    run<4, false>(4, "4 chains");
    run<4, false>(8, "4 chains");
    run<8, false>(4, "8 chains");
    run<8, false>(8, "8 chains");
    run<4, true>(4, "4 chains + tanh");
    run<4, true>(8, "4 chains + tanh");
    run<8, true>(4, "8 chains + tanh");
    run<8, true>(8, "8 chains + tanh");
    return 0;
}
