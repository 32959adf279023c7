// Microbenchmark: v_mfma_f32_16x16x4_f32 issue rate on gfx950 for the rollout kernel's
// shapes: (a) register operands, (b) A operand from LDS via ds_read_b128 one k-step ahead,
// with 1 or 2 waves per SIMD.  Prints achieved TFLOP/s and the in-kernel clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512, 1) void k(float* out, int iters, unsigned long long* clk) {
    __shared__ __attribute__((aligned(16))) float L[64 * 64];
    for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) L[i] = 1e-3f * (i % 7);
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    f32x4 acc[4];
    for (int b = 0; b < 4; ++b) acc[b] = f32x4{0, 0, 0, 0};
    float h[16];
    for (int r = 0; r < 16; ++r) h[r] = 1e-3f * (lane + r);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) {
#pragma unroll
            for (int s = 0; s < 16; ++s)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(h[s], h[(s + b) & 15], acc[b], 0, 0, 0);
        } else {
            f32x4 wn = *reinterpret_cast<const f32x4*>(L + (4 * g) * 64 + 4 * j);
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const f32x4 w = wn;
                if (s < 15) wn = *reinterpret_cast<const f32x4*>(L + ((s + 1 + 4 * g) & 63) * 64 + 4 * j);
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[b], h[s], acc[b], 0, 0, 0);
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0 && blockIdx.x == 0) clk[threadIdx.x >> 6] = t1 - t0;
    float s = 0;
    for (int b = 0; b < 4; ++b) s += acc[b][0] + acc[b][1] + acc[b][2] + acc[b][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
void run(int threads, const char* name) {
    const int blocks = 256, iters = 2000;
    float* out; unsigned long long* clk;
    hipMalloc(&out, sizeof(float) * blocks * threads);
    hipMalloc(&clk, sizeof(unsigned long long) * 8);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, out, iters, clk);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, out, iters, clk);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    unsigned long long c[8]; hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
    const double flop = 2.0 * 16 * 16 * 4 * 64.0 * iters * (threads / 64) * blocks;
    printf("%s threads=%d: %.3f ms, %.1f TFLOP/s, wave0 cycles %llu -> %.2f GHz, cyc/mfma/wave %.1f\n", name, threads, ms,
           flop / ms / 1e9, c[0], c[0] / (ms * 1e6), (double)c[0] / (64.0 * iters));
}

int main() {
    run<0>(256, "regs");
    run<0>(512, "regs");
    run<1>(256, "lds-A");
    run<1>(512, "lds-A");
    return 0;
}
