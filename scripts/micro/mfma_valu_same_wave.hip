// Microbenchmark: VALU instructions interleaved with independent v_mfma_f32_16x16x4_f32 in
// ONE wave (1 wave per SIMD): how many VALU ops per MFMA are hidden?
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NV>   // VALU fmas per MFMA
__global__ __launch_bounds__(256, 1) void k(float* out, int iters) {
    const int lane = threadIdx.x & 63;
    f32x4 acc[4] = {};
    float h[4], v[8];
    for (int r = 0; r < 4; ++r) h[r] = 1e-3f * (lane + r);
    for (int r = 0; r < 8; ++r) v[r] = 1e-3f * (lane * 2 + r);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int x = 0; x < 16; ++x)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(h[x & 3], h[(x + b) & 3], acc[b], 0, 0, 0);
#pragma unroll
                for (int q = 0; q < NV; ++q) v[q & 7] = __builtin_fmaf(v[q & 7], 0.999f, 1e-4f);
            }
    }
    float s = 0;
    for (int b = 0; b < 4; ++b) s += acc[b][0];
    for (int r = 0; r < 8; ++r) s += v[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NV>
void run(int iters = 1000) {
    float* out;
    (void)hipMalloc(&out, sizeof(float) * 256 * 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k<NV>, dim3(256), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<NV>, dim3(256), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("valu per mfma %2d: %.3f ms\n", NV, ms);
    (void)hipFree(out);
}

int main() {
    run<0>(); run<1>(); run<2>(); run<4>(); run<6>(); run<8>(); run<12>(); run<16>();
    return 0;
}
