// Microbenchmark: does a VALU-only wave overlap a v_mfma_f32_16x16x4_f32-only wave on the
// same SIMD (512-thread WG: waves w and w+4 share a SIMD)?  Compare wall time of
// MFMA-only, VALU-only, and mixed (waves 0-3 MFMA, 4-7 VALU) launches.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int ROLE_LO, int ROLE_HI>   // role: 0 idle, 1 f32 mfma, 2 valu fma, 3 bf16 mfma
__global__ __launch_bounds__(512, 1) void k(float* out, int iters) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int role = wave < 4 ? ROLE_LO : ROLE_HI;
    float s = 0;
    if (role == 1) {
        f32x4 acc[4] = {};
        float h[4];
        for (int r = 0; r < 4; ++r) h[r] = 1e-3f * (lane + r);
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int x = 0; x < 16; ++x)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(h[x & 3], h[(x + b) & 3], acc[b], 0, 0, 0);
        for (int b = 0; b < 4; ++b) s += acc[b][0];
    } else if (role == 3) {
        f32x4 acc[4] = {};
        bf16x8 av, bv;
        for (int r = 0; r < 8; ++r) { av[r] = (short)(lane + r); bv[r] = (short)(lane * 3 + r); }
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int x = 0; x < 16; ++x)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[b], 0, 0, 0);
        for (int b = 0; b < 4; ++b) s += acc[b][0];
    } else if (role == 2) {
        float v[16];
        for (int r = 0; r < 16; ++r) v[r] = 1e-3f * (lane + r);
        // 16 independent fma chains; per iteration 16*16 = 256 v_fma (comparable issue time
        // to 64 f32 MFMAs x 32 cycles = 2048 cycles at 4+ cycles per VALU op... 512+)
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int x = 0; x < 32; ++x)
#pragma unroll
                for (int r = 0; r < 16; ++r) v[r] = __builtin_fmaf(v[r], 0.999f, 1e-4f);
        for (int r = 0; r < 16; ++r) s += v[r];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int A, int B>
float run(const char* name, int iters = 1000) {
    float* out;
    (void)hipMalloc(&out, sizeof(float) * 256 * 512);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k<A, B>), dim3(256), dim3(512), 0, 0, out, iters);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k<A, B>), dim3(256), dim3(512), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %.3f ms\n", name, ms);
    (void)hipFree(out);
    return ms;
}

int main() {
    run<1, 0>("f32 mfma only (lo)");
    run<2, 0>("valu only (lo)");
    run<1, 2>("f32 mfma lo + valu hi");
    run<1, 1>("f32 mfma lo + hi");
    run<3, 0>("bf16 mfma only (lo)");
    run<3, 2>("bf16 mfma lo + valu hi");
    return 0;
}
