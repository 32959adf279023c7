// Streaming-copy ceiling on one MI355X (diagnostic): dst = src with 4-, 8- and 16-B accesses
// per lane, grid-stride, vs the rd_step_kernel's measured rate.  Build:
//   hipcc -O3 --offload-arch=gfx950 -o scripts/micro/copy_bw scripts/micro/copy_bw.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

template <typename T>
__global__ __launch_bounds__(256) void copy_kernel(const T* __restrict__ src, T* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

template <typename T>
double run(const char* name, void* a, void* b, size_t bytes, int blocks) {
    const size_t n = bytes / sizeof(T);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(copy_kernel<T>, dim3(blocks), dim3(256), 0, 0, (const T*)a, (T*)b, n);
    hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(copy_kernel<T>, dim3(blocks), dim3(256), 0, 0, (const T*)a, (T*)b, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double tbs = 2.0 * bytes * reps / (ms * 1e-3) / 1e12;
    printf("{\"access\": \"%s\", \"blocks\": %d, \"bytes\": %zu, \"TB_per_s\": %.3f}\n", name, blocks, bytes, tbs);
    return tbs;
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    void *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    for (int blocks : {1024, 4096, 16384, 65536}) {
        run<float>("4B", a, b, bytes, blocks);
        run<float2>("8B", a, b, bytes, blocks);
        run<float4>("16B", a, b, bytes, blocks);
    }
    hipFree(a);
    hipFree(b);
    return 0;
}
