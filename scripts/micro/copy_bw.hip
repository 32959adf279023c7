// Streaming-copy ceiling on one MI355X (measurement tool, not the product): dst = src with 4-,
// 8- and 16-B accesses per lane, grid-stride, plus a one-shot float4 form that keeps UNROLL
// 16-B loads per lane in flight before its stores (plain or non-temporal).  bench.py quotes the
// standalone env kernel's HBM rate against the best of these measured in the same run
// (MI355X_MICROARCH.md: 6.29 TB/s measured for a float4 copy).
//   shared library (bench.py, __graft_entry__.build): hipcc -O3 --offload-arch=gfx950 -shared -fPIC
//       -DCOPY_BW_LIB -o scripts/micro/libcopybw.so scripts/micro/copy_bw.hip
//   stand-alone:  hipcc -O3 --offload-arch=gfx950 -o scripts/micro/copy_bw scripts/micro/copy_bw.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__global__ __launch_bounds__(256) void copy_kernel(const T* __restrict__ src, T* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

// one-shot: block b copies float4s [b * 256 * U, (b + 1) * 256 * U), lane-contiguous per step
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy4_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst, size_t n) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) v[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) {
            if (NT) __builtin_nontemporal_store(v[u], dst + i);
            else dst[i] = v[u];
        }
    }
}

// the env kernel's read:write mix (40 B read, 73 B written per env-step ~ 1 : 2): block b reads
// float4s [b * 256 * U, ...) of src once and writes each twice, to dst[i] and dst[n + i] (dst
// holds 2n float4s); bytes counted = 3 x 16 B per source float4
template <int U, bool NT>
__global__ __launch_bounds__(256) void mix12_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst, size_t n) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) v[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) {
            if (NT) {
                __builtin_nontemporal_store(v[u], dst + i);
                __builtin_nontemporal_store(v[u], dst + n + i);
            } else {
                dst[i] = v[u];
                dst[n + i] = v[u];
            }
        }
    }
}

template <typename F>
static double timed(F&& launch, size_t bytes, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) launch();
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 2.0 * bytes * reps / (ms * 1e-3) / 1e12;   // read + write bytes per second, TB/s
}

// variant: 0 = grid-stride 4 B, 1 = 8 B, 2 = 16 B (`blocks` workgroups); 3 = one-shot float4
// x4 per lane, 4 = the same non-temporal, 5 = one-shot x8, 6 = x8 non-temporal, 7 / 8 = the
// 1 : 2 read:write mix (mix12_kernel), non-temporal / plain
static double run(void* a, void* b, size_t bytes, int variant, int blocks, int reps) {
    const size_t n4 = bytes / 16;
    switch (variant) {
        case 0: return timed([&] { hipLaunchKernelGGL(copy_kernel<float>, dim3(blocks), dim3(256), 0, 0, (const float*)a, (float*)b, bytes / 4); }, bytes, reps);
        case 1: return timed([&] { hipLaunchKernelGGL(copy_kernel<float2>, dim3(blocks), dim3(256), 0, 0, (const float2*)a, (float2*)b, bytes / 8); }, bytes, reps);
        case 2: return timed([&] { hipLaunchKernelGGL(copy_kernel<f32x4>, dim3(blocks), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)b, n4); }, bytes, reps);
        case 3: return timed([&] { hipLaunchKernelGGL((copy4_kernel<4, false>), dim3((n4 + 1023) / 1024), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)b, n4); }, bytes, reps);
        case 4: return timed([&] { hipLaunchKernelGGL((copy4_kernel<4, true>), dim3((n4 + 1023) / 1024), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)b, n4); }, bytes, reps);
        case 5: return timed([&] { hipLaunchKernelGGL((copy4_kernel<8, false>), dim3((n4 + 2047) / 2048), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)b, n4); }, bytes, reps);
        case 6: return timed([&] { hipLaunchKernelGGL((copy4_kernel<8, true>), dim3((n4 + 2047) / 2048), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)b, n4); }, bytes, reps);
        // read:write 1:2 over a third of the buffer as source (timed() counts 2 x bytes; the
        // mix moves 3 x bytes / 3 read + 2 x bytes / 3 written = the same total)
        case 7: { const size_t m = n4 / 3; return timed([&] { hipLaunchKernelGGL((mix12_kernel<4, true>), dim3((m + 1023) / 1024), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)b, m); }, m * 16 * 3 / 2, reps); }
        case 8: { const size_t m = n4 / 3; return timed([&] { hipLaunchKernelGGL((mix12_kernel<4, false>), dim3((m + 1023) / 1024), dim3(256), 0, 0, (const f32x4*)a, (f32x4*)b, m); }, m * 16 * 3 / 2, reps); }
        default: return -1.0;
    }
}

static const char* kName[] = {"grid-stride 4B", "grid-stride 8B", "grid-stride 16B", "one-shot 16B x4",
                              "one-shot 16B x4 nt", "one-shot 16B x8", "one-shot 16B x8 nt",
                              "read 1 : write 2, 16B x4 nt", "read 1 : write 2, 16B x4"};

#ifdef COPY_BW_LIB
extern "C" {
// TB/s (read + write) of one copy variant over `bytes` (two device buffers allocated here), or < 0
double copy_bw_tbs(size_t bytes, int variant, int blocks, int reps) {
    void *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess) return -1.0;
    if (hipMalloc(&b, bytes) != hipSuccess) {
        (void)hipFree(a);
        return -1.0;
    }
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 0, bytes);
    const double t = run(a, b, bytes, variant, blocks, reps);
    (void)hipFree(a);
    (void)hipFree(b);
    return t;
}
const char* copy_bw_name(int variant) { return variant >= 0 && variant < 9 ? kName[variant] : ""; }
}
#else
int main() {
    const size_t bytes = (size_t)1 << 30;
    void *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 0, bytes);
    for (int blocks : {1024, 4096, 16384, 65536})
        for (int v = 0; v < 3; ++v)
            printf("{\"access\": \"%s\", \"blocks\": %d, \"bytes\": %zu, \"TB_per_s\": %.3f}\n", kName[v], blocks, bytes,
                   run(a, b, bytes, v, blocks, 20));
    for (int v = 3; v < 9; ++v)
        printf("{\"access\": \"%s\", \"bytes\": %zu, \"TB_per_s\": %.3f}\n", kName[v], bytes, run(a, b, bytes, v, 0, 20));
    (void)hipFree(a);
    (void)hipFree(b);
    return 0;
}
#endif
