// copy_probe.hip — which flat copy reaches the HBM ceiling on this box?
// Variants: load/store cache policy (plain / nt), grid size, unroll.
// Build: hipcc --offload-arch=gfx950 -O3 -o copy_probe copy_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int LD, int ST, int U>
__global__ void __launch_bounds__(256) k_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n16) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = LD ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (ST) __builtin_nontemporal_store(v[u], dst + i + u * stride);
            else dst[i + u * stride] = v[u];
        }
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

template <int LD, int ST, int U>
void run(const char* name, const u32x4* a, u32x4* b, int64_t n16, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_copy<LD, ST, U>), dim3(blocks), dim3(256), 0, 0, a, b, n16);
    hipEventRecord(e0);
    const int reps = 10;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_copy<LD, ST, U>), dim3(blocks), dim3(256), 0, 0, a, b, n16);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("%-12s U=%d blocks=%6d  %8.1f GB/s\n", name, U, blocks, 2.0 * 16.0 * n16 / (ms * 1e-3) / 1e9);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    for (int64_t bytes : {(int64_t)1 << 30, (int64_t)4 << 30}) {
        const int64_t n16 = bytes / 16;
        u32x4 *a, *b;
        if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
        hipMemset(a, 1, bytes);
        printf("--- %lld MiB\n", (long long)(bytes >> 20));
        for (int blocks : {1024, 2048, 4096, 16384, 65536}) {
            run<0, 0, 4>("plain/plain", a, b, n16, blocks);
            run<0, 1, 4>("plain/nt", a, b, n16, blocks);
            run<1, 1, 4>("nt/nt", a, b, n16, blocks);
            run<1, 0, 4>("nt/plain", a, b, n16, blocks);
        }
        run<0, 0, 1>("plain/plain", a, b, n16, 1 << 20);
        run<0, 1, 1>("plain/nt", a, b, n16, 1 << 20);
        hipFree(a);
        hipFree(b);
    }
    return 0;
}
