// lds_dma_probe.hip — semantics of the 16-byte LDS-DMA loads on gfx950 that
// a staged H pass would rely on:
//   1. buffer_load_dwordx4 ... lds and global_load_lds_dwordx4 at byte
//      offsets that are 16-, 4- and 1-aligned: are the bytes right?
//   2. buffer range check on a 16-byte load that straddles num_records: which
//      dwords come back (per dword, per byte, or all zero)?
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_dma_probe lds_dma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void* lds_ptr;

// mode 0: buffer lds x4, 1: global lds x4.  Lane l loads 16 B at byte
// offset base_off + 16 l (+ 0 for the straddle test) into LDS[16 l].
__global__ void k_dma(const uint8_t* src, int nrec, int base_off, int mode, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t s[64 * 16];
    for (int i = threadIdx.x; i < 64 * 16; i += 64) s[i] = 0xEE;
    __syncthreads();
    if (mode == 0) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nrec, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)s, 16, base_off + 16 * threadIdx.x, 0, 0, 0);
    } else {
        __builtin_amdgcn_global_load_lds((const void*)(src + base_off + 16 * threadIdx.x), (lds_ptr)s, 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 16; i += 64) out[i] = s[i];
}

int main() {
    const int N = 4096;
    std::vector<uint8_t> h(N);
    for (int i = 0; i < N; ++i) h[i] = (uint8_t)(i * 7 + 3);
    uint8_t *d, *o;
    hipMalloc(&d, N);
    hipMalloc(&o, 1024);
    hipMemcpy(d, h.data(), N, hipMemcpyHostToDevice);
    std::vector<uint8_t> r(1024);
    for (int mode = 0; mode < 2; ++mode)
        for (int off : {0, 4, 8, 1, 2, 3, 5}) {
            hipLaunchKernelGGL(k_dma, dim3(1), dim3(64), 0, 0, d, N, off, mode, o);
            hipMemcpy(r.data(), o, 1024, hipMemcpyDeviceToHost);
            int bad = 0, first = -1;
            for (int i = 0; i < 1024; ++i)
                if (r[i] != h[off + i]) { if (first < 0) first = i; ++bad; }
            printf("%s offset %d: %d wrong bytes (first %d)\n", mode ? "global_load_lds_dwordx4" : "buffer_load_dwordx4 lds",
                   off, bad, first);
        }
    // straddle: num_records = 16*k + t; lane k's load covers [16k, 16k+16)
    for (int t : {1, 3, 4, 5, 8, 13}) {
        const int nrec = 16 * 10 + t;
        hipLaunchKernelGGL(k_dma, dim3(1), dim3(64), 0, 0, d, nrec, 0, 0, o);
        hipMemcpy(r.data(), o, 1024, hipMemcpyDeviceToHost);
        printf("straddle nrec=16*10+%2d, lane 10 bytes:", t);
        for (int i = 160; i < 176; ++i) printf(" %s", r[i] == h[i] ? "d" : (r[i] == 0 ? "0" : "?"));
        printf("   lane 9 ok=%d lane 11 zero=%d\n", (int)(r[159] == h[159]), (int)(r[176] == 0));
    }
    hipFree(d);
    hipFree(o);
    return 0;
}
