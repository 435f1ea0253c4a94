// Probe: does v_ashr_pk_u8_i32 preserve bits 16-31 of its destination on gfx950?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
    unsigned d = 0xDEADBEEFu;
    int a = 100 << 22, b = 7 << 22;
    asm volatile("v_ashr_pk_u8_i32 %0, %1, %2, 22" : "+v"(d) : "v"(a), "v"(b));
    out[threadIdx.x] = d;
}
int main() {
    unsigned* o; hipMalloc(&o, 256); hipLaunchKernelGGL(k, 1, 64, 0, 0, o);
    unsigned h[64]; hipMemcpy(h, o, 256, hipMemcpyDeviceToHost);
    printf("v_ashr_pk_u8_i32 dst=0xDEADBEEF a=100<<22 b=7<<22 -> 0x%08X (zeroed upper: 0x%08X)\n", h[0], 0x0764u);
    return 0;
}
