// Probe of the v_mfma_i32_16x16x64_i8 operand layout on gfx950 with exact
// integer data and an asymmetric B.  Hypothesis (bf16 16x16x32 analogue):
//   lane l holds A[row l&15][k = 16(l>>4) + j] and B[k = 16(l>>4) + j][col l&15],
//   j = 0..15 (byte j of its 4-VGPR fragment); D: col = l&15, row = 4(l>>4) + r.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const int8_t* A, const int8_t* B, int32_t* C) {
    const int l = threadIdx.x;
    i32x4 a, b;
    int8_t* pa = reinterpret_cast<int8_t*>(&a);
    int8_t* pb = reinterpret_cast<int8_t*>(&b);
    for (int j = 0; j < 16; ++j) {
        pa[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
        pb[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
    }
    i32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
    int8_t A[16 * 64], B[64 * 16];
    for (int i = 0; i < 16; ++i)
        for (int kk = 0; kk < 64; ++kk) A[i * 64 + kk] = (int8_t)((i * 7 + kk * 3) % 23 - 11);
    for (int kk = 0; kk < 64; ++kk)
        for (int j = 0; j < 16; ++j) B[kk * 16 + j] = (int8_t)((kk * 5 + j * 11 + kk * j) % 29 - 14);
    int8_t *dA, *dB;
    int32_t* dC;
    hipMalloc(&dA, sizeof(A));
    hipMalloc(&dB, sizeof(B));
    hipMalloc(&dC, 256 * 4);
    hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
    hipMemcpy(dB, B, sizeof(B), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    int32_t C[256];
    hipMemcpy(C, dC, sizeof(C), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            int32_t s = 0;
            for (int kk = 0; kk < 64; ++kk) s += A[i * 64 + kk] * B[kk * 16 + j];
            if (s != C[i * 16 + j]) ++bad;
        }
    printf("mfma_i32_16x16x64_i8 layout hypothesis: %d / 256 mismatches\n", bad);
    return bad != 0;
}
