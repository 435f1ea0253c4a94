// ta_probe.hip — cost of one vector-memory load instruction on the texture
// path (TA → TCP → TD) by access shape, from an L1-resident footprint, every
// CU busy.  Each wave issues `iters` × 8 loads of one shape in flight groups
// of 8 (vmcnt waits only between groups), addresses re-randomised per group
// inside a 16 KB window per block, and folds the data so nothing is dead.
// Prints ns per wave-instruction per CU and CU cycles per wave-instruction at
// the measured clock (GRBM-free: wall time × 2.4 GHz nominal, relative only).
//   shapes: dword / dwordx2 / dwordx4, aligned or byte-unaligned, random lanes
//   or one 16-row × 4-column quad map like the H pass, EXEC 64 / 32 / 16 lanes,
//   broadcast, contiguous.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o ta_probe ta_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

namespace {

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum Shape { RAND_DW_AL, RAND_DW_UN, RAND_X2_AL, RAND_X2_UN, RAND_X4_AL, RAND_X4_UN, RAND_DW_E32, RAND_DW_E16,
             BCAST_DW, CONTIG_DW, CONTIG_X4, ROWS16_DW_UN, ROWS16_X2_UN, ROWS16_X4_UN, CONTIG_X4_E16, CONTIG_X4_E32, CONTIG_X2, NSHAPE };
const char* kName[NSHAPE] = {"rand dword aligned", "rand dword unaligned", "rand dwordx2 aligned",
                             "rand dwordx2 unaligned", "rand dwordx4 aligned", "rand dwordx4 unaligned",
                             "rand dword, 32 lanes", "rand dword, 16 lanes", "broadcast dword",
                             "contiguous dword (256 B)", "contiguous dwordx4 (1 KB)",
                             "16 rows x 4 px dword (H-pass quad map)", "16 rows x 4 px dwordx2",
                             "16 rows x 4 px dwordx4", "contiguous dwordx4, 16 lanes", "contiguous dwordx4, 32 lanes",
                             "contiguous dwordx2 (512 B)"};

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

template <int S>
__global__ void __launch_bounds__(256) k_probe(const uint8_t* __restrict__ buf, int iters, uint32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint8_t* base = buf + (blockIdx.x & 1023) * 16384;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, 16384 + 64, 0x00020000);
    uint32_t acc = 0;
    uint32_t seed = hash(blockIdx.x * 256 + threadIdx.x);
    const bool act = (S == RAND_DW_E32 || S == CONTIG_X4_E32) ? lane < 32 : ((S == RAND_DW_E16 || S == CONTIG_X4_E16) ? lane < 16 : true);
    uint32_t r0[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r0[k] = hash(seed + (uint32_t)k * 0x9E3779B9u);
    const bool al = S == RAND_DW_AL || S == RAND_X2_AL || S == RAND_X4_AL || S == RAND_DW_E32 || S == RAND_DW_E16;
    const int r = 2 * (lane >> 3) + ((lane >> 1) & 1), c = 8 * ((lane >> 2) & 1) + (lane & 1);
    const uint32_t quad = (uint32_t)r * 300u + 3u * (uint32_t)c;
    for (int it = 0; it < iters; ++it) {
        uint32_t off[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t u = (uint32_t)(it * 8 + k);  // uniform
            uint32_t o;
            if (S == BCAST_DW) o = (u & 255u) * 64u;
            else if (S == CONTIG_DW) o = (u & 63u) * 256u + (uint32_t)lane * 4u;
            else if (S == CONTIG_X4 || S == CONTIG_X4_E16 || S == CONTIG_X4_E32) o = (u & 15u) * 1024u + (uint32_t)lane * 16u;
            else if (S == CONTIG_X2) o = (u & 31u) * 512u + (uint32_t)lane * 8u;
            else if (S >= ROWS16_DW_UN && S <= ROWS16_X4_UN) {
                // lane quad = 2x2 pixels, 16 rows x 4 columns of a 3-byte image of pitch 300 B,
                // window origin moving per instruction (uniform)
                const uint32_t org = ((u * 7u) % 40u) * 300u + ((u * 13u) % 60u) * 3u;
                o = org + quad;
            } else {
                o = (r0[k] + u * 0x2A4u) & 0x3FFFu;  // byte offset in 16 KB
                if (al) o &= ~3u;
            }
            off[k] = o;
        }
        if (act) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (S == RAND_X2_AL || S == RAND_X2_UN || S == ROWS16_X2_UN || S == CONTIG_X2) {
                    const u32x2 v = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off[k], 0, 0));
                    acc += v.x ^ v.y;
                } else if (S == RAND_X4_AL || S == RAND_X4_UN || S == CONTIG_X4 || S == ROWS16_X4_UN || S == CONTIG_X4_E16 || S == CONTIG_X4_E32) {
                    const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off[k], 0, 0));
                    acc += v.x ^ v.y ^ v.z ^ v.w;
                } else {
                    acc += __builtin_amdgcn_raw_buffer_load_b32(rs, off[k], 0, 0);
                }
            }
        }
    }
    if (acc == 0x12345678u) out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int S>
float run(const uint8_t* buf, uint32_t* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_probe<S>, dim3(blocks), dim3(256), 0, 0, buf, iters, out);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_probe<S>, dim3(blocks), dim3(256), 0, 0, buf, iters, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

template <int S>
void one(const uint8_t* buf, uint32_t* out, int blocks, int iters, int cus) {
    const float ms = run<S>(buf, out, blocks, iters);
    const double instr = (double)blocks * 4 * iters * 8;  // wave-instructions
    const double per_cu_ns = ms * 1e6 / (instr / cus);
    printf("%-42s %8.3f ms  %7.2f ns/instr/CU  %6.1f cyc@2.4GHz\n", kName[S], ms, per_cu_ns, per_cu_ns * 2.4);
    fflush(stdout);
}

}  // namespace

int main() {
    uint8_t* buf;
    uint32_t* out;
    const size_t bytes = (size_t)1024 * 16384 + 4096;
    if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
    hipMemset(buf, 0x5A, bytes);
    if (hipMalloc(&out, (size_t)1 << 24) != hipSuccess) return 1;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8, iters = 512;
    printf("%d CUs, %d blocks x 4 waves, %d loads per wave\n", cus, blocks, iters * 8);
    one<RAND_DW_AL>(buf, out, blocks, iters, cus);
    one<RAND_DW_UN>(buf, out, blocks, iters, cus);
    one<RAND_X2_AL>(buf, out, blocks, iters, cus);
    one<RAND_X2_UN>(buf, out, blocks, iters, cus);
    one<RAND_X4_AL>(buf, out, blocks, iters, cus);
    one<RAND_X4_UN>(buf, out, blocks, iters, cus);
    one<RAND_DW_E32>(buf, out, blocks, iters, cus);
    one<RAND_DW_E16>(buf, out, blocks, iters, cus);
    one<BCAST_DW>(buf, out, blocks, iters, cus);
    one<CONTIG_DW>(buf, out, blocks, iters, cus);
    one<CONTIG_X4>(buf, out, blocks, iters, cus);
    one<ROWS16_DW_UN>(buf, out, blocks, iters, cus);
    one<ROWS16_X2_UN>(buf, out, blocks, iters, cus);
    one<ROWS16_X4_UN>(buf, out, blocks, iters, cus);
    one<CONTIG_X4_E32>(buf, out, blocks, iters, cus);
    one<CONTIG_X4_E16>(buf, out, blocks, iters, cus);
    one<CONTIG_X2>(buf, out, blocks, iters, cus);
    hipFree(buf);
    hipFree(out);
    return 0;
}
