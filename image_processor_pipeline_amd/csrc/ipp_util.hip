// ipp_util.hip — measurement helper: the on-box HBM copy ceiling.
//
// SURVEY §8(d) asks for the roofline fraction against the 8 TB/s spec AND
// against a copy kernel measured on the same box.  This is that copy: a flat
// byte stream moved with 16-B loads and stores, four in flight per thread,
// grid-strided so every CU keeps the same share of the stream.  bench.py times
// it with HIP events right before the pipe and reports
// (read + written bytes) / time as `hbm_copy_ceiling_gbps`.
#include "ipp_device.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_stream_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                     int64_t n16) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], dst + i + u * stride);
    }
    for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ void k_tail_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

}  // namespace

extern "C" int ipp_stream_copy(const uint8_t* src, uint8_t* dst, int64_t nbytes, void* stream) {
    if (nbytes == 0) return IPP_OK;
    if (!src || !dst || nbytes < 0) return IPP_E_ARG;
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) != 0) return IPP_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    const int64_t n16 = nbytes >> 4;
    if (n16 > 0) {
        // 8 blocks of 256 threads per CU on 256 CUs
        const int64_t want = (n16 + 255) / 256;
        const uint32_t blocks = (uint32_t)(want < 2048 ? want : 2048);
        hipLaunchKernelGGL(k_stream_copy, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const u32x4*>(src),
                           reinterpret_cast<u32x4*>(dst), n16);
    }
    const int64_t tail = nbytes - (n16 << 4);
    if (tail > 0)
        hipLaunchKernelGGL(k_tail_copy, dim3(1), dim3(256), 0, s, src + (n16 << 4), dst + (n16 << 4), tail);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
