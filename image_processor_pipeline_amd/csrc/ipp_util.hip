// ipp_util.hip — measurement helper: the on-box HBM copy ceiling.
//
// SURVEY §8(d) asks for the roofline fraction against the 8 TB/s spec AND
// against a copy kernel measured on the same box.  This is that copy: a flat
// byte stream moved with 16-B loads and stores, one vector per thread.
// bench.py times it with HIP events right before the pipe and reports
// (read + written bytes) / time as roofline.copy_ceiling.
#include "ipp_device.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// One 16-B vector per thread, no grid-stride loop: on MI355X this one-shot
// form reaches the HBM ceiling (≈6.3 TB/s for a 1 GiB copy), while
// grid-strided loops with 4 vectors in flight per thread top out near
// 5.4 TB/s (tools/probes/copy_probe.hip, measured on the box).
__global__ void __launch_bounds__(256) k_stream_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                     int64_t n16) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) __builtin_nontemporal_store(src[i], dst + i);
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
        const int64_t blocks = (n16 + 255) / 256;
        if (blocks >= INT32_MAX) return IPP_E_ARG;
        hipLaunchKernelGGL(k_stream_copy, dim3((uint32_t)blocks), dim3(256), 0, s, reinterpret_cast<const u32x4*>(src),
                           reinterpret_cast<u32x4*>(dst), n16);
    }
    const int64_t tail = nbytes - (n16 << 4);
    if (tail > 0)
        hipLaunchKernelGGL(k_tail_copy, dim3(1), dim3(256), 0, s, src + (n16 << 4), dst + (n16 << 4), tail);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
