// ipp_hsv.hip — K6+K7 standalone: BGR(A) image → BGRA with α from the HSV
// range masks (filtres_liste.py:84-134).  One pass, 4 pixels per thread,
// dwordx4 stores of the BGRA output.
#include "ipp_hsv.h"

namespace {
constexpr int TILE_W = 64, TILE_H = 16, PX = 4;

__global__ void __launch_bounds__(256)
k_hsv_mask(const uint8_t* __restrict__ src, const ipp_image_desc* __restrict__ sd,
           uint8_t* __restrict__ dst, const ipp_image_desc* __restrict__ dd,
           int tiles_x, int tiles_y, ipp_hsv_params p) {
    __shared__ HsvLds s;
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int per_img = tiles_x * tiles_y;
    const int im = b / per_img;
    const int t = b - im * per_img;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const ipp_image_desc in = sd[im];
    const ipp_image_desc out = dd[im];
    hsv_lds_init(s, p, in.w, in.h);
    __syncthreads();
    const int y = ty * TILE_H + (int)(threadIdx.x >> 4);
    const int x0 = tx * TILE_W + (int)(threadIdx.x & 15) * PX;
    if (y >= in.h || x0 >= in.w) return;
    const uint8_t* row = src + in.off + (int64_t)y * in.pitch;
    uint32_t o[PX];
#pragma unroll
    for (int k = 0; k < PX; ++k) {
        const int x = x0 + k;
        uint32_t px = 0;
        if (x < in.w) {
            if (in.cn == 4) {
                px = reinterpret_cast<const uint32_t*>(row)[x];
            } else {
                const bool wide_ok = (y < in.h - 1) || (x < in.w - 1);
                px = load_rgb_opaque(row + 3 * x, wide_ok);
            }
        }
        o[k] = (px & 0x00FFFFFFu) | (hsv_keep_alpha(s, px, p.bgr, x, y) << 24);
    }
    uint8_t* op = dst + out.off + (int64_t)y * out.pitch + 4 * x0;
    if (x0 + PX <= in.w && ((reinterpret_cast<uintptr_t>(op) & 15u) == 0)) {
        *reinterpret_cast<uint4*>(op) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
        for (int k = 0; k < PX; ++k)
            if (x0 + k < in.w) reinterpret_cast<uint32_t*>(op)[k] = o[k];
    }
}
}  // namespace

extern "C" int ipp_hsv_mask(const uint8_t* src, const ipp_image_desc* src_descs, uint8_t* dst,
                            const ipp_image_desc* dst_descs, int32_t n_images, int32_t max_w, int32_t max_h,
                            const ipp_hsv_params* params, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !dst || !src_descs || !dst_descs || !params || n_images < 0 || max_w <= 0 || max_h <= 0)
        return IPP_E_ARG;
    if (params->n_ranges < 0 || params->n_ranges > IPP_MAX_HSV_RANGES) return IPP_E_ARG;
    const int tx = (max_w + TILE_W - 1) / TILE_W, ty = (max_h + TILE_H - 1) / TILE_H;
    const int64_t blocks = (int64_t)tx * ty * n_images;
    if (blocks <= 0 || blocks >= INT32_MAX) return IPP_E_ARG;
    hipLaunchKernelGGL(k_hsv_mask, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, src, src_descs, dst,
                       dst_descs, tx, ty, *params);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
