// ipp_resample.hip — K8 LANCZOS separable passes and K9 paste/blend.
//
// Reference: overlays.py:129 ``overlay.resize((w, h), LANCZOS)`` → Pillow
// Image.resize (RGBA → RGBa convert, ImagingResample horizontal pass over rows
// [ybox_first, ybox_last), vertical pass, RGBa → RGBA) and overlays.py:138-139
// ``background.copy(); paste(ov, (x, y), ov)`` → Paste.c paste_mask_RGBA.
// Arithmetic: int32 accumulators seeded with 1 << 21, 22-bit taps, clip8 of
// ss >> 22 (Resample.c, PRECISION_BITS = 22); DIV255 blend (Paste.c BLEND).
// 8-bit × 24-bit products use v_mad_i32_i24 (taps |k| < 2^23).
#include "ipp_device.h"

namespace {

__device__ __forceinline__ int32_t mad24(int32_t a, int32_t b, int32_t c) { return __mul24(a, b) + c; }

// H pass: one output pixel per thread; block = 64 outputs × 4 rows.
__global__ void __launch_bounds__(256)
k_lanczos_h(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, const int32_t* __restrict__ coefs,
            const ipp_resample_desc* __restrict__ descs, int tiles_x, int tiles_y, int flags) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int per_img = tiles_x * tiles_y;
    const int im = b / per_img;
    const int t = b - im * per_img;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const ipp_resample_desc d = descs[im];
    const int xo = tx * 64 + (int)(threadIdx.x & 63);
    const int row = ty * 4 + (int)(threadIdx.x >> 6);
    if (xo >= d.out_len || row >= d.lines) return;
    const int32_t* bnd = coefs + d.coef_off;
    const int32_t* kk = bnd + 2 * d.out_len + (int64_t)xo * d.ksize;
    const int xmin = bnd[2 * xo], cnt = bnd[2 * xo + 1];
    const uint32_t* in =
        reinterpret_cast<const uint32_t*>(src + d.src_off + (int64_t)(d.line0 + row) * d.src_pitch) + xmin;
    int32_t s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21, s3 = 1 << 21;
    const bool pm = flags & IPP_RS_PREMULTIPLY;
    for (int k = 0; k < cnt; ++k) {
        uint32_t p = in[k];
        if (pm) p = premultiply(p);
        const int32_t w = kk[k];
        s0 = mad24((int32_t)(p & 0xFF), w, s0);
        s1 = mad24((int32_t)((p >> 8) & 0xFF), w, s1);
        s2 = mad24((int32_t)((p >> 16) & 0xFF), w, s2);
        s3 = mad24((int32_t)(p >> 24), w, s3);
    }
    uint32_t o = clip8(s0) | (clip8(s1) << 8) | (clip8(s2) << 16) | (clip8(s3) << 24);
    if (flags & IPP_RS_UNPREMULTIPLY) o = unpremultiply(o);
    reinterpret_cast<uint32_t*>(dst + d.dst_off + (int64_t)row * d.dst_pitch)[xo] = o;
}

// V pass: one output pixel per thread; block = 64 columns × 4 output rows.
__global__ void __launch_bounds__(256)
k_lanczos_v(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, const int32_t* __restrict__ coefs,
            const ipp_resample_desc* __restrict__ descs, int tiles_x, int tiles_y, int flags) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int per_img = tiles_x * tiles_y;
    const int im = b / per_img;
    const int t = b - im * per_img;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const ipp_resample_desc d = descs[im];
    const int col = tx * 64 + (int)(threadIdx.x & 63);
    const int yo = ty * 4 + (int)(threadIdx.x >> 6);
    if (col >= d.lines || yo >= d.out_len) return;
    const int32_t* bnd = coefs + d.coef_off;
    const int32_t* kk = bnd + 2 * d.out_len + (int64_t)yo * d.ksize;
    const int ymin = bnd[2 * yo], cnt = bnd[2 * yo + 1];
    const uint8_t* in = src + d.src_off + (int64_t)ymin * d.src_pitch + 4 * (int64_t)col;
    int32_t s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21, s3 = 1 << 21;
    const bool pm = flags & IPP_RS_PREMULTIPLY;
    for (int k = 0; k < cnt; ++k) {
        uint32_t p = *reinterpret_cast<const uint32_t*>(in + (int64_t)k * d.src_pitch);
        if (pm) p = premultiply(p);
        const int32_t w = kk[k];
        s0 = mad24((int32_t)(p & 0xFF), w, s0);
        s1 = mad24((int32_t)((p >> 8) & 0xFF), w, s1);
        s2 = mad24((int32_t)((p >> 16) & 0xFF), w, s2);
        s3 = mad24((int32_t)(p >> 24), w, s3);
    }
    uint32_t o = clip8(s0) | (clip8(s1) << 8) | (clip8(s2) << 16) | (clip8(s3) << 24);
    if (flags & IPP_RS_UNPREMULTIPLY) o = unpremultiply(o);
    reinterpret_cast<uint32_t*>(dst + d.dst_off + (int64_t)yo * d.dst_pitch)[col] = o;
}

// Paste: dst = bg (RGB) with the RGBA overlay blended at (x, y).  Each thread
// owns 16 bytes of one output row; a block covers 4 rows × 64 chunks.
__global__ void __launch_bounds__(256)
k_paste_blend(const uint8_t* __restrict__ bg, const uint8_t* __restrict__ ov, uint8_t* __restrict__ dst,
              const ipp_paste_desc* __restrict__ descs, int tiles_x, int tiles_y) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int per_img = tiles_x * tiles_y;
    const int im = b / per_img;
    const int t = b - im * per_img;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const ipp_paste_desc d = descs[im];
    const int y = ty * 4 + (int)(threadIdx.x >> 6);
    const int c0 = (tx * 64 + (int)(threadIdx.x & 63)) * 16;
    const int row_bytes = 3 * d.bg_w;
    if (y >= d.bg_h || c0 >= row_bytes) return;
    const uint8_t* brow = bg + d.bg_off + (int64_t)y * d.bg_pitch;
    uint8_t* orow = dst + d.dst_off + (int64_t)y * d.dst_pitch;
    const int nbytes = min(16, row_bytes - c0);
    const bool vec = nbytes == 16 && ((reinterpret_cast<uintptr_t>(brow + c0) | reinterpret_cast<uintptr_t>(orow + c0)) & 15u) == 0;
    uint32_t w[4];
    load16(brow + c0, nbytes, vec, w);
    const int oy = y - d.y;
    if ((unsigned)oy < (unsigned)d.ov_h && c0 + nbytes > 3 * d.x && c0 < 3 * (d.x + d.ov_w)) {
        const uint32_t* orow_ov = reinterpret_cast<const uint32_t*>(ov + d.ov_off + (int64_t)oy * d.ov_pitch);
        blend16(w, c0, nbytes, d.x, d.ov_w, [&](int ox) { return orow_ov[ox]; });
    }
    store16(orow + c0, nbytes, vec, w);
}

inline int64_t nblocks(int tx, int ty, int n) { return (int64_t)tx * ty * n; }

}  // namespace

extern "C" int ipp_lanczos_h(const uint8_t* src, uint8_t* dst, const int32_t* coefs, const ipp_resample_desc* descs,
                             int32_t n_images, int32_t max_out, int32_t max_lines, int32_t flags, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !dst || !coefs || !descs || n_images < 0 || max_out <= 0 || max_lines <= 0) return IPP_E_ARG;
    const int tx = (max_out + 63) / 64, ty = (max_lines + 3) / 4;
    const int64_t blocks = nblocks(tx, ty, n_images);
    if (blocks >= INT32_MAX) return IPP_E_ARG;
    hipLaunchKernelGGL(k_lanczos_h, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, src, dst, coefs, descs,
                       tx, ty, flags);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_lanczos_v(const uint8_t* src, uint8_t* dst, const int32_t* coefs, const ipp_resample_desc* descs,
                             int32_t n_images, int32_t max_out, int32_t max_lines, int32_t flags, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !dst || !coefs || !descs || n_images < 0 || max_out <= 0 || max_lines <= 0) return IPP_E_ARG;
    const int tx = (max_lines + 63) / 64, ty = (max_out + 3) / 4;
    const int64_t blocks = nblocks(tx, ty, n_images);
    if (blocks >= INT32_MAX) return IPP_E_ARG;
    hipLaunchKernelGGL(k_lanczos_v, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, src, dst, coefs, descs,
                       tx, ty, flags);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_paste_blend(const uint8_t* bg, const uint8_t* ov, uint8_t* dst, const ipp_paste_desc* descs,
                               int32_t n_images, int32_t bg_w, int32_t bg_h, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!bg || !ov || !dst || !descs || n_images < 0 || bg_w <= 0 || bg_h <= 0) return IPP_E_ARG;
    const int tx = (3 * bg_w + 16 * 64 - 1) / (16 * 64), ty = (bg_h + 3) / 4;
    const int64_t blocks = nblocks(tx, ty, n_images);
    if (blocks >= INT32_MAX) return IPP_E_ARG;
    hipLaunchKernelGGL(k_paste_blend, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, bg, ov, dst, descs,
                       tx, ty);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
