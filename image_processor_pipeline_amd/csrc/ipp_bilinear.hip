// ipp_bilinear.hip — opt-in BILINEAR rotation (Pillow rotate(angle,
// expand=True, resample=BILINEAR)).
//
// north_star names "rotations.py (bilinear)"; the reference's own call
// (transforms/rotations.py:96) passes no resample and runs NEAREST, which
// ipp_rotate_flip_nearest reproduces.  This kernel is the opt-in mode
// (process_rotations(..., resample="bilinear")), bit-exact with Pillow 12.2.0:
//   * PIL/Image.py:2978-2983 — an RGBA image is transformed as RGBa
//     (premultiplied, Convert.c rgbA2rgba: c' = DIV255(c·α)) and converted
//     back (rgba2rgbA: α ∈ {0, 255} unchanged, else min(255, 255c / α));
//   * Geometry.c affine_transform — source point of output (x, y) is
//     a0(x + .5) + a1(y + .5) + a2 (and a3.., a5) in double, evaluated as
//     (a0·x + a1·y) + a2 without fused multiply-adds (x86-64 baseline build);
//   * Geometry.c bilinear_filter32RGB — reject x ∉ [0, w) or y ∉ [0, h) (fill
//     0), shift by -0.5, floor, clamp the x neighbours and the first row, fall
//     back to row y when y + 1 is outside, v = a + (b - a)·d in double twice,
//     truncate to uint8.
// SURVEY Appendix A9.  The 0/90/180/270 fast paths are exact transposes and
// go through ipp_rotate_flip_nearest.
#include "ipp_device.h"

namespace {

constexpr int BW = 64, BH = 4;

// Built with -ffp-contract=off (Makefile): the pragma below covers this
// file's expressions, the flag also covers the HIP header helpers inlined
// here — a fused multiply-add changes the last bit that the truncation to
// uint8 then exposes.
#pragma clang fp contract(off)

__device__ __forceinline__ uint32_t fetch_rgba_premul(const uint8_t* p, int cn) {
    if (cn == 3) return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | 0xFF000000u;
    const uint32_t px = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    return premultiply(px);
}

__device__ __forceinline__ double lerp_c(double a, double b, double d) {
    // BILINEAR(v, a, b, d): v = a + (b - a) * d, separately rounded
    return a + (b - a) * d;
}

__global__ void __launch_bounds__(256) k_rotate_bilinear(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                         const ipp_affine_desc* __restrict__ descs, int tx, int ty) {
    const int per = tx * ty;
    const int im = blockIdx.x / per;
    const int t = blockIdx.x - im * per;
    const int bx = t % tx, by = t / tx;
    const ipp_affine_desc d = descs[im];
    const int x = bx * BW + (threadIdx.x % BW), y = by * BH + (threadIdx.x / BW);
    if (x >= d.out_w || y >= d.out_h) return;
    const int cx = (d.flip & 1) ? d.out_w - 1 - x : x;   // canvas pixel this output shows
    const int cy = (d.flip & 2) ? d.out_h - 1 - y : y;
    const double X = (double)cx + 0.5, Y = (double)cy + 0.5;
    const double xin = (d.m[0] * X + d.m[1] * Y) + d.m[2];
    const double yin = (d.m[3] * X + d.m[4] * Y) + d.m[5];
    uint32_t out = 0u;
    if (xin >= 0.0 && xin < (double)d.in_w && yin >= 0.0 && yin < (double)d.in_h) {
        const double xs = xin - 0.5, ys = yin - 0.5;
        const double xf = floor(xs), yf = floor(ys);
        const int xi = (int)xf, yi = (int)yf;
        const double dx = xs - xf, dy = ys - yf;
        const int x0 = min(max(xi, 0), d.in_w - 1), x1 = min(max(xi + 1, 0), d.in_w - 1);
        const int y0 = min(max(yi, 0), d.in_h - 1);
        const bool y1ok = yi + 1 >= 0 && yi + 1 < d.in_h;
        const uint8_t* base = src + d.src_off + (int64_t)d.in_y0 * d.src_pitch + (int64_t)d.in_x0 * d.src_cn;
        const uint8_t* r0 = base + (int64_t)y0 * d.src_pitch;
        const uint32_t p00 = fetch_rgba_premul(r0 + x0 * d.src_cn, d.src_cn);
        const uint32_t p01 = fetch_rgba_premul(r0 + x1 * d.src_cn, d.src_cn);
        uint32_t p10 = 0u, p11 = 0u;
        if (y1ok) {
            const uint8_t* r1 = base + (int64_t)(yi + 1) * d.src_pitch;
            p10 = fetch_rgba_premul(r1 + x0 * d.src_cn, d.src_cn);
            p11 = fetch_rgba_premul(r1 + x1 * d.src_cn, d.src_cn);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const double a = (double)((p00 >> (8 * c)) & 0xFFu), b = (double)((p01 >> (8 * c)) & 0xFFu);
            const double v1 = lerp_c(a, b, dx);
            double v2 = v1;
            if (y1ok) v2 = lerp_c((double)((p10 >> (8 * c)) & 0xFFu), (double)((p11 >> (8 * c)) & 0xFFu), dx);
            const double v = lerp_c(v1, v2, dy);
            out |= ((uint32_t)(int)v & 0xFFu) << (8 * c);
        }
        out = unpremultiply(out);
    }
    *reinterpret_cast<uint32_t*>(dst + d.dst_off + (int64_t)y * d.dst_pitch + 4 * (int64_t)x) = out;
}

}  // namespace

extern "C" int ipp_rotate_bilinear(const uint8_t* src, uint8_t* dst, const ipp_affine_desc* descs, int32_t n_images,
                                   int32_t max_out_w, int32_t max_out_h, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !dst || !descs || n_images < 0 || max_out_w <= 0 || max_out_h <= 0) return IPP_E_ARG;
    const int tx = (max_out_w + BW - 1) / BW, ty = (max_out_h + BH - 1) / BH;
    const int64_t blocks = (int64_t)tx * ty * n_images;
    if (blocks >= INT32_MAX) return IPP_E_ARG;
    hipLaunchKernelGGL(k_rotate_bilinear, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, src, dst, descs,
                       tx, ty);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
