// ipp_pipe.hip — the fused 5-stage pipe (BASELINE configs 3/4):
//
//   crop_from_border → process_rotations (RGBA, NEAREST, expand, bbox crop)
//   → generate_symmetries (flip) → process_images_with_color_masks (HSV α)
//   → paste_overlay_onto_background (LANCZOS resize + alpha paste)
//
// Stage chain of the reference (files between steps, one library pass per
// op): recadrages.py:46 → rotations.py:55,96,99-101 → symmetry.py:114-119 →
// filtres_liste.py:84-134 → overlays.py:129,138-139.  Here the RGBA cut-out
// (the pipe image "M") is never materialised: the LANCZOS horizontal pass
// computes each M pixel on the fly from the source (gather → HSV α →
// premultiply) into an LDS window and runs the taps over it; the vertical pass
// is fused with unpremultiply, the alpha blend and the background copy, so the
// composite is written once with dwordx4 stores.
//
// HBM traffic per image (algorithmic): source crop 3·Hc·Wc read, T (H-pass
// output, 4·W'·rows) written + read, background 3·HW read, composite 3·HW
// written.  See DESIGN.md §Kernels for the roofline accounting.
#include "ipp_hsv.h"

namespace {

constexpr int HX = 64;          // H-pass outputs per block (one per lane)
constexpr int HR = 8;           // H-pass rows per block (2 per thread)
constexpr int HWIN = 1024;      // LDS window width in pixels
constexpr int VR = 4;           // composite rows per vblend block

__device__ __forceinline__ int32_t mad24(int32_t a, int32_t b, int32_t c) { return __mul24(a, b) + c; }

// Pixel (x, y) of the pipe image M, premultiplied (Convert.c rgbA2rgba): the
// flipped, bbox-cropped, rotated crop with α replaced by the HSV keep mask.
__device__ __forceinline__ uint32_t pipe_pixel(const uint8_t* __restrict__ src, const ipp_gather_desc& g,
                                               const HsvLds& hs, int x, int y) {
    const int fx = (g.flip & 1) ? g.out_w - 1 - x : x;
    const int fy = (g.flip & 2) ? g.out_h - 1 - y : y;
    const int X = g.off_x + fx, Y = g.off_y + fy;
    const int32_t xx = (int32_t)((uint32_t)g.a2 + (uint32_t)Y * (uint32_t)g.a1 + (uint32_t)X * (uint32_t)g.a0);
    const int32_t yy = (int32_t)((uint32_t)g.a5 + (uint32_t)Y * (uint32_t)g.a4 + (uint32_t)X * (uint32_t)g.a3);
    const int xin = xx >> 16, yin = yy >> 16;
    uint32_t px = 0u;
    if ((unsigned)xin < (unsigned)g.in_w && (unsigned)yin < (unsigned)g.in_h) {
        const int sx = g.in_x0 + xin, sy = g.in_y0 + yin;
        const uint8_t* p = src + g.src_off + (int64_t)sy * g.src_pitch;
        if (g.src_cn == 4) {
            px = reinterpret_cast<const uint32_t*>(p)[sx];
        } else {
            const bool wide_ok = (sy < g.src_h - 1) || (sx < g.src_w - 1);
            px = load_rgb_opaque(p + 3 * sx, wide_ok);
        }
    }
    const uint32_t a = hsv_keep_alpha(hs, px, 0, x, y);
    return premultiply((px & 0x00FFFFFFu) | (a << 24));
}

__global__ void __launch_bounds__(256)
k_pipe_hpass(const uint8_t* __restrict__ src, uint8_t* __restrict__ tmp, const int32_t* __restrict__ coefs,
             const ipp_pipe_desc* __restrict__ descs, int tiles_x, int tiles_y, ipp_hsv_params hp) {
    __shared__ HsvLds hs;
    __shared__ uint32_t win[HR][HWIN];
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int per_img = tiles_x * tiles_y;
    const int im = b / per_img;
    const int t = b - im * per_img;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const ipp_gather_desc g = descs[im].g;
    const ipp_resample_desc h = descs[im].h;
    const int xo0 = tx * HX, row0 = ty * HR;
    if (xo0 >= h.out_len || row0 >= h.lines) return;  // block-uniform
    hsv_lds_init(hs, hp, g.out_w, g.out_h);
    const int32_t* bnd = coefs + h.coef_off;
    const int32_t* taps = bnd + 2 * h.out_len;
    const int xo_end = min(xo0 + HX, h.out_len);
    const int lane = threadIdx.x & 63, rsub = threadIdx.x >> 6;  // rsub in [0,4)
    const int nrows = min(HR, h.lines - row0);
    __syncthreads();

    // Sub-chunks of outputs whose input window fits the LDS window.
    for (int s0 = xo0; s0 < xo_end;) {
        int s1 = xo_end;
        while (s1 - s0 > 1 && bnd[2 * (s1 - 1)] + bnd[2 * (s1 - 1) + 1] - bnd[2 * s0] > HWIN)
            s1 = s0 + (s1 - s0 + 1) / 2;
        const int wlo = bnd[2 * s0];
        const int ww = bnd[2 * (s1 - 1)] + bnd[2 * (s1 - 1) + 1] - wlo;
        for (int i = threadIdx.x; i < nrows * ww; i += 256) {
            const int r = i / ww, c = i - r * ww;
            win[r][c] = pipe_pixel(src, g, hs, wlo + c, h.line0 + row0 + r);
        }
        __syncthreads();
        const int xo = s0 + lane;
        if (xo < s1) {
            const int xmin = bnd[2 * xo] - wlo, cnt = bnd[2 * xo + 1];
            const int32_t* kk = taps + (int64_t)xo * h.ksize;
            for (int r = rsub; r < nrows; r += 4) {
                int32_t a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21, a3 = 1 << 21;
                const uint32_t* w = &win[r][xmin];
                for (int k = 0; k < cnt; ++k) {
                    const uint32_t p = w[k];
                    const int32_t c = kk[k];
                    a0 = mad24((int32_t)(p & 0xFF), c, a0);
                    a1 = mad24((int32_t)((p >> 8) & 0xFF), c, a1);
                    a2 = mad24((int32_t)((p >> 16) & 0xFF), c, a2);
                    a3 = mad24((int32_t)(p >> 24), c, a3);
                }
                const uint32_t o = clip8(a0) | (clip8(a1) << 8) | (clip8(a2) << 16) | (clip8(a3) << 24);
                reinterpret_cast<uint32_t*>(tmp + h.dst_off + (int64_t)(row0 + r) * h.dst_pitch)[xo] = o;
            }
        }
        __syncthreads();
        s0 = s1;
    }
}

__global__ void __launch_bounds__(256)
k_pipe_vblend(const uint8_t* __restrict__ tmp, const uint8_t* __restrict__ bg, uint8_t* __restrict__ dst,
              const int32_t* __restrict__ coefs, const ipp_pipe_desc* __restrict__ descs, int tiles_y, int bg_w_max) {
    extern __shared__ __attribute__((aligned(16))) uint32_t orow[];  // [VR][bg_w_max]
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / tiles_y;
    const int ty = b - im * tiles_y;
    const ipp_resample_desc v = descs[im].v;
    const ipp_resample_desc h = descs[im].h;
    const ipp_paste_desc p = descs[im].p;
    const int y0 = ty * VR;
    if (y0 >= p.bg_h) return;
    const int nrows = min(VR, p.bg_h - y0);

    // Phase 1: overlay rows of this band — V pass over T, unpremultiply.
    const int32_t* bnd = coefs + v.coef_off;
    const int32_t* taps = bnd + 2 * v.out_len;
    bool any = false;
    for (int r = 0; r < nrows; ++r) {
        const int oy = y0 + r - p.y;
        if ((unsigned)oy >= (unsigned)p.ov_h) continue;
        any = true;
        const int ymin = bnd[2 * oy], cnt = bnd[2 * oy + 1];
        const int32_t* kk = taps + (int64_t)oy * v.ksize;
        for (int x = threadIdx.x; x < p.ov_w; x += 256) {
            const uint8_t* col = tmp + h.dst_off + (int64_t)ymin * h.dst_pitch + 4 * (int64_t)x;
            int32_t a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21, a3 = 1 << 21;
            for (int k = 0; k < cnt; ++k) {
                const uint32_t q = *reinterpret_cast<const uint32_t*>(col + (int64_t)k * h.dst_pitch);
                const int32_t c = kk[k];
                a0 = mad24((int32_t)(q & 0xFF), c, a0);
                a1 = mad24((int32_t)((q >> 8) & 0xFF), c, a1);
                a2 = mad24((int32_t)((q >> 16) & 0xFF), c, a2);
                a3 = mad24((int32_t)(q >> 24), c, a3);
            }
            orow[r * bg_w_max + x] =
                unpremultiply(clip8(a0) | (clip8(a1) << 8) | (clip8(a2) << 16) | (clip8(a3) << 24));
        }
    }
    if (any) __syncthreads();

    // Phase 2: composite rows = background bytes, blended inside the footprint.
    const int row_bytes = 3 * p.bg_w;
    const int chunks = (row_bytes + 15) >> 4;
    for (int i = threadIdx.x; i < nrows * chunks; i += 256) {
        const int r = i / chunks, c0 = (i - r * chunks) << 4;
        const int y = y0 + r;
        const uint8_t* brow = bg + p.bg_off + (int64_t)y * p.bg_pitch;
        uint8_t* drow = dst + p.dst_off + (int64_t)y * p.dst_pitch;
        const int nbytes = min(16, row_bytes - c0);
        const bool vec = nbytes == 16 &&
                         ((reinterpret_cast<uintptr_t>(brow + c0) | reinterpret_cast<uintptr_t>(drow + c0)) & 15u) == 0;
        uint8_t vb[16];
        if (vec) {
            *reinterpret_cast<uint4*>(vb) = *reinterpret_cast<const uint4*>(brow + c0);
        } else {
            for (int j = 0; j < nbytes; ++j) vb[j] = brow[c0 + j];
        }
        const int oy = y - p.y;
        if ((unsigned)oy < (unsigned)p.ov_h && c0 + nbytes > 3 * p.x && c0 < 3 * (p.x + p.ov_w)) {
            int px = c0 / 3, ch = c0 - 3 * px;
            for (int j = 0; j < nbytes; ++j) {
                const int ox = px - p.x;
                if ((unsigned)ox < (unsigned)p.ov_w) {
                    const uint32_t o = orow[r * bg_w_max + ox];
                    const uint32_t a = o >> 24;
                    vb[j] = (uint8_t)div255((uint32_t)vb[j] * (255u - a) + ((o >> (8 * ch)) & 0xFFu) * a);
                }
                if (++ch == 3) { ch = 0; ++px; }
            }
        }
        if (vec) {
            *reinterpret_cast<uint4*>(drow + c0) = *reinterpret_cast<const uint4*>(vb);
        } else {
            for (int j = 0; j < nbytes; ++j) drow[c0 + j] = vb[j];
        }
    }
}

}  // namespace

extern "C" int ipp_pipe_hpass(const uint8_t* src, uint8_t* tmp, const int32_t* coefs, const ipp_pipe_desc* descs,
                              int32_t n_images, int32_t max_out_w, int32_t max_rows, const ipp_hsv_params* hsv,
                              void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !tmp || !coefs || !descs || !hsv || n_images < 0 || max_out_w <= 0 || max_rows <= 0) return IPP_E_ARG;
    if (hsv->n_ranges < 0 || hsv->n_ranges > IPP_MAX_HSV_RANGES) return IPP_E_ARG;
    const int tx = (max_out_w + HX - 1) / HX, ty = (max_rows + HR - 1) / HR;
    const int64_t blocks = (int64_t)tx * ty * n_images;
    if (blocks >= INT32_MAX) return IPP_E_ARG;
    hipLaunchKernelGGL(k_pipe_hpass, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, src, tmp, coefs,
                       descs, tx, ty, *hsv);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_pipe_vblend(const uint8_t* tmp, const uint8_t* bg, uint8_t* dst, const int32_t* coefs,
                               const ipp_pipe_desc* descs, int32_t n_images, int32_t bg_w, int32_t bg_h,
                               void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!tmp || !bg || !dst || !coefs || !descs || n_images < 0 || bg_w <= 0 || bg_h <= 0) return IPP_E_ARG;
    const size_t shmem = (size_t)VR * bg_w * sizeof(uint32_t);
    if (shmem > 160 * 1024) return IPP_E_ARG;
    const int ty = (bg_h + VR - 1) / VR;
    const int64_t blocks = (int64_t)ty * n_images;
    if (blocks >= INT32_MAX) return IPP_E_ARG;
    hipLaunchKernelGGL(k_pipe_vblend, dim3((uint32_t)blocks), dim3(256), shmem, (hipStream_t)stream, tmp, bg, dst,
                       coefs, descs, ty, bg_w);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
