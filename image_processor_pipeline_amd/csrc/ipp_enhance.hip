// ipp_enhance.hip — tranfo.enhance_image (transforms/tranfo.py:37-53) on RGB:
//
//   img = Brightness(img).enhance(f1)   Image.blend(black, img, f1)
//   img = Contrast(img).enhance(f2)     Image.blend(gray(mean L), img, f2)
//   img = Color(img).enhance(f3)        Image.blend(L(img) as RGB, img, f3)
//   [GaussianBlur(r)]                   BoxBlur.c: 3 box passes per axis
//   [r/g/b point(LUT)]                  256-entry table per channel
//
// Bit-exact with Pillow 12.2.0 (libImaging Blend.c, Convert.c rgb2l,
// ImageStat mean, BoxBlur.c):
//   * blend: t = (float)in1 + α·(float)(in2 - in1), α = float32(factor), two
//     float32 roundings (no FMA: this file is built with -ffp-contract=off);
//     α ∈ [0, 1] truncates, otherwise clips to [0, 255] then truncates;
//     α = 0 / 1 copy an input;
//   * L = (19595 R + 38470 G + 7471 B + 0x8000) >> 16;
//   * contrast mean = int(ΣL / N + 0.5) in double (ImageStat sums exactly);
//   * box pass: out[x] = (acc·ww + (in[x-r-1] + in[x+r+1])·fw + 2^23) >> 24
//     in uint32 arithmetic, acc = Σ in[clamp(i)], i ∈ [x-r, x+r]; ww, fw, r
//     come from the host (float32 box radius of _gaussian_blur_radius).
//
// Launches: ipp_enhance_lsum (Σ L of the brightened image per image, 64-bit
// atomics), ipp_enhance_color (brightness → contrast → color [→ LUT]) and,
// with blur, 2 × passes ipp_box_pass launches (rows, then columns; the last
// one applies the LUT).
#include "ipp_device.h"

namespace {

#pragma clang fp contract(off)

__device__ __forceinline__ uint32_t blend_c(uint32_t in1, uint32_t in2, float a) {
    if (a == 0.0f) return in1;
    if (a == 1.0f) return in2;
    const float t = (float)(int)in1 + a * (float)((int)in2 - (int)in1);
    if (a >= 0.0f && a <= 1.0f) return (uint32_t)(int)t & 0xFFu;
    if (t <= 0.0f) return 0u;
    if (t >= 255.0f) return 255u;
    return (uint32_t)(int)t;
}

__device__ __forceinline__ uint32_t rgb2l(uint32_t r, uint32_t g, uint32_t b) {
    return (r * 19595u + g * 38470u + b * 7471u + 0x8000u) >> 16;
}

__device__ __forceinline__ void load_rgb(const uint8_t* p, uint32_t& r, uint32_t& g, uint32_t& b) {
    r = p[0];
    g = p[1];
    b = p[2];
}

__device__ __forceinline__ void brighten(uint32_t& r, uint32_t& g, uint32_t& b, float f1) {
    r = blend_c(0u, r, f1);
    g = blend_c(0u, g, f1);
    b = blend_c(0u, b, f1);
}

constexpr int TILE = 1024;   // pixels per block (4 per thread)

__global__ void __launch_bounds__(256) k_enh_lsum(const uint8_t* __restrict__ src,
                                                  const ipp_enhance_desc* __restrict__ descs, int tiles,
                                                  unsigned long long* __restrict__ sums) {
    const int im = blockIdx.x / tiles, t = blockIdx.x - im * tiles;
    const ipp_enhance_desc d = descs[im];
    const int64_t npx = (int64_t)d.w * d.h;
    uint32_t acc = 0;
    for (int k = 0; k < 4; ++k) {
        const int64_t i = (int64_t)t * TILE + k * 256 + threadIdx.x;
        if (i < npx) {
            const int y = (int)(i / d.w), x = (int)(i - (int64_t)y * d.w);
            uint32_t r, g, b;
            load_rgb(src + d.src_off + (int64_t)y * d.src_pitch + 3 * x, r, g, b);
            brighten(r, g, b, d.f_brightness);
            acc += rgb2l(r, g, b);
        }
    }
    // wave reduction, then one 64-bit atomic per wave
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(&sums[im], (unsigned long long)acc);
}

template <bool LUT>
__global__ void __launch_bounds__(256) k_enh_color(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   const ipp_enhance_desc* __restrict__ descs, int tiles,
                                                   const unsigned long long* __restrict__ sums,
                                                   const uint8_t* __restrict__ luts) {
    const int im = blockIdx.x / tiles, t = blockIdx.x - im * tiles;
    const ipp_enhance_desc d = descs[im];
    const int64_t npx = (int64_t)d.w * d.h;
    // ImageStat: mean = sum / count in double; Contrast: int(mean + 0.5)
    const uint32_t mean = (uint32_t)(int)((double)sums[im] / (double)npx + 0.5);
    const bool lut = LUT && (d.flags & IPP_ENH_LUT) && !(d.flags & IPP_ENH_BLUR);
    const uint8_t* lt = luts + d.lut_off;
    for (int k = 0; k < 4; ++k) {
        const int64_t i = (int64_t)t * TILE + k * 256 + threadIdx.x;
        if (i >= npx) continue;
        const int y = (int)(i / d.w), x = (int)(i - (int64_t)y * d.w);
        uint32_t r, g, b;
        load_rgb(src + d.src_off + (int64_t)y * d.src_pitch + 3 * x, r, g, b);
        brighten(r, g, b, d.f_brightness);
        r = blend_c(mean, r, d.f_contrast);
        g = blend_c(mean, g, d.f_contrast);
        b = blend_c(mean, b, d.f_contrast);
        const uint32_t l = rgb2l(r, g, b);
        r = blend_c(l, r, d.f_color);
        g = blend_c(l, g, d.f_color);
        b = blend_c(l, b, d.f_color);
        if (lut) {
            r = lt[r];
            g = lt[256 + g];
            b = lt[512 + b];
        }
        uint8_t* q = dst + d.dst_off + (int64_t)y * d.dst_pitch + 3 * x;
        q[0] = (uint8_t)r;
        q[1] = (uint8_t)g;
        q[2] = (uint8_t)b;
    }
}

// One box pass along x (AXIS 0) or y (AXIS 1) over tightly packed RGB planes
// (pitch 3·w).  Last pass of a blur may apply the LUT.
template <int AXIS, bool LUT>
__global__ void __launch_bounds__(256) k_box_pass(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  const ipp_enhance_desc* __restrict__ descs, int tiles,
                                                  const int64_t* __restrict__ offs, const uint8_t* __restrict__ luts,
                                                  int final_dst) {
    const int im = blockIdx.x / tiles, t = blockIdx.x - im * tiles;
    const ipp_enhance_desc d = descs[im];
    const int64_t npx = (int64_t)d.w * d.h;
    const int64_t i = (int64_t)t * 256 + threadIdx.x;
    if (i >= npx) return;
    const int y = (int)(i / d.w), x = (int)(i - (int64_t)y * d.w);
    const uint8_t* base = src + offs[im];
    const int pitch = 3 * d.w;
    const int r = d.box_r, n = AXIS == 0 ? d.w : d.h, pos = AXIS == 0 ? x : y;
    auto at = [&](int j, int c) -> uint32_t {
        j = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
        return AXIS == 0 ? base[(int64_t)y * pitch + 3 * j + c] : base[(int64_t)j * pitch + 3 * x + c];
    };
    uint32_t o[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        uint32_t acc = 0;
        for (int j = pos - r; j <= pos + r; ++j) acc += at(j, c);
        const uint32_t bulk = acc * d.box_ww + (at(pos - r - 1, c) + at(pos + r + 1, c)) * d.box_fw;
        o[c] = ((bulk + (1u << 23)) >> 24) & 0xFFu;
    }
    if (LUT && (d.flags & IPP_ENH_LUT)) {
        const uint8_t* lt = luts + d.lut_off;
        o[0] = lt[o[0]];
        o[1] = lt[256 + o[1]];
        o[2] = lt[512 + o[2]];
    }
    uint8_t* q = final_dst ? dst + d.dst_off + (int64_t)y * d.dst_pitch + 3 * x : dst + offs[im] + (int64_t)y * pitch + 3 * x;
    q[0] = (uint8_t)o[0];
    q[1] = (uint8_t)o[1];
    q[2] = (uint8_t)o[2];
}

}  // namespace

extern "C" int ipp_enhance_lsum(const uint8_t* src, const ipp_enhance_desc* descs, int32_t n_images,
                                int64_t max_pixels, uint64_t* sums, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !descs || !sums || n_images < 0 || max_pixels <= 0) return IPP_E_ARG;
    const int64_t tiles = (max_pixels + TILE - 1) / TILE;
    if (tiles * n_images >= INT32_MAX) return IPP_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(sums, 0, sizeof(uint64_t) * n_images, s) != hipSuccess) return IPP_E_LAUNCH;
    hipLaunchKernelGGL(k_enh_lsum, dim3((uint32_t)(tiles * n_images)), dim3(256), 0, s, src, descs, (int)tiles,
                       reinterpret_cast<unsigned long long*>(sums));
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_enhance_color(const uint8_t* src, uint8_t* dst, const ipp_enhance_desc* descs, int32_t n_images,
                                 int64_t max_pixels, const uint64_t* sums, const uint8_t* luts, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !dst || !descs || !sums || n_images < 0 || max_pixels <= 0) return IPP_E_ARG;
    const int64_t tiles = (max_pixels + TILE - 1) / TILE;
    if (tiles * n_images >= INT32_MAX) return IPP_E_ARG;
    const auto* sm = reinterpret_cast<const unsigned long long*>(sums);
    if (luts)
        hipLaunchKernelGGL(k_enh_color<true>, dim3((uint32_t)(tiles * n_images)), dim3(256), 0, (hipStream_t)stream,
                           src, dst, descs, (int)tiles, sm, luts);
    else
        hipLaunchKernelGGL(k_enh_color<false>, dim3((uint32_t)(tiles * n_images)), dim3(256), 0, (hipStream_t)stream,
                           src, dst, descs, (int)tiles, sm, luts);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_box_pass(const uint8_t* src, uint8_t* dst, const ipp_enhance_desc* descs, int32_t n_images,
                            int64_t max_pixels, const int64_t* offs, int32_t axis, const uint8_t* luts,
                            int32_t final_dst, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !dst || !descs || !offs || n_images < 0 || max_pixels <= 0 || (axis != 0 && axis != 1)) return IPP_E_ARG;
    const int64_t tiles = (max_pixels + 255) / 256;
    if (tiles * n_images >= INT32_MAX) return IPP_E_ARG;
    const dim3 g((uint32_t)(tiles * n_images));
    hipStream_t s = (hipStream_t)stream;
    if (axis == 0) {
        if (luts) hipLaunchKernelGGL((k_box_pass<0, true>), g, dim3(256), 0, s, src, dst, descs, (int)tiles, offs, luts, final_dst);
        else hipLaunchKernelGGL((k_box_pass<0, false>), g, dim3(256), 0, s, src, dst, descs, (int)tiles, offs, luts, final_dst);
    } else {
        if (luts) hipLaunchKernelGGL((k_box_pass<1, true>), g, dim3(256), 0, s, src, dst, descs, (int)tiles, offs, luts, final_dst);
        else hipLaunchKernelGGL((k_box_pass<1, false>), g, dim3(256), 0, s, src, dst, descs, (int)tiles, offs, luts, final_dst);
    }
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
