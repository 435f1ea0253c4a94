// ipp_sampler.h — branch-free NEAREST gather of the rotated / flipped /
// bbox-cropped source (Pillow Geometry.c affine_fixed: 16.16 int32
// accumulation, arithmetic >> 16, out-of-range → transparent), shared by the
// standalone gather (ipp_gather.hip) and the fused pipe (ipp_pipe.hip).
#pragma once
#include "ipp_device.h"

// Source sampling for M pixel (x, y): flip + bbox offset folded into the 16.16
// map so xx = B2 + y*B1 + x*B0 (int32 wrap-around arithmetic, as Pillow).
struct Sampler {
    const uint8_t* base;  // source pixel (in_x0, in_y0)
    uint32_t pitch, lim;  // lim: last byte offset from base where a dword load fits
    int32_t b0, b1, b2, b3, b4, b5;
    int32_t in_w, in_h;
};

#ifndef IPP_SAMPLER_PREPARED
#define IPP_SAMPLER_PREPARED 1  // (0: A/B builds recompute the sampler per block)
#endif
__device__ __forceinline__ Sampler make_sampler(const uint8_t* src, const ipp_gather_desc& g) {
    Sampler s;
    if (IPP_SAMPLER_PREPARED && g.prepared) {  // ipp_gather_prepare did the arithmetic below once per image (block-uniform)
        s.base = src + g.base_off;
        s.pitch = (uint32_t)g.src_pitch;
        s.lim = g.lim;
        s.b0 = g.b[0];
        s.b1 = g.b[1];
        s.b2 = g.b[2];
        s.b3 = g.b[3];
        s.b4 = g.b[4];
        s.b5 = g.b[5];
        s.in_w = g.in_w;
        s.in_h = g.in_h;
        return s;
    }
    s.base = src + g.src_off + (int64_t)g.in_y0 * g.src_pitch + (int64_t)g.in_x0 * g.src_cn;
    s.pitch = (uint32_t)g.src_pitch;
    const int64_t avail = (int64_t)(g.src_h - g.in_y0) * g.src_pitch - (int64_t)g.in_x0 * g.src_cn;
    s.lim = (uint32_t)(avail - 4);
    const int sgx = (g.flip & 1) ? -1 : 1, sgy = (g.flip & 2) ? -1 : 1;
    const uint32_t sx0 = (uint32_t)(g.off_x + ((g.flip & 1) ? g.out_w - 1 : 0));
    const uint32_t sy0 = (uint32_t)(g.off_y + ((g.flip & 2) ? g.out_h - 1 : 0));
    s.b0 = (int32_t)((uint32_t)sgx * (uint32_t)g.a0);
    s.b1 = (int32_t)((uint32_t)sgy * (uint32_t)g.a1);
    s.b2 = (int32_t)((uint32_t)g.a2 + sy0 * (uint32_t)g.a1 + sx0 * (uint32_t)g.a0);
    s.b3 = (int32_t)((uint32_t)sgx * (uint32_t)g.a3);
    s.b4 = (int32_t)((uint32_t)sgy * (uint32_t)g.a4);
    s.b5 = (int32_t)((uint32_t)g.a5 + sy0 * (uint32_t)g.a4 + sx0 * (uint32_t)g.a3);
    s.in_w = g.in_w;
    s.in_h = g.in_h;
    return s;
}

// Four horizontally adjacent M pixels: issue the four (branch-free) loads.
// Invalid lanes read the window origin; `valid` masks them afterwards.
template <int CN>
struct Gather4 {
    uint32_t raw[4];
    uint32_t sh[4];   // right shift (0 or 8) for a clamped tail load
    uint32_t valid;   // bit k: pixel k inside the source
};

template <int CN>
__device__ __forceinline__ void gather4_issue(const Sampler& S, uint32_t xx, uint32_t yy, Gather4<CN>& G) {
    G.valid = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int xin = (int32_t)xx >> 16, yin = (int32_t)yy >> 16;
        const bool ok = ((uint32_t)xin < (uint32_t)S.in_w) & ((uint32_t)yin < (uint32_t)S.in_h);
        const uint32_t off_any = (uint32_t)__umul24(yin, S.pitch) + (uint32_t)__umul24(xin, CN);
        uint32_t off = ok ? off_any : 0u;
        if (CN == 3) {
            const uint32_t offc = min(off, S.lim);
            G.sh[k] = (off - offc) << 3;
            off = offc;
        }
        G.raw[k] = *reinterpret_cast<const ipp_u32_unaligned*>(S.base + off);
        G.valid |= (ok ? 1u : 0u) << k;
        xx += (uint32_t)S.b0;
        yy += (uint32_t)S.b3;
    }
}

template <int CN>
__device__ __forceinline__ uint32_t gather4_pixel(const Gather4<CN>& G, int k) {
    // 3-channel sources are opaque (RGB → RGBA adds α = 255); 4-channel ones keep α
    const uint32_t p = CN == 3 ? ((G.raw[k] >> G.sh[k]) | 0xFF000000u) : G.raw[k];
    return ((G.valid >> k) & 1u) ? p : 0u;
}

// Four M pixels at the corners of an 8×8 square: (0,0), (0,8), (8,0), (8,8)
// (x, y offsets).  With lanes laid out as 8 rows × 8 columns, each load
// instruction then reads one dense 8×8 block: a compact source footprint
// (fewer cache lines per wave instruction than 16 rows × 4 spread columns).
template <int CN>
__device__ __forceinline__ void gather4_issue_sq8(const Sampler& S, uint32_t xx, uint32_t yy, Gather4<CN>& G) {
    G.valid = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t xk = xx + (k & 1) * 8u * (uint32_t)S.b0 + (k >> 1) * 8u * (uint32_t)S.b1;
        const uint32_t yk = yy + (k & 1) * 8u * (uint32_t)S.b3 + (k >> 1) * 8u * (uint32_t)S.b4;
        const int xin = (int32_t)xk >> 16, yin = (int32_t)yk >> 16;
        const bool ok = ((uint32_t)xin < (uint32_t)S.in_w) & ((uint32_t)yin < (uint32_t)S.in_h);
        const uint32_t off_any = (uint32_t)__umul24(yin, S.pitch) + (uint32_t)__umul24(xin, CN);
        uint32_t off = ok ? off_any : 0u;
        if (CN == 3) {
            const uint32_t offc = min(off, S.lim);
            G.sh[k] = (off - offc) << 3;
            off = offc;
        }
        G.raw[k] = *reinterpret_cast<const ipp_u32_unaligned*>(S.base + off);
        G.valid |= (ok ? 1u : 0u) << k;
    }
}
