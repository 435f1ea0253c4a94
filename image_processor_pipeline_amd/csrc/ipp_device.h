// ipp_device.h — device helpers shared by the gfx950 kernels.
//
// Pixels travel packed little-endian in one dword: byte 0 = channel 0 at the
// lowest address (R for Pillow-order images, B for cv2-order images), byte 3 =
// alpha.  All arithmetic is integer and reproduces the library code the
// reference calls bit-for-bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ipp.h"

#define IPP_CHECK_LAUNCH()                                  \
    do {                                                    \
        if (hipGetLastError() != hipSuccess) return IPP_E_LAUNCH; \
    } while (0)

// A dword load from a byte address with no alignment promise.  gfx950 runs the
// HSA queues in unaligned-access mode, so global_load_dword needs no 4-byte
// alignment; the caller guarantees the 4 bytes are inside the allocation.
typedef uint32_t __attribute__((aligned(1), may_alias)) ipp_u32_unaligned;

__device__ __forceinline__ uint32_t ld_u32_unaligned(const uint8_t* p) {
    return *reinterpret_cast<const ipp_u32_unaligned*>(p);
}

// RGB (3 bytes at p) → packed RGBA with alpha 255 (Pillow convert('RGBA'),
// rotations.py:55).  `wide_ok` says a 4-byte read at p stays inside the image.
__device__ __forceinline__ uint32_t load_rgb_opaque(const uint8_t* p, bool wide_ok) {
    if (wide_ok) return ld_u32_unaligned(p) | 0xFF000000u;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | 0xFF000000u;
}

// 4×4 transpose of dwords across a quad of lanes: lane i of the quad ends
// with element i of each of the four lanes (element j from lane j).
__device__ __forceinline__ void quad_transpose4(uint32_t (&a)[4], int lane) {
    const bool o1 = lane & 1;
    const uint32_t r0 = __shfl_xor(o1 ? a[0] : a[1], 1), r2 = __shfl_xor(o1 ? a[2] : a[3], 1);
    if (o1) {
        a[0] = r0;
        a[2] = r2;
    } else {
        a[1] = r0;
        a[3] = r2;
    }
    const bool o2 = lane & 2;
    const uint32_t q0 = __shfl_xor(o2 ? a[0] : a[2], 2), q1 = __shfl_xor(o2 ? a[1] : a[3], 2);
    if (o2) {
        a[0] = q0;
        a[1] = q1;
    } else {
        a[2] = q0;
        a[3] = q1;
    }
}

// MULDIV255 / DIV255 of libImaging (Convert.c, Paste.c):
//   DIV255(v) = ((v + 128) + ((v + 128) >> 8)) >> 8
__device__ __forceinline__ uint32_t div255(uint32_t v) {
    v += 128u;
    return (v + (v >> 8)) >> 8;
}

// Convert.c rgbA2rgba: c' = MULDIV255(c, a) for the three colour bytes.
__device__ __forceinline__ uint32_t premultiply(uint32_t px) {
    uint32_t a = px >> 24;
    if (a == 255u) return px;
    if (a == 0u) return 0u;
    uint32_t c0 = div255((px & 0xFFu) * a);
    uint32_t c1 = div255(((px >> 8) & 0xFFu) * a);
    uint32_t c2 = div255(((px >> 16) & 0xFFu) * a);
    return c0 | (c1 << 8) | (c2 << 16) | (a << 24);
}

// Convert.c rgba2rgbA: alpha 0 or 255 → unchanged, else min(255, 255*c / a)
// (integer division).  The float quotient is corrected by ±1 so the result is
// the exact floor whatever the division's rounding.
__device__ __forceinline__ uint32_t unpremultiply(uint32_t px) {
    uint32_t a = px >> 24;
    if (a == 255u || a == 0u) return px;
    float ra = __builtin_amdgcn_rcpf((float)a);
    uint32_t out = a << 24;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        uint32_t n = 255u * ((px >> (8 * c)) & 0xFFu);
        uint32_t q = (uint32_t)((float)n * ra);
        if ((q + 1u) * a <= n) ++q;
        if (q * a > n) --q;
        out |= (q > 255u ? 255u : q) << (8 * c);
    }
    return out;
}

// unpremultiply with the per-α division by a magic multiplier: M[a] =
// floor(2^31 / a) + 1 gives floor(255·c / a) = (510·c · M[a]) >> 32 exactly
// for every a in 1..255 and c in 0..255 (checked exhaustively by
// tests/test_host_plan.py::test_unpremultiply_magic_table_is_exact).  M[0] is
// unused (α 0 returns the pixel, as above).
__host__ __device__ constexpr uint32_t unpremul_magic(uint32_t a) { return a ? (uint32_t)((1ull << 31) / a + 1ull) : 0u; }
__device__ __forceinline__ uint32_t unpremultiply_magic(uint32_t px, const uint32_t* __restrict__ M) {
    const uint32_t a = px >> 24;
    const uint32_t m = M[a];
    uint32_t out = a << 24;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const uint32_t q = __umulhi(510u * ((px >> (8 * c)) & 0xFFu), m);
        out |= (q > 255u ? 255u : q) << (8 * c);
    }
    return a == 0u ? px : out;
}

// Resample.c clip8: clamp(ss >> 22, 0, 255) with an arithmetic shift.
//
// The empty asm is an optimisation barrier: ROCm 7.2's gfx950 backend fuses
// "clamp(a >> 22) | clamp(b >> 22) << 8" into v_ashr_pk_u8_i32 and then ORs
// further bytes into bits 16-31 of that register as if the instruction had
// zeroed them; on MI355X the upper half keeps its previous contents, which
// corrupted bytes 2/3 of packed results (found by tests/test_gpu_parity.py,
// diagnosed in DESIGN.md §Toolchain notes).
__device__ __forceinline__ uint32_t clip8(int32_t ss) {
    int32_t v = ss >> 22;
    asm volatile("" : "+v"(v));
    return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// Four clip8 results packed into one dword (byte k = clip8(sk)): two
// v_ashr_pk_u8_i32 (each gives two saturated bytes and leaves bits 16-31 of
// its register as they were — here undefined, and discarded) and one v_perm
// taking the low halves; 3 VALU instead of about 11.  In the pipe's H and V
// epilogues: H launch 8.77 -> 8.64 ms (round 5, alternating runs on one box,
// profiles/r05/ab_packed_clip_r05ao.txt).
//
// The compiler's hazard recognizer does not look inside inline asm, so an asm
// operand written by an MFMA gets none of the wait states a VALU read of an
// MFMA result needs: the inputs here must come from ordinary (compiler-seen)
// instructions — planes3 below, or the shift of clip8x4_mfma.
__device__ __forceinline__ uint32_t clip8x4(int32_t s0, int32_t s1, int32_t s2, int32_t s3) {
    uint32_t lo, hi;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 22" : "=v"(lo) : "v"(s0), "v"(s1));
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 22" : "=v"(hi) : "v"(s2), "v"(s3));
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// clip8x4 of four MFMA results: the >> 22 in plain code (hazard-checked),
// then the packed saturation with shift 0.
__device__ __forceinline__ uint32_t clip8x4_mfma(int32_t s0, int32_t s1, int32_t s2, int32_t s3) {
    const int32_t v0 = s0 >> 22, v1 = s1 >> 22, v2 = s2 >> 22, v3 = s3 >> 22;
    uint32_t lo, hi;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 0" : "=v"(lo) : "v"(v0), "v"(v1));
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 0" : "=v"(hi) : "v"(v2), "v"(v3));
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// clip8x4(s) ^ 0x80808080 for s already lowered by 128 << 22 (folded into the
// MFMA bias): clamp(v - 128, -128, 127) as a byte is clamp(v, 0, 255) ^ 0x80,
// and v_ashr_pk_i8_i32 saturates to exactly that range.  (Inputs: as clip8x4.)
__device__ __forceinline__ uint32_t clip8x4_x80(int32_t s0, int32_t s1, int32_t s2, int32_t s3) {
    uint32_t lo, hi;
    asm("v_ashr_pk_i8_i32 %0, %1, %2, 22" : "=v"(lo) : "v"(s0), "v"(s1));
    asm("v_ashr_pk_i8_i32 %0, %1, %2, 22" : "=v"(hi) : "v"(s2), "v"(s3));
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// a0 + (a1 << 8) + (a2 << 16) (the three tap byte planes' accumulators) as
// ((a2 << 8) + a1 << 8) + a0: two v_lshl_add_u32 (left alone, the compiler
// re-associates it into two shifts and an add3).  Plain code where it reads
// the MFMA results, so they get their wait states (see clip8x4); the empty
// asm only pins the intermediate (a VALU result).
__device__ __forceinline__ int32_t planes3(int32_t a0, int32_t a1, int32_t a2) {
    uint32_t t = ((uint32_t)a2 << 8) + (uint32_t)a1;
    asm("" : "+v"(t));
    return (int32_t)((t << 8) + (uint32_t)a0);
}

// Python slice(start, stop).indices(length) for step 1 (zone masks,
// filtres_liste.py:102-103: mask[t : H-b, l : W-r] = 255).
__device__ __forceinline__ void slice_indices(int start, int stop, int length, int& lo, int& hi) {
    if (start < 0) { start += length; if (start < 0) start = 0; } else if (start > length) start = length;
    if (stop < 0) { stop += length; if (stop < 0) stop = 0; } else if (stop > length) stop = length;
    lo = start;
    hi = stop < start ? start : stop;
}

// Division of block indices by a launch-invariant divisor without the ~30
// instructions of a runtime integer division (a float reciprocal and two
// fix-ups): q = umulhi(n, m) >> sh with m = ceil(2^(31 + l) / d), l =
// ceil(log2 d), exact for every n < 2^31 (the error n·(m·d − 2^(31+l)) /
// (d·2^(31+l)) stays below 1/d).  d = 1 is its own case (m would be 2^32).
struct FastDiv {
    uint32_t d, m, sh;
};

inline FastDiv fast_div(uint32_t d) {
    FastDiv f{d, 0u, 0u};
    if (d > 1) {
        uint32_t l = 0;
        while ((1ull << l) < d) ++l;
        f.m = (uint32_t)(((1ull << (31 + l)) + d - 1) / d);
        f.sh = l - 1;
    }
    return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    return f.d == 1u ? n : __umulhi(n, f.m) >> f.sh;
}

// XCD-aware block remap (cdna_hip_programming.md §5.5 T1): the dispatcher deals
// linear block ids round-robin over the 8 XCDs; remap so that consecutive
// logical tiles (the tiles of one image) share an XCD and its L2.  Bijective
// for any count.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nblocks) {
    uint32_t xcd = b & 7u, slot = b >> 3;
    uint32_t q = nblocks >> 3, r = nblocks & 7u;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

// 16 composite bytes (RGB, 3 per pixel) starting at row byte c0, blended with
// the RGBA overlay row `ov` (pixels [ox0, ox0 + ov_w)) — Paste.c
// paste_mask_RGBA: out = DIV255(bg * (255 - a) + ov * a) per channel.  Fully
// unrolled over register dwords (a dynamically indexed byte array would live
// in scratch memory).
template <typename OvFetch>
__device__ __forceinline__ void blend16(uint32_t w[4], int c0, int nbytes, int ox0, int ov_w, OvFetch fetch) {
    int px = c0 / 3, ch = c0 - 3 * px;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int ox = px - ox0;
        if (j < nbytes && (unsigned)ox < (unsigned)ov_w) {
            const uint32_t o = fetch(ox);
            const uint32_t a = o >> 24;
            const uint32_t bgb = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            const uint32_t v = div255(bgb * (255u - a) + ((o >> (8 * ch)) & 0xFFu) * a);
            w[j >> 2] = (w[j >> 2] & ~(0xFFu << (8 * (j & 3)))) | (v << (8 * (j & 3)));
        }
        if (++ch == 3) { ch = 0; ++px; }
    }
}

// Load / store up to 16 bytes of a row into 4 register dwords (vector path
// when 16-B aligned and complete, byte path otherwise).
__device__ __forceinline__ void load16(const uint8_t* p, int nbytes, bool vec, uint32_t w[4]) {
    if (vec) {
        const uint4 v = *reinterpret_cast<const uint4*>(p);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
        w[0] = w[1] = w[2] = w[3] = 0u;
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (j < nbytes) w[j >> 2] |= (uint32_t)p[j] << (8 * (j & 3));
    }
}

// Store policy for write-once outputs: 0 plain, 1 sc1 (line dropped from the
// XCD L2 after write-back), 2 nt.  (MI355X_MICROARCH.md: plain/nt keep the
// line in L2, sc1 drops it; 16-B sc1 stores run at the plain rate.)
template <int POLICY = 0>
__device__ __forceinline__ void store16(uint8_t* p, int nbytes, bool vec, const uint32_t w[4]) {
    if (vec) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = {w[0], w[1], w[2], w[3]};
        if (POLICY == 1)
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
        else if (POLICY == 2)
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
        else
            *reinterpret_cast<u32x4*>(p) = v;
    } else {
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (j < nbytes) p[j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    }
}
