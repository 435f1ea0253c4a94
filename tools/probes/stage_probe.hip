// stage_probe.hip — phase 1 of the pipe's H pass (gather → HSV → planar LDS
// ring) in two forms, to decide whether LDS staging of the source beats the
// per-pixel texture-path gathers:
//   direct : every M pixel is one buffer_load_dword gather (the shipped form,
//            2×2 lane quads, 4 pixels per lane and step, one step ahead);
//   staged : per block step (64 M columns × 16 rows) the source rows of the
//            step's footprint parallelogram are copied into LDS by 16-byte
//            LDS-DMA pieces (buffer_load_dwordx4 … lds), D steps ahead, in a
//            sheared row layout (row j starts at source column XL(j), a linear
//            function of j); every M pixel then reads its source pixel from
//            LDS (one unaligned ds_read_b32).
// Both run the same table HSV test and write the same ring bytes; each thread
// XOR-folds what it writes, and the two forms must agree thread for thread.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I../../image_processor_pipeline_amd/csrc
//        -o stage_probe stage_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "ipp_hsv.h"

namespace {

constexpr int HR = 16, RING = 512, WSTRIDE = 544;
constexpr int NR = 4;
constexpr int STAGE_BYTES = 8192;  // one buffer: ≤ 512 pieces of 16 B

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

struct Geo {
    int32_t b0, b3, b1, b4;  // 16.16 per M column (b0, b3) and per M row (b1, b4)
    int32_t c, f;            // 16.16 source position of M pixel (0, 0)
    int32_t in_w, in_h, pitch;
    int32_t mw, mh;
};

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ void transpose4(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t ch[4]) {
    const uint32_t lo01 = perm(p1, p0, 0x05010400u), hi01 = perm(p1, p0, 0x07030602u);
    const uint32_t lo23 = perm(p3, p2, 0x05010400u), hi23 = perm(p3, p2, 0x07030602u);
    ch[0] = perm(lo23, lo01, 0x05040100u);
    ch[1] = perm(lo23, lo01, 0x07060302u);
    ch[2] = perm(hi23, hi01, 0x05040100u);
    ch[3] = perm(hi23, hi01, 0x07060302u);
}
__device__ __forceinline__ void pair_regroup(uint32_t (&a)[4], bool o1) {
    const uint32_t s0 = o1 ? a[0] : a[2], s1 = o1 ? a[1] : a[3];
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s0, 0xB1, 0xF, 0xF, false);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s1, 0xB1, 0xF, 0xF, false);
    const uint32_t b0 = o1 ? r0 : a[0], b1 = o1 ? a[2] : r0, b2 = o1 ? r1 : a[1], b3 = o1 ? a[3] : r1;
    a[0] = b0; a[1] = b1; a[2] = b2; a[3] = b3;
}

template <bool HSV>
__device__ __forceinline__ uint32_t win_px(const HsvTables<NR>& T, uint32_t raw) {
    if (!HSV) return (raw | 0xFF000000u) ^ 0x80808080u;
    const uint32_t ex = hsv_tab_excl<NR, false>(T, raw);
    const uint32_t t = (raw | 0xFF000000u) ^ 0x80808080u;
    return ex ? 0x80808080u : t;
}

struct Lds {
    uint8_t win[4][HR][WSTRIDE];
    HsvTables<NR> T;
};
template <int NB>
struct LdsS {
    uint8_t win[4][HR][WSTRIDE];
    HsvTables<NR> T;
    __attribute__((aligned(16))) uint8_t stage[NB][STAGE_BYTES];
    uint32_t zero[4];
};

// 4 pixels of a lane → ring (same as the shipped kernel's phase 1 tail).
template <bool HSV>
__device__ __forceinline__ uint32_t ring_write(const HsvTables<NR>& T, uint8_t (&win)[4][HR][WSTRIDE], uint32_t (&p)[4],
                                               int lane, int r, int x) {
    uint32_t px[4], ch[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) px[k] = win_px<HSV>(T, p[k] & 0xFFFFFFu);
    pair_regroup(px, lane & 1);
    transpose4(px[0], px[1], px[2], px[3], ch);
    const int pos = x & (RING - 1);
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        *reinterpret_cast<uint32_t*>(&win[c][r][pos]) = ch[c];
        acc ^= ch[c] * (2 * c + 1);
    }
    return acc;
}

// ---------------------------------------------------------------------------
template <bool HSV>
__global__ void __launch_bounds__(256) k_direct(const uint8_t* __restrict__ src, int64_t item_bytes, Geo g, int bands,
                                                ipp_hsv_params hp, uint32_t* __restrict__ out) {
    __shared__ Lds L;
    const int item = blockIdx.x / bands, band = blockIdx.x - item * bands;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    hsv_tables_init<NR>(L.T, hp);
    __syncthreads();
    const uint8_t* base = src + item * item_bytes;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)item_bytes, 0x00020000);
    const int r = 2 * (lane >> 3) + ((lane >> 1) & 1);
    const int y = band * HR + r;
    uint32_t acc = 0;
    const int nsteps = (g.mw + 63) / 64;
    auto issue = [&](int st, uint32_t (&p)[4]) {
        const int x0 = 64 * st + 16 * wave + 8 * ((lane >> 2) & 1) + (lane & 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int x = x0 + 2 * k;
            const int xx = g.b0 * x + g.b1 * y + g.c, yy = g.b3 * x + g.b4 * y + g.f;
            const int xi = xx >> 16, yi = yy >> 16;
            const bool ok = (uint32_t)xi < (uint32_t)g.in_w && (uint32_t)yi < (uint32_t)g.in_h && x < g.mw;
            const uint32_t off = ok ? (uint32_t)__mul24(yi, g.pitch) + (uint32_t)__mul24(xi, 3) : 0xFFFFFFFFu;
            p[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
        }
    };
    uint32_t A[4], Bq[4];
    issue(0, A);
    for (int st = 0; st < nsteps; ++st) {
        if (st + 1 < nsteps) issue(st + 1, Bq);
        const int x = 64 * st + 16 * wave + 8 * ((lane >> 2) & 1) + 4 * (lane & 1);
        acc ^= ring_write<HSV>(L.T, L.win, A, lane, r, x) + st;
#pragma unroll
        for (int k = 0; k < 4; ++k) A[k] = Bq[k];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// ---------------------------------------------------------------------------
// Staged form.  Per block: the shear K (16.16 source columns per source row)
// along the parallelogram edge with the larger source-row extent, the piece
// count P per staged row (row bytes RB = 16 P), the row bound RMAX; per step:
// the first staged row jlo and XL(jlo) in 16.16 (BASE).  XL(jlo + t) =
// (BASE + K t) >> 16 for staging and reading alike.
struct StageGeo {
    int32_t K, P, RB, RMAX, magic;  // magic: i / P = (i * magic) >> 16 for i < 1024
    int32_t ymin_rel, xpmin;        // corner offsets: min source y (16.16), min sheared x (16.16)
    bool ok;                        // RMAX * P <= 512
};

__device__ __forceinline__ StageGeo stage_geo(const Geo& g) {
    StageGeo s;
    const float k16 = 1.0f / 65536.0f;
    const float vdy = 63.0f * g.b3, udy = 15.0f * g.b4;
    const bool useV = fabsf(vdy) >= fabsf(udy);
    const float bx = useV ? (float)g.b0 : (float)g.b1, by = useV ? (float)g.b3 : (float)g.b4;
    s.K = (int32_t)rintf(65536.0f * bx / by);
    // corners relative to the step origin (16.16)
    const int32_t cx[4] = {0, 63 * g.b0, 15 * g.b1, 63 * g.b0 + 15 * g.b1};
    const int32_t cy[4] = {0, 63 * g.b3, 15 * g.b4, 63 * g.b3 + 15 * g.b4};
    int32_t ymin = 0, ymax = 0;
    float xpmin = 1e30f, xpmax = -1e30f;
    for (int c = 0; c < 4; ++c) {
        ymin = min(ymin, cy[c]);
        ymax = max(ymax, cy[c]);
        const float xp = (float)cx[c] - (float)s.K * k16 * (float)cy[c];
        xpmin = fminf(xpmin, xp);
        xpmax = fmaxf(xpmax, xp);
    }
    s.ymin_rel = ymin;
    s.xpmin = (int32_t)floorf(xpmin) - 65536;  // 1 px slack on the left
    const float w = (xpmax - xpmin) * k16 + fabsf((float)s.K * k16) + 4.0f;  // px, slack both sides
    s.P = ((int)ceilf(3.0f * w) + 1 + 15) / 16;
    s.RB = 16 * s.P;
    s.RMAX = (int)((ymax - ymin) >> 16) + 3;
    s.magic = (65536 + s.P - 1) / s.P;
    s.ok = s.RMAX * s.P <= STAGE_BYTES / 16;
    return s;
}

template <int NB, int D, bool HSV>
__global__ void __launch_bounds__(256) k_staged(const uint8_t* __restrict__ src, int64_t item_bytes, Geo g, int bands,
                                                ipp_hsv_params hp, uint32_t* __restrict__ out) {
    static_assert(NB >= D + 1, "stage ring");
    __shared__ LdsS<NB> L;
    const int item = blockIdx.x / bands, band = blockIdx.x - item * bands;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    hsv_tables_init<NR>(L.T, hp);
    if (threadIdx.x < 4) L.zero[threadIdx.x] = 0u;
    const uint8_t* base = src + item * item_bytes;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)item_bytes, 0x00020000);
    const StageGeo sg = stage_geo(g);
    const int r = 2 * (lane >> 3) + ((lane >> 1) & 1);
    const int Y = band * HR, y = Y + r;
    uint32_t acc = 0;
    const int nsteps = (g.mw + 63) / 64;
    // step origin (16.16) and its staged-row geometry
    auto step_jlo = [&](int st, int& jlo, int32_t& basex) {
        const int32_t ox = g.c + 64 * st * g.b0 + Y * g.b1, oy = g.f + 64 * st * g.b3 + Y * g.b4;
        jlo = ((oy + sg.ymin_rel) >> 16) - 1;
        // XL(jlo) = floor(ox + xpmin + K (jlo - oy) + min(0, K))
        const int64_t dy = (int64_t)jlo * 65536 - oy;
        basex = ox + sg.xpmin + (int32_t)(((int64_t)sg.K * dy) >> 16) + min(0, sg.K);
    };
    // piece i of step st → this lane's DMA
    auto issue = [&](int st) {
        int jlo;
        int32_t bx;
        step_jlo(st, jlo, bx);
        uint8_t* stg = L.stage[st % NB];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int i = 64 * (wave + 4 * q) + lane;
            const int t = (i * sg.magic) >> 16, p = i - t * sg.P;
            const int j = jlo + t;
            const int xl = (bx + sg.K * t) >> 16;
            uint32_t off = (uint32_t)(j * g.pitch + 3 * xl + 16 * p);
            if ((uint32_t)j >= (uint32_t)g.in_h || t >= sg.RMAX) off = 0xFFFFFFFFu;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void*)(stg + 1024 * (wave + 4 * q)), 16, off, 0, 0, 0);
        }
    };
    __syncthreads();
    if (!sg.ok) {
        out[blockIdx.x * 256 + threadIdx.x] = 0xDEADBEEFu;
        return;
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (d < nsteps) issue(d);
    for (int st = 0; st < nsteps; ++st) {
        // wait for this wave's pieces of step st (2 instructions per later step issued)
        if (st + D - 1 < nsteps && D >= 2) {
            if (D == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // LDS writes/reads of the previous step done, then a bare barrier (a
        // __syncthreads() fence would wait for the DMA issued ahead: vmcnt(0))
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (st + D < nsteps) issue(st + D);
        int jlo;
        int32_t bx;
        step_jlo(st, jlo, bx);
        const uint8_t* stg = L.stage[st % NB];
        const int x0 = 64 * st + 16 * wave + 8 * ((lane >> 2) & 1) + (lane & 1);
        uint32_t p[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int x = x0 + 2 * k;
            const int xx = g.b0 * x + g.b1 * y + g.c, yy = g.b3 * x + g.b4 * y + g.f;
            const int xi = xx >> 16, yi = yy >> 16;
            const bool ok = (uint32_t)xi < (uint32_t)g.in_w && (uint32_t)yi < (uint32_t)g.in_h && x < g.mw;
            const int t = yi - jlo;
            const int xl = (bx + sg.K * t) >> 16;
            const int a = t * sg.RB + 3 * (xi - xl);
            const uint8_t* ap = ok ? stg + a : reinterpret_cast<const uint8_t*>(L.zero);
            p[k] = *reinterpret_cast<const ipp_u32_unaligned*>(ap);
        }
        const int x = 64 * st + 16 * wave + 8 * ((lane >> 2) & 1) + 4 * (lane & 1);
        acc ^= ring_write<HSV>(L.T, L.win, p, lane, r, x) + st;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <typename F>
float timeit(F launch) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch();
    hipEventRecord(e0);
    const int reps = 5;
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

}  // namespace

int main() {
    const int S = 896, items = 1024;
    const int64_t item_bytes = (int64_t)S * S * 3;
    uint8_t* src;
    uint32_t* out;
    if (hipMalloc(&src, item_bytes * items) != hipSuccess) return 1;
    {
        std::vector<uint8_t> h(item_bytes * 4);
        uint32_t st = 12345u;
        for (auto& b : h) { st = st * 1664525u + 1013904223u; b = (uint8_t)(st >> 24); }
        for (int i = 0; i < items; i += 4) hipMemcpy(src + item_bytes * i, h.data(), h.size(), hipMemcpyHostToDevice);
    }
    const int maxb = items * 80;
    if (hipMalloc(&out, (size_t)maxb * 256 * 4) != hipSuccess) return 1;
    // the reference's four ranges (filtres_liste.py:186-190, cvRound-ed)
    ipp_hsv_params hp{};
    hp.n_ranges = 4;
    const int rr[4][6] = {{0, 0, 0, 180, 255, 150}, {15, 60, 200, 35, 255, 255}, {15, 76, 140, 30, 153, 204},
                          {15, 153, 153, 30, 191, 230}};
    for (int k = 0; k < 4; ++k)
        for (int c = 0; c < 3; ++c) {
            hp.r[k].lo[c] = rr[k][c];
            hp.r[k].hi[c] = rr[k][3 + c];
        }
    printf("ms per 1024 items of 896^2 (phase 1 only: gather/stage + HSV + ring)\n");
    printf("angle canvas | direct  staged(3,2) staged(2,1) | noHSV: direct staged(3,2) | mismatch(3,2) (2,1)\n");
    for (double deg : {0.0, 5.0, 10.0, 13.4, 20.0, 30.0, 45.0, 60.0, 80.0, 90.0, 100.0, 135.0, 200.0, 300.0}) {
        const double a = deg * M_PI / 180.0, c = cos(a), s = sin(a);
        const int mw = (int)ceil(S * (fabs(c) + fabs(s))), mh = mw;
        Geo g;
        g.b0 = (int32_t)lrint(c * 65536), g.b1 = (int32_t)lrint(s * 65536);
        g.b3 = (int32_t)lrint(-s * 65536), g.b4 = (int32_t)lrint(c * 65536);
        const double cx = mw / 2.0, cy = mh / 2.0;
        g.c = (int32_t)lrint((S / 2.0 - c * cx - s * cy) * 65536);
        g.f = (int32_t)lrint((S / 2.0 + s * cx - c * cy) * 65536);
        g.in_w = S, g.in_h = S, g.mw = mw, g.mh = mh, g.pitch = 3 * S;
        const int bands = (mh + 15) / 16;
        const dim3 grid(items * bands);
        const size_t n = (size_t)items * bands * 256;
        std::vector<uint32_t> h0(n), h1(n), h2(n);
        float t[5];
        t[0] = timeit([&] { hipLaunchKernelGGL(k_direct<true>, grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out); });
        hipMemcpy(h0.data(), out, n * 4, hipMemcpyDeviceToHost);
        t[1] = timeit([&] { hipLaunchKernelGGL((k_staged<3, 2, true>), grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out); });
        hipMemcpy(h1.data(), out, n * 4, hipMemcpyDeviceToHost);
        t[2] = timeit([&] { hipLaunchKernelGGL((k_staged<2, 1, true>), grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out); });
        hipMemcpy(h2.data(), out, n * 4, hipMemcpyDeviceToHost);
        t[3] = timeit([&] { hipLaunchKernelGGL(k_direct<false>, grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out); });
        t[4] = timeit([&] { hipLaunchKernelGGL((k_staged<3, 2, false>), grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out); });
        size_t bad1 = 0, bad2 = 0, dead = 0;
        for (size_t i = 0; i < n; ++i) {
            bad1 += h0[i] != h1[i];
            bad2 += h0[i] != h2[i];
            dead += h1[i] == 0xDEADBEEFu;
        }
        printf("%5.1f %5d | %7.3f %7.3f %7.3f | %7.3f %7.3f | %zu %zu (overflow %zu)\n", deg, mw, t[0], t[1], t[2], t[3],
               t[4], bad1, bad2, dead);
        fflush(stdout);
    }
    hipFree(src);
    hipFree(out);
    return 0;
}
