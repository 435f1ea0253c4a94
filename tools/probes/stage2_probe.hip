// stage2_probe.hip — phase 1 of the pipe's H pass (M pixels → HSV → planar LDS
// ring) with the source staged through LDS in sheared row spans, against the
// shipped per-pixel texture-path gathers.
//   direct : every M pixel is one buffer_load_dword gather (2×2 lane quads,
//            4 pixels per lane and step, one step ahead) — the shipped form;
//   staged : per sub-chunk of SC M columns × 16 rows, the source rows of the
//            sub-chunk's footprint parallelogram are loaded with coalesced
//            12-byte loads (4 pixels per lane), widened to one dword per pixel
//            and written to an LDS stage whose rows are sheared along the
//            parallelogram edge that gives the smaller stage (row j holds
//            source columns [XL(j), XL(j) + SR), XL linear in j); each M pixel
//            then reads its source pixel with one aligned ds_read_b32
//            (out-of-window source pixels are zeros in the stage).
// Both forms run the same table HSV test and write the same ring bytes: each
// block folds an order-free hash of every ring dword it writes, and the two
// forms must agree block for block.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I../../image_processor_pipeline_amd/csrc
//        -o stage2_probe stage2_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "ipp_hsv.h"

namespace {

constexpr int HR = 16, RING = 512, WSTRIDE = 544;
constexpr int NR = 4;

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
    const uint32_t t = (raw | 0xFF000000u) ^ 0x80808080u;
    if (!HSV) return t;
    const uint32_t ex = hsv_tab_excl<NR, false>(T, raw);
    return ex ? 0x80808080u : t;
}

__device__ __forceinline__ uint32_t hsh(uint32_t x, uint32_t r, uint32_t c, uint32_t v) {
    uint32_t h = v * 0x9E3779B1u ^ (x * 0x85EBCA77u + r * 0xC2B2AE3Du + c * 0x27D4EB2Fu);
    return h ^ (h >> 15);
}

// 4 channel dwords of 4 consecutive columns x..x+3 of row r → ring (+ hash).
__device__ __forceinline__ uint32_t ring_put(uint8_t (&win)[4][HR][WSTRIDE], const uint32_t (&ch)[4], int r, int x) {
    const int pos = x & (RING - 1);
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        *reinterpret_cast<uint32_t*>(&win[c][r][pos]) = ch[c];
        acc += hsh((uint32_t)x, (uint32_t)r, (uint32_t)c, ch[c]);
    }
    return acc;
}

struct Lds {
    uint8_t win[4][HR][WSTRIDE];
    HsvTables<NR> T;
    uint32_t red[4];
};

__device__ __forceinline__ void block_out(uint32_t acc, uint32_t* red, uint32_t* out) {
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
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
        uint32_t px[4], ch[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) px[k] = win_px<HSV>(L.T, A[k] & 0xFFFFFFu);
        pair_regroup(px, lane & 1);
        transpose4(px[0], px[1], px[2], px[3], ch);
        acc += ring_put(L.win, ch, r, x);
#pragma unroll
        for (int k = 0; k < 4; ++k) A[k] = Bq[k];
    }
    block_out(acc, L.red, out);
}

// ---------------------------------------------------------------------------
// Staged form.
template <int STG>
struct LdsS {
    uint8_t win[4][HR][WSTRIDE];
    HsvTables<NR> T;
    uint32_t red[4];
    __attribute__((aligned(16))) uint32_t stage[STG / 4];
};

// Per-block shear: the stage rows run along the parallelogram edge e (0: the
// M-column direction (b0, b3), 1: the M-row direction (b1, b4)); K = dx/dy of
// that edge in 16.16.  Chosen per block for the smaller stage of a typical
// sub-chunk.
struct Shear {
    int32_t K;
};

template <int SC, int STG, bool HSV, bool CHK>
__global__ void __launch_bounds__(256) k_staged(const uint8_t* __restrict__ src, int64_t item_bytes, Geo g, int bands,
                                                ipp_hsv_params hp, uint32_t* __restrict__ out,
                                                uint32_t* __restrict__ err) {
    __shared__ LdsS<STG> L;
    const int item = blockIdx.x / bands, band = blockIdx.x - item * bands;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    hsv_tables_init<NR>(L.T, hp);
    const uint8_t* base = src + item * item_bytes;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)item_bytes, 0x00020000);
    const int Y = band * HR;
    // ---- shear choice (block-uniform; float geometry with slack)
    const float k16 = 1.0f / 65536.0f;
    const float ex_x = (float)g.b0 * k16 * (SC - 1), ex_y = (float)g.b3 * k16 * (SC - 1);   // M-column edge
    const float ey_x = (float)g.b1 * k16 * (HR - 1), ey_y = (float)g.b4 * k16 * (HR - 1);   // M-row edge
    float Kf[2], Wf[2];
    {
        // shear along the column edge: width = x'-extent of the row edge
        const bool ok0 = fabsf(ex_y) > 1e-3f;
        Kf[0] = ok0 ? ex_x / ex_y : 0.0f;
        Wf[0] = ok0 && fabsf(Kf[0]) < 64.0f ? fabsf(ey_x - Kf[0] * ey_y) + 2.0f * fabsf(Kf[0]) + 6.0f : 1e9f;
        const bool ok1 = fabsf(ey_y) > 1e-3f;
        Kf[1] = ok1 ? ey_x / ey_y : 0.0f;
        Wf[1] = ok1 && fabsf(Kf[1]) < 64.0f ? fabsf(ex_x - Kf[1] * ex_y) + 2.0f * fabsf(Kf[1]) + 6.0f : 1e9f;
    }
    const int e = Wf[1] < Wf[0] ? 1 : 0;
    const int32_t K = __builtin_amdgcn_readfirstlane((int32_t)lrintf(Kf[e] * 65536.0f));
    const int SR = __builtin_amdgcn_readfirstlane(((int)ceilf(Wf[e]) + 3) & ~3);  // stage row stride (px)
    const int NV = SR >> 2;                                                    // 4-px vectors per row
    const int lgv = 32 - __builtin_clz(max(NV, 1) - 1);                       // log2 of NV rounded up
    const int NVp = 1 << lgv;
    const int RPI = 64 / NVp;                                                  // rows per wave instruction
    __syncthreads();

    // corner offsets of a sub-chunk (16.16, relative to its origin), once per block
    const int32_t cxs[4] = {0, (SC - 1) * g.b0, (HR - 1) * g.b1, (SC - 1) * g.b0 + (HR - 1) * g.b1};
    const int32_t cys[4] = {0, (SC - 1) * g.b3, (HR - 1) * g.b4, (SC - 1) * g.b3 + (HR - 1) * g.b4};
    int32_t dymin = 0, dymax = 0, dxp = 0x7FFFFFFF;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        dymin = min(dymin, cys[q]);
        dymax = max(dymax, cys[q]);
        dxp = min(dxp, cxs[q] - (int32_t)(((int64_t)K * cys[q]) >> 16));
    }
    dymin = __builtin_amdgcn_readfirstlane(dymin);
    dymax = __builtin_amdgcn_readfirstlane(dymax);
    dxp = __builtin_amdgcn_readfirstlane(dxp);
    const int32_t slack = (int32_t)((abs(K) >> 16) + 3) * 65536;
    struct SG { int J0, R; int32_t BX; };
    auto geo = [&](int X) {
        SG q;
        const int32_t ox = g.c + X * g.b0 + Y * g.b1, oy = g.f + X * g.b3 + Y * g.b4;
        q.J0 = ((oy + dymin) >> 16) - 1;
        q.R = ((oy + dymax) >> 16) - q.J0 + 2;
        // x'(sample) = xx - K yy / 2^16; XL(j) = (BX + K j) >> 16 covers x' - K (J0 + j) with slack
        const int64_t xpmin = (int64_t)ox - (((int64_t)K * oy) >> 16) + dxp;
        q.BX = (int32_t)(xpmin + (((int64_t)K * q.J0 * 65536) >> 16) - slack);
        return q;
    };
    typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
    constexpr int NS = 4;  // staging load slots per thread
    u32x3 ld[NS];
    auto issue = [&](const SG& q) {
#pragma unroll
        for (int p = 0; p < NS; ++p) {
            const int j = wave * RPI + p * 4 * RPI + (lane >> lgv), v = lane & (NVp - 1);
            const int sy = q.J0 + j;
            const int x0 = ((q.BX + K * j) >> 16) + 4 * v;
            const bool ok = j < q.R && v < NV && (uint32_t)sy < (uint32_t)g.in_h;
            const uint32_t off = ok ? (uint32_t)(sy * g.pitch + 3 * x0) : 0x80000000u;
            ld[p] = u32x3{0u, 0u, 0u};
            if (p * 4 * RPI < q.R) ld[p] = __builtin_bit_cast(u32x3, __builtin_amdgcn_raw_buffer_load_b96(rs, off, 0, 0));
        }
    };
    auto put = [&](const SG& q) {
#pragma unroll
        for (int p = 0; p < NS; ++p) {
            const int j = wave * RPI + p * 4 * RPI + (lane >> lgv), v = lane & (NVp - 1);
            if (j < q.R && v < NV) {
                const u32x3 d = ld[p];
                const int x0 = ((q.BX + K * j) >> 16) + 4 * v;
                uint32_t px[4];
                // px1 = d.x[3], d.y[0], d.y[1]; px2 = d.y[2], d.y[3], d.z[0]; px3 = d.z[1..3]
                px[0] = d.x & 0xFFFFFFu;
                px[1] = perm(d.y, d.x, 0x0c050403u);
                px[2] = perm(d.z, d.y, 0x0c040302u);
                px[3] = d.z >> 8;
                if (x0 < 0 || x0 + 4 > g.in_w) {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if ((uint32_t)(x0 + k) >= (uint32_t)g.in_w) px[k] = 0u;
                }
                *reinterpret_cast<uint4*>(&L.stage[j * SR + 4 * v]) = make_uint4(px[0], px[1], px[2], px[3]);
            }
        }
    };

    const int cg = lane & 7, rr0 = lane >> 3;  // fetch map: 8 rows x 8 column groups per instruction
    uint32_t acc = 0;
    const int XE = 64 * ((g.mw + 63) / 64);
    SG cur = geo(0);
    if (cur.R * SR * 4 > STG || cur.R > NS * 4 * RPI) {
        if (tid == 0) atomicAdd(err + 1, 1u);
    }
    issue(cur);
    for (int X = 0; X < XE; X += SC) {
        if (X > 0) __syncthreads();  // the previous sub-chunk's fetches are done with the stage
        put(cur);
        SG nxt = cur;
        if (X + SC < XE) {
            nxt = geo(X + SC);
            if (CHK && tid == 0 && (nxt.R * SR * 4 > STG || nxt.R > NS * 4 * RPI)) atomicAdd(err + 1, 1u);
            issue(nxt);
        }
        __syncthreads();
        const int J0 = cur.J0, R = cur.R;
        const int32_t BX = cur.BX;
        // ---- fetch: wave covers 8 rows x 32 columns per instruction group
        for (int blk = wave; blk < 2 * (SC / 32); blk += 4) {
            const int h = blk & 1, cb = blk >> 1;
            if (X + 32 * cb >= XE) break;
            const int r = rr0 + 8 * h, x0 = X + 32 * cb + 4 * cg, y = Y + r;
            int32_t xx = g.c + x0 * g.b0 + y * g.b1, yy = g.f + x0 * g.b3 + y * g.b4 - J0 * 65536;
            uint32_t px[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int sx = xx >> 16, j = yy >> 16;
                const int a = __mul24(j, SR) + sx - ((BX + K * j) >> 16);
                if (CHK && (a < 0 || a >= R * SR)) atomicAdd(err, 1u);
                uint32_t raw = L.stage[a];
                raw = (x0 + k < g.mw) ? raw : 0u;
                px[k] = win_px<HSV>(L.T, raw);
                xx += g.b0;
                yy += g.b3;
            }
            uint32_t ch[4];
            transpose4(px[0], px[1], px[2], px[3], ch);
            acc += ring_put(L.win, ch, r, x0);
        }
        cur = nxt;
    }
    block_out(acc, L.red, out);
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
    uint32_t *out, *err;
    if (hipMalloc(&src, item_bytes * items) != hipSuccess) return 1;
    {
        std::vector<uint8_t> h(item_bytes * 4);
        uint32_t st = 12345u;
        for (auto& b : h) { st = st * 1664525u + 1013904223u; b = (uint8_t)(st >> 24); }
        for (int i = 0; i < items; i += 4) hipMemcpy(src + item_bytes * i, h.data(), h.size(), hipMemcpyHostToDevice);
    }
    const int maxb = items * 80;
    if (hipMalloc(&out, (size_t)maxb * 4) != hipSuccess) return 1;
    if (hipMalloc(&err, 16) != hipSuccess) return 1;
    ipp_hsv_params hp{};
    hp.n_ranges = 4;
    const int rr[4][6] = {{0, 0, 0, 180, 255, 150}, {15, 60, 200, 35, 255, 255}, {15, 76, 140, 30, 153, 204},
                          {15, 153, 153, 30, 191, 230}};
    for (int k = 0; k < 4; ++k)
        for (int c = 0; c < 3; ++c) {
            hp.r[k].lo[c] = rr[k][c];
            hp.r[k].hi[c] = rr[k][3 + c];
        }
    printf("ms per 1024 items of 896^2 (phase 1 only: M pixels + HSV + ring), whole canvas\n");
    printf("angle canvas | direct  st64/12K st128/20K | noHSV: direct st64 | mismatch 64 128 | err64 oflow64 err128 oflow128\n");
    for (double deg : {0.0, 3.6, 10.0, 20.0, 30.0, 45.0, 60.0, 80.0, 90.0, 100.0, 135.0, 200.0, 300.0, 357.0}) {
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
        const size_t n = (size_t)items * bands;
        std::vector<uint32_t> h0(n), h1(n), h2(n);
        uint32_t he[4][4] = {};
        float t[5];
        t[0] = timeit([&] { hipLaunchKernelGGL(k_direct<true>, grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out); });
        hipMemcpy(h0.data(), out, n * 4, hipMemcpyDeviceToHost);
        hipMemset(err, 0, 16);
        hipLaunchKernelGGL((k_staged<64, 12288, true, true>), grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out, err);
        hipMemcpy(he[0], err, 16, hipMemcpyDeviceToHost);
        t[1] = timeit([&] { hipLaunchKernelGGL((k_staged<64, 12288, true, false>), grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out, err); });
        hipMemcpy(h1.data(), out, n * 4, hipMemcpyDeviceToHost);
        hipMemset(err, 0, 16);
        hipLaunchKernelGGL((k_staged<128, 20480, true, true>), grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out, err);
        hipMemcpy(he[1], err, 16, hipMemcpyDeviceToHost);
        t[2] = timeit([&] { hipLaunchKernelGGL((k_staged<128, 20480, true, false>), grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out, err); });
        hipMemcpy(h2.data(), out, n * 4, hipMemcpyDeviceToHost);
        t[3] = timeit([&] { hipLaunchKernelGGL(k_direct<false>, grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out); });
        t[4] = timeit([&] { hipLaunchKernelGGL((k_staged<64, 12288, false, false>), grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out, err); });
        size_t bad1 = 0, bad2 = 0;
        for (size_t i = 0; i < n; ++i) {
            bad1 += h0[i] != h1[i];
            bad2 += h0[i] != h2[i];
        }
        printf("%5.1f %5d | %7.3f %7.3f %7.3f | %7.3f %7.3f | %zu %zu | %u %u %u %u\n", deg, mw, t[0], t[1], t[2], t[3],
               t[4], bad1, bad2, he[0][0], he[0][1], he[1][0], he[1][1]);
        fflush(stdout);
    }
    hipFree(src);
    hipFree(out);
    hipFree(err);
    return 0;
}
