// pair_probe.hip — does loading two M pixels per lane access pay?  The H
// pass's gathers are bound by the CU's L1 (TCP) accesses, about one per lane
// per dword gather.  Here every wave step covers 16 M rows × 16 columns (4 px
// per lane) of a rotated 3-byte-per-pixel source, and only the load form
// varies:
//   A  2×2 lane quads, 4 buffer_load_dword gathers per lane (the shipped form)
//   B  2 runs of 2 M pixels along the M axis closest to the source rows
//      (rows when |b0| >= |b3|, else columns): one unaligned
//      buffer_load_dwordx2 at the run's leftmost source pixel, plus a masked
//      dword for the second pixel when the run changes source row
//   D  one buffer_load_dwordx4 per lane and step at the first pixel (wrong
//      bytes whenever the 4 pixels leave that row: a lower bound only)
// Every pixel value is folded with its M position into an order-free XOR
// hash per block (A and B must agree).  HSV=1 adds the table HSV test.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -I../../include
//        -I../../image_processor_pipeline_amd/csrc -o pair_probe pair_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "ipp_hsv.h"

namespace {

constexpr int NR = 4;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Geo {
    int32_t b0, b3, b1, b4, c, f;
    int32_t in_w, in_h, pitch, mw, mh;
};

__device__ __forceinline__ uint32_t hash(uint32_t x, uint32_t y, uint32_t v) {
    uint32_t h = (v & 0xFFFFFFu) * 0x9E3779B1u ^ (x * 0x85EBCA77u + y * 0xC2B2AE3Du);
    return h ^ (h >> 15);
}

template <bool HSV>
__device__ __forceinline__ uint32_t fold(const HsvTables<NR>& T, uint32_t x, uint32_t y, uint32_t raw) {
    uint32_t v = raw & 0xFFFFFFu;
    if (HSV) v = hsv_tab_excl<NR, false>(T, v) ? 0x80808080u : v;
    return hash(x, y, v);
}

template <int V, bool HSV>
__global__ void __launch_bounds__(256) k_probe(const uint8_t* __restrict__ src, int64_t item_bytes, Geo g, int bands,
                                               ipp_hsv_params hp, uint32_t* __restrict__ out) {
    __shared__ HsvTables<NR> T;
    __shared__ uint32_t red[4];
    hsv_tables_init<NR>(T, hp);
    __syncthreads();
    const int item = blockIdx.x / bands, band = blockIdx.x - item * bands;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint8_t* base = src + item * item_bytes;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)item_bytes, 0x00020000);
    const bool rowdom = abs(g.b0) >= abs(g.b3);
    uint32_t acc = 0;
    const int nsteps = (g.mw + 63) / 64;
    for (int st = 0; st < nsteps; ++st) {
        const int X = 64 * st + 16 * wave, Y = band * 16;
        if (V == 0) {
            const int r = 2 * (lane >> 3) + ((lane >> 1) & 1);
            const int y = Y + r;
            const int x0 = X + 8 * ((lane >> 2) & 1) + (lane & 1);
            uint32_t p[4];
            int xs[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int x = x0 + 2 * k;
                xs[k] = x;
                const int xx = g.b0 * x + g.b1 * y + g.c, yy = g.b3 * x + g.b4 * y + g.f;
                const int xi = xx >> 16, yi = yy >> 16;
                const bool ok = (uint32_t)xi < (uint32_t)g.in_w && (uint32_t)yi < (uint32_t)g.in_h && x < g.mw;
                const uint32_t off = ok ? (uint32_t)__mul24(yi, g.pitch) + (uint32_t)__mul24(xi, 3) : 0xFFFFFFFFu;
                p[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) acc ^= fold<HSV>(T, xs[k], y, p[k]);
        } else {
            // lane → 4 M pixels along the dominant axis: rows: (X + 4 (lane >> 4) + k, Y + (lane & 15));
            // columns: (X + (lane & 15), Y + 4 (lane >> 4) + k)
            const int a = lane & 15, bq = lane >> 4;
            const int px0 = rowdom ? X + 4 * bq : X + a, py0 = rowdom ? Y + a : Y + 4 * bq;
            const int dx = rowdom ? 1 : 0, dy = rowdom ? 0 : 1;
            int xi[4], yi[4];
            bool ok[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int x = px0 + k * dx, y = py0 + k * dy;
                const int xx = g.b0 * x + g.b1 * y + g.c, yy = g.b3 * x + g.b4 * y + g.f;
                xi[k] = xx >> 16;
                yi[k] = yy >> 16;
                ok[k] = (uint32_t)xi[k] < (uint32_t)g.in_w && (uint32_t)yi[k] < (uint32_t)g.in_h && x < g.mw;
            }
            if (V == 2) {
                const uint32_t off = ok[0] ? (uint32_t)__mul24(yi[0], g.pitch) + (uint32_t)__mul24(xi[0], 3) : 0xFFFFFFFFu;
                const u32x4 w = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off & ~3u, 0, 0));
#pragma unroll
                for (int k = 0; k < 4; ++k) acc ^= fold<HSV>(T, px0 + k * dx, py0 + k * dy, w[k]);
            } else {
                uint32_t v[4];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int k0 = 2 * q, k1 = k0 + 1;
                    const bool same = yi[k0] == yi[k1] && ok[k0] && ok[k1];
                    const int xm = min(xi[k0], xi[k1]);
                    // the pair's first access: both pixels when they share a source row
                    const int xa = same ? xm : xi[k0];
                    const uint32_t offa = ok[k0] || same ? (uint32_t)__mul24(yi[k0], g.pitch) + (uint32_t)__mul24(xa, 3)
                                                         : 0xFFFFFFFFu;
                    const u32x2 w = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, offa, 0, 0));
                    uint32_t s = 0;
                    if (!same && ok[k1]) {
                        s = __builtin_amdgcn_raw_buffer_load_b32(
                            rs, (uint32_t)__mul24(yi[k1], g.pitch) + (uint32_t)__mul24(xi[k1], 3), 0, 0);
                    }
                    const uint32_t hi = __builtin_amdgcn_alignbyte(w.y, w.x, 3);
                    v[k0] = !ok[k0] ? 0u : (same && xi[k0] != xm ? hi : w.x);
                    v[k1] = !ok[k1] ? 0u : (same ? (xi[k1] != xm ? hi : w.x) : s);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) acc ^= fold<HSV>(T, px0 + k * dx, py0 + k * dy, ok[k] ? v[k] : 0u);
            }
        }
    }
    // order-free block hash
    for (int o = 32; o > 0; o >>= 1) acc ^= __shfl_xor(acc, o);
    if (lane == 0) red[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = red[0] ^ red[1] ^ red[2] ^ red[3];
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

int main(int argc, char** argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;  // rocprof: one variant (0..5), one angle
    const int S = 896, items = 1024;
    const int64_t item_bytes = (int64_t)S * S * 3;
    uint8_t* src;
    uint32_t* out;
    if (hipMalloc(&src, item_bytes * items + 64) != hipSuccess) return 1;
    {
        std::vector<uint8_t> h(item_bytes * 4);
        uint32_t st = 12345u;
        for (auto& b : h) { st = st * 1664525u + 1013904223u; b = (uint8_t)(st >> 24); }
        for (int i = 0; i < items; i += 4) hipMemcpy(src + item_bytes * i, h.data(), h.size(), hipMemcpyHostToDevice);
    }
    if (hipMalloc(&out, (size_t)items * 80 * 4) != hipSuccess) return 1;
    ipp_hsv_params hp{};
    hp.n_ranges = 4;
    const int rr[4][6] = {{0, 0, 0, 180, 255, 150}, {15, 60, 200, 35, 255, 255}, {15, 76, 140, 30, 153, 204},
                          {15, 153, 153, 30, 191, 230}};
    for (int k = 0; k < 4; ++k)
        for (int c = 0; c < 3; ++c) {
            hp.r[k].lo[c] = rr[k][c];
            hp.r[k].hi[c] = rr[k][3 + c];
        }
    printf("ms per 1024 items of 896^2, whole canvas (fill lanes load nothing useful)\n");
    printf("angle canvas |  A quads  B pairs  D x4(lb) | HSV: A  B | mismatch B\n");
    std::vector<double> angles = {0.0, 10.0, 20.0, 30.0, 45.0, 60.0, 80.0, 100.0, 135.0, 200.0};
    if (only >= 0) angles = {30.0};
    for (double deg : angles) {
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
        std::vector<uint32_t> hA(n), hB(n);
        float t[6] = {0, 0, 0, 0, 0, 0};
#define RUN(i, V, H) \
        if (only < 0 || only == i) t[i] = timeit([&] { hipLaunchKernelGGL((k_probe<V, H>), grid, dim3(256), 0, 0, src, item_bytes, g, bands, hp, out); });
        RUN(0, 0, false)
        hipMemcpy(hA.data(), out, n * 4, hipMemcpyDeviceToHost);
        RUN(1, 1, false)
        hipMemcpy(hB.data(), out, n * 4, hipMemcpyDeviceToHost);
        RUN(2, 2, false)
        RUN(3, 0, true)
        RUN(4, 1, true)
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i) bad += hA[i] != hB[i];
        printf("%5.1f %5d | %8.3f %8.3f %8.3f | %8.3f %8.3f | %zu\n", deg, mw, t[0], t[1], t[2], t[3], t[4], bad);
        fflush(stdout);
    }
    return 0;
}
