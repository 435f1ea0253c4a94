// gather_probe.hip — what does one rotated-pixel gather cost on the texture
// path?  Mimics the H pass's phase-1 access pattern (a 16-row band of a
// rotated 3-byte-per-pixel image; a lane quad takes a 2x2 block of M pixels,
// 4 pixels per lane and step, 16 columns per wave step) without the HSV and
// MFMA work, and varies only the load form:
//   0  buffer_load_dword   at 3x            (the shipped form: 3/4 unaligned)
//   1  buffer_load_dword   at 3x & ~3       (aligned, wrong bytes: cost of alignment)
//   2  buffer_load_dwordx2 at 3x & ~3       (aligned, always covers the pixel)
//   3  buffer_load_ubyte x3                 (three aligned byte loads)
//   4  global_load_dword   at 3x            (flat/global address path)
//   5  buffer_load_dword   at 4x            (an RGBA source: all aligned)
//   6  source box of each 64x16 M segment staged in LDS by 16-B LDS-DMA
//      loads (global_load_lds_dwordx4), pixels read from LDS (single buffer)
// Variant 6 must XOR to the same value as variant 0 (checked).
// The result is XOR-reduced into one dword per thread so nothing is dead.
// Build: hipcc --offload-arch=gfx950 -O3 -o gather_probe gather_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

struct Geo {
    int32_t b0, b3, b1, b4;  // 16.16 affine: xx = b0*x + b1*y + c, yy = b3*x + b4*y + f
    int32_t c, f;
    int32_t in_w, in_h, pitch;
    int32_t mw, mh;          // M canvas
};

template <int V>
__global__ void __launch_bounds__(256) k_gather(const uint8_t* __restrict__ src, int64_t item_bytes, Geo g,
                                                int bands, uint32_t* __restrict__ out) {
    const int item = blockIdx.x / bands, band = blockIdx.x - item * bands;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint8_t* base = src + item * item_bytes;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)item_bytes, 0x00020000);
    const int y = band * 16 + 2 * (lane >> 3) + ((lane >> 1) & 1);
    const int cn = V == 5 ? 4 : 3;
    uint32_t acc = 0;
    // columns of this wave: steps of 64 columns over the block, 16 per wave
    for (int x0 = 16 * wave; x0 < g.mw; x0 += 64) {
        uint32_t off[4];
        bool ok[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int x = x0 + 8 * ((lane >> 2) & 1) + (lane & 1) + 2 * k;
            const int xx = g.b0 * x + g.b1 * y + g.c, yy = g.b3 * x + g.b4 * y + g.f;
            const int xi = xx >> 16, yi = yy >> 16;
            ok[k] = (uint32_t)xi < (uint32_t)g.in_w && (uint32_t)yi < (uint32_t)g.in_h;
            off[k] = ok[k] ? (uint32_t)(yi * g.pitch + xi * cn) : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t v;
            if (V == 0 || V == 5) v = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off[k], 0, 0);
            else if (V == 1) v = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off[k] & ~3u, 0, 0);
            else if (V == 2) {
                typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 w = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off[k] & ~3u, 0, 0));
                v = __builtin_amdgcn_alignbyte(w.y, w.x, off[k] & 3u);
            } else if (V == 3) {
                v = __builtin_amdgcn_raw_buffer_load_b8(rsrc, off[k], 0, 0) |
                    (__builtin_amdgcn_raw_buffer_load_b8(rsrc, off[k] + 1, 0, 0) << 8) |
                    (__builtin_amdgcn_raw_buffer_load_b8(rsrc, off[k] + 2, 0, 0) << 16);
            } else {
                v = ok[k] ? *reinterpret_cast<const uint32_t*>(base + off[k]) : 0u;
            }
            acc ^= v + k;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// Variant 6: per block (16-row band) and segment of 64 M columns, the
// source bounding box is copied to LDS with 16-B LDS-DMA loads, then every
// lane reads its 4 pixels from LDS.  Pitch must be a multiple of 16.
constexpr int STAGE_BYTES = 16384;
__global__ void __launch_bounds__(256) k_staged(const uint8_t* __restrict__ src, int64_t item_bytes, Geo g,
                                                int bands, uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE_BYTES + 64];
    const int item = blockIdx.x / bands, band = blockIdx.x - item * bands;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint8_t* base = src + item * item_bytes;
    const int Y = band * 16;
    const int y = Y + 2 * (lane >> 3) + ((lane >> 1) & 1);
    uint32_t acc = 0;
    int overflow = 0;
    for (int X = 0; X < g.mw; X += 64) {
        // box of the segment's source footprint (corners, inclusive)
        int sxl = 1 << 30, sxh = -(1 << 30), syl = 1 << 30, syh = -(1 << 30);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int cx = X + (c & 1) * 63, cy = Y + (c >> 1) * 15;
            const int xx = (g.b0 * cx + g.b1 * cy + g.c) >> 16, yy = (g.b3 * cx + g.b4 * cy + g.f) >> 16;
            sxl = min(sxl, xx); sxh = max(sxh, xx); syl = min(syl, yy); syh = max(syh, yy);
        }
        sxl = max(sxl, 0); syl = max(syl, 0); sxh = min(sxh, g.in_w - 1); syh = min(syh, g.in_h - 1);
        const bool empty = sxl > sxh || syl > syh;
        const int b0 = (3 * sxl) & ~15;
        const int n16 = empty ? 0 : (3 * (sxh + 1) - b0 + 15) >> 4;
        const int rows = empty ? 0 : syh - syl + 1;
        const int total = rows * n16;
        if (total * 16 > STAGE_BYTES) { overflow = 1; continue; }
        const int ninst = (total + 63) >> 6;
        for (int j = wave; j < ninst; j += 4) {
            const int idx = 64 * j + lane;
            const int row = idx / n16, k = idx - row * n16;
            const int rr = min(row, rows - 1);
            const uint8_t* gp = base + (int64_t)(syl + rr) * g.pitch + b0 + 16 * k;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(gp),
                                             (__attribute__((address_space(3))) void*)(stage + 1024 * j), 16, 0, 0);
        }
        __syncthreads();
        const int RS = 16 * n16;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int x = X + 16 * wave + 8 * ((lane >> 2) & 1) + (lane & 1) + 2 * k;
            if (x >= g.mw) continue;
            const int xx = g.b0 * x + g.b1 * y + g.c, yy = g.b3 * x + g.b4 * y + g.f;
            const int xi = xx >> 16, yi = yy >> 16;
            const bool ok = (uint32_t)xi < (uint32_t)g.in_w && (uint32_t)yi < (uint32_t)g.in_h;
            uint32_t v = 0;
            if (ok) {
                const int a = (yi - syl) * RS + 3 * xi - b0;
                const uint32_t* w = reinterpret_cast<const uint32_t*>(stage + (a & ~3));
                v = __builtin_amdgcn_alignbyte(w[1], w[0], a & 3) & 0xFFFFFFu;
            }
            acc ^= v + k;
        }
        __syncthreads();
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc + overflow * 0x40000000u;
}

// Variant 7: per-wave row-span staging.  For each wave step (16 M columns ×
// 16 rows) the source rows its pixels fall in are copied to a wave-private
// LDS stage with 16-B LDS-DMA loads (buffer_load_dwordx4 … lds), one row per
// 6 lanes = 96 bytes = 32 px starting at the row's left bound from the
// footprint's slab edges; a per-row table gives each row's LDS origin; the
// lanes then read their pixels from LDS.  No block barriers.
constexpr int ST_ROWS = 28, ST_RB = 96;
__global__ void __launch_bounds__(256) k_staged_rows(const uint8_t* __restrict__ src, int64_t item_bytes, Geo g,
                                                     int bands, uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t stage_all[4][ST_ROWS * ST_RB + 64];
    __shared__ int32_t tab_all[4][ST_ROWS];
    const int item = blockIdx.x / bands, band = blockIdx.x - item * bands;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint8_t* stage = stage_all[wave];
    int32_t* tab = tab_all[wave];
    const uint8_t* base = src + item * item_bytes;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)item_bytes, 0x00020000);
    const int Y = band * 16;
    const int y = Y + 2 * (lane >> 3) + ((lane >> 1) & 1);
    // slab constants (pixel units): u per M column, v per M row
    const float ux = g.b0 / 65536.0f, uy = g.b3 / 65536.0f, vx = g.b1 / 65536.0f, vy = g.b4 / 65536.0f;
    const bool hu = fabsf(uy) > 1e-6f, hv = fabsf(vy) > 1e-6f;
    const float ku = hu ? ux / uy : 0.0f, kv = hv ? vx / vy : 0.0f;
    uint32_t acc = 0;
    int overflow = 0;
    for (int x0 = 16 * wave; x0 < g.mw; x0 += 64) {
        const int xx0 = g.b0 * x0 + g.b1 * Y + g.c, yy0 = g.b3 * x0 + g.b4 * Y + g.f;
        int ylo = 1 << 30, yhi = -(1 << 30);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int yyc = yy0 + (c & 1) * 15 * g.b3 + (c >> 1) * 15 * g.b4;
            ylo = min(ylo, yyc >> 16);
            yhi = max(yhi, yyc >> 16);
        }
        const int syl = max(ylo, 0), syh = min(yhi, g.in_h - 1);
        const int R = syh - syl + 1;
        if (R > ST_ROWS) { overflow = 1; continue; }
        const float px = xx0 / 65536.0f, py = yy0 / 65536.0f;
        // u-slab: lines through P and P + 15v, direction u
        const float cu1 = px - py * ku, cu2 = (px + 15 * vx) - (py + 15 * vy) * ku;
        const float cv1 = px - py * kv, cv2 = (px + 15 * ux) - (py + 15 * uy) * kv;
        const float culo = fminf(cu1, cu2) + fminf(0.0f, ku), cvlo = fminf(cv1, cv2) + fminf(0.0f, kv);
        const float cuhi = fmaxf(cu1, cu2) + fmaxf(0.0f, ku), cvhi = fmaxf(cv1, cv2) + fmaxf(0.0f, kv);
        if (R > 0) {
#pragma unroll
            for (int j = 0; j < (ST_ROWS * 6 + 63) / 64; ++j) {
                const int i = 64 * j + lane;
                const int r = (i * 683) >> 12, k = i - 6 * r;
                if (r < R) {
                    const int sy = syl + r;
                    const float lo = fmaxf(hu ? culo + ku * sy : -1e9f, hv ? cvlo + kv * sy : -1e9f);
                    const float hi = fminf(hu ? cuhi + ku * sy : 1e9f, hv ? cvhi + kv * sy : 1e9f);
                    const int xl = max((int)floorf(lo) - 1, 0);
                    const int xh = min((int)floorf(hi) + 1, g.in_w - 1);
                    overflow |= xh - xl + 1 > 32;
                    if (k == 0) tab[r] = ST_RB * r - 3 * xl;
                    const uint32_t off = (uint32_t)(sy * g.pitch + 3 * xl + 16 * k);
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rsrc, (__attribute__((address_space(3))) void*)(stage + 1024 * j), 16, off, 0, 0, 0);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int x = x0 + 8 * ((lane >> 2) & 1) + (lane & 1) + 2 * k;
            const int xx = g.b0 * x + g.b1 * y + g.c, yy = g.b3 * x + g.b4 * y + g.f;
            const int xi = xx >> 16, yi = yy >> 16;
            const bool ok = x < g.mw && (uint32_t)xi < (uint32_t)g.in_w && (uint32_t)yi < (uint32_t)g.in_h;
            uint32_t v = 0;
            if (ok) {
                const int a = tab[yi - syl] + 3 * xi;
                const uint32_t* w = reinterpret_cast<const uint32_t*>(stage + (a & ~3));
                v = __builtin_amdgcn_alignbyte(w[1], w[0], a & 3) & 0xFFFFFFu;
            }
            acc ^= v + k;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();  // reads done before the next step's DMA overwrites the stage
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc + overflow * 0x40000000u;
}

// reference for variant 6's check: variant 0's pixel values, masked to 3 bytes
__global__ void __launch_bounds__(256) k_ref3(const uint8_t* __restrict__ src, int64_t item_bytes, Geo g, int bands,
                                              uint32_t* __restrict__ out) {
    const int item = blockIdx.x / bands, band = blockIdx.x - item * bands;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint8_t* base = src + item * item_bytes;
    const int y = band * 16 + 2 * (lane >> 3) + ((lane >> 1) & 1);
    uint32_t acc = 0;
    for (int X = 0; X < g.mw; X += 64)
        for (int k = 0; k < 4; ++k) {
            const int x = X + 16 * wave + 8 * ((lane >> 2) & 1) + (lane & 1) + 2 * k;
            if (x >= g.mw) continue;
            const int xx = g.b0 * x + g.b1 * y + g.c, yy = g.b3 * x + g.b4 * y + g.f;
            const int xi = xx >> 16, yi = yy >> 16;
            const bool ok = (uint32_t)xi < (uint32_t)g.in_w && (uint32_t)yi < (uint32_t)g.in_h;
            uint32_t v = 0;
            if (ok) { const uint8_t* p = base + (int64_t)yi * g.pitch + 3 * xi; v = p[0] | (p[1] << 8) | (p[2] << 16); }
            acc ^= v + k;
        }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int V>
float run(const uint8_t* src, int64_t item_bytes, int items, const Geo& g, uint32_t* out) {
    const int bands = (g.mh + 15) / 16;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto launch = [&] {
        if (V == 6) hipLaunchKernelGGL(k_staged, dim3(items * bands), dim3(256), 0, 0, src, item_bytes, g, bands, out);
        else if (V == 7) hipLaunchKernelGGL(k_ref3, dim3(items * bands), dim3(256), 0, 0, src, item_bytes, g, bands, out);
        else if (V == 8) hipLaunchKernelGGL(k_staged_rows, dim3(items * bands), dim3(256), 0, 0, src, item_bytes, g, bands, out);
        else hipLaunchKernelGGL(k_gather<V>, dim3(items * bands), dim3(256), 0, 0, src, item_bytes, g, bands, out);
    };
    launch();
    hipEventRecord(e0);
    const int reps = 5;
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms / reps;
}

int main() {
    const int S = 896, items = 1024;
    const int64_t item_bytes = (int64_t)S * S * 4;  // room for the RGBA variant
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
    printf("variant: 0 dword@3x  1 dword aligned  2 dwordx2 aligned  3 ubyte x3  4 global dword  5 dword@4x (RGBA)  6 LDS-staged box\n");
    for (double deg : {0.0, 10.0, 30.0, 45.0}) {
        const double a = deg * M_PI / 180.0, c = cos(a), s = sin(a);
        const int mw = (int)ceil(S * (fabs(c) + fabs(s))), mh = mw;
        Geo g;
        // inverse map of an expand rotation about the canvas centre
        g.b0 = (int32_t)lrint(c * 65536), g.b1 = (int32_t)lrint(s * 65536);
        g.b3 = (int32_t)lrint(-s * 65536), g.b4 = (int32_t)lrint(c * 65536);
        const double cx = mw / 2.0, cy = mh / 2.0;
        g.c = (int32_t)lrint((S / 2.0 - c * cx - s * cy) * 65536);
        g.f = (int32_t)lrint((S / 2.0 + s * cx - c * cy) * 65536);
        g.in_w = S, g.in_h = S, g.mw = mw, g.mh = mh;
        float t[9];
        g.pitch = 3 * S;
        t[0] = run<0>(src, item_bytes, items, g, out);
        t[1] = run<1>(src, item_bytes, items, g, out);
        t[2] = run<2>(src, item_bytes, items, g, out);
        t[3] = run<3>(src, item_bytes, items, g, out);
        t[4] = run<4>(src, item_bytes, items, g, out);
        t[6] = run<6>(src, item_bytes, items, g, out);
        const int nb = items * ((mh + 15) / 16);
        std::vector<uint32_t> h6((size_t)nb * 256), h7((size_t)nb * 256), h8((size_t)nb * 256);
        hipMemcpy(h6.data(), out, h6.size() * 4, hipMemcpyDeviceToHost);
        t[8] = run<8>(src, item_bytes, items, g, out);
        hipMemcpy(h8.data(), out, h8.size() * 4, hipMemcpyDeviceToHost);
        run<7>(src, item_bytes, items, g, out);
        hipMemcpy(h7.data(), out, h7.size() * 4, hipMemcpyDeviceToHost);
        size_t bad = 0, bad8 = 0;
        for (size_t i = 0; i < h6.size(); ++i) bad += h6[i] != h7[i];
        for (size_t i = 0; i < h8.size(); ++i) bad8 += h8[i] != h7[i];
        g.pitch = 4 * S;
        t[5] = run<5>(src, item_bytes, items, g, out);
        const double px = (double)mw * mh * items;
        printf("angle %4.0f  canvas %4d  ms:", deg, mw);
        for (int v = 0; v < 7; ++v) printf(" %7.3f", t[v]);
        printf("   Gpx/s:");
        for (int v = 0; v < 7; ++v) printf(" %6.1f", px / (t[v] * 1e-3) / 1e9);
        printf("   staged mismatches %zu   rows-staged %7.3f ms (%6.1f Gpx/s) mismatches %zu\n", bad, t[8],
               px / (t[8] * 1e-3) / 1e9, bad8);
    }
    hipFree(src);
    hipFree(out);
    return 0;
}
