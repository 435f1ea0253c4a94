// map_probe.hip — does a lane map that follows the source rows cut the cost
// of the H pass's gathers?  The texture path charges a gather instruction
// roughly per distinct 64-B sector its 64 lanes touch (ta_probe.hip).  The
// shipped map (2×2 lane quads over 16 M rows × 4 columns) touches ~16-30
// source rows per instruction when the item is rotated.  A map whose lanes run
// along "digital lines" of M pixels that stay in one source row touches a few:
//   steep items (|b3| >= |b4|, the source row direction is within 45° of the M
//   columns): lane (g, r) takes row r of the band at column L + off(r),
//   off(r) = round(t r), t = -b4 / b3, L = 4g + k + step base: every line is
//   one source row, the 4 lines of an instruction are 4 adjacent lines;
//   shallow items: lane (j, q) takes column X + j at band row
//   (4k + q + round(s j)) mod 16, s = -b3 / b4: 16 columns along a line,
//   wrapped inside the band.
// Both maps cover every M pixel of the band exactly once and fold an
// order-free hash of (x, y, pixel): the totals must agree.  Pure gathers (no
// HSV, no ring), 1024 items of 896², whole canvas, ms per launch.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o map_probe map_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

namespace {

struct Geo {
    int32_t b0, b3, b1, b4, c, f;
    int32_t in_w, in_h, pitch, mw, mh;
    float t;      // steep: column shift per row along a source row (-b4 / b3)
    float s;      // shallow: row shift per column (-b3 / b4)
    int steep;
};

__device__ __forceinline__ uint32_t hsh(uint32_t x, uint32_t y, uint32_t v) {
    uint32_t h = (v & 0xFFFFFFu) * 0x9E3779B1u ^ (x * 0x85EBCA77u + y * 0xC2B2AE3Du);
    return h ^ (h >> 15);
}

__device__ __forceinline__ void block_out(uint32_t acc, uint32_t* red, uint32_t* out) {
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, red[0] + red[1] + red[2] + red[3]);
}

__device__ __forceinline__ uint32_t offset_of(const Geo& g, int x, int y, bool& ok) {
    const int xx = g.b0 * x + g.b1 * y + g.c, yy = g.b3 * x + g.b4 * y + g.f;
    const int xi = xx >> 16, yi = yy >> 16;
    ok = (uint32_t)xi < (uint32_t)g.in_w && (uint32_t)yi < (uint32_t)g.in_h && (uint32_t)x < (uint32_t)g.mw &&
         (uint32_t)y < (uint32_t)g.mh;
    return ok ? (uint32_t)__mul24(yi, g.pitch) + (uint32_t)__mul24(xi, 3) : 0xFFFFFFFFu;
}

// MAP 0: shipped 2x2 quads; MAP 1: source-row lines.
template <int MAP>
__global__ void __launch_bounds__(256) k_map(const uint8_t* __restrict__ src, int64_t item_bytes, Geo g, int bands,
                                             uint32_t* __restrict__ out) {
    __shared__ uint32_t red[4];
    const int item = blockIdx.x / bands, band = blockIdx.x - item * bands;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint8_t* base = src + item * item_bytes;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)item_bytes, 0x00020000);
    const int Y = band * 16;
    uint32_t acc = 0;
    if (MAP == 0) {
        const int r = 2 * (lane >> 3) + ((lane >> 1) & 1), y = Y + r;
        const int nsteps = (g.mw + 63) / 64;
        for (int st = 0; st < nsteps; ++st) {
            const int x0 = 64 * st + 16 * wave + 8 * ((lane >> 2) & 1) + (lane & 1);
            uint32_t p[4];
            int xs[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                xs[k] = x0 + 2 * k;
                bool ok;
                const uint32_t off = offset_of(g, xs[k], y, ok);
                p[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) acc += (xs[k] < g.mw) ? hsh(xs[k], y, p[k]) : 0u;
        }
    } else if (MAP == 2 && !g.steep) {
        // ring-compatible shallow map: a lane's 4 pixels are 4 consecutive
        // columns of one row; the 16 column groups of a line index q follow
        // the source row (row shift round(s 4m) per group), wrapped in the band
        const int m = lane & 15, q = (lane >> 4) + 4 * wave;
        const int sh = (int)rintf(g.s * (float)(4 * m)) & 15;
        const int y = Y + ((q + sh) & 15);
        const int nsteps = (g.mw + 63) / 64;
        for (int st = 0; st < nsteps; ++st) {
            const int x0 = 64 * st + 4 * m;
            uint32_t p[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                bool ok;
                const uint32_t o = offset_of(g, x0 + k, y, ok);
                p[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) acc += (x0 + k < g.mw) ? hsh(x0 + k, y, p[k]) : 0u;
        }
    } else if (MAP == 2) {
        // ring-compatible steep map: lane (gq, r): row r, 4 consecutive columns
        // of the column group G = L + gq + round(t r / 4)
        const int gq = lane >> 4, r = lane & 15, y = Y + r;
        const int o4 = (int)rintf(g.t * (float)r * 0.25f);
        const int G0 = (g.mw + 3) / 4;
        const int lo = -4, hi = G0 + 4;
        for (int L0 = lo + 4 * wave; L0 < hi; L0 += 16) {
            const int G = L0 + gq + o4;
            uint32_t p[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                bool ok;
                const uint32_t o = offset_of(g, 4 * G + k, y, ok);
                p[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
            }
            const bool own = G >= 0 && G < G0 && L0 + gq < hi;
#pragma unroll
            for (int k = 0; k < 4; ++k) acc += (own && 4 * G + k < g.mw) ? hsh(4 * G + k, y, p[k]) : 0u;
        }
    } else if (g.steep) {
        const int gq = lane >> 4, r = lane & 15, y = Y + r;
        const int off = (int)rintf(g.t * (float)r);
        // line bases L: every x in [0, mw) of every row once
        const int lo = -16, hi = g.mw + 16;
        for (int L0 = lo + 16 * wave; L0 < hi; L0 += 64) {
            uint32_t p[4];
            int xs[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int L = L0 + 4 * gq + k;
                xs[k] = L + off;
                bool ok;
                const uint32_t o = offset_of(g, xs[k], y, ok);
                p[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int L = L0 + 4 * gq + k;
                // line L owns x = L + off(r) only when that x is in [0, mw) (each x exactly once)
                acc += ((uint32_t)xs[k] < (uint32_t)g.mw && L >= lo && L < hi) ? hsh(xs[k], y, p[k]) : 0u;
            }
        }
    } else {
        const int j = lane & 15, q = lane >> 4;
        const int sh = (int)rintf(g.s * (float)j) & 15;
        const int nsteps = (g.mw + 63) / 64;
        for (int st = 0; st < nsteps; ++st) {
            const int x = 64 * st + 16 * wave + j;
            uint32_t p[4];
            int ys[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ys[k] = Y + ((4 * k + q + sh) & 15);
                bool ok;
                const uint32_t o = offset_of(g, x, ys[k], ok);
                p[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) acc += (x < g.mw) ? hsh(x, ys[k], p[k]) : 0u;
        }
    }
    block_out(acc, red, out);
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
    if (hipMalloc(&out, 64) != hipSuccess) return 1;
    printf("ms per launch, 1024 items of 896^2, whole canvas, gathers only\n");
    printf("angle canvas  steep | quads   lines  ringmap | ratios | hash equal\n");
    for (double deg : {0.0, 5.0, 10.0, 20.0, 30.0, 40.0, 45.0, 50.0, 60.0, 70.0, 80.0, 90.0, 100.0, 135.0, 200.0, 300.0}) {
        const double a = deg * M_PI / 180.0, c = cos(a), s = sin(a);
        const int mw = (int)ceil(S * (fabs(c) + fabs(s))), mh = mw;
        Geo g;
        g.b0 = (int32_t)lrint(c * 65536), g.b1 = (int32_t)lrint(s * 65536);
        g.b3 = (int32_t)lrint(-s * 65536), g.b4 = (int32_t)lrint(c * 65536);
        const double cx = mw / 2.0, cy = mh / 2.0;
        g.c = (int32_t)lrint((S / 2.0 - c * cx - s * cy) * 65536);
        g.f = (int32_t)lrint((S / 2.0 + s * cx - c * cy) * 65536);
        g.in_w = S, g.in_h = S, g.mw = mw, g.mh = mh, g.pitch = 3 * S;
        g.steep = abs(g.b3) >= abs(g.b4);
        g.t = g.steep ? -(float)g.b4 / (float)g.b3 : 0.0f;
        g.s = g.steep ? 0.0f : -(float)g.b3 / (float)g.b4;
        const int bands = (mh + 15) / 16;
        const dim3 grid(items * bands);
        uint32_t h0 = 0, h1 = 0;
        hipMemset(out, 0, 4);
        hipLaunchKernelGGL(k_map<0>, grid, dim3(256), 0, 0, src, item_bytes, g, bands, out);
        hipMemcpy(&h0, out, 4, hipMemcpyDeviceToHost);
        hipMemset(out, 0, 4);
        hipLaunchKernelGGL(k_map<1>, grid, dim3(256), 0, 0, src, item_bytes, g, bands, out);
        hipMemcpy(&h1, out, 4, hipMemcpyDeviceToHost);
        const float t0 = timeit([&] { hipLaunchKernelGGL(k_map<0>, grid, dim3(256), 0, 0, src, item_bytes, g, bands, out); });
        const float t1 = timeit([&] { hipLaunchKernelGGL(k_map<1>, grid, dim3(256), 0, 0, src, item_bytes, g, bands, out); });
        uint32_t h2 = 0;
        hipMemset(out, 0, 4);
        hipLaunchKernelGGL(k_map<2>, grid, dim3(256), 0, 0, src, item_bytes, g, bands, out);
        hipMemcpy(&h2, out, 4, hipMemcpyDeviceToHost);
        const float t2 = timeit([&] { hipLaunchKernelGGL(k_map<2>, grid, dim3(256), 0, 0, src, item_bytes, g, bands, out); });
        printf("%5.1f %5d %6d | %7.3f %7.3f %7.3f | %5.2f %5.2f | %s %s\n", deg, mw, g.steep, t0, t1, t2, t1 / t0, t2 / t0,
               h0 == h1 ? "yes" : "NO", h0 == h2 ? "yes" : "NO");
        fflush(stdout);
    }
    hipFree(src);
    hipFree(out);
    return 0;
}
