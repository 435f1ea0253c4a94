// ipp_taps.hip — device tap planner of the fused pipe (gfx950).
//
// Builds, directly in HBM, the MFMA tile format the pipe kernels read (see
// ipp_host.cpp ipp_plan_mfma_from_taps for the format): per axis hdr[4T],
// bias[16T] and the i8 B/A blocks, tile t's blocks at uint4 offset t·nkb·192.
// The taps are Pillow's LANCZOS taps (Resample.c precompute_coeffs +
// normalize_coeffs_8bpc, reference call site overlays.py:129), computed in
// fp64 exactly as the host code computes them except for sin(): this file is
// compiled with -ffp-contract=off, so every other operation (bounds, filter
// argument, running sum, division, quantisation) rounds as on the host.  The
// device sin and libm's differ by at most an ulp or so, which moves a
// quantised tap's pre-truncation value v·2^22 ± 0.5 by < 1e-8; a tile with any
// tap whose value lies within 2^-22 of an integer is listed and rebuilt on the
// host with libm (ipp_plan_mfma_tile), so the result is bit-exact.
//
// One block per axis, one wave per 16-output tile.  A wave first evaluates
// the filter for all (output, tap) pairs of its tile across its 64 lanes
// (weights cached in LDS), sums each output's weights in Pillow's order on
// one lane, then lane (seg, col) builds the 16-byte chunks of output col at
// K offsets 16·seg + 64·s — exactly one lane owns each chunk, so every block
// is written once, with full 16-byte stores and no memset.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "ipp.h"

namespace {

constexpr int TAP_WAVES = 4;
constexpr int TAP_CACHE = 64;       // cached weights per output (more: recomputed)
constexpr int TAP_FLAG_CAP = 1 << 16;
constexpr double TAP_NEAR = 1.0 / 4194304.0;  // 2^-22

__device__ inline double d_sinc(double x) {
    if (x == 0.0) return 1.0;
    x = x * M_PI;
    return sin(x) / x;
}

__device__ inline double d_lanczos(double x) {
    if (-3.0 <= x && x < 3.0) return d_sinc(x) * d_sinc(x / 3);
    return 0.0;
}

// Resample.c filter argument for tap q of an output: (x + xmin - center + 0.5)·ss
__device__ inline double d_weight(int q, int xmin, double center, double ss) {
    return d_lanczos(((double)(q + xmin) - center + 0.5) * ss);
}

inline __device__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(256) void k_plan_taps(const ipp_tap_axis* __restrict__ axes,
                                                   int32_t* __restrict__ coefs, int32_t* __restrict__ ctl,
                                                   int2* __restrict__ flags) {
    __shared__ double wcache[TAP_WAVES][16][TAP_CACHE];
    __shared__ double s_ww[TAP_WAVES][16];
    __shared__ double s_center[TAP_WAVES][16];
    __shared__ int s_xmin[TAP_WAVES][16];
    __shared__ int s_pre[TAP_WAVES][16];
    __shared__ int s_cnt[TAP_WAVES][16];
    const ipp_tap_axis a = axes[blockIdx.x];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, col = lane & 15, seg = lane >> 4;
    const double scale = (double)((float)a.in_size) / a.out_size;
    const double fs = scale < 1.0 ? 1.0 : scale;
    const double support = 3.0 * fs, ss = 1.0 / fs;
    int32_t* hdr = coefs + a.coef_off;
    int32_t* bias = hdr + 4 * (int64_t)a.n_tiles;
    uint4* blk = reinterpret_cast<uint4*>(hdr + 20 * (int64_t)a.n_tiles);
    double* wc = &wcache[wave][0][0];

    for (int t = wave; t < a.n_tiles; t += TAP_WAVES) {
        const int o0 = 16 * t - a.phase, o = o0 + col;
        const int oa = max(o0, 0), o1 = min(o0 + 16, a.out_size);
        const bool valid = o >= oa && o < o1;
        int xmin = 0, cnt = 0;
        double center = 0.0;
        if (valid) {
            if (a.identity) {
                xmin = o;
                cnt = 1;
            } else {
                center = 0.0 + (o + 0.5) * scale;
                xmin = (int)(center - support + 0.5);
                if (xmin < 0) xmin = 0;
                int xmax = (int)(center + support + 0.5);
                if (xmax > a.in_size) xmax = a.in_size;
                cnt = xmax - xmin;
            }
        }
        const int xs = xmin - a.shift;
        const int K0 = __shfl(xs, oa - o0) & ~15;
        int end = valid ? xs + cnt : K0;
        for (int m = 32; m >= 1; m >>= 1) end = max(end, __shfl_xor(end, m));
        int nK = (max(end, K0) - K0 + 63) >> 6;
        if (nK > a.nkb) {  // the planner's bound was wrong: report, stay in bounds
            if (lane == 0) atomicOr(ctl + 1, 1);
            nK = a.nkb;
        }
        const int64_t boff = (int64_t)t * a.nkb * 192;
        if (lane == 0) *reinterpret_cast<int4*>(hdr + 4 * t) = make_int4(K0, nK, (int)boff, 0);

        // ---- filter weights of the tile, all lanes busy --------------------
        double ww = 0.0;
        if (!a.identity) {
            if (seg == 0) {
                s_center[wave][col] = center;
                s_xmin[wave][col] = xmin;
            }
            int pre = 0, total = 0;  // prefix of cached tap counts over columns
            for (int c = 0; c < 16; ++c) {
                const int nc = min(__shfl(cnt, c), TAP_CACHE);
                if (c < col) pre += nc;
                total += nc;
            }
            if (seg == 0) {
                s_pre[wave][col] = pre;
                s_cnt[wave][col] = min(cnt, TAP_CACHE);
            }
            wave_sync();
            for (int p = lane; p < total; p += 64) {
                int c = 0, base = 0;
                for (int k = 0; k < 16; ++k) {  // column of pair p
                    const int bk = s_pre[wave][k];
                    if (bk <= p && s_cnt[wave][k] > 0) {
                        c = k;
                        base = bk;
                    }
                }
                const int q = p - base;
                wc[c * TAP_CACHE + q] = d_weight(q, s_xmin[wave][c], s_center[wave][c], ss);
            }
            wave_sync();
            if (seg == 0 && valid) {  // Pillow's running sum, in tap order
                for (int q = 0; q < cnt; ++q)
                    ww += q < TAP_CACHE ? wc[col * TAP_CACHE + q] : d_weight(q, xmin, center, ss);
                s_ww[wave][col] = ww;
            }
            wave_sync();
            ww = s_ww[wave][col];
        }

        // ---- chunks of output col at K offset 64s + 16seg ------------------
        int64_t sum = 0;
        bool near = false;
        for (int s = 0; s < nK; ++s) {
            uint32_t P[3][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
            const int qb = K0 + 64 * s + 16 * seg - xs;
            if (valid && qb < cnt && qb + 16 > 0) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int q = qb + j;
                    if (q < 0 || q >= cnt) continue;
                    int32_t k;
                    if (a.identity) {
                        k = 1 << 22;
                    } else {
                        double v = q < TAP_CACHE ? wc[col * TAP_CACHE + q] : d_weight(q, xmin, center, ss);
                        if (ww != 0.0) v = v / ww;
                        const double x = v < 0 ? -0.5 + v * 4194304.0 : 0.5 + v * 4194304.0;
                        k = (int32_t)x;
                        near |= fabs(x - rint(x)) < TAP_NEAR;
                    }
                    sum += k;
                    int32_t r = k;
#pragma unroll
                    for (int p = 0; p < 3; ++p) {  // balanced signed bytes
                        const int32_t lo = ((r + 128) & 255) - 128;
                        P[p][j >> 2] |= (uint32_t)(uint8_t)lo << (8 * (j & 3));
                        r = (r - lo) >> 8;
                    }
                }
            }
#pragma unroll
            for (int p = 0; p < 3; ++p)
                blk[boff + (int64_t)(s * 3 + p) * 64 + lane] = make_uint4(P[p][0], P[p][1], P[p][2], P[p][3]);
        }
        sum += __shfl_xor((long long)sum, 16);
        sum += __shfl_xor((long long)sum, 32);
        if (seg == 0) bias[16 * t + col] = valid ? (int32_t)((1 << 21) + 128 * sum) : 0;
        if (__any(near) && lane == 0) {
            const int idx = atomicAdd(ctl, 1);
            if (idx < TAP_FLAG_CAP) flags[idx] = make_int2((int)blockIdx.x, t);
        }
        wave_sync();  // the next tile reuses the weight cache
    }
}

inline int64_t align256(int64_t x) { return (x + 255) / 256 * 256; }

}  // namespace

extern "C" int64_t ipp_pipe_taps_scratch_bytes(int32_t n_axes) {
    if (n_axes <= 0) return IPP_E_ARG;
    return align256((int64_t)n_axes * (int64_t)sizeof(ipp_tap_axis)) + 256 + 8 * (int64_t)TAP_FLAG_CAP;
}

extern "C" int ipp_pipe_plan_taps(const ipp_tap_axis* axes, int32_t n_axes, int32_t* coefs, void* scratch,
                                  int64_t* stats, void* stream) {
    if (!axes || n_axes <= 0 || !coefs || !scratch || !stats) return IPP_E_ARG;
    for (int32_t j = 0; j < n_axes; ++j) {
        const ipp_tap_axis& a = axes[j];
        if (a.in_size <= 0 || a.out_size <= 0 || a.phase < 0 || a.phase > 15 || a.nkb <= 0 ||
            a.n_tiles != (a.out_size + a.phase + 15) / 16 || (int64_t)a.n_tiles * a.nkb * 192 > INT32_MAX ||
            a.coef_off < 0 || (a.coef_off & 3))
            return IPP_E_ARG;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint8_t* sb = reinterpret_cast<uint8_t*>(scratch);
    ipp_tap_axis* d_axes = reinterpret_cast<ipp_tap_axis*>(sb);
    int32_t* d_ctl = reinterpret_cast<int32_t*>(sb + align256((int64_t)n_axes * sizeof(ipp_tap_axis)));
    int2* d_flags = reinterpret_cast<int2*>(d_ctl + 64);
    if (hipMemcpyAsync(d_axes, axes, (size_t)n_axes * sizeof(ipp_tap_axis), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(d_ctl, 0, 256, s) != hipSuccess)
        return IPP_E_LAUNCH;
    hipLaunchKernelGGL(k_plan_taps, dim3(n_axes), dim3(256), 0, s, d_axes, coefs, d_ctl, d_flags);
    if (hipGetLastError() != hipSuccess) return IPP_E_LAUNCH;
    int32_t ctl[2] = {0, 0};
    if (hipMemcpyAsync(ctl, d_ctl, sizeof ctl, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return IPP_E_LAUNCH;
    stats[0] = ctl[0];
    stats[1] = ctl[1];
    if (ctl[0] > TAP_FLAG_CAP) return IPP_E_RANGE;
    if (ctl[0] == 0) return IPP_OK;
    std::vector<int2> fl(ctl[0]);
    // on `s`, not the null stream (which would wait for unrelated work, e.g.
    // the batch running on another stream while this one is planned)
    if (hipMemcpyAsync(fl.data(), d_flags, fl.size() * sizeof(int2), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return IPP_E_LAUNCH;
    // Rebuild the flagged tiles on the host (libm sin) and copy them over.
    int maxnk = 1;
    for (const int2& f : fl) maxnk = std::max(maxnk, axes[f.x].nkb);
    std::vector<int32_t> bias(16 * fl.size());
    std::vector<uint8_t> blocks((size_t)maxnk * 3072 * fl.size());
    // Every tile is rebuilt before any copy is queued, and the copies (which
    // read `bias` / `blocks`) have completed before this function returns on
    // every path.
    std::vector<int32_t> hdrs(4 * fl.size());
    for (size_t i = 0; i < fl.size(); ++i) {
        const int e = ipp_plan_mfma_tile(&axes[fl[i].x], fl[i].y, hdrs.data() + 4 * i, bias.data() + 16 * i,
                                         blocks.data() + i * (size_t)maxnk * 3072, (int64_t)maxnk * 3072);
        if (e) return e;
    }
    int rc = IPP_OK;
    for (size_t i = 0; i < fl.size() && rc == IPP_OK; ++i) {
        const ipp_tap_axis& a = axes[fl[i].x];
        const int t = fl[i].y;
        const int32_t* hdr = hdrs.data() + 4 * i;
        int32_t* base = coefs + a.coef_off;
        if (hipMemcpyAsync(base + 4 * (int64_t)a.n_tiles + 16 * t, bias.data() + 16 * i, 64, hipMemcpyHostToDevice,
                           s) != hipSuccess ||
            hipMemcpyAsync(base + 20 * (int64_t)a.n_tiles + 4 * (int64_t)hdr[2],
                           blocks.data() + i * (size_t)maxnk * 3072, (size_t)hdr[1] * 3072, hipMemcpyHostToDevice,
                           s) != hipSuccess)
            rc = IPP_E_LAUNCH;
    }
    if (hipStreamSynchronize(s) != hipSuccess) return IPP_E_LAUNCH;
    return rc;
}
