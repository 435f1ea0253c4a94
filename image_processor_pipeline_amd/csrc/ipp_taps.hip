// ipp_taps.hip — device tap planner of the fused pipe (gfx950).
//
// Builds, directly in HBM, the MFMA tile format the pipe kernels read (see
// ipp_host.cpp ipp_plan_mfma_from_taps for the format): per axis hdr[4T],
// bias[16T] and the i8 B/A blocks, tile t's blocks at uint4 offset t·nkb·192.
// The taps are Pillow's LANCZOS taps (Resample.c precompute_coeffs +
// normalize_coeffs_8bpc, reference call site overlays.py:129), computed in
// fp64 as the host code computes them except for the filter's sines (a short
// series, d_sinpi) and the normalisation (a multiply by 1/ww): this file is
// compiled with -ffp-contract=off, so every other operation (bounds, filter
// argument, running sum, quantisation) rounds as on the host.  Those two
// differ from the host's libm sin and division by a few ulps, which moves a
// quantised tap's pre-truncation value v·2^22 ± 0.5 by < 1e-8; a tile with any
// tap whose value lies within 2^-22 of an integer is listed and rebuilt on the
// host with libm (ipp_plan_mfma_tile), so the result is bit-exact.
//
// One block per axis, one wave per 16-output tile.  Lane (seg, col) owns taps
// q = seg + 4i of output col: it evaluates their weights into an LDS cache,
// one lane per output sums them in Pillow's order, then every
// lane quantises its own taps and writes their three byte planes into an LDS
// staging area laid out as the tile's blocks (dense: a window of K steps at a
// time; compact: the whole 196-uint4 tile), which the wave stores with full
// 16-byte coalesced stores.  The VALU work is per (output, tap) pair, not per
// (output, K position): ~5x fewer lanes idle than a chunk-per-lane build.
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
constexpr int TAP_NI = TAP_CACHE / 4;  // weights per lane in registers (4 lanes per output)
constexpr int TAP_STAGE_U4 = 16 * TAP_CACHE * 8 / 16;  // per wave: the weight cache = the staging area
constexpr int TAP_STAGE_K = TAP_STAGE_U4 / 192;         // dense K steps per staging window
static_assert(TAP_STAGE_U4 >= 196 && TAP_STAGE_K >= 1, "staging area holds a compact tile");
constexpr int TAP_FLAG_CAP = 1 << 16;
constexpr double TAP_NEAR = 1.0 / 4194304.0;  // 2^-22

// sin(π t) for |t| ≤ 1.5: t = n/2 + f with |f| ≤ 1/4 (exact), then the
// Taylor series of sin(π f) / cos(π f) to ~1e-17.  A few ulps from libm's
// sin(fl(π x)), far inside the 2^-22 margin of the near-boundary check below
// (a deviation δ of a weight moves the quantised value by 2^22 δ / ww).
__device__ inline double d_sinpi(double t) {
    const double n = rint(2.0 * t);
    const double f = t - 0.5 * n;
    const double x = M_PI * f, z = x * x;
    double sp = 1.0 / 355687428096000.0;             // 1/17!
    sp = sp * z - 1.0 / 1307674368000.0;              // 1/15!
    sp = sp * z + 1.0 / 6227020800.0;                 // 1/13!
    sp = sp * z - 1.0 / 39916800.0;
    sp = sp * z + 1.0 / 362880.0;
    sp = sp * z - 1.0 / 5040.0;
    sp = sp * z + 1.0 / 120.0;
    sp = sp * z - 1.0 / 6.0;
    sp = x + x * z * sp;
    double cp = 1.0 / 6402373705728000.0;            // 1/18!
    cp = cp * z - 1.0 / 20922789888000.0;             // 1/16!
    cp = cp * z + 1.0 / 87178291200.0;                // 1/14!
    cp = cp * z - 1.0 / 479001600.0;
    cp = cp * z + 1.0 / 3628800.0;
    cp = cp * z - 1.0 / 40320.0;
    cp = cp * z + 1.0 / 720.0;
    cp = cp * z - 1.0 / 24.0;
    cp = cp * z + 0.5;
    cp = 1.0 - z * cp;
    const int q = (int)n & 3;
    const double r = (q & 1) ? cp : sp;
    return (q & 2) ? -r : r;
}

// Pillow's lanczos(x) = sinc(x) sinc(x / 3), sinc(x) = sin(π x) / (π x), with
// sin(π x) = sin(3 θ) = s (3 - 4 s²), s = sin(θ), θ = π x / 3: one series.
__device__ inline double d_lanczos(double x) {
    if (-3.0 <= x && x < 3.0) {
        if (x == 0.0) return 1.0;
        const double t = x / 3;
        const double s3 = d_sinpi(t);
        const double s1 = s3 * (3.0 - 4.0 * s3 * s3);
        return (s1 * s3) / ((x * M_PI) * (t * M_PI));
    }
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

// Pillow's 8bpc normalisation of one weight (Resample.c normalize_coeffs_8bpc,
// PRECISION_BITS 22): k = trunc(v·2^22 ± 0.5), v = w / ww; `near` when the
// pre-truncation value is within 2^-22 of an integer (the host rebuilds that
// tile with libm).
__device__ inline int32_t d_quant(double w, double rww, bool& near) {
    const double v = w * rww;
    const double x = v < 0 ? -0.5 + v * 4194304.0 : 0.5 + v * 4194304.0;
    near |= fabs(x - rint(x)) < TAP_NEAR;
    return (int32_t)x;
}

// Byte address, in the wave's staging area, of plane p of tap K index kidx
// (relative to the tile's K0) of output col.  Dense: chunk (s, p, seg, col)
// at uint4 (3s + p)·64 + 16·seg + col of the window that starts at K step s0.
// Compact: block gbase + (kidx >> 4) - g0 of plane p, after the 4 meta uint4.
__device__ inline int stage_byte(bool compact, int kidx, int p, int col, int s0, int g0, int gbase) {
    const int u = compact ? 4 + p * 64 + gbase + (kidx >> 4) - g0
                          : ((((kidx >> 6) - s0) * 3 + p) * 64 + ((kidx >> 4) & 3) * 16 + col);
    return 16 * u + (kidx & 15);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_plan_taps(
    const ipp_tap_axis* __restrict__ axes, int32_t* __restrict__ coefs, int32_t* __restrict__ ctl,
    int2* __restrict__ flags) {
    // per wave: the weight cache of the running sums, then (same bytes) the
    // staging area the tile's blocks are assembled in
    __shared__ uint4 s_wave[TAP_WAVES][TAP_STAGE_U4];
    const ipp_tap_axis a = axes[blockIdx.x];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, col = lane & 15, seg = lane >> 4;
    const double scale = (double)((float)a.in_size) / a.out_size;
    const double fs = scale < 1.0 ? 1.0 : scale;
    const double support = 3.0 * fs, ss = 1.0 / fs;
    int32_t* hdr = coefs + a.coef_off;
    int32_t* bias = hdr + 4 * (int64_t)a.n_tiles;
    uint4* blk = reinterpret_cast<uint4*>(hdr + 20 * (int64_t)a.n_tiles);
    double* wc = reinterpret_cast<double*>(&s_wave[wave][0]);    // [16][TAP_CACHE]
    uint8_t* stage = reinterpret_cast<uint8_t*>(&s_wave[wave][0]);
    uint4* stage4 = &s_wave[wave][0];

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
        int end = valid ? xs + cnt : K0, maxcnt = cnt;
        for (int m = 32; m >= 1; m >>= 1) {
            end = max(end, __shfl_xor(end, m));
            maxcnt = max(maxcnt, __shfl_xor(maxcnt, m));
        }
        int nK = (max(end, K0) - K0 + 63) >> 6;
        if (nK > a.nkb) {  // the planner's bound was wrong: report, stay in bounds
            if (lane == 0) atomicOr(ctl + 1, 1);
            nK = a.nkb;
        }
        const int niter = (maxcnt + 3) >> 2;   // lane (seg, col) holds taps q = seg + 4i of output col
        const int64_t boff = (int64_t)t * a.nkb * 192;
        // Compact layout (ipp.h, ipp_plan_mfma_tile): the 16 outputs' nonzero
        // 16-column groups g0 .. g0 + len - 1, packed at base = the sum of the
        // earlier outputs' len.
        const bool cval = valid && cnt > 0;
        const int g0 = cval ? (xs - K0) >> 4 : 0;
        const int glen = cval ? ((xs + cnt - 1 - K0) >> 4) - g0 + 1 : 0;
        int gbase = 0, nb = 0;
        for (int c = 0; c < 16; ++c) {
            const int lc = __shfl(glen, c);
            gbase += c < col ? lc : 0;
            nb += lc;
        }
        const bool compact = a.compact && !a.identity && nK >= 2 && nb <= 64;  // wave-uniform
        if (lane == 0) *reinterpret_cast<int4*>(hdr + 4 * t) = make_int4(K0, nK, (int)boff, compact ? 1 : 0);

        // ---- filter weights: lane (seg, col) evaluates taps seg + 4i --------
        double ww = 0.0;
        if (!a.identity) {
            for (int i = 0; i < min(niter, TAP_NI); ++i) {
                const int q = 4 * i + seg;
                if (q < cnt) wc[col * TAP_CACHE + q] = d_weight(q, xmin, center, ss);
            }
            wave_sync();
            if (seg == 0 && valid) {  // Pillow's running sum, in tap order
                for (int q = 0; q < cnt; ++q)
                    ww += q < TAP_CACHE ? wc[col * TAP_CACHE + q] : d_weight(q, xmin, center, ss);
            }
            ww = __shfl(ww, col);
        }

        // ---- quantised taps: per lane its K indices and packed byte planes --
        const double rww = ww != 0.0 ? 1.0 / ww : 1.0;  // (a few ulps from v / ww: see d_sinpi)
        int32_t kx[TAP_NI];                     // K index rel. K0 (-1: none)
        uint32_t pb[TAP_NI];                    // balanced signed bytes of the three planes
        int64_t sum = 0;
        bool near = false;
        auto pack = [](int32_t k) {
            uint32_t b = 0;
            int32_t r = k;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const int32_t lo = ((r + 128) & 255) - 128;
                b |= (uint32_t)(lo & 255) << (8 * p);
                r = (r - lo) >> 8;
            }
            return b;
        };
#pragma unroll
        for (int i = 0; i < TAP_NI; ++i) {
            const int q = 4 * i + seg;
            kx[i] = -1;
            pb[i] = 0;
            if (i < niter && q < cnt) {
                const int32_t k = a.identity ? (1 << 22) : d_quant(wc[col * TAP_CACHE + q], rww, near);
                sum += k;
                kx[i] = xs + q - K0;
                pb[i] = pack(k);
            }
        }
        for (int i = TAP_NI; i < niter; ++i) {  // beyond the register set (scale > 10.5): recomputed
            const int q = 4 * i + seg;
            if (q < cnt) sum += d_quant(d_weight(q, xmin, center, ss), rww, near);
        }
        wave_sync();                            // the staging area reuses the cache

        // ---- assemble the blocks in LDS, window by window, then store ------
        const int sw = compact ? nK : TAP_STAGE_K;
        for (int s0 = 0; s0 < nK; s0 += sw) {
            const int nu = compact ? 196 : 192 * min(sw, nK - s0);
            for (int u = lane; u < nu; u += 64) stage4[u] = make_uint4(0u, 0u, 0u, 0u);
            if (compact && seg == 0) reinterpret_cast<int32_t*>(stage)[col] = g0 | glen << 8 | gbase << 16;
            wave_sync();
            auto put = [&](int kidx, uint32_t b) {
                asm volatile("" : "+v"(kidx));  // per window: nothing of it hoisted out of the window loop
                if (kidx < 0 || (!compact && ((kidx >> 6) < s0 || (kidx >> 6) >= s0 + sw))) return;
                // planes 64 uint4 (1 KB) apart in both layouts
                uint8_t* d = stage + stage_byte(compact, kidx, 0, col, s0, g0, gbase);
                d[0] = (uint8_t)b;
                d[1024] = (uint8_t)(b >> 8);
                d[2048] = (uint8_t)(b >> 16);
            };
#pragma unroll
            for (int i = 0; i < TAP_NI; ++i)
                if (i < niter) put(kx[i], pb[i]);
            wave_sync();
            for (int u = lane; u < nu; u += 64) blk[boff + 192 * (int64_t)s0 + u] = stage4[u];
            wave_sync();                        // the next window / tile rewrites the area
        }
        if (niter > TAP_NI) {
            // taps past the register set (scale > 10.5): recomputed and stored
            // as bytes over the zeros just written, at stage_byte's position for
            // the tile's layout — compact too (a partial last tile whose few
            // long-filter outputs keep ≤ 64 nonzero groups over nK ≥ 2 steps)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            uint8_t* tile = reinterpret_cast<uint8_t*>(blk + boff);
            for (int i = TAP_NI; i < niter; ++i) {
                const int q = 4 * i + seg;
                bool nr = false;
                if (q >= cnt) continue;
                const int kidx = xs + q - K0;
                if ((kidx >> 6) >= nK) continue;
                const uint32_t b = pack(d_quant(d_weight(q, xmin, center, ss), rww, nr));
                uint8_t* d = tile + stage_byte(compact, kidx, 0, col, 0, g0, gbase);
                d[0] = (uint8_t)b;
                d[1024] = (uint8_t)(b >> 8);
                d[2048] = (uint8_t)(b >> 16);
            }
        }
        if (compact)  // the zero tail of the tile's area
            for (int u = 196 + lane; u < nK * 192; u += 64) blk[boff + u] = make_uint4(0u, 0u, 0u, 0u);

        sum += __shfl_xor((long long)sum, 16);
        sum += __shfl_xor((long long)sum, 32);
        if (seg == 0) bias[16 * t + col] = valid ? (int32_t)((1 << 21) + 128 * sum) : 0;
        if (__any(near) && lane == 0) {
            const int idx = atomicAdd(ctl, 1);
            if (idx < TAP_FLAG_CAP) flags[idx] = make_int2((int)blockIdx.x, t);
        }
    }
}

inline int64_t align256(int64_t x) { return (x + 255) / 256 * 256; }

// Host-rebuilt tiles are uploaded in one packed copy and put in place by one
// launch (instead of two small pageable copies per tile, which cost ≈ 0.1 ms
// each).  Pack: int64 count, int64 record offsets, then per record
// {int64 bias word offset, int64 block word offset, int64 block bytes, pad},
// 16 bias words and the blocks, every record 16-byte aligned.
constexpr int64_t TAP_PACK_BYTES = 4 << 20;

__global__ __launch_bounds__(256) void k_put_tiles(const uint8_t* __restrict__ pack, int32_t* __restrict__ coefs) {
    const int64_t* hdr = reinterpret_cast<const int64_t*>(pack);
    const uint8_t* rec = pack + hdr[1 + blockIdx.x];
    const int64_t* m = reinterpret_cast<const int64_t*>(rec);
    const uint4* b = reinterpret_cast<const uint4*>(rec + 32);
    if (threadIdx.x < 4) reinterpret_cast<uint4*>(coefs + m[0])[threadIdx.x] = b[threadIdx.x];
    uint4* d = reinterpret_cast<uint4*>(coefs + m[1]);
    for (int64_t i = threadIdx.x; i < m[2] / 16; i += 256) d[i] = b[4 + i];
}

}  // namespace

extern "C" int64_t ipp_pipe_taps_scratch_bytes(int32_t n_axes) {
    if (n_axes <= 0) return IPP_E_ARG;
    return align256((int64_t)n_axes * (int64_t)sizeof(ipp_tap_axis)) + 256 + 8 * (int64_t)TAP_FLAG_CAP + TAP_PACK_BYTES;
}

extern "C" int ipp_pipe_plan_taps_cap(const ipp_tap_axis* axes, int32_t n_axes, int32_t* coefs, void* scratch,
                                      int64_t* stats, int64_t pack_cap, void* stream) {
    if (pack_cap < 0 || pack_cap > TAP_PACK_BYTES) return IPP_E_ARG;
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
    // one packed upload + one launch when the rebuilt tiles fit the pack region
    std::vector<int64_t> recoff(fl.size());
    int64_t pbytes = (8 * (1 + (int64_t)fl.size()) + 15) & ~(int64_t)15;
    for (size_t i = 0; i < fl.size(); ++i) {
        recoff[i] = pbytes;
        pbytes += 32 + 64 + (int64_t)hdrs[4 * i + 1] * 3072;
    }
    std::vector<uint8_t> pack;
    if (pbytes <= pack_cap) {
        pack.assign((size_t)pbytes, 0);
        int64_t* ph = reinterpret_cast<int64_t*>(pack.data());
        ph[0] = (int64_t)fl.size();
        for (size_t i = 0; i < fl.size(); ++i) {
            const ipp_tap_axis& a = axes[fl[i].x];
            const int t = fl[i].y;
            ph[1 + i] = recoff[i];
            int64_t* m = reinterpret_cast<int64_t*>(pack.data() + recoff[i]);
            m[0] = a.coef_off + 4 * (int64_t)a.n_tiles + 16 * t;
            m[1] = a.coef_off + 20 * (int64_t)a.n_tiles + 4 * (int64_t)hdrs[4 * i + 2];
            m[2] = (int64_t)hdrs[4 * i + 1] * 3072;
            memcpy(pack.data() + recoff[i] + 32, bias.data() + 16 * i, 64);
            memcpy(pack.data() + recoff[i] + 96, blocks.data() + i * (size_t)maxnk * 3072, (size_t)m[2]);
        }
        uint8_t* d_pack = reinterpret_cast<uint8_t*>(d_flags + TAP_FLAG_CAP);
        if (hipMemcpyAsync(d_pack, pack.data(), (size_t)pbytes, hipMemcpyHostToDevice, s) != hipSuccess) {
            rc = IPP_E_LAUNCH;
        } else {
            hipLaunchKernelGGL(k_put_tiles, dim3((uint32_t)fl.size()), dim3(256), 0, s, d_pack, coefs);
            if (hipGetLastError() != hipSuccess) rc = IPP_E_LAUNCH;
        }
    } else {
        for (size_t i = 0; i < fl.size() && rc == IPP_OK; ++i) {
            const ipp_tap_axis& a = axes[fl[i].x];
            const int t = fl[i].y;
            const int32_t* hdr = hdrs.data() + 4 * i;
            int32_t* base = coefs + a.coef_off;
            if (hipMemcpyAsync(base + 4 * (int64_t)a.n_tiles + 16 * t, bias.data() + 16 * i, 64,
                               hipMemcpyHostToDevice, s) != hipSuccess ||
                hipMemcpyAsync(base + 20 * (int64_t)a.n_tiles + 4 * (int64_t)hdr[2],
                               blocks.data() + i * (size_t)maxnk * 3072, (size_t)hdr[1] * 3072, hipMemcpyHostToDevice,
                               s) != hipSuccess)
                rc = IPP_E_LAUNCH;
        }
    }
    if (hipStreamSynchronize(s) != hipSuccess) return IPP_E_LAUNCH;
    return rc;
}

extern "C" int ipp_pipe_plan_taps(const ipp_tap_axis* axes, int32_t n_axes, int32_t* coefs, void* scratch,
                                  int64_t* stats, void* stream) {
    return ipp_pipe_plan_taps_cap(axes, n_axes, coefs, scratch, stats, TAP_PACK_BYTES, stream);
}
