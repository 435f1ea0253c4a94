// ipp_host.cpp — host-side planning for the hot path (CPU, C ABI).
//
// These functions reproduce the HOST arithmetic of the libraries the
// reference calls, so the device kernels receive the exact integers Pillow
// would use:
//   * ipp_plan_lanczos: Pillow Resample.c precompute_coeffs +
//     normalize_coeffs_8bpc for the LANCZOS filter (support 3, sinc·sinc/3,
//     double precision, the same libm sin()), PRECISION_BITS = 22 — the taps
//     behind overlays.py:129.
//   * ipp_plan_opaque_bbox: the getbbox() of rotations.py:99 for an opaque
//     source, solved per canvas row from the 16.16 affine map with exact
//     integer inequalities (no canvas is materialised).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "ipp.h"

namespace {

inline double sinc_filter(double x) {
    if (x == 0.0) return 1.0;
    x = x * M_PI;
    return sin(x) / x;
}

inline double lanczos_filter(double x) {
    if (-3.0 <= x && x < 3.0) return sinc_filter(x) * sinc_filter(x / 3);
    return 0.0;
}

inline int ksize_of(double in0, double in1, int out_size) {
    const double scale = (double)((float)in1 - (float)in0) / out_size;
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 3.0 * filterscale;
    return (int)ceil(support) * 2 + 1;
}

// floor(a / b) and ceil(a / b) for b != 0 (int64).
inline int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b, r = a % b;
    return (r != 0 && ((r < 0) != (b < 0))) ? q - 1 : q;
}
inline int64_t ceildiv(int64_t a, int64_t b) { return -floordiv(-a, b); }

// X range where lo <= c + X*a <= hi (inclusive); returns false if empty.
inline bool solve_range(int64_t c, int64_t a, int64_t lo, int64_t hi, int64_t& xlo, int64_t& xhi) {
    if (a == 0) {
        if (c < lo || c > hi) return false;
        xlo = INT64_MIN / 4;
        xhi = INT64_MAX / 4;
        return true;
    }
    if (a > 0) {
        xlo = ceildiv(lo - c, a);
        xhi = floordiv(hi - c, a);
    } else {
        xlo = ceildiv(hi - c, a);
        xhi = floordiv(lo - c, a);
    }
    return xlo <= xhi;
}

}  // namespace

extern "C" int32_t ipp_plan_lanczos_ksize(double in0, double in1, int32_t out_size) {
    if (out_size <= 0) return IPP_E_ARG;
    return ksize_of(in0, in1, out_size);
}

namespace {
// One output of Resample.c precompute_coeffs + normalize_coeffs_8bpc: its
// bounds and its `ksize` quantised taps (zero past the support).
inline void lanczos_one(int32_t in_size, float fin0, double scale, double support, double ss, int xx, int ksize,
                        double* k, int32_t* kq, int& xmin_out, int& cnt_out) {
    const double center = fin0 + (xx + 0.5) * scale;
    double ww = 0.0;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    for (int x = 0; x < xmax; ++x) {
        const double w = lanczos_filter((x + xmin - center + 0.5) * ss);
        k[x] = w;
        ww += w;
    }
    for (int x = 0; x < xmax; ++x)
        if (ww != 0.0) k[x] /= ww;
    for (int x = 0; x < ksize; ++x) {
        const double v = x < xmax ? k[x] : 0.0;
        kq[x] = v < 0 ? (int32_t)(-0.5 + v * (1 << 22)) : (int32_t)(0.5 + v * (1 << 22));
    }
    xmin_out = xmin;
    cnt_out = xmax;
}
}  // namespace

extern "C" int64_t ipp_plan_lanczos(int32_t in_size, double in0, double in1, int32_t out_size, int32_t* out,
                                    int64_t out_capacity) {
    if (in_size <= 0 || out_size <= 0) return IPP_E_ARG;
    const float fin0 = (float)in0, fin1 = (float)in1;  // Resample.c takes float box[4]
    const double scale = (double)(fin1 - fin0) / out_size;
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 3.0 * filterscale;
    const int ksize = (int)ceil(support) * 2 + 1;
    const int64_t need = 2 * (int64_t)out_size + (int64_t)out_size * ksize;
    if (out == nullptr) return -need;
    if (out_capacity < need) return IPP_E_ARG;
    int32_t* bounds = out;
    int32_t* kk = out + 2 * (int64_t)out_size;
    std::vector<double> k(ksize);
    const double ss = 1.0 / filterscale;
    for (int xx = 0; xx < out_size; ++xx) {
        int xmin, cnt;
        lanczos_one(in_size, fin0, scale, support, ss, xx, ksize, k.data(), kk + (int64_t)xx * ksize, xmin, cnt);
        bounds[2 * xx] = xmin;
        bounds[2 * xx + 1] = cnt;
    }
    return ksize;
}

// Batch planner: n independent axes, written at int32 offsets; threads split
// the list.  Returns 0 or the first error.
extern "C" int ipp_plan_lanczos_batch(int32_t n, const int32_t* in_sizes, const int32_t* out_sizes,
                                      const int64_t* offsets, int32_t* out, int64_t out_capacity,
                                      int32_t n_threads) {
    if (n < 0 || (n > 0 && (!in_sizes || !out_sizes || !offsets || !out))) return IPP_E_ARG;
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min(nt, 64));
    std::vector<int> err(nt, 0);
    auto work = [&](int t) {
        for (int i = t; i < n; i += nt) {
            const int64_t r = ipp_plan_lanczos(in_sizes[i], 0.0, (double)in_sizes[i], out_sizes[i], out + offsets[i],
                                               out_capacity - offsets[i]);
            if (r < 0) err[t] = (int)r;
        }
    };
    if (nt == 1 || n < 64) {
        nt = 1;
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
        for (auto& x : th) x.join();
    }
    for (int e : err)
        if (e) return e;
    return IPP_OK;
}

extern "C" int ipp_plan_opaque_bbox(int32_t in_w, int32_t in_h, const int32_t a[6], int32_t nw, int32_t nh,
                                    int32_t bbox[4]) {
    if (in_w <= 0 || in_h <= 0 || nw <= 0 || nh <= 0 || !a || !bbox) return IPP_E_ARG;
    int64_t x0 = INT64_MAX, x1 = -1, y0 = INT64_MAX, y1 = -1;
    const int64_t ux = (int64_t)in_w * 65536 - 1, uy = (int64_t)in_h * 65536 - 1;
    for (int64_t Y = 0; Y < nh; ++Y) {
        const int64_t cx = (int64_t)a[2] + Y * a[1];
        const int64_t cy = (int64_t)a[5] + Y * a[4];
        int64_t lo1, hi1, lo2, hi2;
        if (!solve_range(cx, a[0], 0, ux, lo1, hi1)) continue;
        if (!solve_range(cy, a[3], 0, uy, lo2, hi2)) continue;
        const int64_t lo = std::max<int64_t>(std::max(lo1, lo2), 0);
        const int64_t hi = std::min<int64_t>(std::min(hi1, hi2), nw - 1);
        if (lo > hi) continue;
        x0 = std::min(x0, lo);
        x1 = std::max(x1, hi);
        y0 = std::min(y0, Y);
        y1 = std::max(y1, Y);
    }
    if (x1 < 0) {
        bbox[0] = bbox[1] = bbox[2] = bbox[3] = -1;
    } else {
        bbox[0] = (int32_t)x0;
        bbox[1] = (int32_t)y0;
        bbox[2] = (int32_t)x1 + 1;
        bbox[3] = (int32_t)y1 + 1;
    }
    return IPP_OK;
}

extern "C" const char* ipp_version(void) { return "ipp 0.1.0 (gfx950)"; }

// The gather sampler of ipp_sampler.h make_sampler, once per image on the
// host (rotations.py:96 affine with symmetry.py:114-119's flip and the bbox
// crop of :99-101 folded in; 32-bit wrap-around as in the kernels).
extern "C" int ipp_gather_prepare(ipp_gather_desc* descs, int32_t n) {
    if (n < 0 || (n > 0 && !descs)) return IPP_E_ARG;
    for (int32_t i = 0; i < n; ++i) {
        ipp_gather_desc& g = descs[i];
        g.base_off = g.src_off + (int64_t)g.in_y0 * g.src_pitch + (int64_t)g.in_x0 * g.src_cn;
        const int64_t avail = (int64_t)(g.src_h - g.in_y0) * g.src_pitch - (int64_t)g.in_x0 * g.src_cn;
        g.lim = (uint32_t)(avail - 4);
        const uint32_t sgx = (g.flip & 1) ? 0xFFFFFFFFu : 1u, sgy = (g.flip & 2) ? 0xFFFFFFFFu : 1u;
        const uint32_t sx0 = (uint32_t)(g.off_x + ((g.flip & 1) ? g.out_w - 1 : 0));
        const uint32_t sy0 = (uint32_t)(g.off_y + ((g.flip & 2) ? g.out_h - 1 : 0));
        g.b[0] = (int32_t)(sgx * (uint32_t)g.a0);
        g.b[1] = (int32_t)(sgy * (uint32_t)g.a1);
        g.b[2] = (int32_t)((uint32_t)g.a2 + sy0 * (uint32_t)g.a1 + sx0 * (uint32_t)g.a0);
        g.b[3] = (int32_t)(sgx * (uint32_t)g.a3);
        g.b[4] = (int32_t)(sgy * (uint32_t)g.a4);
        g.b[5] = (int32_t)((uint32_t)g.a5 + sy0 * (uint32_t)g.a4 + sx0 * (uint32_t)g.a3);
        g.prepared = 1;
    }
    return IPP_OK;
}

// Balanced signed bytes of a 22-bit tap: k = b0 + 256 b1 + 65536 b2, each
// b in [-128, 127] (the MFMA tile format below).
namespace {

inline void balanced_bytes(int32_t k, int8_t b[3]) {
    int32_t r = k;
    for (int p = 0; p < 3; ++p) {
        int32_t lo = ((r + 128) & 255) - 128;
        b[p] = (int8_t)lo;
        r = (r - lo) >> 8;
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// MFMA tile format (fused pipe, v_mfma_i32_16x16x64_i8).  Outputs are grouped
// in tiles of 16, tile t covering outputs [16t - phase, 16t - phase + 16) ∩
// [0, out) (phase lets the V pass align tiles with 16-row background bands);
// input indices are shifted by `shift` (the V pass's ybox_first).  For tile t:
//   hdr[t]  = (K0, nK, boff, 0)   K0 = first input column of the tile rounded
//                                 down to 16, nK = 64-column K steps, boff =
//                                 uint4 index of the tile's B blocks
//   bias[16t + c] = 2^21 + 128·Σk of the tile's output c (0 for padding)
//   block (s, p), s < nK, p < 3: 64 lanes × 16 B; lane l holds bytes
//           j = 0..15 = balanced byte p of the tap of the tile's output l&15
//           at input K0 + 64s + 16(l>>4) + j (0 outside its support).  This is
//           the B operand B[k][col] of the H pass and, unchanged, the A
//           operand A[row][k] of the V pass (same lane map).
// so that with pixels stored XOR 0x80 the i8 MFMA accumulators give
//   2^21 + Σ p·k = bias + Σ_p 2^(8p) acc_p   exactly.
// Layout per axis (int32 units): hdr[4T], bias[16T], blocks (4 int32 each).
// ---------------------------------------------------------------------------
namespace {
inline int mfma_nk_bound(int32_t in_size, int32_t out_size, int32_t ksize) {
    const double scale = (double)in_size / (double)out_size;
    return (int)((16 + (int64_t)ceil(15.0 * scale) + 2 + ksize + 63) / 64);
}
}  // namespace

extern "C" int64_t ipp_plan_mfma_size(int32_t in_size, int32_t out_size, int32_t ksize) {
    if (in_size <= 0 || out_size <= 0 || ksize <= 0) return IPP_E_ARG;
    const int64_t T = (out_size + 15) / 16 + 1;  // + 1: a phase may add a tile
    return 20 * T + T * mfma_nk_bound(in_size, out_size, ksize) * 3 * 64 * 4;
}

extern "C" int32_t ipp_plan_mfma_nk_bound(int32_t in_size, int32_t out_size, int32_t ksize) {
    if (in_size <= 0 || out_size <= 0 || ksize <= 0) return IPP_E_ARG;
    return mfma_nk_bound(in_size, out_size, ksize);
}

extern "C" int ipp_plan_mfma_from_taps(int32_t in_size, int32_t out_size, int32_t ksize, const int32_t* std_taps,
                                       int32_t shift, int32_t phase, int32_t* out) {
    if (in_size <= 0 || out_size <= 0 || ksize <= 0 || !std_taps || !out || phase < 0 || phase > 15)
        return IPP_E_ARG;
    const int T = (out_size + phase + 15) / 16;
    const int nkb = mfma_nk_bound(in_size, out_size, ksize);
    const int32_t* bounds = std_taps;
    const int32_t* kk = std_taps + 2 * (int64_t)out_size;
    int32_t* hdr = out;
    int32_t* bias = out + 4 * (int64_t)T;
    uint8_t* blocks = reinterpret_cast<uint8_t*>(out + 20 * (int64_t)T);
    int64_t boff = 0;  // in uint4 units
    for (int t = 0; t < T; ++t) {
        const int o0 = 16 * t - phase, o1 = std::min(o0 + 16, (int)out_size), oa = std::max(o0, 0);
        if (bounds[2 * oa] - shift < 0) return IPP_E_RANGE;
        const int K0 = (bounds[2 * oa] - shift) & ~15;
        int end = K0;
        for (int o = oa; o < o1; ++o) end = std::max(end, bounds[2 * o] - shift + bounds[2 * o + 1]);
        const int nK = (end - K0 + 63) / 64;
        if (nK > nkb) return IPP_E_RANGE;
        hdr[4 * t] = K0;
        hdr[4 * t + 1] = nK;
        hdr[4 * t + 2] = (int32_t)boff;
        hdr[4 * t + 3] = 0;
        uint8_t* tb = blocks + 16 * boff;
        memset(tb, 0, (size_t)nK * 3 * 64 * 16);
        for (int col = 0; col < 16; ++col) {
            const int o = o0 + col;
            if (o < oa || o >= o1) {
                bias[16 * t + col] = 0;
                continue;
            }
            const int xmin = bounds[2 * o] - shift, cnt = bounds[2 * o + 1];
            int64_t sum = 0;
            for (int q = 0; q < cnt; ++q) {
                const int32_t k = kk[(int64_t)o * ksize + q];
                sum += k;
                int8_t b[3];
                balanced_bytes(k, b);
                const int rel = xmin + q - K0, s = rel / 64, kin = rel % 64;
                const int lane = 16 * (kin / 16) + col, j = kin % 16;
                for (int p = 0; p < 3; ++p) tb[((int64_t)(s * 3 + p) * 64 + lane) * 16 + j] = (uint8_t)b[p];
            }
            bias[16 * t + col] = (int32_t)((1 << 21) + 128 * sum);
        }
        boff += (int64_t)nK * 3 * 64;
    }
    return IPP_OK;
}

// One tile of an axis in the layout of the device tap planner (tile t's
// blocks at uint4 offset t·nkb·192), from Pillow's taps computed here.
extern "C" int ipp_plan_mfma_tile(const ipp_tap_axis* a, int32_t t, int32_t hdr[4], int32_t bias[16],
                                  uint8_t* blocks, int64_t blocks_cap) {
    if (!a || !hdr || !bias || !blocks || a->in_size <= 0 || a->out_size <= 0 || a->phase < 0 || a->phase > 15 ||
        t < 0 || t >= (a->out_size + a->phase + 15) / 16)
        return IPP_E_ARG;
    const int in = a->in_size, out = a->out_size, shift = a->shift;
    const int o0 = 16 * t - a->phase, o1 = std::min(o0 + 16, out), oa = std::max(o0, 0);
    const float fin0 = 0.0f, fin1 = (float)in;
    const double scale = (double)(fin1 - fin0) / out;
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 3.0 * filterscale, ss = 1.0 / filterscale;
    const int ksize = a->identity ? 1 : (int)ceil(support) * 2 + 1;
    std::vector<double> kd(ksize);
    std::vector<int32_t> kq(16 * (size_t)ksize);
    int xs[16], cn[16];
    for (int o = oa; o < o1; ++o) {
        const int c = o - o0;
        if (a->identity) {
            xs[c] = o;
            cn[c] = 1;
            kq[(size_t)c * ksize] = 1 << 22;
        } else {
            lanczos_one(in, fin0, scale, support, ss, o, ksize, kd.data(), kq.data() + (size_t)c * ksize, xs[c],
                        cn[c]);
        }
        xs[c] -= shift;
    }
    if (xs[oa - o0] < 0) return IPP_E_RANGE;
    const int K0 = xs[oa - o0] & ~15;
    int end = K0;
    for (int o = oa; o < o1; ++o) end = std::max(end, xs[o - o0] + cn[o - o0]);
    const int nK = (end - K0 + 63) / 64;
    if (nK > a->nkb || (int64_t)nK * 3072 > blocks_cap) return IPP_E_RANGE;
    // compact layout (ipp.h): each output's nonzero 16-column groups
    int g0[16], len[16], base[16], nb = 0;
    for (int col = 0; col < 16; ++col) {
        const int o = o0 + col;
        const bool valid = o >= oa && o < o1 && cn[col] > 0;
        g0[col] = valid ? (xs[col] - K0) >> 4 : 0;
        len[col] = valid ? ((xs[col] + cn[col] - 1 - K0) >> 4) - g0[col] + 1 : 0;
        base[col] = nb;
        nb += len[col];
    }
    const bool compact = a->compact && !a->identity && nK >= 2 && nb <= 64;
    hdr[0] = K0;
    hdr[1] = nK;
    hdr[2] = t * a->nkb * 192;
    hdr[3] = compact ? 1 : 0;
    memset(blocks, 0, (size_t)nK * 3072);
    if (compact)
        for (int col = 0; col < 16; ++col) {
            const int32_t m = g0[col] | len[col] << 8 | base[col] << 16;
            memcpy(blocks + 4 * col, &m, 4);
        }
    for (int col = 0; col < 16; ++col) {
        const int o = o0 + col;
        if (o < oa || o >= o1) {
            bias[col] = 0;
            continue;
        }
        int64_t sum = 0;
        for (int q = 0; q < cn[col]; ++q) {
            const int32_t k = kq[(size_t)col * ksize + q];
            sum += k;
            int8_t b[3];
            balanced_bytes(k, b);
            const int rel = xs[col] + q - K0;
            if (compact) {
                const int i = base[col] + (rel >> 4) - g0[col], j = rel & 15;
                for (int p = 0; p < 3; ++p) blocks[64 + ((int64_t)p * 64 + i) * 16 + j] = (uint8_t)b[p];
            } else {
                const int s = rel / 64, kin = rel % 64;
                const int lane = 16 * (kin / 16) + col, j = kin % 16;
                for (int p = 0; p < 3; ++p) blocks[((int64_t)(s * 3 + p) * 64 + lane) * 16 + j] = (uint8_t)b[p];
            }
        }
        bias[col] = (int32_t)((1 << 21) + 128 * sum);
    }
    return IPP_OK;
}

// Plan every axis of a pipe batch in the MFMA tile format.  Axis i resamples
// in_sizes[i] → out_sizes[i]; identity[i] != 0 encodes "no pass on this axis"
// (single 2^22 tap).  For axes with shift_first[i] != 0 the Pillow bounds are
// shifted by their first xmin (ybox_first).  first_last[2i..2i+1] receives
// (ybox_first, ybox_last) of the unshifted bounds.  format[i] = 2 + phase
// (IPP_TAPS_MFMA tiles, tile phase 0..15; any other value: IPP_E_ARG);
// offsets[i] = int32 offset of the axis block in `out`, sized by
// ipp_plan_mfma_size.
extern "C" int ipp_plan_pipe_axes(int32_t n, const int32_t* in_sizes, const int32_t* out_sizes,
                                  const int32_t* identity, const int32_t* shift_first, const int32_t* transposed,
                                  const int64_t* offsets, int32_t* out, int32_t* first_last, int32_t n_threads) {
    if (n < 0 || (n > 0 && (!in_sizes || !out_sizes || !identity || !shift_first || !transposed || !offsets || !out ||
                            !first_last)))
        return IPP_E_ARG;
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min(nt, 64));
    if (n < 64) nt = 1;
    std::vector<int> err(nt, 0);
    auto work = [&](int t) {
        std::vector<int32_t> tmp;
        for (int i = t; i < n; i += nt) {
            const int in = in_sizes[i], o = out_sizes[i];
            int ksize;
            if (identity[i]) {
                ksize = 1;
                tmp.assign(3 * (size_t)o, 0);
                for (int x = 0; x < o; ++x) {
                    tmp[2 * x] = x;
                    tmp[2 * x + 1] = 1;
                    tmp[2 * (size_t)o + x] = 1 << 22;
                }
            } else {
                ksize = ipp_plan_lanczos_ksize(0.0, (double)in, o);
                tmp.assign(2 * (size_t)o + (size_t)o * ksize, 0);
                const int64_t r = ipp_plan_lanczos(in, 0.0, (double)in, o, tmp.data(), (int64_t)tmp.size());
                if (r < 0) { err[t] = (int)r; continue; }
            }
            const int first = tmp[0], last = tmp[2 * (o - 1)] + tmp[2 * (o - 1) + 1];
            first_last[2 * i] = first;
            first_last[2 * i + 1] = last;
            const int e = transposed[i] >= 2
                              ? ipp_plan_mfma_from_taps(in, o, ksize, tmp.data(), shift_first[i] ? first : 0,
                                                        transposed[i] - 2, out + offsets[i])
                              : IPP_E_ARG;
            if (e) err[t] = e;
        }
    };
    if (nt == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
        for (auto& x : th) x.join();
    }
    for (int e : err)
        if (e) return e;
    return IPP_OK;
}
