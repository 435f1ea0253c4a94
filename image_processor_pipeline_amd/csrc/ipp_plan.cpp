// ipp_plan.cpp — batch planner of the fused pipe (host, C ABI, threaded).
//
// One call plans a whole batch of the 5-stage pipe: every random draw of the
// reference's chained file-mode pipeline, in its order, with CPython's own
// generator (MT19937 + random.py's uniform / randint / shuffle / sample), the
// per-item geometry (PIL rotate(expand=True), getbbox of the opaque rotated
// crop, the overlay size of overlays.py:106-126), the pipe descriptors and the
// per-axis records of the device tap planner (ipp_pipe_plan_taps).  The LANCZOS
// taps themselves are not computed here: they are built on the device.
//
// Reference call sites (draw order, pipeline.py:555-566 step-major):
//   rotations.py:89  uniform(angle_min, angle_max)     one per file, all files
//   symmetry.py:122  sample(pool, 1)                  one per file, all files
//   pipeline.py:202  shuffle(backgrounds)             once ('modulo' pairing)
//   overlays.py:108  uniform(scale_min, scale_max)    per item
//   overlays.py:133-134  randint(0, bw - w), randint(0, bh - h)
// Geometry: rotations.py:96-109 (Pillow 12.2.0 Image.rotate, Geometry.c),
// overlays.py:106-126.  The Python restatement of the same plan is
// fused.draw_params / item_geometry / geometry.py (tests cross-check both).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <thread>
#include <vector>

#include "ipp.h"

namespace {

// ---------------------------------------------------------------------------
// CPython 3.10 random: Modules/_randommodule.c (MT19937, init_by_array,
// genrand_res53) and Lib/random.py (uniform, _randbelow_with_getrandbits,
// randrange fast path, shuffle, sample's pool branch).
// ---------------------------------------------------------------------------
struct PyRandom {
    uint32_t mt[624];
    int idx = 625;

    void init_genrand(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        idx = 624;
    }
    void init_by_array(const uint32_t* key, int len) {
        init_genrand(19650218u);
        int i = 1, j = 0;
        for (int k = std::max(624, len); k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
            ++i;
            ++j;
            if (i >= 624) { mt[0] = mt[623]; i = 1; }
            if (j >= len) j = 0;
        }
        for (int k = 623; k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
            ++i;
            if (i >= 624) { mt[0] = mt[623]; i = 1; }
        }
        mt[0] = 0x80000000u;
    }
    // random.seed(n) for an int n: the key is |n| as little-endian 32-bit words.
    void seed(uint64_t mag) {
        uint32_t key[2] = {(uint32_t)mag, (uint32_t)(mag >> 32)};
        init_by_array(key, key[1] ? 2 : 1);
    }
    uint32_t genrand() {
        if (idx >= 624) {
            static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
            int kk;
            for (kk = 0; kk < 624 - 397; ++kk) {
                const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
                mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
            }
            for (; kk < 623; ++kk) {
                const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
                mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
            }
            const uint32_t y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
            mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
            idx = 0;
        }
        uint32_t y = mt[idx++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    double random() {  // genrand_res53
        const uint32_t a = genrand() >> 5, b = genrand() >> 6;
        return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
    }
    double uniform(double a, double b) { return a + (b - a) * random(); }
    uint32_t getrandbits(int k) { return genrand() >> (32 - k); }  // 1 <= k <= 32
    uint32_t randbelow(uint32_t n) {                               // n >= 1
        const int k = 32 - __builtin_clz(n);
        uint32_t r = getrandbits(k);
        while (r >= n) r = getrandbits(k);
        return r;
    }
};

// ---------------------------------------------------------------------------
// Geometry (geometry.py restated; Python float semantics on x86-64 doubles).
// ---------------------------------------------------------------------------
constexpr int32_t FIX_ONE = 65536, HALF = 32768;

enum PlanErr { E_OK = 0, E_CANVAS = 1, E_SCALE_AFFINE = 2, E_OVERLAY = 3, E_FIT = 4, E_RING = 5, E_EMPTY = 6 };

struct Rot {
    int32_t nw, nh;
    int32_t A[6];
};

double py_round15(double x) {  // round(x, 15): correctly rounded decimal, back to double
    char buf[64];
    snprintf(buf, sizeof buf, "%.15f", x);
    return strtod(buf, nullptr);
}

double py_mod360(double x) {  // float.__mod__(x, 360.0)
    double m = fmod(x, 360.0);
    if (m != 0.0) {
        if (m < 0) m += 360.0;
    } else {
        m = 0.0;
    }
    return m;
}

int64_t py_fix(double v) { return (int64_t)floor(v * 65536.0 + 0.5); }

// geometry.rotation_plan (Pillow Image.rotate(angle, expand=True), NEAREST).
int rotation_plan(int32_t w, int32_t h, double angle, Rot& r) {
    angle = py_mod360(angle);
    if (angle == 0.0) {
        r = {w, h, {FIX_ONE, 0, HALF, 0, FIX_ONE, HALF}};
        return E_OK;
    }
    if (angle == 180.0) {
        r = {w, h, {-FIX_ONE, 0, (w - 1) * FIX_ONE + HALF, 0, -FIX_ONE, (h - 1) * FIX_ONE + HALF}};
        return E_OK;
    }
    if (angle == 90.0) {
        r = {h, w, {0, -FIX_ONE, (w - 1) * FIX_ONE + HALF, FIX_ONE, 0, HALF}};
        return E_OK;
    }
    if (angle == 270.0) {
        r = {h, w, {0, FIX_ONE, HALF, -FIX_ONE, 0, (h - 1) * FIX_ONE + HALF}};
        return E_OK;
    }
    const double cx = w / 2.0, cy = h / 2.0;
    const double a = -(angle * (M_PI / 180.0));  // math.radians
    double m[6] = {py_round15(cos(a)), py_round15(sin(a)), 0.0, py_round15(-sin(a)), py_round15(cos(a)), 0.0};
    auto tr = [&](double x, double y, double& ox, double& oy) {
        ox = m[0] * x + m[1] * y + m[2];
        oy = m[3] * x + m[4] * y + m[5];
    };
    double t2, t5;
    tr(-cx - 0, -cy - 0, t2, t5);
    m[2] = t2 + cx;
    m[5] = t5 + cy;
    const double px[4] = {0, (double)w, (double)w, 0}, py[4] = {0, 0, (double)h, (double)h};
    double xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
    for (int k = 0; k < 4; ++k) {
        double X, Y;
        tr(px[k], py[k], X, Y);
        xmin = std::min(xmin, X);
        xmax = std::max(xmax, X);
        ymin = std::min(ymin, Y);
        ymax = std::max(ymax, Y);
    }
    const int64_t nw = (int64_t)ceil(xmax) - (int64_t)floor(xmin);
    const int64_t nh = (int64_t)ceil(ymax) - (int64_t)floor(ymin);
    if (nw <= 0 || nh <= 0 || nw > INT32_MAX / 4 || nh > INT32_MAX / 4) return E_CANVAS;
    tr(-(double)(nw - w) / 2.0, -(double)(nh - h) / 2.0, t2, t5);
    m[2] = t2;
    m[5] = t5;
    r.nw = (int32_t)nw;
    r.nh = (int32_t)nh;
    if (m[1] == 0 && m[3] == 0) {
        // geometry._scale_affine_plan: ImagingScaleAffine's COORD() tables
        auto coords = [](double o, double step, int64_t n, std::vector<int64_t>& out) {
            out.resize(n);
            for (int64_t i = 0; i < n; ++i) {
                out[i] = o < 0.0 ? -1 : (int64_t)o;
                o += step;
            }
        };
        std::vector<int64_t> xt, yt;
        coords(m[2] + m[0] * 0.5, m[0], nw, xt);
        coords(m[5] + m[4] * 0.5, m[4], nh, yt);
        for (auto* t : {&xt, &yt}) {
            const auto& v = *t;
            if (v.size() > 1) {
                for (size_t i = 0; i + 1 < v.size(); ++i)
                    if (v[i + 1] - v[i] != v[1] - v[0]) return E_SCALE_AFFINE;
                if (llabs(v[1] - v[0]) != 1) return E_SCALE_AFFINE;
            }
        }
        const int64_t sx = nw > 1 ? xt[1] - xt[0] : 1, sy = nh > 1 ? yt[1] - yt[0] : 1;
        r.A[0] = (int32_t)(sx * FIX_ONE);
        r.A[1] = 0;
        r.A[2] = (int32_t)(xt[0] * FIX_ONE + HALF);
        r.A[3] = 0;
        r.A[4] = (int32_t)(sy * FIX_ONE);
        r.A[5] = (int32_t)(yt[0] * FIX_ONE + HALF);
        return E_OK;
    }
    const double cxs[4] = {0, (double)nw, 0, (double)nw}, cys[4] = {0, (double)nh, (double)nh, 0};
    for (int k = 0; k < 4; ++k) {
        const double x = cxs[k], y = cys[k];
        if (!(fabs(x * m[0] + y * m[1] + m[2]) < 32768.0 && fabs(x * m[3] + y * m[4] + m[5]) < 32768.0))
            return E_CANVAS;
    }
    const int64_t A[6] = {py_fix(m[0]), py_fix(m[1]), py_fix(m[2] + m[0] * 0.5 + m[1] * 0.5),
                          py_fix(m[3]), py_fix(m[4]), py_fix(m[5] + m[3] * 0.5 + m[4] * 0.5)};
    for (int k = 0; k < 6; ++k) {
        if (A[k] < INT32_MIN || A[k] > INT32_MAX) return E_CANVAS;
        r.A[k] = (int32_t)A[k];
    }
    return E_OK;
}

// floor(N / a) tracked along N += d (a > 0): division-free per step.
struct FloorTrack {
    int64_t q, r, a, dq, dr;
    static int64_t fdiv(int64_t n, int64_t a) {
        int64_t q = n / a, m = n % a;
        return (m != 0 && ((m < 0) != (a < 0))) ? q - 1 : q;
    }
    void init(int64_t n0, int64_t a_, int64_t d) {  // a_ > 0
        a = a_;
        q = fdiv(n0, a);
        r = n0 - q * a;
        dq = fdiv(d, a);
        dr = d - dq * a;
    }
    void step() {
        q += dq;
        r += dr;
        if (r >= a) { r -= a; ++q; }
    }
};

// The X range lo <= c + X*a <= hi of one row, for c = c0 + Y*dc, as Y steps.
struct RangeTrack {
    bool konst;       // a == 0
    bool ok_const;    // a == 0: whole row inside?
    int64_t c, dc, lo, hi;
    FloorTrack xlo_neg, xhi;  // xlo = -floor(...) (ceil), xhi = floor(...)
    void init(int64_t c0, int64_t dc_, int64_t a, int64_t lo_, int64_t hi_) {
        c = c0;
        dc = dc_;
        lo = lo_;
        hi = hi_;
        konst = a == 0;
        if (konst) return;
        // a > 0: xlo = ceil((lo - c)/a) = -floor((c - lo)/a), xhi = floor((hi - c)/a)
        // a < 0: xlo = ceil((hi - c)/a) = -floor((c - hi)/(-a)) ... written with a' = -a > 0:
        //        xlo = ceil((c - hi)/a') = -floor((hi - c)/a'), xhi = floor((c - lo)/a')
        if (a > 0) {
            xlo_neg.init(c0 - lo, a, dc);
            xhi.init(hi - c0, a, -dc);
        } else {
            xlo_neg.init(hi - c0, -a, -dc);
            xhi.init(c0 - lo, -a, dc);
        }
    }
    bool get(int64_t& xl, int64_t& xh) {
        if (konst) {
            if (c < lo || c > hi) return false;
            xl = INT64_MIN / 4;
            xh = INT64_MAX / 4;
            return true;
        }
        xl = -xlo_neg.q;
        xh = xhi.q;
        return xl <= xh;
    }
    void step() {
        if (konst) {
            c += dc;
            return;
        }
        xlo_neg.step();
        xhi.step();
    }
};

// getbbox() of the rotated canvas of an opaque in_w × in_h image
// (ipp_plan_opaque_bbox, incremental form).  bbox = (x0, y0, x1, y1) or -1s.
void opaque_bbox(int32_t in_w, int32_t in_h, const int32_t* a, int32_t nw, int32_t nh, int32_t bbox[4]) {
    int64_t x0 = INT64_MAX, x1 = -1, y0 = INT64_MAX, y1 = -1;
    const int64_t ux = (int64_t)in_w * 65536 - 1, uy = (int64_t)in_h * 65536 - 1;
    RangeTrack rx, ry;
    rx.init(a[2], a[1], a[0], 0, ux);
    ry.init(a[5], a[4], a[3], 0, uy);
    for (int64_t Y = 0; Y < nh; ++Y, rx.step(), ry.step()) {
        int64_t lo1, hi1, lo2, hi2;
        if (!rx.get(lo1, hi1) || !ry.get(lo2, hi2)) continue;
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
}

// CPython 3.10 math.hypot (Modules/mathmodule.c vector_norm, n = 2).
double py_hypot(double x, double y) {
    double vec[2] = {fabs(x), fabs(y)};
    const double mx = std::max(vec[0], vec[1]);
    if (isinf(mx)) return mx;
    if (isnan(vec[0]) || isnan(vec[1])) return NAN;
    if (mx == 0.0) return mx;
    const double T27 = 134217729.0;
    int max_e;
    frexp(mx, &max_e);
    if (max_e < -1023) return sqrt(vec[0] * vec[0] + vec[1] * vec[1]);  // not reached for pixel sizes
    const double scale = ldexp(1.0, -max_e);
    double csum = 1.0, frac1 = 0.0, frac2 = 0.0, frac3 = 0.0, oldcsum, t, hi, lo, h, v;
    for (int i = 0; i < 2; ++i) {
        v = vec[i] * scale;
        t = v * T27;
        hi = t - (t - v);
        lo = v - hi;
        v = hi * hi;
        oldcsum = csum;
        csum += v;
        frac1 += (oldcsum - csum) + v;
        v = 2.0 * hi * lo;
        oldcsum = csum;
        csum += v;
        frac2 += (oldcsum - csum) + v;
        frac3 += lo * lo;
    }
    h = sqrt(csum - 1.0 + (frac1 + frac2 + frac3));
    v = h;
    t = v * T27;
    hi = t - (t - v);
    lo = v - hi;
    v = -hi * hi;
    oldcsum = csum;
    csum += v;
    frac1 += (oldcsum - csum) + v;
    v = -2.0 * hi * lo;
    oldcsum = csum;
    csum += v;
    frac2 += (oldcsum - csum) + v;
    v = -lo * lo;
    oldcsum = csum;
    csum += v;
    frac3 += (oldcsum - csum) + v;
    v = csum - 1.0 + (frac1 + frac2 + frac3);
    return (h + v / (2.0 * h)) / scale;
}

// geometry.overlay_size (overlays.py:106-126).
int overlay_size(int32_t ov_w, int32_t ov_h, int32_t bg_w, int32_t bg_h, double ratio, int32_t& nw, int32_t& nh) {
    const double bg_diag = py_hypot((double)bg_w, (double)bg_h);
    const double target = bg_diag * ratio;
    if (ov_h == 0) return E_OVERLAY;
    const double ar = (double)ov_w / (double)ov_h;
    const double h_max = std::min((double)bg_w / ar, (double)bg_h);
    const double max_diag = py_hypot(ar * h_max, h_max);
    const double diag = std::min(target, max_diag);  // Python min keeps the first on ties
    const double hh = sqrt(pow(diag, 2.0) / (pow(ar, 2.0) + 1));
    if (!(hh < 2147483647.0)) return E_OVERLAY;
    const int64_t new_h = (int64_t)hh;
    const double ww = ar * (double)new_h;
    if (!(ww < 2147483647.0)) return E_OVERLAY;
    nh = (int32_t)new_h;
    nw = (int32_t)(int64_t)ww;
    return E_OK;
}

// Pillow Resample.c bounds of output xx (precompute_coeffs, in0 = 0).
struct AxisBounds {
    double scale, support;
    int32_t in;
    AxisBounds(int32_t in_, int32_t out) : in(in_) {
        scale = (double)((float)in_) / out;
        const double fs = scale < 1.0 ? 1.0 : scale;
        support = 3.0 * fs;
    }
    void at(int xx, int& xmin, int& cnt) const {
        const double center = 0.0 + (xx + 0.5) * scale;
        xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in) xmax = in;
        cnt = xmax - xmin;
    }
};

}  // namespace

extern "C" int ipp_plan_pipe_batch(const ipp_pipe_plan_cfg* cfg, ipp_pipe_item* items, ipp_pipe_desc* descs,
                                   ipp_tap_axis* axes, int64_t* totals) {
    if (!cfg || !items || !descs || !axes || !totals) return IPP_E_ARG;
    const ipp_pipe_plan_cfg& c = *cfg;
    memset(totals, 0, sizeof(int64_t) * IPP_PLAN_TOTALS);
    totals[IPP_PT_ERR_ITEM] = -1;
    const int32_t start = c.start, stop = c.stop, n = stop - start;
    if (n <= 0 || start < 0 || c.n_global < stop || c.n_bg <= 0 || c.n_sym <= 0 || c.n_sym > 4 || c.src_w <= 0 ||
        c.src_h <= 0 || c.bg_w <= 0 || c.bg_h <= 0)
        return IPP_E_ARG;
    const int32_t wc = c.src_w - c.crop_l - c.crop_r, hc = c.src_h - c.crop_t - c.crop_b;
    if (wc <= 0 || hc <= 0 || c.crop_l < 0 || c.crop_r < 0 || c.crop_t < 0 || c.crop_b < 0) return IPP_E_ARG;
    const int64_t src_pitch = c.src_pitch > 0 ? c.src_pitch : 3 * (int64_t)c.src_w;
    const int32_t bw = c.bg_w, bh = c.bg_h;
    int nt = c.n_threads > 0 ? c.n_threads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min(nt, 64));
    const int64_t ring = c.ring_cols > 0 ? c.ring_cols : 512;  // ipp_pipe.hip RING

    auto fail = [&](int64_t item, int code) {
        totals[IPP_PT_ERR_ITEM] = item;
        totals[IPP_PT_ERR_CODE] = code;
        return IPP_E_RANGE;
    };

    // ---- draws of steps 2, 3 and the background shuffle ------------------
    PyRandom rng;
    std::vector<double> angles;
    std::vector<int32_t> syms, order(c.n_bg);
    if (!c.given) {
        rng.seed(c.seed);
        angles.resize(c.n_global);
        syms.resize(c.n_global);
        for (int32_t g = 0; g < c.n_global; ++g) angles[g] = rng.uniform(c.angle_min, c.angle_max);
        for (int32_t g = 0; g < c.n_global; ++g) syms[g] = (int32_t)rng.randbelow((uint32_t)c.n_sym);
        std::iota(order.begin(), order.end(), 0);
        for (int32_t i = c.n_bg - 1; i >= 1; --i) std::swap(order[i], order[rng.randbelow((uint32_t)i + 1)]);
    }

    // ---- geometry of items [0, stop) (rotation + bbox), threaded ----------
    // Items before `start` still draw their ratio and position (their ranges
    // depend on their geometry), so the whole prefix is planned.
    const int32_t g0 = c.given ? start : 0;
    const int32_t ng = stop - g0;
    std::vector<Rot> rot(ng);
    std::vector<int32_t> box(4 * (size_t)ng);
    std::vector<int> gerr(ng, E_OK);
    auto geo = [&](int t) {
        for (int32_t k = t; k < ng; k += nt) {
            const int32_t gi = g0 + k;
            const double ang = c.given ? items[gi - start].angle : angles[gi];
            Rot& r = rot[k];
            gerr[k] = rotation_plan(wc, hc, ang, r);
            if (gerr[k]) continue;
            int32_t bb[4];
            opaque_bbox(wc, hc, r.A, r.nw, r.nh, bb);
            if (bb[0] >= 0 && bb[2] > bb[0] && bb[3] > bb[1]) {
                box[4 * k] = bb[0];
                box[4 * k + 1] = bb[1];
                box[4 * k + 2] = bb[2] - bb[0];
                box[4 * k + 3] = bb[3] - bb[1];
            } else {
                box[4 * k] = box[4 * k + 1] = 0;
                box[4 * k + 2] = r.nw;
                box[4 * k + 3] = r.nh;
            }
        }
    };
    if (nt == 1 || ng < 256) {
        nt = 1;
        geo(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back(geo, t);
        for (auto& x : th) x.join();
    }
    for (int32_t k = 0; k < ng; ++k)
        if (gerr[k]) return fail(g0 + k, gerr[k]);

    // ---- sequential step-5 draws and the per-item records -----------------
    for (int32_t k = 0; k < ng; ++k) {
        const int32_t gi = g0 + k;
        double ratio;
        int32_t nw_, nh_;
        if (!c.given) {
            ratio = rng.uniform(c.scale_min, c.scale_max);
        } else {
            ratio = items[gi - start].ratio;
        }
        if (overlay_size(box[4 * k + 2], box[4 * k + 3], bw, bh, ratio, nw_, nh_)) return fail(gi, E_OVERLAY);
        if (nw_ <= 0 || nh_ <= 0) return fail(gi, E_OVERLAY);
        int32_t x, y;
        if (!c.given) {
            if (bw - nw_ < 0 || bh - nh_ < 0) return fail(gi, E_EMPTY);
            x = (int32_t)rng.randbelow((uint32_t)(bw - nw_) + 1);
            y = (int32_t)rng.randbelow((uint32_t)(bh - nh_) + 1);
        } else {
            const ipp_pipe_item& it = items[gi - start];
            x = it.x;
            y = it.y;
            if (!(0 <= x && x <= bw - nw_ && 0 <= y && y <= bh - nh_ && 0 <= it.bg_index && it.bg_index < c.n_bg &&
                  0 <= it.sym && it.sym < c.n_sym))
                return fail(gi, E_FIT);
        }
        if (gi < start) continue;
        ipp_pipe_item& it = items[gi - start];
        if (!c.given) {
            it.angle = angles[gi];
            it.ratio = ratio;
            it.sym = syms[gi];
            it.bg_index = order[gi % c.n_bg];
        }
        it.x = x;
        it.y = y;
        it.rot_w = rot[k].nw;
        it.rot_h = rot[k].nh;
        it.cut_x = box[4 * k];
        it.cut_y = box[4 * k + 1];
        it.cut_w = box[4 * k + 2];
        it.cut_h = box[4 * k + 3];
        it.ov_w = nw_;
        it.ov_h = nh_;
    }

    // ---- axes, descriptors, totals -----------------------------------------
    int64_t coef_words = 0, tmp_off = 0, algo_h = 0, algo_v = 0, copy_rows = 0, copy_band_bytes = 0;
    int32_t max_out_w = 1, max_rows = 1, max_ov_w = 1, max_ov_h = 1, max_tiles = 1;
    std::vector<ipp_pipe_desc> d(n);
    for (int32_t i = 0; i < n; ++i) {
        const ipp_pipe_item& it = items[i];
        const Rot& r = rot[i + start - g0];
        const int32_t rw = it.cut_w, rh = it.cut_h, nw_ = it.ov_w, nh_ = it.ov_h;
        const bool same = nw_ == rw && nh_ == rh;
        const bool id_h = same || nw_ == rw, id_v = same || nh_ == rh;
        ipp_tap_axis& ah = axes[2 * i];
        ipp_tap_axis& av = axes[2 * i + 1];
        const int32_t ks_h = id_h ? 1 : ipp_plan_lanczos_ksize(0.0, (double)rw, nw_);
        const int32_t ks_v = id_v ? 1 : ipp_plan_lanczos_ksize(0.0, (double)rh, nh_);
        // V rows: Pillow's ybox_first/last when the H pass runs first
        int32_t y0 = 0, y1 = rh;
        if (!id_h && !id_v) {
            AxisBounds b(rh, nh_);
            int xm, cn;
            b.at(0, xm, cn);
            y0 = xm;
            b.at(nh_ - 1, xm, cn);
            y1 = xm + cn;
        }
        const int32_t rows = y1 - y0;
        const int32_t nkb_h = ipp_plan_mfma_nk_bound(rw, nw_, ks_h);
        const int32_t nkb_v = ipp_plan_mfma_nk_bound(rh, nh_, ks_v);
        if (!id_h && 64 * (int64_t)nkb_h > ring) return fail(start + i, E_RING);
        ah = {rw, nw_, id_h ? 1 : 0, 0, 0, nkb_h, 1, (nw_ + 15) / 16, coef_words};  // compact H tiles
        coef_words += (ipp_plan_mfma_size(rw, nw_, ks_h) + 3) / 4 * 4;
        const int32_t phase = it.y % 16;
        av = {rh, nh_, id_v ? 1 : 0, (!id_h && !id_v) ? y0 : 0, phase, nkb_v, 0, (nh_ + phase + 15) / 16, coef_words};
        coef_words += (ipp_plan_mfma_size(rh, nh_, ks_v) + 3) / 4 * 4;
        max_tiles = std::max(max_tiles, std::max(ah.n_tiles, av.n_tiles));

        ipp_pipe_desc& D = d[i];
        memset(&D, 0, sizeof D);
        ipp_gather_desc& g = D.g;
        g.src_off = (int64_t)i * c.src_h * src_pitch;
        g.src_pitch = (int32_t)src_pitch;
        g.src_cn = 3;
        g.src_w = c.src_w;
        g.src_h = c.src_h;
        g.in_x0 = c.crop_l;
        g.in_y0 = c.crop_t;
        g.in_w = wc;
        g.in_h = hc;
        g.a0 = r.A[0];
        g.a1 = r.A[1];
        g.a2 = r.A[2];
        g.a3 = r.A[3];
        g.a4 = r.A[4];
        g.a5 = r.A[5];
        g.out_w = rw;
        g.out_h = rh;
        g.off_x = it.cut_x;
        g.off_y = it.cut_y;
        g.flip = c.sym_flip[it.sym];
        ipp_gather_prepare(&g, 1);
        // T rows are grouped by 4; V tiles read up to 64·nK rows past their
        // 16-aligned start
        const int64_t groups = (((int64_t)(rows + 15) / 16) * 16 + 64 * nkb_v + 16) / 4;
        const int64_t pitch = 16 * (int64_t)nw_;
        ipp_resample_desc& h = D.h;
        h.dst_off = tmp_off;
        h.dst_pitch = (int32_t)pitch;
        h.in_len = rw;
        h.out_len = nw_;
        h.lines = rows;
        h.line0 = y0;
        h.ksize = ks_h;
        h.coef_off = ah.coef_off;
        ipp_resample_desc& v = D.v;
        v.src_off = tmp_off;
        v.src_pitch = (int32_t)pitch;
        v.in_len = rows;
        v.out_len = nh_;
        v.lines = nw_;
        v.ksize = ks_v;
        v.coef_off = av.coef_off;
        ipp_paste_desc& p = D.p;
        p.bg_off = (int64_t)it.bg_index * bh * bw * 3;
        p.dst_off = (int64_t)i * bh * bw * 3;
        p.bg_w = bw;
        p.bg_h = bh;
        p.bg_pitch = 3 * bw;
        p.dst_pitch = 3 * bw;
        p.ov_w = nw_;
        p.ov_h = nh_;
        p.ov_pitch = 4 * nw_;
        p.x = it.x;
        p.y = it.y;
        tmp_off += pitch * groups;
        tmp_off = (tmp_off + 255) / 256 * 256;
        max_out_w = std::max(max_out_w, nw_);
        max_rows = std::max(max_rows, rows);
        max_ov_w = std::max(max_ov_w, nw_);
        max_ov_h = std::max(max_ov_h, nh_);
        const int64_t t_bytes = pitch * ((rows + 3) / 4);
        algo_h += 3 * (int64_t)hc * wc + t_bytes;
        algo_v += t_bytes + 6 * (int64_t)bh * bw;
        const int32_t vb0 = (it.y / 16) * 16;
        const int32_t vb1 = std::max(vb0, std::min(bh, (it.y + nh_ + 15) / 16 * 16));
        copy_rows += bh - (vb1 - vb0);
        // the band rows' 16-pixel groups outside the overlay's, copied by the
        // H pass too when ipp_pipe.hip's band_cols_split holds (dense rows;
        // 16-B aligned images assumed)
        const int32_t gx0 = std::max(it.x, 0) >> 4, gx1 = std::min((it.x + nw_ + 15) >> 4, bw >> 4);
        const int64_t lr = 3 * (int64_t)(bw >> 4);
        if ((bw & 15) == 0 && ((int64_t)3 * bh * bw) % 16 == 0 && gx0 < gx1 && (int64_t)bh * lr * lr < (1ll << 32))
            copy_band_bytes += 2 * 48 * (int64_t)(vb1 - vb0) * ((bw >> 4) - (gx1 - gx0));
    }
    // processing order: items grouped by background (stable), see fused.py
    std::vector<int32_t> ord(n);
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(),
                     [&](int32_t a, int32_t b) { return items[a].bg_index < items[b].bg_index; });
    for (int32_t i = 0; i < n; ++i) descs[i] = d[ord[i]];
    // The H launch's copy blocks (ipp_pipe.hip bg_copy_group) load each
    // background vector once per run of same-background items within a group
    // of IPP_PIPE_COPY_GROUP consecutive items and store it to every item of
    // the run that takes it: bytes = the composite bytes written + one
    // background read per (group, run) (IPP_PT_COPY_READS).  (Dense, 16-B aligned images assumed,
    // as the planner lays them out; other layouts copy per item.)
    int64_t copy_runs = 0;
    for (int32_t i = 0; i < n; ++i)
        copy_runs += (i % IPP_PIPE_COPY_GROUP == 0 || items[ord[i]].bg_index != items[ord[i - 1]].bg_index) ? 1 : 0;
    const int64_t copy_bytes = 2 * 3 * (int64_t)bw * copy_rows + copy_band_bytes;
    totals[IPP_PT_COEF_WORDS] = coef_words;
    totals[IPP_PT_TMP_BYTES] = std::max<int64_t>(tmp_off, 256);
    totals[IPP_PT_MAX_OUT_W] = max_out_w;
    totals[IPP_PT_MAX_ROWS] = max_rows;
    totals[IPP_PT_MAX_OV_W] = max_ov_w;
    totals[IPP_PT_MAX_OV_H] = max_ov_h;
    totals[IPP_PT_ALGO_H] = algo_h;
    totals[IPP_PT_ALGO_V] = algo_v;
    totals[IPP_PT_COPY_BYTES] = copy_bytes;
    totals[IPP_PT_COPY_READS] = copy_runs * 3 * (int64_t)bw * bh;
    totals[IPP_PT_MAX_TILES] = max_tiles;
    return IPP_OK;
}

// Single-threaded bbox of the incremental tracker (tests compare it with
// ipp_plan_opaque_bbox) and CPython's hypot restated (tests compare it with
// math.hypot).
extern "C" int ipp_plan_opaque_bbox_fast(int32_t in_w, int32_t in_h, const int32_t a[6], int32_t nw, int32_t nh,
                                         int32_t bbox[4]) {
    if (in_w <= 0 || in_h <= 0 || nw <= 0 || nh <= 0 || !a || !bbox) return IPP_E_ARG;
    opaque_bbox(in_w, in_h, a, nw, nh, bbox);
    return IPP_OK;
}

extern "C" double ipp_plan_py_hypot(double x, double y) { return py_hypot(x, y); }

extern "C" int ipp_plan_rotation(int32_t w, int32_t h, double angle, int32_t out[8]) {
    if (!out) return IPP_E_ARG;
    Rot r;
    const int e = rotation_plan(w, h, angle, r);
    if (e) return IPP_E_RANGE;
    out[0] = r.nw;
    out[1] = r.nh;
    for (int k = 0; k < 6; ++k) out[2 + k] = r.A[k];
    return IPP_OK;
}

extern "C" int ipp_plan_py_random(uint64_t seed, int32_t n, double* out) {
    if (!out || n < 0) return IPP_E_ARG;
    PyRandom r;
    r.seed(seed);
    for (int32_t i = 0; i < n; ++i) out[i] = r.random();
    return IPP_OK;
}
