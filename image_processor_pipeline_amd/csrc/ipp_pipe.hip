// ipp_pipe.hip — the fused 5-stage pipe (BASELINE configs 3/4):
//
//   crop_from_border → process_rotations (RGBA, NEAREST, expand, bbox crop)
//   → generate_symmetries (flip) → process_images_with_color_masks (HSV α)
//   → paste_overlay_onto_background (LANCZOS resize + alpha paste)
//
// Stage chain of the reference (files between steps, one library pass per
// op): recadrages.py:46 → rotations.py:55,96,99-101 → symmetry.py:114-119 →
// filtres_liste.py:84-134 → overlays.py:129,138-139.  The RGBA cut-out "M" is
// never materialised: the LANCZOS horizontal pass computes each M pixel on the
// fly from the source (gather → HSV α → premultiply) into a channel-planar
// LDS window and runs the taps over it on the matrix cores
// (v_mfma_i32_16x16x64_i8); the vertical pass (MFMA too) is fused with
// unpremultiply, the alpha blend and the background copy.
//
// Exact integer arithmetic (Pillow Resample.c): each 22-bit tap k is split into
// three balanced signed bytes (k = k0 + 256 k1 + 65536 k2) and every pixel p is
// stored as p ^ 0x80 (= p - 128 as int8), so
//   2^21 + Σ p·k = bias + Σ_b 2^(8b) Σ_j p_j·kb_j,  bias = 2^21 + 128 Σk
// holds bit-for-bit (ipp_host.cpp builds the tap tiles and the bias).
//
// T (H-pass output) layout per item: [row group g][column x'][4 channels][4
// rows] bytes (16 B per (g, x')), values XOR 0x80.  T rows are M rows
// [line0, line0 + lines).
#include <algorithm>

#include "ipp_hsv.h"
#include "ipp_sampler.h"

namespace {

constexpr int HR = 16;            // H-pass rows per block (one 16-row band)
constexpr int RING = 512;         // window ring: M columns x live at x & (RING - 1)
// LDS bytes per plane row of the window ring.  544 ≡ 8 dwords mod 64 banks:
// the phase-2 ds_read_b128 (4 lane groups of 16, 4 dwords each) then covers
// 64 distinct banks per group (MI355X_MICROARCH.md §LDS).
constexpr int WSTRIDE = 544;
// ipp_pipe_hpass_bgcopy: background-copy blocks per item.  Diagnostic builds
// (-DIPP_DIAG) may override it through the environment; the product build
// reads no environment at all.
#ifdef IPP_DIAG
inline int diag_env(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}
inline int copy_blocks_per_item() {
    static const int v = [] {
        const int k = diag_env("IPP_COPY_BLOCKS", 4);
        return k < 1 ? 1 : (k > 64 ? 64 : k);
    }();
    return v;
}
#else
constexpr int copy_blocks_per_item() { return 4; }
#endif

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// Transpose 4 packed pixels (RGBA each) into 4 channel-planar dwords.
__device__ __forceinline__ void transpose4(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t ch[4]) {
    const uint32_t lo01 = perm(p1, p0, 0x05010400u), hi01 = perm(p1, p0, 0x07030602u);
    const uint32_t lo23 = perm(p3, p2, 0x05010400u), hi23 = perm(p3, p2, 0x07030602u);
    ch[0] = perm(lo23, lo01, 0x05040100u);
    ch[1] = perm(lo23, lo01, 0x07060302u);
    ch[2] = perm(hi23, hi01, 0x05040100u);
    ch[3] = perm(hi23, hi01, 0x07060302u);
}

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// H pass (MFMA taps) over LDS-staged source spans.
//
// Block = one 16-row band of M (the rotated / flipped / cropped cut-out) of
// one item, 4 waves.  It sweeps the band's M columns in chunks of ≤ 4 output
// tiles whose input window fits the 512-column channel-planar LDS ring; phase
// 2 of a chunk runs the LANCZOS taps on the matrix cores (below).
//
// The ring's new columns arrive in "pieces" of C ≤ 128 M columns.  A piece's
// 16 × C M pixels come from a parallelogram of the source (NEAREST rotation,
// rotations.py:96).  For each source row j crossing it, the exact column span
// [x_lo(j), x_hi(j)] is computed from the parallelogram's edges (float, with
// 1/64 px of slack, so a superset of the pixels the 16.16 gather can hit), and
// the block loads those spans with 12-byte (4-pixel) coalesced buffer loads —
// one TA wavefront per 256 source pixels instead of one per 64 gathered M
// pixels.  Each 4-pixel group goes through the table-driven HSV test
// (filtres_liste.py:84-134) right after its load, densely, and lands in the
// stage as 4 window bytes per pixel.  The M pixels then read their source
// pixel from the stage (two ds_read_b32: the row's base, the pixel) and write
// the ring.  No gather goes through the texture path any more.
//
// Source row j of a piece is staged at slots [j·S, j·S + cnt(j)) (16 B each,
// S = a per-block bound on the groups per row, so no prefix sum is needed):
//   rowtab[j] = 16 (j S - x_lo(j)/4),   pixel x of row j at rowtab[j] + 4 x.
//
// Pieces are software-pipelined across two barriers per piece:
//   A: issue the loads of piece q+1, the spans of piece q+2, gather piece q
//      from the stage into the ring;
//   B: HSV + stage writes of piece q+1; phase 2 when q ends its chunk.
// ---------------------------------------------------------------------------
constexpr int HP_THREADS = 256;     // 4 waves, one 16-row band
constexpr int HP_SLOTS = 896;       // stage slots (4 source pixels, 16 B each)
constexpr int HP_MAXROWS = 160;     // staged source rows per piece
constexpr int HP_CMAX = 128;        // M columns per piece (at most)
constexpr float HP_EPS = 1.0f / 64.0f;  // px slack of the span arithmetic (float error < 1e-2 px)

typedef uint8_t WinRing[4][HR][WSTRIDE];   // planar window ring, bytes p ^ 0x80

template <int NR>
struct __attribute__((aligned(16))) Hpass3Lds {
    WinRing win;
    uint32_t stage[4 * (HP_SLOTS + 1)];   // staged pixels; the last slot holds the fill pixel
    int32_t rowinfo[2][HP_MAXROWS];       // per staged row (piece parity): x_lo/4 | cnt << 16
    int32_t rowtab[HP_MAXROWS];           // per staged row: stage byte offset of source column 0
    HsvTables<NR> T;                      // table-driven HSV test (ipp_hsv.h)
};

// What a stage pixel holds.  0: the final window byte quad (no zones);
// 1: RGB | range bits << 24 (zones, ≤ 8 ranges: the zone test needs the M
// position); 2: raw RGB (zones, > 8 ranges: the HSV test runs after the gather).
template <int NR, bool ZONES>
struct StageMode {
    static constexpr int v = !ZONES ? 0 : (NR <= 8 ? 1 : 2);
};

// M pixel → window byte quad (p | α 255) ^ 0x80 when kept, 0x80808080 (transparent black) when excluded.
template <int NR, bool ZONES>
__device__ __forceinline__ uint32_t hsv2_px(const HsvTables<NR>& T, uint32_t raw, uint32_t zbits) {
    uint32_t ex = hsv_tab_excl<NR, false>(T, raw);
    if (ZONES) ex &= zbits;
    const uint32_t t = (raw | 0xFF000000u) ^ 0x80808080u;
    return ex ? 0x80808080u : t;
}

// Diagnostic builds only (-DIPP_DIAG, wrong output): IPP_HP_X bit 0 = no
// HSV in the stage, bit 1 = no gather, bit 2 = no phase 2, bit 3 = no loads.
#if defined(IPP_DIAG) && defined(IPP_HP_X)
constexpr int kHpX = IPP_HP_X;
#else
constexpr int kHpX = 0;
#endif

template <int NR, int MODE>
__device__ __forceinline__ uint32_t stage_px(const HsvTables<NR>& T, uint32_t raw) {
    if (MODE == 2) return raw;
    if (kHpX & 1) return (raw | 0xFF000000u) ^ 0x80808080u;
    const uint32_t ex = hsv_tab_excl<NR, false>(T, raw);
    if (MODE == 1) return (raw & 0xFFFFFFu) | (ex << 24);
    return ex ? 0x80808080u : (raw | 0xFF000000u) ^ 0x80808080u;
}

template <int NR, int MODE>
__device__ __forceinline__ uint32_t window_px(const HsvTables<NR>& T, uint32_t v, uint32_t zb) {
    if (MODE == 0) return v;
    if (MODE == 1) return ((v >> 24) & zb) ? 0x80808080u : (v | 0xFF000000u) ^ 0x80808080u;
    return hsv2_px<NR, true>(T, v, zb);
}

// Per-block state.
struct Hp3Block {
    __amdgpu_buffer_rsrc_t rs;   // source window, records = bytes to the image end
    int32_t nrec;
    uint32_t rowx0, rowy0;       // 16.16 source position of M column 0 of the band's row 0
    int32_t b0, b1, b3, b4;      // 16.16 steps per M column (b0, b3) and per M row (b1, b4)
    int32_t pitch, in_w, in_h;
    int32_t xlo, xhi;            // the band's valid M columns ⊆ [xlo, xhi] (conservative)
    int32_t C, lgcg;             // M columns per piece, log2(C / 4)
    int32_t slots, spx;          // stage slots per staged row, bound on x_hi - x_lo
    float rslots;                // 1 / slots
    bool useV, useU;             // edge pairs usable as x(y) lines (|slope| ≤ 64)
    bool bad;                    // no stage layout fits: nothing is staged (status bit 1)
};

// Bound on a slab's x extent (px) for a parallelogram with sides U (16 M
// rows) and V (a piece's columns), the same formula for the block's bound and
// for every piece: the polygon's x extent, or with both edge pairs usable the
// longest horizontal chord plus the boundary's x drift over a slab of
// height 1 + 2 eps.
__device__ __forceinline__ float hp3_extent(float ux, float uy, float vx, float vy, bool useV, bool useU) {
    float ext = fabsf(vx) + fabsf(ux);
    if (useV && useU) {
        const float chord = fabsf(ux * vy - uy * vx) * __builtin_amdgcn_rcpf(fmaxf(fabsf(vy), fabsf(uy)));
        const float slope = fmaxf(fabsf(vx * __builtin_amdgcn_rcpf(vy)), fabsf(ux * __builtin_amdgcn_rcpf(uy)));
        ext = fminf(ext, chord * (1.0f + 1e-5f) + 2.0f * (1.0f + 2.0f * HP_EPS) * slope * (1.0f + 1e-5f));
    }
    return ext;
}

// Piece width and stage layout for the block: the widest C ∈ {128, 64, 32,
// 16} whose worst-case piece fits the stage.  0 when none does (the affine is
// not a rotation; the pipe plans only rotations).
__device__ __forceinline__ void hp3_layout(Hp3Block& B) {
    const float k16 = 1.0f / 65536.0f;
    B.useV = 64ll * llabs((long long)B.b3) > llabs((long long)B.b0);
    B.useU = 64ll * llabs((long long)B.b4) > llabs((long long)B.b1);
    const float ux = (float)(HR - 1) * (float)B.b1 * k16, uy = (float)(HR - 1) * (float)B.b4 * k16;
    B.C = 0;
    B.lgcg = 2;
    B.slots = 1;
    B.spx = 0;
    B.rslots = 1.0f;
    for (int C = HP_CMAX, lg = 5; C >= 16; C >>= 1, --lg) {
        const float vx = (float)(C - 1) * (float)B.b0 * k16, vy = (float)(C - 1) * (float)B.b3 * k16;
        const int rows = (int)(fabsf(vy) + fabsf(uy) + 4.0f * HP_EPS) + 2;
        const int spx = (int)(hp3_extent(ux, uy, vx, vy, B.useV, B.useU) + 4.0f * HP_EPS) + 1;
        const int slots = (spx + 3) / 4 + 1;
        if (rows <= HP_MAXROWS && rows * slots <= HP_SLOTS) {
            B.C = C;
            B.lgcg = lg;
            B.slots = slots;
            B.spx = spx;
            B.rslots = __builtin_amdgcn_rcpf((float)slots);
            return;
        }
    }
}

struct Hp3Piece {
    int xa, xb;        // M columns [xa, xb) written to the ring
    int s0, s1;        // the chunk's output tiles [s0, s1)
    int last;          // the chunk's last piece: phase 2 follows
    int jlo, rows;     // staged source rows [jlo, jlo + rows); 0: nothing staged
};

// Sticky status of the pipe kernels (ipp_pipe_status): bit 0 = an H-pass
// output tile's input window was wider than the LDS ring (the plan violated
// the ring limit of ipp.h; that tile's T columns are wrong); bit 1 = a band's
// rotation did not fit the source stage (not a rotation, or a source wider
// than 32767 px; its T rows are wrong).
__device__ int32_t g_pipe_status;

// Spans of the piece's source rows → rowinfo (one row per thread).  ga..gb:
// the piece's columns that can hold valid pixels.
__device__ __forceinline__ void hp3_spans(const Hp3Block& B, int ga, int gb, int32_t* __restrict__ rowinfo,
                                          Hp3Piece& pc) {
    pc.jlo = 0;
    pc.rows = 0;
    if (ga >= gb || B.bad) return;
    const float k16 = 1.0f / 65536.0f;
    const float ax = (float)(int32_t)(B.rowx0 + (uint32_t)ga * (uint32_t)B.b0) * k16;
    const float ay = (float)(int32_t)(B.rowy0 + (uint32_t)ga * (uint32_t)B.b3) * k16;
    const float ux = (float)(HR - 1) * (float)B.b1 * k16, uy = (float)(HR - 1) * (float)B.b4 * k16;
    const float vx = (float)(gb - 1 - ga) * (float)B.b0 * k16, vy = (float)(gb - 1 - ga) * (float)B.b3 * k16;
    // vertices A = a, Bv = a + V, Cv = a + U + V, D = a + U
    const float bx = ax + vx, by = ay + vy, cx = bx + ux, cy = by + uy, dx = ax + ux, dy = ay + uy;
    const float xmin = fminf(fminf(ax, bx), fminf(cx, dx)), xmax = fmaxf(fmaxf(ax, bx), fmaxf(cx, dx));
    const float ymin = fminf(fminf(ay, by), fminf(cy, dy)), ymax = fmaxf(fmaxf(ay, by), fmaxf(cy, dy));
    const int jlo = max(0, (int)floorf(fmaxf(ymin - HP_EPS, -1.0f)));
    const int jhi = min(B.in_h - 1, (int)floorf(fminf(ymax + HP_EPS, (float)B.in_h)));
    const int rows = __builtin_amdgcn_readfirstlane(jhi - jlo + 1);
    if (rows <= 0) return;
    if (rows > HP_MAXROWS) {  // cannot happen under the block's layout bound
        if (threadIdx.x == 0) atomicOr(&g_pipe_status, 2);
        return;
    }
    pc.jlo = __builtin_amdgcn_readfirstlane(jlo);
    pc.rows = rows;
    if ((int)threadIdx.x >= rows) return;
    // leftmost / rightmost vertex
    float lx = ax, ly = ay, rx = ax, ry = ay;
    if (bx < lx) { lx = bx; ly = by; }
    if (cx < lx) { lx = cx; ly = cy; }
    if (dx < lx) { lx = dx; ly = dy; }
    if (bx > rx) { rx = bx; ry = by; }
    if (cx > rx) { rx = cx; ry = cy; }
    if (dx > rx) { rx = dx; ry = dy; }
    // Boundary lines x = px + b (y - py).  V edges run through A and D, U
    // edges through A and Bv; the V edge through A bounds the left side iff
    // cross(U, V)·vy > 0, the U edge through A iff cross(U, V)·uy < 0.
    // Near-horizontal edges (|slope| > 64) are dropped: fewer constraints only
    // widen the spans, and they would amplify float error.
    const float cr = ux * vy - uy * vx;
    float l1x = xmin, l1y = 0.0f, l1b = 0.0f, r1x = xmax, r1y = 0.0f, r1b = 0.0f;
    float l2x = xmin, l2y = 0.0f, l2b = 0.0f, r2x = xmax, r2y = 0.0f, r2b = 0.0f;
    if (B.useV) {
        const float bv = vx * __builtin_amdgcn_rcpf(vy);
        const bool aL = cr * vy > 0.0f;
        l1x = aL ? ax : dx; l1y = aL ? ay : dy; l1b = bv;
        r1x = aL ? dx : ax; r1y = aL ? dy : ay; r1b = bv;
    }
    if (B.useU) {
        const float bu = ux * __builtin_amdgcn_rcpf(uy);
        const bool aL = cr * uy < 0.0f;
        l2x = aL ? ax : bx; l2y = aL ? ay : by; l2b = bu;
        r2x = aL ? bx : ax; r2y = aL ? by : ay; r2b = bu;
    }
    if (B.useV && !B.useU) { l2x = l1x; l2y = l1y; l2b = l1b; r2x = r1x; r2y = r1y; r2b = r1b; }
    if (B.useU && !B.useV) { l1x = l2x; l1y = l2y; l1b = l2b; r1x = r2x; r1y = r2y; r1b = r2b; }
    const int t = threadIdx.x;
    const float j = (float)(jlo + t);
    const float yl = fmaxf(j - HP_EPS, ymin), yh = fminf(j + 1.0f + HP_EPS, ymax);
    // left boundary max(L1, L2) is convex in y: its minimum over the slab is at
    // an end or at the leftmost vertex; the right boundary likewise
    float xl = fminf(fmaxf(l1x + l1b * (yl - l1y), l2x + l2b * (yl - l2y)),
                     fmaxf(l1x + l1b * (yh - l1y), l2x + l2b * (yh - l2y)));
    float xr = fmaxf(fminf(r1x + r1b * (yl - r1y), r2x + r2b * (yl - r2y)),
                     fminf(r1x + r1b * (yh - r1y), r2x + r2b * (yh - r2y)));
    if (ly >= yl && ly <= yh) xl = lx;
    if (ry >= yl && ry <= yh) xr = rx;
    xl = fmaxf(xl, xmin);
    xr = fminf(xr, xmax);
    const int x_lo = max(0, (int)floorf(fmaxf(xl - HP_EPS, -1.0f)));
    int x_hi = min(B.in_w - 1, (int)floorf(fminf(xr + HP_EPS, (float)B.in_w)));
    if (x_hi - x_lo > B.spx) {  // cannot happen under the block's layout bound
        atomicOr(&g_pipe_status, 2);
        x_hi = x_lo + B.spx;
    }
    const int gl = x_lo >> 2;
    const int cnt = x_lo <= x_hi ? (x_hi >> 2) - gl + 1 : 0;
    rowinfo[t] = gl | (cnt << 16);
}

// A thread's stage slots of one piece: up to 4 groups of 4 source pixels.
template <int CN>
struct Hp3Loads {
    uint32_t w[4][CN];
    int32_t slot[4];   // stage slot, -1: none
};

// Groups that run past the image end (only at the window's last row, when it
// reaches the source's right edge) are loaded dword by dword, the partial
// dword one to three bytes early and shifted down (bytes past the end are
// never used).
template <int CN>
__device__ __forceinline__ void hp3_load_tail(const Hp3Block& B, uint32_t off, uint32_t (&w)[CN]) {
#pragma unroll
    for (int d = 0; d < CN; ++d) {
        const int32_t o = (int32_t)off + 4 * d;
        uint32_t v = 0u;
        if (o + 4 <= B.nrec) {
            v = __builtin_amdgcn_raw_buffer_load_b32(B.rs, (uint32_t)o, 0, 0);
        } else if (o < B.nrec) {
            v = __builtin_amdgcn_raw_buffer_load_b32(B.rs, (uint32_t)(B.nrec - 4), 0, 0) >> (8 * (o + 4 - B.nrec));
        }
        w[d] = v;
    }
}

// Issue the loads of a piece's stage slots (slot g = thread + 256 i; row
// g / S, group g mod S).  Every rowinfo read is issued before any load.
template <int CN>
__device__ __forceinline__ void hp3_issue(const Hp3Block& B, const Hp3Piece& pc, const int32_t* __restrict__ rowinfo,
                                          Hp3Loads<CN>& L) {
    const int n = pc.rows * B.slots;
    int32_t info[4], jv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int g = (int)threadIdx.x + HP_THREADS * i;
        // j = g / S exactly: g < 2^12, and the fraction stays ≥ 0.5 / S from an integer
        jv[i] = min((int)(((float)g + 0.5f) * B.rslots), HP_MAXROWS - 1);
        info[i] = rowinfo[jv[i]];
    }
    bool tail = false;
    uint32_t off[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int g = (int)threadIdx.x + HP_THREADS * i;
        const int k = g - jv[i] * B.slots;
        const int gl = info[i] & 0xFFFF, cnt = info[i] >> 16;
        const bool on = g < n && k < cnt;
        off[i] = (uint32_t)(pc.jlo + jv[i]) * (uint32_t)B.pitch + (uint32_t)(gl + k) * (uint32_t)(4 * CN);
        L.slot[i] = on ? g : -1;
        const bool fast = !(kHpX & 8) && on && (int32_t)off[i] + 4 * CN <= B.nrec;
        tail |= on && !fast;
        if (fast) {
            if (CN == 3) {
                typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
                const u32x3 v = __builtin_bit_cast(u32x3, __builtin_amdgcn_raw_buffer_load_b96(B.rs, off[i], 0, 0));
                L.w[i][0] = v.x;
                L.w[i][1] = v.y;
                L.w[i][2] = v.z;
            } else {
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(B.rs, off[i], 0, 0));
#pragma unroll
                for (int d = 0; d < CN; ++d) L.w[i][d] = v[d];
            }
        }
    }
    if (tail) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (L.slot[i] >= 0 && (int32_t)off[i] + 4 * CN > B.nrec) hp3_load_tail<CN>(B, off[i], L.w[i]);
    }
}

// HSV of the loaded groups → stage; the row table of the piece.
template <int NR, int MODE, int CN>
__device__ __forceinline__ void hp3_stage(Hpass3Lds<NR>& L, const Hp3Block& B, const Hp3Piece& pc,
                                          const int32_t* __restrict__ rowinfo, const Hp3Loads<CN>& LD) {
    const int t = threadIdx.x;
    if (t < pc.rows) L.rowtab[t] = 16 * (t * B.slots - (rowinfo[t] & 0xFFFF));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (LD.slot[i] < 0) continue;
        uint32_t p[4];
        if (CN == 3) {
            p[0] = LD.w[i][0];
            p[1] = __builtin_amdgcn_alignbit(LD.w[i][1], LD.w[i][0], 24);
            p[2] = __builtin_amdgcn_alignbit(LD.w[i][2], LD.w[i][1], 16);
            p[3] = LD.w[i][2] >> 8;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) p[k] = LD.w[i][k < CN ? k : 0];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) p[k] = stage_px<NR, MODE>(L.T, p[k]);
        *reinterpret_cast<uint4*>(&L.stage[4 * LD.slot[i]]) = make_uint4(p[0], p[1], p[2], p[3]);
    }
}

// Zone bits of 4 M pixels (columns x .. x + 3 of band row rw).
template <int NR, bool ZONES>
__device__ __forceinline__ void hp3_zones(int yrow, int x, const int32_t* zr0, const int32_t* zrh, const int32_t* zc0,
                                          const int32_t* zcw, uint32_t (&zb)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) zb[k] = ~0u;
    if (!ZONES) return;
    uint32_t zrow = 0;
#pragma unroll
    for (int q = 0; q < NR; ++q) zrow |= (uint32_t)((uint32_t)(yrow - zr0[q]) < (uint32_t)zrh[q]) << q;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t zc = 0;
#pragma unroll
        for (int q = 0; q < NR; ++q) zc |= (uint32_t)((uint32_t)(x + k - zc0[q]) < (uint32_t)zcw[q]) << q;
        zb[k] = zc & zrow;
    }
}

__device__ __forceinline__ void ring_write(WinRing& win, int rw, int x, const uint32_t (&px)[4]) {
    uint32_t ch[4];
    transpose4(px[0], px[1], px[2], px[3], ch);
    const int pos = x & (RING - 1);
#pragma unroll
    for (int c = 0; c < 4; ++c) *reinterpret_cast<uint32_t*>(&win[c][rw][pos]) = ch[c];
}

// Gather the piece's 16 × (xb - xa) M pixels into the ring.  Unit = 4
// consecutive columns of one row; unit u: column group u mod C/4 (a 32-lane
// group writes one ring row's consecutive dwords, conflict-free), row
// (u / (C/4)) mod 16, C-block u / 4C.  A live piece (≤ C columns) is ≤ 2 units
// per thread, issued as one batch: 8 row-table reads, then 8 pixel reads.  A
// fill run (nothing staged) may be wider.
template <int NR, bool ZONES, int MODE>
__device__ __forceinline__ void hp3_gather(Hpass3Lds<NR>& L, const Hp3Block& B, const Hp3Piece& pc, int nrows,
                                           int yb, const int32_t* zr0, const int32_t* zrh, const int32_t* zc0,
                                           const int32_t* zcw, uint32_t fill) {
    if (kHpX & 2) return;
    const int ncg = B.C >> 2;
    const int fillofs = 16 * HP_SLOTS;
    const uint8_t* stg = reinterpret_cast<const uint8_t*>(L.stage);
    if (pc.rows == 0) {
        // units: 16 rows × C/4 column groups per C-block
        const int nu = 4 * B.C * ((pc.xb - pc.xa + B.C - 1) >> (B.lgcg + 2));
        // fill run: every pixel is the fill (black); zones still decide its α
        for (int u = threadIdx.x; u < nu; u += HP_THREADS) {
            const int cg = u & (ncg - 1), rw = (u >> B.lgcg) & (HR - 1), cb = u >> (B.lgcg + 4);
            const int x = pc.xa + 4 * cg + B.C * cb;
            if (x >= pc.xb || rw >= nrows) continue;
            uint32_t px[4];
            if (ZONES) {
                uint32_t zb[4];
                hp3_zones<NR, ZONES>(yb + rw, x, zr0, zrh, zc0, zcw, zb);
                const uint32_t v = *reinterpret_cast<const uint32_t*>(stg + fillofs);
#pragma unroll
                for (int k = 0; k < 4; ++k) px[k] = window_px<NR, MODE>(L.T, v, zb[k]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) px[k] = fill;
            }
            ring_write(L.win, rw, x, px);
        }
        return;
    }
    int a[2][4], xs[2], rws[2];
    bool on[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int u = (int)threadIdx.x + HP_THREADS * i;
        const int cg = u & (ncg - 1), rw = (u >> B.lgcg) & (HR - 1);
        const int x = pc.xa + 4 * cg;
        xs[i] = x;
        rws[i] = rw;
        on[i] = u < 4 * B.C && x < pc.xb && rw < nrows;
        uint32_t xx = B.rowx0 + (uint32_t)rw * (uint32_t)B.b1 + (uint32_t)x * (uint32_t)B.b0;
        uint32_t yy = B.rowy0 + (uint32_t)rw * (uint32_t)B.b4 + (uint32_t)x * (uint32_t)B.b3;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int xin = (int32_t)xx >> 16, yin = (int32_t)yy >> 16;
            const bool ok = ((uint32_t)xin < (uint32_t)B.in_w) & ((uint32_t)yin < (uint32_t)B.in_h);
            const int jj = min(max(yin - pc.jlo, 0), pc.rows - 1);
            // row table read now, pixel read below: all 8 in flight together
            // (rb feeds both arms of the select, so the read is not sunk into
            // a branch of its own)
            const int rb = L.rowtab[jj];
            a[i][k] = rb + (ok ? 4 * xin : fillofs - rb);
            xx += (uint32_t)B.b0;
            yy += (uint32_t)B.b3;
        }
    }
    uint32_t v[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) v[i][k] = *reinterpret_cast<const uint32_t*>(stg + a[i][k]);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        if (!on[i]) continue;
        uint32_t zb[4], px[4];
        hp3_zones<NR, ZONES>(yb + rws[i], xs[i], zr0, zrh, zc0, zcw, zb);
#pragma unroll
        for (int k = 0; k < 4; ++k) px[k] = window_px<NR, MODE>(L.T, v[i][k], zb[k]);
        ring_write(L.win, rws[i], xs[i], px);
    }
}

// Chunks: ≤ 4 output tiles whose input window fits the ring.
struct Hp3Chunk {
    int s0, s1;   // tiles [s0, s1)
    int c0, cend; // new M columns [c0, cend)
};

__device__ __forceinline__ Hp3Chunk hp3_chunk(const int4* hdr, int s0, int ntiles, int& filled) {
    Hp3Chunk c;
    c.s0 = s0;
    const int W0 = hdr[s0].x;
    int s1 = min(s0 + 4, ntiles), W1;
    for (;;) {
        W1 = W0;
        for (int t = s0; t < s1; ++t) W1 = max(W1, hdr[t].x + 64 * hdr[t].y);
        if (s1 - s0 == 1 || W1 - W0 <= RING) break;
        --s1;
    }
    c.s1 = s1;
    if (W1 - W0 > RING && threadIdx.x == 0) atomicOr(&g_pipe_status, 1);  // single tile beyond the ring
    c.c0 = max(filled, W0);
    c.cend = max(c.c0, W1);
    filled = max(filled, W1);
    return c;
}

template <int NR, bool ZONES, int CN>
__device__ __forceinline__ void hpass3_body(Hpass3Lds<NR>& L, const Hp3Block& B, uint8_t* __restrict__ tmp,
                                            const int32_t* __restrict__ coefs, const ipp_resample_desc& h, int row0,
                                            int nrows, const int32_t* zr0, const int32_t* zrh, const int32_t* zc0,
                                            const int32_t* zcw, uint32_t fill) {
    constexpr int MODE = StageMode<NR, ZONES>::v;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ntiles = (h.out_len + 15) >> 4;
    const int4* hdr = reinterpret_cast<const int4*>(coefs + h.coef_off);
    const int32_t* tbias = coefs + h.coef_off + 4 * (int64_t)ntiles;
    const uint4* tblk = reinterpret_cast<const uint4*>(coefs + h.coef_off + 20 * (int64_t)ntiles);
    const int yb = h.line0 + row0;  // M row of the band's row 0
    const int C = B.C;

    // Piece generator over the chunks.  A piece is ≤ C live columns, or a
    // fill run (columns outside the band's valid range [xlo, xhi], nothing to
    // stage) up to the next live column or the chunk's end; a chunk with no
    // new columns still yields one empty piece, so its phase 2 runs.
    int filled = hdr[0].x;
    Hp3Chunk gch = hp3_chunk(hdr, 0, ntiles, filled);
    int gx = gch.c0;
    bool gemitted = false;
    auto gen = [&](Hp3Piece& p) -> bool {
        if (gx >= gch.cend && gemitted) {
            if (gch.s1 >= ntiles) return false;
            gch = hp3_chunk(hdr, gch.s1, ntiles, filled);
            gx = gch.c0;
            gemitted = false;
        }
        p.xa = gx;
        int xb;
        if (gx > B.xhi) xb = gch.cend;                                          // past the live columns
        else if (gx + C <= B.xlo) xb = min(gch.cend, max(gx + 4, B.xlo & ~3));  // before them
        else xb = min(gx + C, gch.cend);
        p.xb = max(gx, xb);
        gx = p.xb;
        gemitted = true;
        p.s0 = gch.s0;
        p.s1 = gch.s1;
        p.last = gx >= gch.cend;
        return true;
    };
    auto spans = [&](Hp3Piece& p, int par) {
        hp3_spans(B, max(p.xa, B.xlo), min(p.xb, B.xhi + 1), L.rowinfo[par], p);
    };

    Hp3Piece q, nq, nnq;
    gen(q);
    spans(q, 0);
    bool hnq = gen(nq);
    if (hnq) spans(nq, 1);
    __syncthreads();
    Hp3Loads<CN> LD;
    hp3_issue<CN>(B, q, L.rowinfo[0], LD);
    hp3_stage<NR, MODE, CN>(L, B, q, L.rowinfo[0], LD);
    if (hnq) hp3_issue<CN>(B, nq, L.rowinfo[1], LD);
    __syncthreads();
    int par = 0;  // q's rowinfo buffer
    for (;;) {
        // ---- A: spans of q+2; q → ring; taps of q's chunk
        const bool hnnq = hnq && gen(nnq);
        if (hnnq) spans(nnq, par);
        const int t = q.s0 + wave;
        const bool has_tile = !(kHpX & 4) && q.last && t < q.s1;
        int4 th = make_int4(0, 0, 0, 0);
        uint4 bn[3];
        int32_t bias = 0;
        const uint4* bt = tblk + lane;
        if (has_tile) {
            th = hdr[t];
            bt += th.z;
#pragma unroll
            for (int p = 0; p < 3; ++p) bn[p] = bt[p * 64];
            bias = tbias[min(16 * t + (lane & 15), h.out_len - 1)];
        }
        hp3_gather<NR, ZONES, MODE>(L, B, q, nrows, yb, zr0, zrh, zc0, zcw, fill);
        __syncthreads();
        // ---- B: q+1 → stage; loads of q+2 (in flight until the next B);
        // phase 2 at a chunk's end
        if (hnq) hp3_stage<NR, MODE, CN>(L, B, nq, L.rowinfo[par ^ 1], LD);
        if (hnnq) hp3_issue<CN>(B, nnq, L.rowinfo[par], LD);
        if (has_tile) {
            // Phase 2 (mfma): wave w takes tile s0 + w; A = 16 window rows ×
            // 64 columns of one channel (lane l: row l&15, bytes
            // 16(l>>4)..+15), B = 64 columns × 16 outputs of one tap byte
            // plane.  D lane l = output l&15, rows 4(l>>4)..+3 = exactly one
            // 16-B T group.
            i32x4 acc[4][3];
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int p = 0; p < 3; ++p) acc[c][p] = i32x4{0, 0, 0, 0};
            const int arow = lane & 15, akoff = 16 * (lane >> 4);
#pragma unroll 1
            for (int ks = 0; ks < th.y; ++ks) {
                i32x4 bq[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) bq[p] = __builtin_bit_cast(i32x4, bn[p]);
                if (ks + 1 < th.y) {
#pragma unroll
                    for (int p = 0; p < 3; ++p) bn[p] = bt[((ks + 1) * 3 + p) * 64];
                }
                const int pos = (th.x + 64 * ks + akoff) & (RING - 1);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const i32x4 a = *reinterpret_cast<const i32x4*>(&L.win[c][arow][pos]);
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        acc[c][p] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bq[p], acc[c][p], 0, 0, 0);
                }
            }
            const int xo = 16 * t + (lane & 15);
            if (xo < h.out_len) {
                uint32_t outc[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int32_t ss = bias + acc[c][0][rr] + (acc[c][1][rr] << 8) + (acc[c][2][rr] << 16);
                        outc[c] |= clip8(ss) << (8 * rr);
                    }
                const int grp = (row0 >> 2) + (lane >> 4);
                uint4* dst = reinterpret_cast<uint4*>(tmp + h.dst_off + (int64_t)grp * h.dst_pitch) + xo;
                *dst = make_uint4(outc[0] ^ 0x80808080u, outc[1] ^ 0x80808080u, outc[2] ^ 0x80808080u,
                                  outc[3] ^ 0x80808080u);
            }
        }
        __syncthreads();
        if (!hnq) break;
        q = nq;
        nq = nnq;
        hnq = hnnq;
        par ^= 1;
    }
}

// Composite rows outside the overlay's 16-row bands [vb0, vb1) are plain
// copies of the background (Paste.c leaves them untouched).  Dedicated copy
// blocks of the H-pass launch write them, so ipp_pipe_vblend_bands then only
// visits the bands the overlay touches.
__device__ __forceinline__ void paste_bands(const ipp_paste_desc& p, int& vb0, int& vb1) {
    vb0 = (p.y >> 4) << 4;
    vb1 = min(p.bg_h, ((p.y + p.ov_h + 15) >> 4) << 4);
    vb1 = max(vb1, vb0);
}

template <int NT = 256>
__device__ __forceinline__ void bg_copy_outside_bands(const ipp_paste_desc& p, const uint8_t* __restrict__ bg,
                                                      uint8_t* __restrict__ dst, int share, int nshare) {
    int vb0, vb1;
    paste_bands(p, vb0, vb1);
    const int rb = 3 * p.bg_w;
    const uint8_t* sb = bg + p.bg_off;
    uint8_t* db = dst + p.dst_off;
    const bool flat = p.bg_pitch == rb && p.dst_pitch == rb && (rb & 15) == 0 &&
                      ((reinterpret_cast<uintptr_t>(sb) | reinterpret_cast<uintptr_t>(db)) & 15u) == 0;
    if (flat) {
        // Two flat byte ranges [0, vb0·rb) and [vb1·rb, bg_h·rb) in 16-B vectors.
        const int64_t n0 = (int64_t)vb0 * rb / 16, n1 = (int64_t)(p.bg_h - vb1) * rb / 16, V = n0 + n1;
        const int64_t a = V * share / nshare, e = V * (share + 1) / nshare;
        const int64_t skip = (int64_t)vb1 * rb / 16 - n0;  // vector index gap over the bands
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* s4 = reinterpret_cast<const u32x4*>(sb);
        u32x4* d4 = reinterpret_cast<u32x4*>(db);
        for (int64_t i0 = a + threadIdx.x; i0 < e; i0 += 8 * NT) {
            u32x4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int64_t i = i0 + NT * j;
                if (i < e) v[j] = s4[i < n0 ? i : i + skip];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int64_t i = i0 + NT * j;
                if (i < e) __builtin_nontemporal_store(v[j], d4 + (i < n0 ? i : i + skip));
            }
        }
        return;
    }
    // General pitches: whole rows, 16-B chunks with byte tails.
    const int R = vb0 + (p.bg_h - vb1);
    const int ra = (int)((int64_t)R * share / nshare), re = (int)((int64_t)R * (share + 1) / nshare);
    const int chunks = (rb + 15) >> 4;
    for (int rr = ra; rr < re; ++rr) {
        const int y = rr < vb0 ? rr : rr - vb0 + vb1;
        const uint8_t* brow = sb + (int64_t)y * p.bg_pitch;
        uint8_t* drow = db + (int64_t)y * p.dst_pitch;
        for (int ci = threadIdx.x; ci < chunks; ci += NT) {
            const int c0 = ci << 4, nb = min(16, rb - c0);
            const bool vec = nb == 16 && ((reinterpret_cast<uintptr_t>(brow + c0) | reinterpret_cast<uintptr_t>(drow + c0)) & 15u) == 0;
            uint32_t w[4];
            load16(brow + c0, nb, vec, w);
            store16<2>(drow + c0, nb, vec, w);
        }
    }
}

template <int NR, bool ZONES, int CN, bool COPY>
__global__ void __launch_bounds__(HP_THREADS) __attribute__((amdgpu_waves_per_eu(3)))
k_pipe_hpass3(const uint8_t* __restrict__ src, uint8_t* __restrict__ tmp, const int32_t* __restrict__ coefs,
              const ipp_pipe_desc* __restrict__ descs, int tiles_y, ipp_hsv_params hp, const uint8_t* __restrict__ bg,
              uint8_t* __restrict__ dst, int cpi) {
    __shared__ Hpass3Lds<NR> L;
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    // tiles_y = H-pass blocks per item.  COPY: each item owns tiles_y H-pass
    // blocks followed by cpi background-copy blocks, so the copies run beside
    // the H pass on every XCD.
    const int per_item = tiles_y + (COPY ? cpi : 0);
    const int im = b / per_item;
    const int tb = b - im * per_item;
    if (COPY && tb >= tiles_y) {
        bg_copy_outside_bands<HP_THREADS>(descs[im].p, bg, dst, tb - tiles_y, cpi);
        return;
    }
    const ipp_gather_desc g = descs[im].g;
    const ipp_resample_desc h = descs[im].h;
    const int row0 = tb * HR;
    if (row0 >= h.lines) return;  // block-uniform

    hsv_tables_init<NR>(L.T, hp);

    // Zones (filtres_liste.py:102-103): per range the M rows [zr0, zr0 + zrh)
    // and columns [zc0, zc0 + zcw).
    int32_t zr0[ZONES ? NR : 1], zrh[ZONES ? NR : 1], zc0[ZONES ? NR : 1], zcw[ZONES ? NR : 1];
    if (ZONES) {
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            int a, bb, cc, dd;
            slice_indices(hp.r[k].zone[0], g.out_h - hp.r[k].zone[1], g.out_h, a, bb);
            slice_indices(hp.r[k].zone[2], g.out_w - hp.r[k].zone[3], g.out_w, cc, dd);
            zr0[k] = a;
            zrh[k] = bb - a;
            zc0[k] = cc;
            zcw[k] = dd - cc;
        }
    }

    // Source window as a buffer resource (32-bit scalar arithmetic: a 64-bit
    // value would land in VGPRs and turn every buffer load into a waterfall
    // loop; items are < 2 GiB, checked on the host).
    const Sampler S = make_sampler(src, g);
    const int nrec = (g.src_h - g.in_y0) * g.src_pitch - g.in_x0 * g.src_cn;
    const uint64_t sbu = reinterpret_cast<uint64_t>(S.base);
    Hp3Block B;
    B.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(sbu), (short)0, nrec, 0x00020000);
    B.nrec = nrec;
    const int y0 = h.line0 + row0;
    B.rowx0 = (uint32_t)S.b2 + (uint32_t)y0 * (uint32_t)S.b1;
    B.rowy0 = (uint32_t)S.b5 + (uint32_t)y0 * (uint32_t)S.b4;
    B.b0 = S.b0;
    B.b1 = S.b1;
    B.b3 = S.b3;
    B.b4 = S.b4;
    B.pitch = (int32_t)S.pitch;
    B.in_w = S.in_w;
    B.in_h = S.in_h;
    hp3_layout(B);
    B.bad = B.C == 0 || S.in_w > 32767;  // not a rotation, or columns beyond the 16-bit span fields
    if (B.bad) {
        if (threadIdx.x == 0) atomicOr(&g_pipe_status, 2);
        B.C = HP_CMAX;
        B.lgcg = 5;
    }
    {
        // Row r's valid columns: 0 <= xx(x) < in_w·2^16 and 0 <= yy(x) < in_h·2^16,
        // both linear in x; ±2 columns of slack absorb the rounding.  Union
        // over the band's 16 rows (lane r holds row r) by readlane.
        const int r = threadIdx.x & 15;
        const uint32_t rx = B.rowx0 + (uint32_t)r * (uint32_t)B.b1, ry = B.rowy0 + (uint32_t)r * (uint32_t)B.b4;
        float lo = -1e9f, hi = 1e9f;
        auto clip = [&](float a, float bb, float lim) {
            if (bb == 0.0f) {
                if (!(a >= 0.0f && a < lim)) { lo = 1e9f; hi = -1e9f; }
            } else {
                const float t1 = -a / bb, t2 = (lim - a) / bb;
                lo = fmaxf(lo, fminf(t1, t2));
                hi = fminf(hi, fmaxf(t1, t2));
            }
        };
        clip((float)(int32_t)rx, (float)S.b0, 65536.0f * (float)S.in_w);
        clip((float)(int32_t)ry, (float)S.b3, 65536.0f * (float)S.in_h);
        const int ilo = lo > hi ? 0x3FFFFFFF : (int)fmaxf(lo - 2.0f, -1e8f);
        const int ihi = lo > hi ? -0x3FFFFFFF : (int)fminf(hi + 2.0f, 1e8f);
        int blo = 0x3FFFFFFF, bhi = -0x3FFFFFFF;
#pragma unroll
        for (int rr = 0; rr < HR; ++rr) {
            blo = min(blo, __builtin_amdgcn_readlane(ilo, rr));
            bhi = max(bhi, __builtin_amdgcn_readlane(ihi, rr));
        }
        B.xlo = blo;
        B.xhi = bhi;
    }

    __syncthreads();  // tables visible
    // Fill (raw 0 = black, rotations.py's transparent fill read back without
    // alpha): uniform over the block except for zone bits.
    constexpr int MODE = StageMode<NR, ZONES>::v;
    const uint32_t fill = hsv2_px<NR, false>(L.T, 0u, ~0u);
    if (threadIdx.x == 0) L.stage[4 * HP_SLOTS] = stage_px<NR, MODE>(L.T, 0u);
    const int nrows = min(HR, h.lines - row0);
    hpass3_body<NR, ZONES, CN>(L, B, tmp, coefs, h, row0, nrows, zr0, zrh, zc0, zcw, fill);
}

// V pass on MFMA (tap tiles aligned with 16-row background bands: the plan's
// phase = p.y mod 16) → unpremultiply → blend onto the background, fused with
// the background copy.  Block = 16 composite rows of one item.  A = taps of
// the band's 16 overlay rows (lane l: row l&15, T rows 16(l>>4)..+15 of the K
// step), B = 64 T rows × 16 overlay columns of one channel (four 16-B T groups
// per lane give all four channels), D lane l = column l&15, rows 4(l>>4)..+3.
constexpr int VBR = 16;

template <int STORE, int DBG = 0, bool BANDS = false>
__global__ void __launch_bounds__(256)
k_pipe_vblend_mfma(const uint8_t* __restrict__ tmp, const uint8_t* __restrict__ bg, uint8_t* __restrict__ dst,
                   const int32_t* __restrict__ coefs, const ipp_pipe_desc* __restrict__ descs, int tiles_y,
                   int ov_w_max) {
    extern __shared__ __attribute__((aligned(16))) uint32_t orow[];  // [VBR][ov_w_max]
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / tiles_y;
    const int ty = b - im * tiles_y;
    const ipp_paste_desc p = descs[im].p;
    int y0 = ty * VBR;
    if (BANDS) {  // only the 16-row bands the overlay touches (the rest: ipp_pipe_hpass_bgcopy)
        int vb0, vb1;
        paste_bands(p, vb0, vb1);
        y0 += vb0;
        if (y0 >= vb1) return;
    }
    if (y0 >= p.bg_h) return;
    const int nrows = min(VBR, p.bg_h - y0);
    const int oy_lo = max(0, y0 - p.y), oy_hi = min(p.ov_h, y0 + nrows - p.y);
    const bool any = (DBG & 2) ? false : oy_lo < oy_hi;  // block-uniform
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

    if (any) {
        const ipp_resample_desc v = descs[im].v;
        const int phase = p.y & 15;
        const int ntiles = (v.out_len + phase + 15) >> 4;
        const int t = (y0 - p.y + phase) >> 4;  // the band's tap tile
        const int4* thdr = reinterpret_cast<const int4*>(coefs + v.coef_off);
        const int32_t* tbias = coefs + v.coef_off + 4 * (int64_t)ntiles;
        const uint4* tblk = reinterpret_cast<const uint4*>(coefs + v.coef_off + 20 * (int64_t)ntiles);
        const int4 th = thdr[t];
        const int ctiles = (p.ov_w + 15) >> 4;
        const int gstride = v.src_pitch >> 4;  // uint4 per T group row
        const int x_l = lane & 15;
        for (int ct = wave; ct < ctiles; ct += 4) {
            const int x = 16 * ct + x_l;
            const int xs = min(x, p.ov_w - 1);
            i32x4 acc[4][3];
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int q = 0; q < 3; ++q) acc[c][q] = i32x4{0, 0, 0, 0};
#pragma unroll 1
            for (int ks = 0; ks < th.y; ++ks) {
                i32x4 a[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) a[q] = __builtin_bit_cast(i32x4, tblk[th.z + (ks * 3 + q) * 64 + lane]);
                const int G = (th.x + 64 * ks + 16 * (lane >> 4)) >> 2;
                const uint4* tq = reinterpret_cast<const uint4*>(tmp + v.src_off + (int64_t)G * v.src_pitch) + xs;
                const uint4 g0 = tq[0], g1 = tq[gstride], g2 = tq[2 * gstride], g3 = tq[3 * gstride];
                const i32x4 bq[4] = {i32x4{(int)g0.x, (int)g1.x, (int)g2.x, (int)g3.x},
                                     i32x4{(int)g0.y, (int)g1.y, (int)g2.y, (int)g3.y},
                                     i32x4{(int)g0.z, (int)g1.z, (int)g2.z, (int)g3.z},
                                     i32x4{(int)g0.w, (int)g1.w, (int)g2.w, (int)g3.w}};
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        acc[c][q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[q], bq[c], acc[c][q], 0, 0, 0);
            }
            if (x < p.ov_w) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 4 * (lane >> 4) + r;   // band row = tile row
                    const int o = y0 + row - p.y;           // overlay row
                    if (o >= oy_lo && o < oy_hi) {
                        const int32_t bias = tbias[16 * t + row];
                        uint32_t px = 0;
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            px |= clip8(bias + acc[c][0][r] + (acc[c][1][r] << 8) + (acc[c][2][r] << 16)) << (8 * c);
                        orow[row * ov_w_max + x] = unpremultiply(px);
                    }
                }
            }
        }
        __syncthreads();
    }

    // Phase 2: composite rows = background bytes, blended inside the footprint.
    // Four 16-B chunks per thread are loaded before any is stored, so each
    // wave keeps four background reads in flight.
    const int row_bytes = 3 * p.bg_w;
    const int chunks = (row_bytes + 15) >> 4;
    const int total = nrows * chunks;
    for (int base = threadIdx.x; base < total; base += 4 * 256) {
        uint32_t w[4][4];
        int rr[4], c0[4], nb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int idx = base + u * 256;
            rr[u] = idx / chunks;
            c0[u] = (idx - rr[u] * chunks) << 4;
            nb[u] = idx < total ? min(16, row_bytes - c0[u]) : 0;
            if (nb[u] > 0) {
                const uint8_t* bp = bg + p.bg_off + (int64_t)(y0 + rr[u]) * p.bg_pitch + c0[u];
                if (DBG & 1) {
                    w[u][0] = w[u][1] = w[u][2] = w[u][3] = (uint32_t)c0[u];
                } else {
                    load16(bp, nb[u], nb[u] == 16 && (reinterpret_cast<uintptr_t>(bp) & 15u) == 0, w[u]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (nb[u] <= 0) continue;
            const int o = y0 + rr[u] - p.y;
            if (any && o >= oy_lo && o < oy_hi && c0[u] + nb[u] > 3 * p.x && c0[u] < 3 * (p.x + p.ov_w)) {
                const uint32_t* orw = orow + rr[u] * ov_w_max;
                blend16(w[u], c0[u], nb[u], p.x, p.ov_w, [&](int ox) { return orw[ox]; });
            }
            uint8_t* dp = dst + p.dst_off + (int64_t)(y0 + rr[u]) * p.dst_pitch + c0[u];
            store16<STORE>(dp, nb[u], nb[u] == 16 && (reinterpret_cast<uintptr_t>(dp) & 15u) == 0, w[u]);
        }
    }
}

template <int NR, bool ZONES, int CN>
void launch_hpass(dim3 grid, hipStream_t s, const uint8_t* src, uint8_t* tmp, const int32_t* coefs,
                  const ipp_pipe_desc* descs, int ty, const ipp_hsv_params& hp, const uint8_t* bg, uint8_t* dst) {
    const int n = grid.x / ty;
    if (bg && dst) {  // H pass + the background rows outside the overlay bands
        const int cpi = copy_blocks_per_item();
        hipLaunchKernelGGL((k_pipe_hpass3<NR, ZONES, CN, true>), dim3((uint32_t)(n * (ty + cpi))), dim3(HP_THREADS), 0,
                           s, src, tmp, coefs, descs, ty, hp, bg, dst, cpi);
        return;
    }
    hipLaunchKernelGGL((k_pipe_hpass3<NR, ZONES, CN, false>), grid, dim3(HP_THREADS), 0, s, src, tmp, coefs, descs, ty,
                       hp, bg, dst, 0);
}

template <int NR>
void launch_hpass_nr(bool zones, int cn, dim3 grid, hipStream_t s, const uint8_t* src, uint8_t* tmp,
                     const int32_t* coefs, const ipp_pipe_desc* descs, int ty, const ipp_hsv_params& hp,
                     const uint8_t* bg, uint8_t* dst) {
    if (zones) {
        if (cn == 4) launch_hpass<NR, true, 4>(grid, s, src, tmp, coefs, descs, ty, hp, bg, dst);
        else launch_hpass<NR, true, 3>(grid, s, src, tmp, coefs, descs, ty, hp, bg, dst);
    } else {
        if (cn == 4) launch_hpass<NR, false, 4>(grid, s, src, tmp, coefs, descs, ty, hp, bg, dst);
        else launch_hpass<NR, false, 3>(grid, s, src, tmp, coefs, descs, ty, hp, bg, dst);
    }
}

}  // namespace

static int pipe_hpass_impl(const uint8_t* src, uint8_t* tmp, const int32_t* coefs, const ipp_pipe_desc* descs,
                           int32_t n_images, int32_t max_out_w, int32_t max_rows, int32_t src_cn,
                           const ipp_hsv_params* hsv, int32_t tap_format, const uint8_t* bg, uint8_t* dst,
                           void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !tmp || !coefs || !descs || !hsv || n_images < 0 || max_out_w <= 0 || max_rows <= 0) return IPP_E_ARG;
    if (src_cn != 3 && src_cn != 4) return IPP_E_ARG;
    if (tap_format != IPP_TAPS_MFMA) return IPP_E_ARG;  // the VALU dot4 kernels were retired
    const int ty = (max_rows + HR - 1) / HR;  // one block per 16-row band
    const int64_t blocks = (int64_t)ty * n_images;
    if ((int64_t)(ty + (bg ? copy_blocks_per_item() : 0)) * n_images >= INT32_MAX) return IPP_E_ARG;
    const dim3 grid((uint32_t)blocks);
    hipStream_t s = (hipStream_t)stream;
    // Zones are needed unless every range's zone is the whole image (all
    // margins 0).  The source channel count is uniform over the batch.
    bool zones = false;
    for (int k = 0; k < hsv->n_ranges; ++k)
        for (int m = 0; m < 4; ++m) zones |= hsv->r[k].zone[m] != 0;
    const int cn = src_cn;
    // A range that never matches: lo_v = 1 > hi_v = 0 (cv::inRange's empty range).
    const ipp_hsv_range never = ipp_hsv_range{{0, 0, 1}, {180, 255, 0}, {0, 0, 0, 0}};
    switch (hsv->n_ranges) {
        case 1: launch_hpass_nr<1>(zones, cn, grid, s, src, tmp, coefs, descs, ty, *hsv, bg, dst); break;
        case 2: launch_hpass_nr<2>(zones, cn, grid, s, src, tmp, coefs, descs, ty, *hsv, bg, dst); break;
        case 3: launch_hpass_nr<3>(zones, cn, grid, s, src, tmp, coefs, descs, ty, *hsv, bg, dst); break;
        case 4: launch_hpass_nr<4>(zones, cn, grid, s, src, tmp, coefs, descs, ty, *hsv, bg, dst); break;
        case 5: case 6: {
            ipp_hsv_params q = *hsv;  // pad with never-matching ranges (lo > hi in v)
            for (int k = q.n_ranges; k < 6; ++k) q.r[k] = never;
            launch_hpass_nr<6>(zones, cn, grid, s, src, tmp, coefs, descs, ty, q, bg, dst);
            break;
        }
        default: {
            if (hsv->n_ranges > IPP_MAX_HSV_RANGES) return IPP_E_ARG;
            ipp_hsv_params q = *hsv;
            for (int k = q.n_ranges; k < IPP_MAX_HSV_RANGES; ++k) q.r[k] = never;
            launch_hpass_nr<IPP_MAX_HSV_RANGES>(zones, cn, grid, s, src, tmp, coefs, descs, ty, q, bg, dst);
            break;
        }
    }
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_pipe_hpass(const uint8_t* src, uint8_t* tmp, const int32_t* coefs, const ipp_pipe_desc* descs,
                              int32_t n_images, int32_t max_out_w, int32_t max_rows, int32_t src_cn,
                              const ipp_hsv_params* hsv, int32_t tap_format, void* stream) {
    return pipe_hpass_impl(src, tmp, coefs, descs, n_images, max_out_w, max_rows, src_cn, hsv, tap_format, nullptr,
                           nullptr, stream);
}

extern "C" int ipp_pipe_hpass_bgcopy(const uint8_t* src, uint8_t* tmp, const int32_t* coefs,
                                     const ipp_pipe_desc* descs, int32_t n_images, int32_t max_out_w,
                                     int32_t max_rows, int32_t src_cn, const ipp_hsv_params* hsv,
                                     int32_t tap_format, const uint8_t* bg, uint8_t* dst, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!bg || !dst || tap_format != IPP_TAPS_MFMA) return IPP_E_ARG;
    return pipe_hpass_impl(src, tmp, coefs, descs, n_images, max_out_w, max_rows, src_cn, hsv, tap_format, bg, dst,
                           stream);
}

extern "C" int ipp_pipe_status(int32_t* status, void* stream) {
    if (!status) return IPP_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    const int32_t zero = 0;
    if (hipMemcpyFromSymbolAsync(status, HIP_SYMBOL(g_pipe_status), sizeof(int32_t), 0, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipMemcpyToSymbolAsync(HIP_SYMBOL(g_pipe_status), &zero, sizeof(int32_t), 0, hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return IPP_E_LAUNCH;
    return IPP_OK;
}

extern "C" int ipp_pipe_vblend_bands(const uint8_t* tmp, const uint8_t* bg, uint8_t* dst, const int32_t* coefs,
                                     const ipp_pipe_desc* descs, int32_t n_images, int32_t bg_w, int32_t bg_h,
                                     int32_t max_ov_w, int32_t max_ov_h, int32_t tap_format, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!tmp || !bg || !dst || !coefs || !descs || n_images < 0 || bg_w <= 0 || bg_h <= 0) return IPP_E_ARG;
    if (tap_format != IPP_TAPS_MFMA || max_ov_w <= 0 || max_ov_w > bg_w || max_ov_h <= 0 || max_ov_h > bg_h)
        return IPP_E_ARG;
    const size_t sm = (size_t)VBR * max_ov_w * sizeof(uint32_t);
    // an overlay of height H at any y spans at most ceil((15 + H) / 16) bands
    const int tyb = std::min((max_ov_h + 15 + VBR - 1) / VBR, (bg_h + VBR - 1) / VBR);
    const int64_t nb = (int64_t)tyb * n_images;
    if (nb >= INT32_MAX || sm > 64 * 1024) return IPP_E_ARG;
    hipLaunchKernelGGL((k_pipe_vblend_mfma<2, 0, true>), dim3((uint32_t)nb), dim3(256), sm, (hipStream_t)stream, tmp,
                       bg, dst, coefs, descs, tyb, max_ov_w);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_pipe_vblend(const uint8_t* tmp, const uint8_t* bg, uint8_t* dst, const int32_t* coefs,
                               const ipp_pipe_desc* descs, int32_t n_images, int32_t bg_w, int32_t bg_h,
                               int32_t max_ov_w, int32_t tap_format, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!tmp || !bg || !dst || !coefs || !descs || n_images < 0 || bg_w <= 0 || bg_h <= 0) return IPP_E_ARG;
    if (tap_format != IPP_TAPS_MFMA || max_ov_w <= 0 || max_ov_w > bg_w) return IPP_E_ARG;
    const size_t sm = (size_t)VBR * max_ov_w * sizeof(uint32_t);
    const int tyb = (bg_h + VBR - 1) / VBR;
    const int64_t nb = (int64_t)tyb * n_images;
    if (nb >= INT32_MAX || sm > 64 * 1024) return IPP_E_ARG;
    const dim3 grid((uint32_t)nb);
    hipStream_t st = (hipStream_t)stream;
#ifdef IPP_DIAG
    // store policy 0 plain / 1 sc1 / 2 nt; experiment kernels (WRONG output):
    // 9 no background reads, 10 no V pass, 11 stores only
    static const int pol = diag_env("IPP_VB_STORE", 2);
    switch (pol) {
        case 0: hipLaunchKernelGGL(k_pipe_vblend_mfma<0>, grid, dim3(256), sm, st, tmp, bg, dst, coefs, descs, tyb, max_ov_w); break;
        case 1: hipLaunchKernelGGL(k_pipe_vblend_mfma<1>, grid, dim3(256), sm, st, tmp, bg, dst, coefs, descs, tyb, max_ov_w); break;
        case 9: hipLaunchKernelGGL((k_pipe_vblend_mfma<2, 1>), grid, dim3(256), sm, st, tmp, bg, dst, coefs, descs, tyb, max_ov_w); break;
        case 10: hipLaunchKernelGGL((k_pipe_vblend_mfma<2, 2>), grid, dim3(256), sm, st, tmp, bg, dst, coefs, descs, tyb, max_ov_w); break;
        case 11: hipLaunchKernelGGL((k_pipe_vblend_mfma<2, 3>), grid, dim3(256), sm, st, tmp, bg, dst, coefs, descs, tyb, max_ov_w); break;
        default: hipLaunchKernelGGL(k_pipe_vblend_mfma<2>, grid, dim3(256), sm, st, tmp, bg, dst, coefs, descs, tyb, max_ov_w); break;
    }
#else
    // nt stores: the write-once composite does not evict the shared backgrounds
    hipLaunchKernelGGL(k_pipe_vblend_mfma<2>, grid, dim3(256), sm, st, tmp, bg, dst, coefs, descs, tyb, max_ov_w);
#endif
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
