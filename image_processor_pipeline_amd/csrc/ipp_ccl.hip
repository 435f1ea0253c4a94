// ipp_ccl.hip — K10..K13: pixels_isolés.keep_largest_component, and the fused
// config-5 chain (filtres_liste HSV mask → keep largest → crop-fit).
//
// Reference: pixels_isolés.py:32 threshold(α, 1, 255, BINARY) → fg = α > 1;
// :35 connectedComponentsWithStats(fg, connectivity=8); :38-44 largest area,
// strict '>' so the lowest OpenCV label wins ties; :47-55 α := 0 outside it
// (when there is no foreground at all, label 0 — the background — is "kept"
// and α is left unchanged); :74-81 crop-fit to the bbox of α ≠ 0.
//
// Component identity.  Pixel (x, y) has the BLOCK-RASTER index
//   L = ((y >> 1) * wb + (x >> 1)) * 4 + (y & 1) * 2 + (x & 1),  wb = ⌈w/2⌉,
// and every union links the larger index under the smaller, so a component's
// root is its minimum L: root >> 2 is the first 2×2 scan block (blocks in
// raster order) that touches it — the order in which OpenCV's block-based
// 8-connectivity labelling (Spaghetti/BBDT) numbers components.  The tie rule
// is therefore "smallest root" (restated; UNPINNED: OpenCV is absent here).
//
// Algorithm (tile-local labelling, then border merging):
//   K1 k_ccl_tile     one 64×32 tile per block, one wave per row: fg bits
//                     (α > 1, or the fused HSV mask) by ballot → horizontal
//                     runs labelled without atomics (run start = highest
//                     clear bit below the lane) → one LDS union per pair of
//                     8-adjacent runs in consecutive rows → per-pixel local
//                     root (uint16, raster) → per-component area and row /
//                     column masks (bbox) by wave-aggregated LDS atomics →
//                     one entry per local
//                     component {global root, area, bbox}; P[root] = root.
//   K2 k_ccl_border   unites the local roots of 8-adjacent fg pixel pairs
//                     straddling a tile border, skipping pairs a neighbouring
//                     border pixel already unites (global atomicMin
//                     union-find on P, touched only at local roots).
//   K3 k_ccl_resolve  per entry: R = find(P, L); A[R] += area; P[L] = R.
//   K4 k_ccl_best     per global root: atomicMax of (area << 32 | ~root).
//   K5 k_ccl_bbox     per entry of the best component: bbox atomics.
//   K6 k_ccl_emit     per tile meeting the output: flags of its local roots
//                     (in the best component?) in LDS, then per pixel α := 0
//                     outside it in place (plugin path), or the crop-fit
//                     written as BGRA from the BGR frame (fused chain).
// Pixels are read once in K1 and once in K6 (within the crop for the fused
// chain); everything else is per component.
#include <algorithm>

#include <type_traits>

#include "ipp_hsv.h"

namespace {

constexpr int TW = 64, TH = 32, TPX = TW * TH;  // tile (2048 pixels)
constexpr uint16_t NOFG = 0xFFFF;

struct Frame {
    int w, h, wb, tiles_x, tiles_y;
};

__device__ __forceinline__ Frame frame_of(const ipp_image_desc& d) {
    Frame f;
    f.w = d.w;
    f.h = d.h;
    f.wb = (d.w + 1) >> 1;
    f.tiles_x = (d.w + TW - 1) / TW;
    f.tiles_y = (d.h + TH - 1) / TH;
    return f;
}

__device__ __forceinline__ int32_t gidx(const Frame& f, int x, int y) {
    return (((y >> 1) * f.wb + (x >> 1)) << 2) + ((y & 1) << 1) + (x & 1);
}

// Local (in-tile) index with the same ordering as gidx among the tile's pixels.
__device__ __forceinline__ int lidx(int lx, int ly) {
    return (((ly >> 1) * (TW / 2) + (lx >> 1)) << 2) + ((ly & 1) << 1) + (lx & 1);
}
__device__ __forceinline__ void lpos(int li, int& lx, int& ly) {
    const int blk = li >> 2;
    ly = ((blk / (TW / 2)) << 1) + ((li >> 1) & 1);
    lx = ((blk % (TW / 2)) << 1) + (li & 1);
}

// Global index of the local root `lr` of tile (tx, ty).
__device__ __forceinline__ int32_t root_gidx(const Frame& f, int tx, int ty, int lr) {
    int lx, ly;
    lpos(lr, lx, ly);
    return gidx(f, tx * TW + lx, ty * TH + ly);
}

__device__ __forceinline__ int32_t ld(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int32_t gfind(const int32_t* P, int32_t x) {
    int32_t p = ld(P + x);
    while (p != x) {
        x = p;
        p = ld(P + x);
    }
    return x;
}

__device__ __forceinline__ void gunite(int32_t* P, int32_t a, int32_t b) {
    for (;;) {
        a = gfind(P, a);
        b = gfind(P, b);
        if (a == b) return;
        if (a > b) {
            const int32_t t = a;
            a = b;
            b = t;
        }
        const int32_t old = atomicMin(P + b, a);
        if (old == b) return;
        b = old;
    }
}

__device__ __forceinline__ int lld(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ int lfind(const int* lab, int x) {
    int p = lld(lab + x);
    while (p != x) {
        x = p;
        p = lld(lab + x);
    }
    return x;
}

__device__ __forceinline__ void lunite(int* lab, int a, int b) {
    for (;;) {
        a = lfind(lab, a);
        b = lfind(lab, b);
        if (a == b) return;
        if (a > b) {
            const int t = a;
            a = b;
            b = t;
        }
        const int old = atomicMin(lab + b, a);
        if (old == b) return;
        b = old;
    }
}

// Scratch layout per image (offsets in the ipp_ccl_work descriptor).
struct Work {
    uint16_t* lab16;   // w*h local roots (raster); NOFG for background
    int32_t* P;        // 4*wb*hb parent array (touched at local roots only)
    uint32_t* A;       // 4*wb*hb areas (touched at roots only)
    int32_t* entL;     // per local component: global root index
    uint32_t* entA;    // ... its in-tile area
    int4* entB;        // ... its bbox (x0, y0, x1, y1), image coordinates
    int2* tile;        // per tile: (first entry, entry count)
};

__device__ __forceinline__ Work work_of(uint8_t* scratch, const ipp_ccl_work& w) {
    Work k;
    k.lab16 = reinterpret_cast<uint16_t*>(scratch + w.lab_off);
    k.P = reinterpret_cast<int32_t*>(scratch + w.p_off);
    k.A = reinterpret_cast<uint32_t*>(scratch + w.a_off);
    k.entL = reinterpret_cast<int32_t*>(scratch + w.ent_off);
    k.entA = reinterpret_cast<uint32_t*>(scratch + w.ent_off) + w.ent_cap;
    k.entB = reinterpret_cast<int4*>(scratch + w.ent_off + 8 * w.ent_cap);
    k.tile = reinterpret_cast<int2*>(scratch + w.tile_off);
    return k;
}

// Local index of the pixel with global block-raster index L inside tile (tx, ty).
__device__ __forceinline__ int local_of(const Frame& f, int32_t L, int tx, int ty) {
    const int32_t blk = L >> 2;
    const int by = blk / f.wb, bx = blk - by * f.wb;
    const int y = 2 * by + ((L >> 1) & 1), x = 2 * bx + (L & 1);
    return lidx(x - tx * TW, y - ty * TH);
}

// Foreground source: α > 1 of a 4-channel image, or the HSV mask of a
// 3-channel BGR image (fused chain).
enum { SRC_ALPHA = 0, SRC_HSV = 1 };

constexpr int NT = 4;            // tiles per labelling block: a 64×128 strip
constexpr int MAXC = TPX / 4;    // ≤ one 8-connected component per 2×2 block of a tile

// Per-lane source samples of one tile (8 rows of the lane's column): the raw
// pixel dword (HSV source) or the alpha byte (α source).  Loads of tile t+1 are
// issued before tile t is labelled, so their latency hides behind its work.
template <int SRC>
__device__ __forceinline__ void ccl_load(const uint8_t* __restrict__ img, const ipp_image_desc& d, int x, int ty,
                                         int wave, uint32_t (&raw)[TH / 4]) {
#pragma unroll
    for (int j = 0; j < TH / 4; ++j) {
        const int y = ty * TH + wave + 4 * j;
        raw[j] = 0u;
        if (x < d.w && y < d.h) {
            const uint8_t* row = img + d.off + (int64_t)y * d.pitch;
            if (SRC == SRC_ALPHA) {
                raw[j] = row[4 * x + 3];
            } else {
                const bool wide_ok = (y < d.h - 1) || (x < d.w - 1);
                raw[j] = load_rgb_opaque(row + 3 * x, wide_ok);
            }
        }
    }
}

// K1: one block labels NT vertically consecutive 64×32 tiles.  Per tile:
//   A  fg bits per row (ballot) → run labels (each pixel points at its run
//      start, the run minimum) — no atomics;
//   B  one LDS union per pair of 8-adjacent runs in consecutive rows;
//   C  local root of every pixel (run starts walk the forest, the run takes
//      its start's root by shuffle);
//   C2 roots get compact ids 0..n-1 (per-component LDS arrays of TPX/4, not
//      per-pixel ones: 20 KB of LDS per block, 8 blocks per CU);
//   D  area and row/column masks per component by wave-aggregated LDS
//      atomics; the uint16 local-root plane; the tile's entry range from one
//      global atomic whose latency hides behind D;
//   E  one entry {global root, area, bbox} per component; P[root] = root.
template <int SRC, int NR, bool ZONES>
__global__ void __launch_bounds__(256)
k_ccl_tile(const uint8_t* __restrict__ img, const ipp_image_desc* __restrict__ descs,
           const ipp_ccl_work* __restrict__ works, uint8_t* __restrict__ scratch, int32_t* __restrict__ counts,
           int strips_per_img, int tiles_x_max, ipp_hsv_params hp) {
    constexpr int RPW = TH / 4;  // rows per wave
    __shared__ int lab[TPX];     // union-find parents; then, at roots, the component id
    __shared__ uint32_t c_area[MAXC];
    __shared__ unsigned long long c_cols[MAXC];
    __shared__ uint32_t c_rows[MAXC];
    __shared__ uint16_t c_root[MAXC];
    __shared__ unsigned long long rowbits[TH];
    struct NoTables {};
    __shared__ typename std::conditional<SRC == SRC_HSV, HsvTables<NR>, NoTables>::type T;
    __shared__ int nroots, base;
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / strips_per_img;
    const int s = b - im * strips_per_img;
    const int sy = s / tiles_x_max, tx = s - sy * tiles_x_max;
    const ipp_image_desc d = descs[im];
    const Frame f = frame_of(d);
    const int ty0 = sy * NT;
    if (tx >= f.tiles_x || ty0 >= f.tiles_y) return;  // block-uniform
    const int ntile = min(NT, f.tiles_y - ty0);
    const Work k = work_of(scratch, works[im]);
    uint32_t cur[RPW], nxt[RPW];
    ccl_load<SRC>(img, d, tx * TW + (int)(threadIdx.x & 63), ty0, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                  cur);
    Ranges<SRC == SRC_HSV ? NR : 1> R;  // zones only (the test itself is table-driven)
    if constexpr (SRC == SRC_HSV) {
        hsv_tables_init<NR>(T, hp);
        if (ZONES) ranges_init<NR, ZONES>(R, hp, d.w, d.h);
    }

#pragma unroll 1
    for (int it = 0; it < ntile; ++it) {
        // Per-lane values are re-derived every tile from an opaque copy of the
        // lane id: hoisted out of the loop they would pin ~70 VGPRs for the
        // whole strip and halve the occupancy.
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int x = tx * TW + lane;
        const unsigned long long below = (1ull << lane) - 1ull;
        const int ty = ty0 + it;
        if (it + 1 < ntile) ccl_load<SRC>(img, d, x, ty + 1, wave, nxt);
        if (threadIdx.x == 0) nroots = 0;
        if (SRC == SRC_HSV && it == 0) __syncthreads();  // tables visible

        // A. fg bits per row and run labels.
        uint32_t fgmask = 0;
        int startlane[RPW];
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int ly = wave + 4 * j, y = ty * TH + ly;
            bool fg = false;
            if (x < d.w && y < d.h) {
                if (SRC == SRC_ALPHA) {
                    fg = cur[j] > 1u;
                } else if constexpr (SRC == SRC_HSV) {
                    uint32_t ex = hsv_tab_excl<NR, true>(T, cur[j]);
                    if (ZONES) {
                        uint32_t zb = 0;
#pragma unroll
                        for (int q = 0; q < NR; ++q)
                            zb |= (uint32_t)(((uint32_t)(y - R.r0[q]) < (uint32_t)R.rh[q]) &
                                             ((uint32_t)(x - R.c0[q]) < (uint32_t)R.cw[q])) << q;
                        ex &= zb;
                    }
                    fg = ex == 0u;
                }
            }
            const unsigned long long bits = __ballot(fg);
            const unsigned long long gaps = ~bits & below;
            const int start = gaps ? 64 - __clzll(gaps) : 0;
            startlane[j] = start;
            lab[lidx(lane, ly)] = fg ? lidx(start, ly) : -1;
            if (lane == 0) rowbits[ly] = bits;
            fgmask |= (fg ? 1u : 0u) << j;
        }
        __syncthreads();

        // B. one union per pair of 8-adjacent runs in rows ly-1, ly: the run
        //    start takes the pixels above-left and above; every pixel takes
        //    the one above-right when it starts a run segment above.
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int ly = wave + 4 * j;
            if (ly == 0 || !((fgmask >> j) & 1u)) continue;
            const unsigned long long up = rowbits[ly - 1];
            const int li = lidx(lane, ly);
            const bool at_start = lane == 0 || !((rowbits[ly] >> (lane - 1)) & 1ull);
            const bool u = (up >> lane) & 1ull;
            if (at_start) {
                if (lane > 0 && ((up >> (lane - 1)) & 1ull)) lunite(lab, li, lidx(lane - 1, ly - 1));
                if (u) lunite(lab, li, lidx(lane, ly - 1));
            }
            if (lane < TW - 1 && ((up >> (lane + 1)) & 1ull) && !u) lunite(lab, li, lidx(lane + 1, ly - 1));
        }
        __syncthreads();

        // C. local root of every pixel.
        int root[RPW];
        uint32_t rootmask = 0;
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int li = lidx(lane, wave + 4 * j);
            const bool fg = (fgmask >> j) & 1u;
            const int rs = (fg && startlane[j] == lane) ? lfind(lab, li) : 0;
            const int rr = __shfl(rs, startlane[j]);
            root[j] = fg ? rr : -1;
            rootmask |= (root[j] == li ? 1u : 0u) << j;
        }
        __syncthreads();

        // C2. compact component ids at the roots.
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            if (!((rootmask >> j) & 1u)) continue;
            const int li = lidx(lane, wave + 4 * j);
            const int c = atomicAdd(&nroots, 1);
            lab[li] = c;
            c_root[c] = (uint16_t)li;
            c_area[c] = 0u;
            c_cols[c] = 0ull;
            c_rows[c] = 0u;
        }
        __syncthreads();

        // D. per row, per distinct component in the wave: area and bbox masks
        //    (one set of LDS atomics per component, by its lowest lane);
        //    the local-root plane; the tile's entry range.
        int gbase = 0;
        const int n = nroots;
        if (threadIdx.x == 0 && n > 0) gbase = atomicAdd(&counts[im], n);
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int ly = wave + 4 * j, y = ty * TH + ly;
            const bool fg = (fgmask >> j) & 1u;
            const int cid = fg ? lab[root[j]] : -1;
            unsigned long long pending = __ballot(fg);
            while (pending) {
                const int leader = __ffsll((long long)pending) - 1;
                const int c = __shfl(cid, leader);
                const unsigned long long same = __ballot(cid == c) & pending;
                if (lane == leader) {
                    atomicAdd(&c_area[c], (uint32_t)__popcll(same));
                    atomicOr(&c_cols[c], same);
                    atomicOr(&c_rows[c], 1u << ly);
                }
                pending &= ~same;
            }
            if (x < d.w && y < d.h) k.lab16[(int64_t)y * d.w + x] = fg ? (uint16_t)root[j] : NOFG;
        }
        if (threadIdx.x == 0) {
            base = gbase;
            k.tile[ty * f.tiles_x + tx] = make_int2(gbase, n);
        }
        __syncthreads();

        // E. one entry per component.
        const int x0 = tx * TW, y0 = ty * TH;
        for (int c = threadIdx.x; c < n; c += 256) {
            const int li = c_root[c];
            int lx, ly;
            lpos(li, lx, ly);
            const int32_t L = gidx(f, x0 + lx, y0 + ly);
            const int e = base + c;
            k.entL[e] = L;
            k.entA[e] = c_area[c];
            const unsigned long long cm = c_cols[c];
            const uint32_t rm = c_rows[c];
            k.entB[e] = make_int4(x0 + __ffsll((long long)cm) - 1, y0 + __ffs((int)rm) - 1, x0 + 64 - __clzll(cm),
                                  y0 + 32 - __clz((int)rm));
            k.P[L] = L;
            k.A[L] = 0u;
        }
        __syncthreads();  // LDS reused by the next tile
#pragma unroll
        for (int j = 0; j < RPW; ++j) cur[j] = nxt[j];
    }
}

// Pixel (x, y) of tile-local root → global root index, or -1 for background.
__device__ __forceinline__ int32_t root_of(const Frame& f, const Work& k, int x, int y) {
    const uint16_t r = k.lab16[(int64_t)y * f.w + x];
    if (r == NOFG) return -1;
    return root_gidx(f, x / TW, y / TH, r);
}

// Border pairs.  Thread i < vert owns left pixel (64*bx - 1, y) of a vertical
// tile border and its 8-neighbours (64*bx, y-1..y+1); the rest own the upper
// pixel (x, 32*by - 1) of a horizontal border and (x-1..x+1, 32*by).  Along a
// border, consecutive owners usually see the same pair of roots: a pair is
// skipped when the previous (next) owner with the same near-side root takes
// it, so a long shared boundary costs one union, not one per pixel.
__global__ void __launch_bounds__(256)
k_ccl_border(const ipp_image_desc* __restrict__ descs, const ipp_ccl_work* __restrict__ works,
             uint8_t* __restrict__ scratch, int chunks) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / chunks;
    const int64_t i = (int64_t)(b - (uint32_t)im * chunks) * 256 + threadIdx.x;
    const ipp_image_desc d = descs[im];
    const Frame f = frame_of(d);
    const Work k = work_of(scratch, works[im]);
    const int64_t vert = (int64_t)(f.tiles_x - 1) * f.h;
    const int64_t horz = (int64_t)(f.tiles_y - 1) * f.w;
    // near side pixel (nx, ny) moving along the border by (sx, sy); far side at +(fx, fy)
    int nx, ny, sx, sy, fx, fy, pos, len;
    if (i < vert) {
        const int bx = 1 + (int)(i / f.h);
        pos = (int)(i % f.h);
        len = f.h;
        nx = bx * TW - 1, ny = pos, sx = 0, sy = 1, fx = 1, fy = 0;
    } else if (i < vert + horz) {
        const int64_t j = i - vert;
        const int by = 1 + (int)(j / f.w);
        pos = (int)(j % f.w);
        len = f.w;
        nx = pos, ny = by * TH - 1, sx = 1, sy = 0, fx = 0, fy = 1;
    } else {
        return;
    }
    const int32_t a = root_of(f, k, nx, ny);
    if (a < 0) return;
    auto near_at = [&](int p) { return (p < 0 || p >= len) ? -1 : root_of(f, k, nx + (p - pos) * sx, ny + (p - pos) * sy); };
    auto far_at = [&](int p) {
        return (p < 0 || p >= len) ? -1 : root_of(f, k, nx + fx + (p - pos) * sx, ny + fy + (p - pos) * sy);
    };
    const int32_t ap = near_at(pos - 1), an = near_at(pos + 1);
    const int32_t cp = far_at(pos - 1), c0 = far_at(pos), cn = far_at(pos + 1);
    if (cp >= 0 && ap != a) gunite(k.P, a, cp);
    if (c0 >= 0 && !(ap == a && cp == c0)) gunite(k.P, a, c0);
    if (cn >= 0 && an != a) gunite(k.P, a, cn);
}

// Entry kernels run ENT_BLOCKS blocks per image striding over the image's
// entry count (known only on the device).
constexpr int ENT_BLOCKS = 32;

__global__ void __launch_bounds__(256)
k_ccl_resolve(const ipp_ccl_work* __restrict__ works, uint8_t* __restrict__ scratch,
              const int32_t* __restrict__ counts) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / ENT_BLOCKS;
    const int n = counts[im];
    const Work k = work_of(scratch, works[im]);
    for (int e = (int)(b - (uint32_t)im * ENT_BLOCKS) * 256 + threadIdx.x; e < n; e += ENT_BLOCKS * 256) {
        const int32_t L = k.entL[e];
        const int32_t R = gfind(k.P, L);
        atomicAdd(k.A + R, k.entA[e]);
        if (R != L) __hip_atomic_store(k.P + L, R, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void __launch_bounds__(256)
k_ccl_best(const ipp_ccl_work* __restrict__ works, uint8_t* __restrict__ scratch, const int32_t* __restrict__ counts,
           unsigned long long* __restrict__ best) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / ENT_BLOCKS;
    const int n = counts[im];
    const Work k = work_of(scratch, works[im]);
    unsigned long long key = 0ull;
    for (int e = (int)(b - (uint32_t)im * ENT_BLOCKS) * 256 + threadIdx.x; e < n; e += ENT_BLOCKS * 256) {
        const int32_t L = k.entL[e];
        if (k.P[L] == L) {
            const unsigned long long kk =
                ((unsigned long long)k.A[L] << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)L);
            key = kk > key ? kk : key;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off);
        key = o > key ? o : key;
    }
    if ((threadIdx.x & 63) == 0 && key) atomicMax(best + im, key);
}

__device__ __forceinline__ int32_t best_root(unsigned long long key) {
    return key ? (int32_t)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull)) : -1;
}

// K5: bbox of the best component = union of its entries' tile bboxes.
__global__ void __launch_bounds__(256)
k_ccl_bbox(const ipp_ccl_work* __restrict__ works, uint8_t* __restrict__ scratch, const int32_t* __restrict__ counts,
           const unsigned long long* __restrict__ best, int32_t* __restrict__ bbox) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / ENT_BLOCKS;
    const int32_t broot = best_root(best[im]);
    int4 bb = make_int4(INT32_MAX, INT32_MAX, -1, -1);
    if (broot >= 0) {
        const int n = counts[im];
        const Work k = work_of(scratch, works[im]);
        for (int e = (int)(b - (uint32_t)im * ENT_BLOCKS) * 256 + threadIdx.x; e < n; e += ENT_BLOCKS * 256) {
            if (k.P[k.entL[e]] == broot) {
                const int4 q = k.entB[e];
                bb = make_int4(min(bb.x, q.x), min(bb.y, q.y), max(bb.z, q.z), max(bb.w, q.w));
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        bb.x = min(bb.x, __shfl_xor(bb.x, off));
        bb.y = min(bb.y, __shfl_xor(bb.y, off));
        bb.z = max(bb.z, __shfl_xor(bb.z, off));
        bb.w = max(bb.w, __shfl_xor(bb.w, off));
    }
    if ((threadIdx.x & 63) == 0 && bb.z >= 0) {
        atomicMin(&bbox[4 * im + 0], bb.x);
        atomicMin(&bbox[4 * im + 1], bb.y);
        atomicMax(&bbox[4 * im + 2], bb.z);
        atomicMax(&bbox[4 * im + 3], bb.w);
    }
}

// Flags (LDS) of a tile's local roots: in the best component?  Returns false
// when the tile has no pixel of it.
__device__ __forceinline__ bool tile_flags(const Frame& f, const Work& k, int tx, int ty, int32_t broot,
                                           uint8_t* flag, int* any) {
    const int2 te = k.tile[ty * f.tiles_x + tx];
    if (threadIdx.x == 0) *any = 0;
    __syncthreads();
    for (int e = threadIdx.x; e < te.y; e += 256) {
        const int32_t L = k.entL[te.x + e];
        const bool in = k.P[L] == broot;
        flag[local_of(f, L, tx, ty)] = in ? 1 : 0;
        if (in) *any = 1;
    }
    __syncthreads();
    return *any != 0;
}

// K6, plugin path: in place on a 4-channel image, α := 0 outside the best
// component (images without any component are left unchanged).
__global__ void __launch_bounds__(256)
k_ccl_apply(uint8_t* __restrict__ img, const ipp_image_desc* __restrict__ descs, const ipp_ccl_work* __restrict__ works,
            uint8_t* __restrict__ scratch, const unsigned long long* __restrict__ best, int tiles_per_img,
            int tiles_x_max) {
    __shared__ uint8_t flag[TPX];
    __shared__ int any;
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / tiles_per_img;
    const int t = b - im * tiles_per_img;
    const int ty = t / tiles_x_max, tx = t - ty * tiles_x_max;
    const ipp_image_desc d = descs[im];
    const Frame f = frame_of(d);
    if (tx >= f.tiles_x || ty >= f.tiles_y) return;
    const int32_t broot = best_root(best[im]);
    if (broot < 0) return;
    const Work k = work_of(scratch, works[im]);
    tile_flags(f, k, tx, ty, broot, flag, &any);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = tx * TW + lane;
    if (x >= d.w) return;
    for (int j = 0; j < TH / 4; ++j) {
        const int y = ty * TH + wave + 4 * j;
        if (y >= d.h) break;
        const uint16_t r = k.lab16[(int64_t)y * d.w + x];
        if (r == NOFG || !flag[r]) {
            uint8_t* a = img + d.off + (int64_t)y * d.pitch + 4 * (int64_t)x + 3;
            if (*a) *a = 0;
        }
    }
}

// K6, fused chain: crop-fit of the BGR frame to the best component's bbox,
// written as BGRA (α = 255 inside the component, 0 elsewhere) into the image's
// output slot; one block per labelling tile that meets the bbox.
__global__ void __launch_bounds__(256)
k_ccl_crop_bgr(const uint8_t* __restrict__ img, const ipp_image_desc* __restrict__ descs,
               const ipp_ccl_work* __restrict__ works, uint8_t* __restrict__ scratch,
               const unsigned long long* __restrict__ best, const int32_t* __restrict__ bbox,
               uint8_t* __restrict__ out, const ipp_image_desc* __restrict__ out_descs, int tiles_per_img,
               int tiles_x_max) {
    __shared__ uint8_t flag[TPX];
    __shared__ int any;
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / tiles_per_img;
    const int t = b - im * tiles_per_img;
    const int ty = t / tiles_x_max, tx = t - ty * tiles_x_max;
    const ipp_image_desc d = descs[im];
    const Frame f = frame_of(d);
    if (tx >= f.tiles_x || ty >= f.tiles_y) return;
    const int32_t broot = best_root(best[im]);
    if (broot < 0) return;
    const int bx0 = bbox[4 * im + 0], by0 = bbox[4 * im + 1], bx1 = bbox[4 * im + 2], by1 = bbox[4 * im + 3];
    if (tx * TW >= bx1 || (tx + 1) * TW <= bx0 || ty * TH >= by1 || (ty + 1) * TH <= by0) return;
    const Work k = work_of(scratch, works[im]);
    tile_flags(f, k, tx, ty, broot, flag, &any);
    const ipp_image_desc od = out_descs[im];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = tx * TW + lane;
    if (x < bx0 || x >= bx1) return;
    for (int j = 0; j < TH / 4; ++j) {
        const int y = ty * TH + wave + 4 * j;
        if (y < by0) continue;
        if (y >= by1) break;
        const bool wide_ok = (y < d.h - 1) || (x < d.w - 1);
        const uint32_t px = load_rgb_opaque(img + d.off + (int64_t)y * d.pitch + 3 * (int64_t)x, wide_ok);
        const uint16_t r = k.lab16[(int64_t)y * d.w + x];
        const bool in = r != NOFG && flag[r];
        reinterpret_cast<uint32_t*>(out + od.off + (int64_t)(y - by0) * od.pitch)[x - bx0] =
            (px & 0x00FFFFFFu) | (in ? 0xFF000000u : 0u);
    }
}

__global__ void k_ccl_prep(int32_t* bbox, unsigned long long* best, int32_t* counts, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        bbox[4 * i + 0] = INT32_MAX;
        bbox[4 * i + 1] = INT32_MAX;
        bbox[4 * i + 2] = -1;
        bbox[4 * i + 3] = -1;
        best[i] = 0ull;
        counts[i] = 0;
    }
}

__global__ void k_ccl_finish(int32_t* bbox, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && bbox[4 * i + 2] < 0) bbox[4 * i + 0] = bbox[4 * i + 1] = bbox[4 * i + 2] = bbox[4 * i + 3] = -1;
}

struct Launch {
    int tiles_x, tiles_y, tiles_per_img, strips_per_img;
    int border_chunks, ent_chunks;
    dim3 tile_grid, strip_grid, border_grid, ent_grid;
    bool ok;
};

Launch plan_launch(int n, int max_w, int max_h, int64_t max_ent) {
    Launch L{};
    L.tiles_x = (max_w + TW - 1) / TW;
    L.tiles_y = (max_h + TH - 1) / TH;
    L.tiles_per_img = L.tiles_x * L.tiles_y;
    L.strips_per_img = L.tiles_x * ((L.tiles_y + NT - 1) / NT);
    const int64_t border = (int64_t)(L.tiles_x - 1) * max_h + (int64_t)(L.tiles_y - 1) * max_w;
    L.border_chunks = (int)std::max<int64_t>(1, (border + 255) / 256);
    (void)max_ent;
    L.ent_chunks = ENT_BLOCKS;
    const int64_t tb = (int64_t)L.tiles_per_img * n, bb = (int64_t)L.border_chunks * n, eb = (int64_t)L.ent_chunks * n;
    L.ok = tb < INT32_MAX && bb < INT32_MAX && eb < INT32_MAX;
    L.tile_grid = dim3((uint32_t)tb);
    L.strip_grid = dim3((uint32_t)((int64_t)L.strips_per_img * n));
    L.border_grid = dim3((uint32_t)bb);
    L.ent_grid = dim3((uint32_t)eb);
    return L;
}

template <int SRC, int NR, bool ZONES>
void launch_tiles(const Launch& L, hipStream_t s, const uint8_t* img, const ipp_image_desc* descs,
                  const ipp_ccl_work* works, uint8_t* scratch, int32_t* counts, const ipp_hsv_params& hp) {
    hipLaunchKernelGGL((k_ccl_tile<SRC, NR, ZONES>), L.strip_grid, dim3(256), 0, s, img, descs, works, scratch,
                       counts, L.strips_per_img, L.tiles_x, hp);
}

// K1..K5 common to both entry points.
int run_labels(int src, const uint8_t* img, const ipp_image_desc* descs, int32_t n, int32_t max_w, int32_t max_h,
               const ipp_hsv_params* hsv, const ipp_ccl_work* works, uint8_t* scratch, int64_t max_ent,
               int32_t* counts, unsigned long long* best, int32_t* bbox, hipStream_t s, Launch& L) {
    L = plan_launch(n, max_w, max_h, max_ent);
    if (!L.ok) return IPP_E_ARG;
    const int nb = (n + 255) / 256;
    hipLaunchKernelGGL(k_ccl_prep, dim3(nb), dim3(256), 0, s, bbox, best, counts, n);
    if (src == SRC_ALPHA) {
        launch_tiles<SRC_ALPHA, 1, false>(L, s, img, descs, works, scratch, counts, ipp_hsv_params{});
    } else {
        const bool zones = hsv_has_zones(*hsv);
        const bool small = hsv->n_ranges <= 4;
        const ipp_hsv_params q = hsv_pad(*hsv, small ? 4 : IPP_MAX_HSV_RANGES);
        if (small && !zones) launch_tiles<SRC_HSV, 4, false>(L, s, img, descs, works, scratch, counts, q);
        else if (small) launch_tiles<SRC_HSV, 4, true>(L, s, img, descs, works, scratch, counts, q);
        else if (!zones) launch_tiles<SRC_HSV, IPP_MAX_HSV_RANGES, false>(L, s, img, descs, works, scratch, counts, q);
        else launch_tiles<SRC_HSV, IPP_MAX_HSV_RANGES, true>(L, s, img, descs, works, scratch, counts, q);
    }
    hipLaunchKernelGGL(k_ccl_border, L.border_grid, dim3(256), 0, s, descs, works, scratch, L.border_chunks);
    hipLaunchKernelGGL(k_ccl_resolve, L.ent_grid, dim3(256), 0, s, works, scratch, counts);
    hipLaunchKernelGGL(k_ccl_best, L.ent_grid, dim3(256), 0, s, works, scratch, counts, best);
    hipLaunchKernelGGL(k_ccl_bbox, L.ent_grid, dim3(256), 0, s, works, scratch, counts, best, bbox);
    return IPP_OK;
}

}  // namespace

extern "C" int64_t ipp_ccl_scratch_layout(int32_t w, int32_t h, ipp_ccl_work* work) {
    if (w <= 0 || h <= 0) return IPP_E_ARG;
    const int64_t wb = (w + 1) / 2, hb = (h + 1) / 2;
    const int64_t slots = 4 * wb * hb;
    if (slots >= INT32_MAX) return IPP_E_RANGE;
    // ≤ one component per 2×2 block of a tile (8-connectivity), per tile
    const int64_t tiles = (int64_t)((w + TW - 1) / TW) * ((h + TH - 1) / TH);
    const int64_t cap = tiles * (TPX / 4);
    auto al = [](int64_t v) { return (v + 255) & ~(int64_t)255; };
    ipp_ccl_work k{};
    k.lab_off = 0;
    k.p_off = al(2 * (int64_t)w * h);
    k.a_off = k.p_off + al(4 * slots);
    k.ent_off = k.a_off + al(4 * slots);
    k.ent_cap = cap;
    k.tile_off = k.ent_off + al(24 * cap);
    const int64_t total = k.tile_off + al(8 * tiles);
    if (work) *work = k;
    return total;
}

extern "C" int ipp_ccl_keep_largest(uint8_t* img, const ipp_image_desc* descs, int32_t n_images, int32_t max_w,
                                    int32_t max_h, const ipp_ccl_work* works, uint8_t* scratch, int64_t max_ent,
                                    int32_t* counts, int64_t* stats, int32_t* bbox, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!img || !descs || !works || !scratch || !counts || !stats || !bbox || n_images < 0 || max_w <= 0 ||
        max_h <= 0 || max_ent <= 0)
        return IPP_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    unsigned long long* best = reinterpret_cast<unsigned long long*>(stats);
    Launch L;
    const int rc = run_labels(SRC_ALPHA, img, descs, n_images, max_w, max_h, nullptr, works, scratch, max_ent, counts,
                              best, bbox, s, L);
    if (rc != IPP_OK) return rc;
    hipLaunchKernelGGL(k_ccl_apply, L.tile_grid, dim3(256), 0, s, img, descs, works, scratch, best, L.tiles_per_img,
                       L.tiles_x);
    hipLaunchKernelGGL(k_ccl_finish, dim3((n_images + 255) / 256), dim3(256), 0, s, bbox, n_images);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_video_keep_largest(const uint8_t* frames, const ipp_image_desc* descs, int32_t n_images,
                                      int32_t max_w, int32_t max_h, const ipp_hsv_params* hsv,
                                      const ipp_ccl_work* works, uint8_t* scratch, int64_t max_ent, int32_t* counts,
                                      int64_t* stats, int32_t* bbox, uint8_t* out,
                                      const ipp_image_desc* out_descs, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!frames || !descs || !hsv || !works || !scratch || !counts || !stats || !bbox || !out || !out_descs ||
        n_images < 0 || max_w <= 0 || max_h <= 0 || max_ent <= 0)
        return IPP_E_ARG;
    if (hsv->n_ranges < 0 || hsv->n_ranges > IPP_MAX_HSV_RANGES) return IPP_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    unsigned long long* best = reinterpret_cast<unsigned long long*>(stats);
    Launch L;
    const int rc = run_labels(SRC_HSV, frames, descs, n_images, max_w, max_h, hsv, works, scratch, max_ent, counts,
                              best, bbox, s, L);
    if (rc != IPP_OK) return rc;
    hipLaunchKernelGGL(k_ccl_crop_bgr, L.tile_grid, dim3(256), 0, s, frames, descs, works, scratch, best, bbox, out,
                       out_descs, L.tiles_per_img, L.tiles_x);
    hipLaunchKernelGGL(k_ccl_finish, dim3((n_images + 255) / 256), dim3(256), 0, s, bbox, n_images);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
