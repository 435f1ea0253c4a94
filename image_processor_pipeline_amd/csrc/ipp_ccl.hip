// ipp_ccl.hip — K10..K13: pixels_isolés.keep_largest_component, and the fused
// config-5 chain (filtres_liste HSV mask → keep largest → crop-fit).
//
// Reference: pixels_isolés.py:32 threshold(α, 1, 255, BINARY) → fg = α > 1;
// :35 connectedComponentsWithStats(fg, connectivity=8); :38-44 largest area,
// strict '>' so the lowest OpenCV label wins ties; :47-55 α := 0 outside it
// (when there is no foreground at all, label 0 — the background — is "kept"
// and α is left unchanged); :74-81 crop-fit to the bbox of α ≠ 0.
//
// Component identity.  A horizontal run of fg pixels starting at (x, y) has
// the RUN-START index
//   G = (((y >> 1) * wb + (x >> 1)) << 1) + (y & 1),  wb = ⌈w/2⌉,
// unique because two run starts of one row are ≥ 2 columns apart (tile
// borders are at even columns).  A component's pixel of minimum block-raster
// order ((y>>1, x>>1), then y&1, x&1) is always a run start, and G orders run
// starts exactly that way, so every union links the larger G under the
// smaller and a component's root is the first 2×2 scan block (blocks in
// raster order) that touches it — the order in which OpenCV's block-based
// 8-connectivity labelling (Spaghetti/BBDT) numbers components.  The tie rule
// is therefore "smallest root" (restated; UNPINNED: OpenCV is absent here).
//
// Algorithm (bit-plane runs; one wave per 64×64 tile, lane = row):
//   K1 k_ccl_label   fg bit per pixel (α > 1, or the fused HSV mask), one
//                    ballot per row → the row's 64-bit mask word in lane r.
//                    Runs come from the word (start = m & ~(m << 1)); each
//                    run unites, through a per-wave LDS union-find over run
//                    slots, with the runs of row r-1 it touches (8-adjacency:
//                    columns a-1 .. b+1).  Compact component ids by a wave
//                    scan; area / row and column masks per component by LDS
//                    atomics in passes of MAXC ids.  A component touching a
//                    tile edge ("open") gets an entry {root G, area, bbox};
//                    one that does not ("closed") is final here and competes
//                    for the image's closed key by one 64-bit atomicMax.
//                    Written per non-empty tile: the 64 mask words, the root
//                    of every edge pixel, a record {components, the only
//                    root, edge flags}.  No per-pixel label plane.
//   K2 k_ccl_border  per tile (64 tiles per wave): unites the roots of 8-adjacent fg
//                    pixel pairs across its right and bottom borders and its
//                    two lower-right corners (only where both edge flags are
//                    set), skipping pairs a neighbouring border pixel already
//                    unites (global atomicMin union-find on P, at roots).
//   K3 k_ccl_resolve per open entry: R = find(P, G); A[R] += area; P[G] = R.
//   K4 k_ccl_best    per open root: atomicMax of (area << 32 | ~root).
//   K5 k_ccl_bbox    the kept component = the better of the open and closed
//                    bests; bbox from the closed key, or from its entries.
//                    (One launch for K3-K5, the image's last block doing K4
//                    and K5 over all its entries, ran 0.2 ms slower per
//                    video4k step: 16 blocks per image are needed there.)
//   K6 k_ccl_apply / k_ccl_inwords, one wave per tile meeting the output:
//                    a one-component tile takes its mask words or nothing; a
//                    tile with several relabels its words (the same
//                    deterministic labelling as K1, so the same ids) and looks
//                    up each component's final root.  Then α := 0 outside the
//                    component in place (plugin path), or (fused chain) the
//                    words are stored and k_ccl_crop_stream writes the crop-fit
//                    as BGRA from the BGR frame in output-row order.
// Pixels are read once in K1 and once in K6 (within the crop for the fused
// chain); everything else is per run, per component or per edge pixel.
#include <algorithm>
#include <type_traits>

#include "ipp_hsv.h"

namespace {

constexpr int TW = 64, TH = 64;        // tile: one wave, lane r owns row r
constexpr int NJ = (TW / 2) * TH;      // run-start slots per tile (row, column pair)
constexpr int MAXC = 32;               // component stats per LDS pass
constexpr int CMAX = (TW / 2) * (TH / 2);  // ≤ one 8-connected component per 2×2 block
constexpr int WAVES = 4;               // tiles (waves) per block
typedef unsigned long long u64;

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

// Run-start slot inside a tile; orders slots as G orders run starts.
__device__ __forceinline__ int slot(int r, int a) { return ((((r >> 1) << 5) + (a >> 1)) << 1) | (r & 1); }

// Global run-start index of slot j of tile (tx, ty).
__device__ __forceinline__ int32_t slot_gidx(const Frame& f, int tx, int ty, int j) {
    const int r = ((j >> 6) << 1) | (j & 1);
    const int y = ty * TH + r;
    return (((y >> 1) * f.wb + tx * (TW / 2) + ((j >> 1) & 31)) << 1) + (y & 1);
}

__device__ __forceinline__ int ctz64(u64 v) { return __ffsll((long long)v) - 1; }

// Calls fn(a, len) for every run of word m (a = first column).
template <class F>
__device__ __forceinline__ void for_runs(u64 m, F fn) {
    u64 s = m & ~(m << 1);
    while (s) {
        const int a = ctz64(s);
        const u64 rest = ~m >> a;
        const int len = rest ? ctz64(rest) : 64 - a;
        fn(a, len);
        s &= s - 1;
    }
}

__device__ __forceinline__ u64 run_mask(int a, int len) {
    return (len >= 64 ? ~0ull : ((1ull << len) - 1ull)) << a;
}

__device__ __forceinline__ int32_t ld(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Find with path halving: each visited node is re-pointed at its grandparent
// by a no-return atomicMin (parents only ever decrease), so the chains that
// concurrent unions build stay short.
__device__ __forceinline__ int32_t gfind(int32_t* P, int32_t x) {
    int32_t p = ld(P + x);
    while (p != x) {
        const int32_t gp = ld(P + p);
        if (gp == p) return p;
        __hip_atomic_fetch_min(P + x, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        x = gp;
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

// Per-wave LDS union-find over run slots, 16-bit entries (slots < NJ, and
// NJ + component id < NJ + CMAX after label_tile): 4 KB per wave.  A union's
// atomicMin is a 32-bit compare-and-swap on the word holding the entry (LDS
// has no 16-bit atomics); plain 16-bit loads and stores elsewhere.
typedef uint16_t Par;

__device__ __forceinline__ int lld(const Par* p) { return *reinterpret_cast<const volatile Par*>(p); }

// Physical position of run slot j in the union-find array.  Slot j's dword
// (two 16-bit entries: rows 2k and 2k+1 of one column pair) sits on bank
// (column pair) mod 32, so the runs of many rows that start in one column — a
// blob crossing the tile's left edge — hit one bank: that is where
// k_ccl_label's LDS bank conflicts come from (2.2e8 of 5.9e8 LDS cycles;
// profiles/r05/ccl/).  Rotating the bank by the row pair cut them to 5.8e7 but
// cost VALU on every union-find access: config 5 0.3-5 % slower (round 5, two
// forms measured), so slots stay in place.
__device__ __forceinline__ int pswz(int j) { return j; }

__device__ __forceinline__ int lfind(const Par* par, int x) {
    int p = lld(par + pswz(x));
    while (p != x) {
        x = p;
        p = lld(par + pswz(x));
    }
    return x;
}

// par[b] = min(par[b], a); returns the previous par[b].
__device__ __forceinline__ int lmin16(Par* par, int b, int a) {
    uint32_t* w = reinterpret_cast<uint32_t*>(par + (pswz(b) & ~1));
    const int sh = (b & 1) * 16;
    uint32_t cur = *reinterpret_cast<volatile uint32_t*>(w);
    for (;;) {
        const int old = (int)((cur >> sh) & 0xFFFFu);
        if (old <= a) return old;
        const uint32_t nw = (cur & ~(0xFFFFu << sh)) | ((uint32_t)a << sh);
        const uint32_t prev = atomicCAS(w, cur, nw);
        if (prev == cur) return old;
        cur = prev;
    }
}

__device__ __forceinline__ void lunite(Par* par, int a, int b) {
    for (;;) {
        a = lfind(par, a);
        b = lfind(par, b);
        if (a == b) return;
        if (a > b) {
            const int t = a;
            a = b;
            b = t;
        }
        const int old = lmin16(par, b, a);
        if (old == b) return;
        b = old;
    }
}

// LDS writes of one lane become visible to the other lanes of its wave.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-wide exclusive prefix sum of v (and the total).
__device__ __forceinline__ int wave_scan_excl(int v, int lane, int& total) {
    int s = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(s, o);
        if (lane >= o) s += t;
    }
    total = __shfl(s, 63);
    return s - v;
}

// (Pointer jumping after the unions: 2.998 -> 2.978 ms per config-5 step;
// tiles where no run touches the row above skip the unions and the root
// pass: 2.957 -> 2.934 ms; round 5, alternating runs on one box.)
// Tile labelling on the mask words (lane r: word m of row r, p of row r-1).
// On return par[slot] holds, for a root run, NJ + its component id, and for
// any other run its root's slot; returns the component count.  Component ids
// follow (row, run) order — a pure function of the words, so K6 relabelling a
// tile reproduces K1's ids.
__device__ __forceinline__ int label_tile(Par* par, int r, int lane, u64 m, u64 p) {
    if (__builtin_amdgcn_ballot_w64((m & (p | (p << 1) | (p >> 1))) != 0ull) == 0ull) {
        // No run touches a run of the row above (a tile of isolated specks):
        // every run is a root, and the ids follow (row, run) order as below.
        int n;
        int cid = wave_scan_excl(__popcll(m & ~(m << 1)), lane, n);
        for_runs(m, [&](int a, int) { par[pswz(slot(r, a))] = NJ + cid++; });
        wave_sync();
        return n;
    }
    for_runs(m, [&](int a, int) { par[pswz(slot(r, a))] = slot(r, a); });
    wave_sync();
    if (p) {
        const u64 ps = p & ~(p << 1);
        for_runs(m, [&](int a, int len) {
            const int me = slot(r, a);
            if (a > 0 && ((p >> (a - 1)) & 1ull)) {
                // the run of row r-1 covering column a-1 starts at the highest
                // start ≤ a-1
                const u64 below = ps & ((a >= 64 ? ~0ull : ((1ull << a) - 1ull)));
                lunite(par, me, slot(r - 1, 63 - __clzll(below)));
            }
            const int hi = min(a + len, 63);  // columns a .. b+1
            u64 hit = ps & (((hi >= 63 ? ~0ull : ((2ull << hi) - 1ull))) & ~((1ull << a) - 1ull));
            while (hit) {
                lunite(par, me, slot(r - 1, ctz64(hit)));
                hit &= hit - 1;
            }
        });
    }
    wave_sync();
    // Pointer jumping: the unions of a column of runs (a blob crossing the
    // tile: each row's run linked under the row above's) leave chains as long
    // as the tile is tall, and the root pass below would walk them lane by
    // lane.  par[j] := par[par[j]] in lockstep halves every depth per round;
    // the wave stops when no lane moved (speck tiles: after one round).
    for (int it = 0; it < 6; ++it) {
        bool moved = false;
        for_runs(m, [&](int a, int) {
            const int j = slot(r, a);
            const int pj = par[pswz(j)];
            const int pp = par[pswz(pj)];
            if (pp != pj) {
                par[pswz(j)] = pp;
                moved = true;
            }
        });
        wave_sync();
        if (__builtin_amdgcn_ballot_w64(moved) == 0ull) break;
    }
    int nroot = 0;
    for_runs(m, [&](int a, int) {
        const int j = slot(r, a);
        const int root = lfind(par, j);
        nroot += root == j;
        if (root != j) par[pswz(j)] = root;
    });
    wave_sync();
    int n;
    int cid = wave_scan_excl(nroot, lane, n);
    for_runs(m, [&](int a, int) {
        const int j = slot(r, a);
        if (par[pswz(j)] == j) par[pswz(j)] = NJ + cid++;
    });
    wave_sync();
    return n;
}

__device__ __forceinline__ int run_root(const Par* par, int j) {
    const int v = par[pswz(j)];
    return v >= NJ ? j : v;
}
__device__ __forceinline__ int run_cid(const Par* par, int j) {
    const int v = par[pswz(j)];
    return (v >= NJ ? v : par[pswz(v)]) - NJ;
}

// Scratch layout per image (offsets in the ipp_ccl_work descriptor).
struct ImgRec {               // per-image record (img_off), zeroed by k_ccl_prep
    u64 ckey;                 // best closed component (closed_key)
    int32_t root;             // the kept component's root G, or -1 (k_ccl_bbox)
    int32_t pad;
};

struct TileRec {              // per tile
    int32_t n;                // components in the tile
    int32_t g1;               // root G of the only component when n == 1
    int32_t flags;            // fg on the tile's top / bottom / left / right edge
    int32_t g1_open;          // that component touches a tile edge (P holds its root)
};
enum { F_TOP = 1, F_BOT = 2, F_LEFT = 4, F_RIGHT = 8 };

struct Work {
    u64* mask;        // per tile 64 row words (tile-major)
    int32_t* edge;    // per tile 4 × 64 edge roots: top, bottom, left, right
    int32_t* P;       // 2*wb*hb parent array (touched at run-start roots only)
    uint32_t* A;      // 2*wb*hb areas (touched at open roots only)
    int32_t* entL;    // per OPEN component: global root index
    uint32_t* entA;   // ... its in-tile area
    int4* entB;       // ... its bbox (x0, y0, x1, y1), image coordinates
    TileRec* tile;
    ImgRec* rec;
};

__device__ __forceinline__ Work work_of(uint8_t* scratch, const ipp_ccl_work& w) {
    Work k;
    k.mask = reinterpret_cast<u64*>(scratch + w.mask_off);
    k.edge = reinterpret_cast<int32_t*>(scratch + w.edge_off);
    k.P = reinterpret_cast<int32_t*>(scratch + w.p_off);
    k.A = reinterpret_cast<uint32_t*>(scratch + w.a_off);
    k.entL = reinterpret_cast<int32_t*>(scratch + w.ent_off);
    k.entA = reinterpret_cast<uint32_t*>(scratch + w.ent_off) + w.ent_cap;
    k.entB = reinterpret_cast<int4*>(scratch + w.ent_off + 8 * w.ent_cap);
    k.tile = reinterpret_cast<TileRec*>(scratch + w.tile_off);
    k.rec = reinterpret_cast<ImgRec*>(scratch + w.img_off);
    return k;
}

enum { E_TOP = 0, E_BOT = 1, E_LEFT = 2, E_RIGHT = 3 };

// Closed components (no pixel on a tile edge) are final after K1: they never
// take part in a union.  Their best is kept per image in one 64-bit key whose
// order is the selection order (area, then smaller root):
//   area (13 bits) << 51 | (~G & 0x7FFFFF) << 24 | in-tile bbox (4 × 6 bits).
// Images with 2·wb·hb > 2^23 run-start slots treat every component as open.
constexpr int64_t CLOSED_SLOTS = 1 << 23;

__device__ __forceinline__ u64 closed_key(uint32_t area, int32_t G, int bx0, int by0, int bx1, int by1) {
    return ((u64)area << 51) | ((u64)(~(uint32_t)G & 0x7FFFFFu) << 24) |
           (u64)(bx0 | (by0 << 6) | ((bx1 - 1) << 12) | ((by1 - 1) << 18));
}

// Foreground source: α > 1 of a 4-channel image, or the HSV mask of a
// 3-channel BGR image (fused chain).
enum { SRC_ALPHA = 0, SRC_HSV = 1 };

constexpr int RB = 16;  // rows per load batch (double-buffered)

// Source samples of RB rows of the lane's column: the raw pixel dword (HSV
// source) or the alpha byte (α source).  FULL: every row is inside the image
// and not its last one, every column inside the image (no checks; a 4-byte
// read at the row's last pixel stays inside the next row).
template <int SRC, bool FULL>
__device__ __forceinline__ void load_rows(const uint8_t* __restrict__ img, const ipp_image_desc& d, int x, int y0,
                                          uint32_t (&raw)[RB]) {
    const uint8_t* base = img + d.off + (int64_t)y0 * d.pitch + (SRC == SRC_ALPHA ? 4 * x + 3 : 3 * x);
#pragma unroll
    for (int k = 0; k < RB; ++k) {
        const uint8_t* p = base + (int64_t)k * d.pitch;
        if (FULL) {
            raw[k] = SRC == SRC_ALPHA ? (uint32_t)*p : ld_u32_unaligned(p);
        } else {
            const int y = y0 + k;
            raw[k] = 0u;
            if (x < d.w && y < d.h) {
                if (SRC == SRC_ALPHA) raw[k] = *p;
                else raw[k] = load_rgb_opaque(p, (y < d.h - 1) || (x < d.w - 1));
            }
        }
    }
}

// v_writelane_b32: lane `lane` of v := s (uniform value and lane).
extern "C" __device__ int32_t ipp_llvm_writelane(int32_t, int32_t, int32_t) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ void writelane(uint32_t& v, uint32_t s, int lane) {
    v = (uint32_t)ipp_llvm_writelane((int32_t)s, lane, (int32_t)v);
}

// Mask words of one tile: lane = column while loading; lane r returns row r's
// word in m and row r-1's in p.
template <int SRC, int NR, bool ZONES, bool FULL>
__device__ __forceinline__ void tile_words(const uint8_t* __restrict__ img, const ipp_image_desc& d, int x, int y0,
                                           int lane, const HsvTables<NR>* T, const Ranges<NR>& R, u64& m, u64& p) {
    uint32_t zx = 0;  // ranges whose zone columns hold this lane's column
    if constexpr (SRC == SRC_HSV && ZONES) {
#pragma unroll
        for (int q = 0; q < NR; ++q) zx |= (uint32_t)((uint32_t)(x - R.c0[q]) < (uint32_t)R.cw[q]) << q;
    }
    const bool xin = x < d.w;
    uint32_t mlo = 0u, mhi = 0u;
    uint32_t bufA[RB], bufB[RB];
    load_rows<SRC, FULL>(img, d, x, y0, bufA);
#pragma unroll
    for (int rb = 0; rb < TH / RB; ++rb) {
        uint32_t(&cur)[RB] = (rb & 1) ? bufB : bufA;
        uint32_t(&nxt)[RB] = (rb & 1) ? bufA : bufB;
        if (rb + 1 < TH / RB) load_rows<SRC, FULL>(img, d, x, y0 + (rb + 1) * RB, nxt);
#pragma unroll
        for (int kk = 0; kk < RB; ++kk) {
            const int r = rb * RB + kk, y = y0 + r;
            bool fg;
            if constexpr (SRC == SRC_ALPHA) {
                fg = cur[kk] > 1u;
            } else {
                uint32_t ex;
                if constexpr (!ZONES && HsvTables<NR>::kDecided)
                    ex = hsv_tab_excl_vfirst<NR, true>(*T, cur[kk]);  // rows decided by v skip s and h
                else
                    ex = hsv_tab_excl<NR, true>(*T, cur[kk]);
                if (ZONES) {
                    uint32_t zy = 0;
#pragma unroll
                    for (int q = 0; q < NR; ++q) zy |= (uint32_t)((uint32_t)(y - R.r0[q]) < (uint32_t)R.rh[q]) << q;
                    ex &= zx & zy;
                }
                fg = ex == 0u;
            }
            if (!FULL) fg = fg && xin && y < d.h;
            const u64 bits = __ballot(fg);
            writelane(mlo, (uint32_t)bits, r);
            writelane(mhi, (uint32_t)(bits >> 32), r);
        }
    }
    m = ((u64)mhi << 32) | mlo;
    p = __shfl_up(m, 1);
    p = lane > 0 ? p : 0ull;
}

// DPP move within 16-lane rows (row_shl:k, lanes past the row end read 0).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

// Mask pass: pixel slots whose 64 pixels all have the wave's reference
// colour skip the HSV test (3.12 -> 2.98 ms per config-5 step on flat
// synthetic frames, round 5, alternating runs on one box;
// profiles/r05/ccl/ab_uniform_slots_r05n.txt).
// Mask words of one interior tile of a 3-channel HSV source (FULL): lane =
// (row rr = lane >> 4 of a 4-row group, pixel quad q = lane & 15), one 12-byte
// load per lane and group = 4 pixels (768 contiguous bytes per row group and
// wave instruction, a quarter of the one-dword-per-lane loads of
// tile_words).  The four fg bits of a lane form a nibble; a 16-lane DPP
// reduction assembles each row's 64-bit word in lane 16·rr, which is moved
// to lane r by readlane/writelane.  Same words as tile_words.
template <int NR>
__device__ __forceinline__ void tile_words_quads(const uint8_t* __restrict__ img, const ipp_image_desc& d, int X0,
                                                 int y0, int lane, const HsvTables<NR>* T, u64& m, u64& p) {
    // 12 bytes at a 3-byte pixel boundary: no alignment promise (the pitch
    // 3·w and the image offset need not be multiples of 4); the queues run in
    // unaligned-access mode, so this is still one global_load_dwordx3
    struct __attribute__((packed, aligned(1), may_alias)) u32x3 {
        uint32_t x, y, z;
    };
    const int q = lane & 15, rr = lane >> 4;
    const uint8_t* base = img + d.off + (int64_t)(y0 + rr) * d.pitch + 3 * (X0 + 4 * q);
    const int64_t gstep = 4 * (int64_t)d.pitch;  // next 4-row group
    constexpr int G = TH / 4, GB = 4;             // 16 groups, loaded 4 at a time (double-buffered)
    u32x3 bufA[GB], bufB[GB];
#pragma unroll
    for (int j = 0; j < GB; ++j) bufA[j] = *reinterpret_cast<const u32x3*>(base + j * gstep);
    uint32_t mlo = 0u, mhi = 0u;
    uint32_t ref_c = 0xFFFFFFFFu, ref_keep = 0u;  // reference colour (none yet) and its nibble
#pragma unroll
    for (int gb = 0; gb < G / GB; ++gb) {
        u32x3(&cur)[GB] = (gb & 1) ? bufB : bufA;
        u32x3(&nxt)[GB] = (gb & 1) ? bufA : bufB;
        if (gb + 1 < G / GB) {
#pragma unroll
            for (int j = 0; j < GB; ++j) nxt[j] = *reinterpret_cast<const u32x3*>(base + ((gb + 1) * GB + j) * gstep);
        }
#pragma unroll
        for (int j = 0; j < GB; ++j) {
            const uint32_t w0 = cur[j].x, w1 = cur[j].y, w2 = cur[j].z;
            const uint32_t px[4] = {w0, __builtin_amdgcn_alignbyte(w1, w0, 3), __builtin_amdgcn_alignbyte(w2, w1, 2),
                                    w2 >> 8};
            uint32_t nib = 0;
            // Pixel slots k whose 64 pixels all have the wave's reference
            // colour (lane 0's first pixel of the group: a frame's flat
            // background or blob) take its cached result instead of the HSV
            // test; the others, or all four, the full test.
            uint32_t need = 0xFu;
            {
                const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(px[0] & 0xFFFFFFu));
                need = 0u;
#pragma unroll
                for (int k = 0; k < 4; ++k) need |= (__builtin_amdgcn_ballot_w64((px[k] & 0xFFFFFFu) != c0) != 0ull) << k;
                if (need != 0xFu && c0 != ref_c) {  // wave-uniform: the reference colour's result, once
                    ref_c = c0;
                    ref_keep = hsv_post<NR>(*T, hsv_pre<NR, true>(*T, c0)) == 0u ? 0xFu : 0u;
                }
            }
            if (need == 0xFu) {
                HsvPre pre[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) pre[k] = hsv_pre<NR, true>(*T, px[k]);
#pragma unroll
                for (int k = 0; k < 4; ++k) nib |= (hsv_post<NR>(*T, pre[k]) == 0u ? 1u : 0u) << k;
            } else {
                nib = ref_keep & ~need;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if ((need >> k) & 1u) nib |= (hsv_post<NR>(*T, hsv_pre<NR, true>(*T, px[k])) == 0u ? 1u : 0u) << k;
            }
            // lanes 16rr + q → lane 16rr: 4 → 8 → 16 → 32 bits, then the high half
            uint32_t t = nib | (dpp<0x101>(nib) << 4);      // row_shl:1
            t = t | (dpp<0x102>(t) << 8);                     // row_shl:2
            t = t | (dpp<0x104>(t) << 16);                    // row_shl:4
            const uint32_t hi = dpp<0x108>(t);                // row_shl:8: bits 32..63
            // lanes 4G..4G+3 (G = this group) take the words of lanes 0, 16, 32, 48
            const int src = 64 * (lane & 3);                  // ds_bpermute byte address of lane 16·(lane & 3)
            const uint32_t wlo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)t);
            const uint32_t whi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)hi);
            const bool mine = (lane >> 2) == gb * GB + j;
            mlo = mine ? wlo : mlo;
            mhi = mine ? whi : mhi;
        }
    }
    m = ((u64)mhi << 32) | mlo;
    p = __shfl_up(m, 1);
    p = lane > 0 ? p : 0ull;
}

// K1: one wave per 64×64 tile, WAVES tiles side by side per block.  Occupancy
// target 6 waves per SIMD: 49-55 VGPRs, 7 waves/SIMD, no spills; 3.44 vs 3.63
// ms per video4k step against the compiler's choice (85-89 VGPRs, 5 waves).
template <int SRC, int NR, bool ZONES>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(6)))
k_ccl_label(const uint8_t* __restrict__ img, const ipp_image_desc* __restrict__ descs,
            const ipp_ccl_work* __restrict__ works, uint8_t* __restrict__ scratch, int32_t* __restrict__ counts,
            int groups_per_img, int groups_x, ipp_hsv_params hp) {
    __shared__ Par par_s[WAVES][NJ];
    __shared__ uint32_t st_area[WAVES][MAXC];
    __shared__ u64 st_rows[WAVES][MAXC], st_cols[WAVES][MAXC];
    __shared__ int st_root[WAVES][MAXC];
    struct NoTables {};
    __shared__ typename std::conditional<SRC == SRC_HSV, HsvTables<NR>, NoTables>::type T;
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / groups_per_img;
    const int g = b - im * groups_per_img;
    const int ty = g / groups_x;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int tx = (g - ty * groups_x) * WAVES + wave;
    const ipp_image_desc d = descs[im];
    const Frame f = frame_of(d);
    Ranges<NR> R;  // zones only (the test itself is table-driven)
    if constexpr (SRC == SRC_HSV) {
        hsv_tables_init<NR>(T, hp);
        if (ZONES) ranges_init<NR, ZONES>(R, hp, d.w, d.h);
        __syncthreads();
    }
    if (tx >= f.tiles_x || ty >= f.tiles_y) return;  // wave-uniform; no barrier follows
    Par* par = par_s[wave];
    const Work k = work_of(scratch, works[im]);
    const int x = tx * TW + lane, y0 = ty * TH, X0 = tx * TW;
    const int tile = ty * f.tiles_x + tx;

    // A. mask words.
    u64 m, p;
    const HsvTables<NR>* Tp = nullptr;
    if constexpr (SRC == SRC_HSV) Tp = &T;
    if constexpr (SRC == SRC_HSV && !ZONES && HsvTables<NR>::kDecided) {
        if (X0 + TW <= d.w && y0 + TH <= d.h)
            tile_words_quads<NR>(img, d, X0, y0, lane, Tp, m, p);
        else
            tile_words<SRC, NR, ZONES, false>(img, d, x, y0, lane, Tp, R, m, p);
    } else if (X0 + TW <= d.w && y0 + TH < d.h)
        tile_words<SRC, NR, ZONES, true>(img, d, x, y0, lane, Tp, R, m, p);
    else
        tile_words<SRC, NR, ZONES, false>(img, d, x, y0, lane, Tp, R, m, p);
    if (__ballot(m != 0ull) == 0ull) {  // no foreground: K2 and K6 skip the tile by its record
        if (lane == 0) k.tile[tile] = TileRec{0, -1, 0, 0};
        return;
    }
    k.mask[(int64_t)tile * TH + lane] = m;

    // B-F. runs, unions, component ids.
    const int r = lane;
    const int n = label_tile(par, r, lane, m, p);
    const bool closed_ok = 2ll * f.wb * ((f.h + 1) >> 1) <= CLOSED_SLOTS;

    int32_t g1 = -1, g1_open = 0;  // the only component's root (n == 1), for K6

    // Stats per component, MAXC ids per pass; open components get entries,
    // closed ones compete for the image's closed key.
    uint32_t* area = st_area[wave];
    u64* rows = st_rows[wave];
    u64* cols = st_cols[wave];
    int* croot = st_root[wave];
    u64 best_closed = 0ull;
    for (int c0 = 0; c0 < n; c0 += MAXC) {
        if (lane < MAXC) {
            area[lane] = 0u;
            rows[lane] = 0ull;
            cols[lane] = 0ull;
        }
        wave_sync();
        for_runs(m, [&](int a, int len) {
            const int j = slot(r, a);
            const int v = par[pswz(j)];
            const int c = (v >= NJ ? v : par[pswz(v)]) - NJ - c0;
            if ((unsigned)c < (unsigned)MAXC) {
                atomicAdd(&area[c], (uint32_t)len);
                atomicOr(&rows[c], 1ull << r);
                atomicOr(&cols[c], run_mask(a, len));
                if (v >= NJ) croot[c] = j;
            }
        });
        wave_sync();
        const bool valid = lane < MAXC && c0 + lane < n;
        u64 cm = 0ull, rm = 0ull;
        uint32_t ar = 0u;
        int32_t G = 0;
        if (valid) {
            cm = cols[lane];
            rm = rows[lane];
            ar = area[lane];
            G = slot_gidx(f, tx, ty, croot[lane]);
        }
        const bool edge = ((cm | rm) & (1ull | (1ull << 63))) != 0ull;
        const bool open = valid && (edge || !closed_ok);
        const int bx0 = ctz64(cm), by0 = ctz64(rm), bx1 = 64 - __clzll(cm), by1 = 64 - __clzll(rm);
        if (valid && !open) {
            const u64 key = closed_key(ar, G, bx0, by0, bx1, by1);
            best_closed = key > best_closed ? key : best_closed;
        }
        if (c0 == 0 && lane == 0) {
            g1 = G;
            g1_open = open;
        }
        const u64 om = __ballot(open);
        if (om) {
            int base = 0;
            if (lane == 0) base = atomicAdd(&counts[im], __popcll(om));
            base = __shfl(base, 0);
            if (open) {
                const int e = base + __popcll(om & ((1ull << lane) - 1ull));
                k.entL[e] = G;
                k.entA[e] = ar;
                k.entB[e] = make_int4(X0 + bx0, y0 + by0, X0 + bx1, y0 + by1);
                k.P[G] = G;  // open roots only: closed ones never take part in a union
                k.A[G] = 0u;
            }
        }
        wave_sync();
    }
    for (int off = 32; off > 0; off >>= 1) {
        const u64 o = __shfl_xor(best_closed, off);
        best_closed = o > best_closed ? o : best_closed;
    }
    if (lane == 0 && best_closed) atomicMax(&k.rec[0].ckey, best_closed);

    // Edge roots (global G of the pixel's root, -1 for background) of the
    // edges that hold foreground, and the tile record.
    int32_t* edge = k.edge + (int64_t)tile * (4 * 64);
    const u64 s = m & ~(m << 1);
    const u64 m0 = __shfl(m, 0), m63 = __shfl(m, TH - 1);
    const u64 lb = __ballot(m & 1ull), rbits = __ballot(m >> 63);
    if (lb) edge[E_LEFT * 64 + lane] = (m & 1ull) ? slot_gidx(f, tx, ty, run_root(par, slot(r, 0))) : -1;
    if (rbits)
        edge[E_RIGHT * 64 + lane] =
            (m >> 63) ? slot_gidx(f, tx, ty, run_root(par, slot(r, 63 - __clzll(s)))) : -1;
    const u64 upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    if (m0)
        edge[E_TOP * 64 + lane] =
            ((m0 >> lane) & 1ull) ? slot_gidx(f, tx, ty, run_root(par, slot(0, 63 - __clzll(m0 & ~(m0 << 1) & upto))))
                                  : -1;
    if (m63)
        edge[E_BOT * 64 + lane] =
            ((m63 >> lane) & 1ull)
                ? slot_gidx(f, tx, ty, run_root(par, slot(TH - 1, 63 - __clzll(m63 & ~(m63 << 1) & upto))))
                : -1;
    if (lane == 0)
        k.tile[tile] = TileRec{n, n == 1 ? g1 : -1,
                               (m0 ? F_TOP : 0) | (m63 ? F_BOT : 0) | (lb ? F_LEFT : 0) | (rbits ? F_RIGHT : 0),
                               g1_open};
}

// K2: per tile T, unions across its right border (pairs with the tile to
// the right, rows of one tile row), its bottom border, and the two corner
// pairs below-right: (63, 63)@T – (0, 0)@T+x+y and (0, 63)@T+x – (63, 0)@T+y.
// One wave takes 64 consecutive tiles: lane i loads the edge flags around tile
// i, and the wave walks only the borders whose both sides have foreground
// (launching a wave per tile made the kernel dispatch-bound).  Along a
// border, consecutive pixels usually see the same pair of roots: a pair is
// skipped when the previous (next) pixel with the same near-side root takes
// it, so a long shared boundary costs one union.
constexpr int ULIST = 256;  // pending unions per wave (LDS), flushed lane-parallel

struct UnionList {
    int2 u[ULIST];
};

__device__ __forceinline__ void flush_unions(int32_t* P, UnionList& L, int& n, int lane) {
    wave_sync();
    for (int i = lane; i < n; i += 64) gunite(P, L.u[i].x, L.u[i].y);
    n = 0;
    wave_sync();
}

// Appends the (a, c) pairs of the lanes with `want` set (wave-aggregated).
__device__ __forceinline__ void push_unions(int32_t* P, UnionList& L, int& n, int lane, bool want, int32_t a,
                                            int32_t c) {
    const u64 wm = __ballot(want);
    if (!wm) return;
    if (n + __popcll(wm) > ULIST) flush_unions(P, L, n, lane);
    if (want) L.u[n + __popcll(wm & ((1ull << lane) - 1ull))] = make_int2(a, c);
    n += __popcll(wm);
}

// One border of 64 pixel pairs (near edge, far edge; lane = position along it).
__device__ __forceinline__ void border_pairs(int32_t* P, UnionList& L, int& n, const int32_t* near,
                                             const int32_t* far, int lane) {
    const int32_t a = near[lane];
    const int32_t ap = lane > 0 ? near[lane - 1] : -1, an = lane < 63 ? near[lane + 1] : -1;
    const int32_t cp = lane > 0 ? far[lane - 1] : -1, c0 = far[lane], cn = lane < 63 ? far[lane + 1] : -1;
    const bool fg = a >= 0;
    push_unions(P, L, n, lane, fg && cp >= 0 && ap != a, a, cp);
    push_unions(P, L, n, lane, fg && c0 >= 0 && !(ap == a && cp == c0), a, c0);
    push_unions(P, L, n, lane, fg && cn >= 0 && an != a, a, cn);
}

__global__ void __launch_bounds__(64 * WAVES)
k_ccl_border(const ipp_image_desc* __restrict__ descs, const ipp_ccl_work* __restrict__ works,
             uint8_t* __restrict__ scratch, int chunks_per_img, int n_images) {
    __shared__ UnionList lists[WAVES];
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int cw = (int)b * WAVES + wave;
    const int im = cw / chunks_per_img;
    if (im >= n_images) return;  // the grid rounds up to whole blocks
    const int t = (cw - im * chunks_per_img) * 64 + lane;
    const ipp_image_desc d = descs[im];
    const Frame f = frame_of(d);
    const int ntiles = f.tiles_x * f.tiles_y;
    if ((cw - im * chunks_per_img) * 64 >= ntiles) return;  // wave-uniform
    const Work k = work_of(scratch, works[im]);
    UnionList& L = lists[wave];
    int n = 0;
    const int ty = t / f.tiles_x, tx = t - ty * f.tiles_x;
    const bool valid = t < ntiles;
    const bool has_r = valid && tx + 1 < f.tiles_x, has_b = valid && ty + 1 < f.tiles_y;
    const int fl = valid ? k.tile[t].flags : 0;
    const int fr = has_r ? k.tile[t + 1].flags : 0;
    const int fb = has_b ? k.tile[t + f.tiles_x].flags : 0;
    const int fd = has_r && has_b ? k.tile[t + f.tiles_x + 1].flags : 0;
    auto E = [&](int u, int which) { return k.edge + (int64_t)u * (4 * 64) + which * 64; };
    // corners: lane-parallel, one pair each at most
    {
        int32_t a = -1, c = -1;
        if ((fl & F_BOT) && (fd & F_TOP)) {
            a = E(t, E_BOT)[63];
            c = E(t + f.tiles_x + 1, E_TOP)[0];
        }
        push_unions(k.P, L, n, lane, a >= 0 && c >= 0, a, c);
        a = c = -1;
        if ((fr & F_BOT) && (fb & F_TOP)) {
            a = E(t + 1, E_BOT)[0];
            c = E(t + f.tiles_x, E_TOP)[63];
        }
        push_unions(k.P, L, n, lane, a >= 0 && c >= 0, a, c);
    }
    u64 hv = __ballot((fl & F_RIGHT) && (fr & F_LEFT));
    u64 vv = __ballot((fl & F_BOT) && (fb & F_TOP));
    const int t0 = t - lane;
    while (hv) {
        const int u = t0 + ctz64(hv);
        border_pairs(k.P, L, n, E(u, E_RIGHT), E(u + 1, E_LEFT), lane);
        hv &= hv - 1;
    }
    while (vv) {
        const int u = t0 + ctz64(vv);
        border_pairs(k.P, L, n, E(u, E_BOT), E(u + f.tiles_x, E_TOP), lane);
        vv &= vv - 1;
    }
    flush_unions(k.P, L, n, lane);
}

// Entry kernels (open components only) run ENT_BLOCKS blocks per image
// striding over the image's entry count (known only on the device).
constexpr int ENT_BLOCKS = 16;

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

// K5: the kept component = the larger of the best open one (best[im]: area
// << 32 | ~root) and the best closed one (rec.ckey), the smaller root on equal
// areas; its bbox = the closed key's tile bbox, or the union of its open
// entries' tile bboxes.  The image's first block records the root for K6.
__global__ void __launch_bounds__(256)
k_ccl_bbox(const ipp_image_desc* __restrict__ descs, const ipp_ccl_work* __restrict__ works,
           uint8_t* __restrict__ scratch, const int32_t* __restrict__ counts,
           const unsigned long long* __restrict__ best, int32_t* __restrict__ bbox) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / ENT_BLOCKS;
    const int blk = b - im * ENT_BLOCKS;
    const Work k = work_of(scratch, works[im]);
    const u64 ko = best[im], kc = k.rec->ckey;
    const uint32_t ao = (uint32_t)(ko >> 32), ac = (uint32_t)(kc >> 51);
    const int32_t go = ko ? (int32_t)(0xFFFFFFFFu - (uint32_t)ko) : -1;
    const int32_t gc = kc ? (int32_t)(~(uint32_t)(kc >> 24) & 0x7FFFFFu) : -1;
    const bool closed_wins = kc && (!ko || ac > ao || (ac == ao && gc < go));
    const int32_t broot = closed_wins ? gc : go;
    if (blk == 0 && threadIdx.x == 0) {
        k.rec->root = broot;
        if (closed_wins) {
            const Frame f = frame_of(descs[im]);
            const int yb = (gc >> 1) / f.wb;
            const int tx = ((gc >> 1) - yb * f.wb) / (TW / 2), ty = (2 * yb + (gc & 1)) / TH;
            const uint32_t q = (uint32_t)(kc & 0xFFFFFFu);
            bbox[4 * im + 0] = tx * TW + (int)(q & 63u);
            bbox[4 * im + 1] = ty * TH + (int)((q >> 6) & 63u);
            bbox[4 * im + 2] = tx * TW + (int)((q >> 12) & 63u) + 1;
            bbox[4 * im + 3] = ty * TH + (int)((q >> 18) & 63u) + 1;
        }
    }
    if (closed_wins || broot < 0) return;
    int4 bb = make_int4(INT32_MAX, INT32_MAX, -1, -1);
    const int n = counts[im];
    for (int e = blk * 256 + threadIdx.x; e < n; e += ENT_BLOCKS * 256) {
        if (k.P[k.entL[e]] == broot) {
            const int4 q = k.entB[e];
            bb = make_int4(min(bb.x, q.x), min(bb.y, q.y), max(bb.z, q.z), max(bb.w, q.w));
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

// K6 front half, one wave per tile: the tile's row words restricted to the
// kept component (lane r: row r).  A tile with one component takes its mask
// words or nothing; a tile with several relabels its words (same ids as K1)
// and looks up each component's final root.
__device__ __forceinline__ u64 tile_in_word(const Frame& f, const Work& k, int tile, int32_t broot, int lane,
                                            Par* par, uint8_t* cflag, uint32_t* cedge, int tx, int ty) {
    const TileRec t = k.tile[tile];
    if (t.n == 0) return 0ull;
    const u64 m = k.mask[(int64_t)tile * TH + lane];
    if (t.n == 1) return (t.g1_open ? k.P[t.g1] == broot : t.g1 == broot) ? m : 0ull;
    const u64 p = __shfl_up(m, 1);
    const int n = label_tile(par, lane, lane, m, lane > 0 ? p : 0ull);
    // which components touch a tile edge (open: P holds their root; closed:
    // the root is their own run-start index, K1's rule)
    for (int i = lane; i < (n + 31) / 32; i += 64) cedge[i] = 0u;
    wave_sync();
    for_runs(m, [&](int a, int len) {
        if (lane == 0 || lane == TH - 1 || a == 0 || a + len == TW) {
            const int c = run_cid(par, slot(lane, a));
            atomicOr(&cedge[c >> 5], 1u << (c & 31));
        }
    });
    wave_sync();
    const bool closed_ok = 2ll * f.wb * ((f.h + 1) >> 1) <= CLOSED_SLOTS;
    for_runs(m, [&](int a, int) {
        const int j = slot(lane, a);
        const int v = par[pswz(j)];
        if (v >= NJ) {
            const int c = v - NJ;
            const int32_t G = slot_gidx(f, tx, ty, j);
            const bool open = !closed_ok || ((cedge[c >> 5] >> (c & 31)) & 1u);
            cflag[c] = (open ? k.P[G] : G) == broot;
        }
    });
    wave_sync();
    u64 w = 0ull;
    for_runs(m, [&](int a, int len) {
        if (cflag[run_cid(par, slot(lane, a))]) w |= run_mask(a, len);
    });
    return w;
}

__device__ __forceinline__ u64 row_word(u64 w, int r) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)w, r);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(w >> 32), r);
    return ((u64)hi << 32) | lo;
}

// K6, plugin path: in place on a 4-channel image, α := 0 outside the kept
// component (images without any component are left unchanged).
__global__ void __launch_bounds__(64 * WAVES)
k_ccl_apply(uint8_t* __restrict__ img, const ipp_image_desc* __restrict__ descs, const ipp_ccl_work* __restrict__ works,
            uint8_t* __restrict__ scratch, int groups_per_img, int groups_x) {
    __shared__ Par par_s[WAVES][NJ];
    __shared__ uint8_t flag_s[WAVES][CMAX];
    __shared__ uint32_t cedge_s[WAVES][CMAX / 32];
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / groups_per_img;
    const int g = b - im * groups_per_img;
    const int ty = g / groups_x;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int tx = (g - ty * groups_x) * WAVES + wave;
    const ipp_image_desc d = descs[im];
    const Frame f = frame_of(d);
    if (tx >= f.tiles_x || ty >= f.tiles_y) return;
    const Work k = work_of(scratch, works[im]);
    const int32_t broot = k.rec->root;
    if (broot < 0) return;
    const u64 w = tile_in_word(f, k, ty * f.tiles_x + tx, broot, lane, par_s[wave], flag_s[wave], cedge_s[wave], tx, ty);
    const int x = tx * TW + lane;
    const int nr = min(TH, d.h - ty * TH);
    for (int r = 0; r < nr; ++r) {
        const u64 rw = row_word(w, r);
        if (x < d.w && !((rw >> lane) & 1ull)) {
            uint8_t* a = img + d.off + (int64_t)(ty * TH + r) * d.pitch + 4 * (int64_t)x + 3;
            if (*a) *a = 0;
        }
    }
}

#ifndef IPP_CCL_CROP_ROWS
#define IPP_CCL_CROP_ROWS 1  // the crop-fit by row waves (k_ccl_crop_rows); 0: the item stream (A/B)
#endif

// K6, fused chain, in two passes.
// (a) k_ccl_inwords: one wave per tile that meets the kept component's bbox
//     overwrites the tile's mask words with its words restricted to the
//     component (tile_in_word; zeros for tiles without foreground).
// (b) k_ccl_crop_stream: the crop-fit of the BGR frame written as BGRA (α =
//     255 inside the component, 0 elsewhere) into the image's output slot,
//     row by row in output order: 4 pixels per thread (three dword loads, one
//     16-byte store), so output lines are written whole whatever the bbox's
//     alignment to the 64-pixel tiles.
__global__ void __launch_bounds__(64 * WAVES)
k_ccl_inwords(const ipp_image_desc* __restrict__ descs, const ipp_ccl_work* __restrict__ works,
              uint8_t* __restrict__ scratch, const int32_t* __restrict__ bbox, int groups_per_img, int groups_x) {
    __shared__ Par par_s[WAVES][NJ];
    __shared__ uint8_t flag_s[WAVES][CMAX];
    __shared__ uint32_t cedge_s[WAVES][CMAX / 32];
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / groups_per_img;
    const int g = b - im * groups_per_img;
    const int ty = g / groups_x;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int tx = (g - ty * groups_x) * WAVES + wave;
    // the bbox alone decides most waves (no kept component: an empty bbox)
    const int bx0 = bbox[4 * im + 0], by0 = bbox[4 * im + 1], bx1 = bbox[4 * im + 2], by1 = bbox[4 * im + 3];
    const int X0 = tx * TW, Y0 = ty * TH;
    if (X0 >= bx1 || X0 + TW <= bx0 || Y0 >= by1 || Y0 + TH <= by0) return;
    const ipp_image_desc d = descs[im];
    const Frame f = frame_of(d);
    if (tx >= f.tiles_x || ty >= f.tiles_y) return;
    const Work k = work_of(scratch, works[im]);
    const int tile = ty * f.tiles_x + tx;
    const u64 w = tile_in_word(f, k, tile, k.rec->root, lane, par_s[wave], flag_s[wave], cedge_s[wave], tx, ty);
    k.mask[(int64_t)tile * TH + lane] = w;
}

constexpr int CROP_BLOCKS = 256;  // blocks per image striding over the crop

__global__ void __launch_bounds__(256)
k_ccl_crop_stream(const uint8_t* __restrict__ img, const ipp_image_desc* __restrict__ descs,
                  const ipp_ccl_work* __restrict__ works, uint8_t* __restrict__ scratch,
                  int32_t* __restrict__ bbox, uint8_t* __restrict__ out,
                  const ipp_image_desc* __restrict__ out_descs) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / CROP_BLOCKS;
    const int rb = b - im * CROP_BLOCKS;
    const int bx0 = bbox[4 * im + 0], by0 = bbox[4 * im + 1], bx1 = bbox[4 * im + 2], by1 = bbox[4 * im + 3];
    if (bx1 <= bx0 || by1 <= by0) {  // no kept component
        // (k_ccl_finish folded in: the image's first block reports the empty
        // bbox as -1s; the other blocks read either form as empty)
        if (rb == 0 && threadIdx.x < 4) bbox[4 * im + threadIdx.x] = -1;
        return;
    }
    const ipp_image_desc d = descs[im];
    const ipp_image_desc od = out_descs[im];
    const Frame f = frame_of(d);
    const Work k = work_of(scratch, works[im]);
    const int cw = bx1 - bx0;
    // all (row, 4-pixel chunk) items of the crop, 256 threads × CROP_BLOCKS
    // blocks striding over them, two items per step for more loads in flight
    const int cpr = (cw + 3) >> 2;  // chunks per row
    const int64_t items = (int64_t)cpr * (by1 - by0);
    const int64_t stride = (int64_t)CROP_BLOCKS * 256;
    auto item = [&](int64_t it, uint32_t (&o)[4], int& n, uint32_t*& q) {
        const int oy = (int)(it / cpr), ox = 4 * (int)(it - (int64_t)oy * cpr);
        const int y = by0 + oy, x = bx0 + ox;
        n = min(4, cw - ox);
        const uint8_t* srow = img + d.off + (int64_t)y * d.pitch;
        const u64* wrow = k.mask + (int64_t)(y / TH) * f.tiles_x * TH + (y & (TH - 1));
        const u64 w0 = wrow[(int64_t)(x >> 6) * TH];
        const u64 w1 = ((x + n - 1) >> 6) != (x >> 6) ? wrow[(int64_t)((x + n - 1) >> 6) * TH] : w0;
        uint32_t px[4];
        if (n == 4) {
            const uint8_t* p = srow + 3 * x;
            const uint32_t d0 = ld_u32_unaligned(p), d1 = ld_u32_unaligned(p + 4), d2 = ld_u32_unaligned(p + 8);
            px[0] = d0;
            px[1] = (d0 >> 24) | (d1 << 8);
            px[2] = (d1 >> 16) | (d2 << 16);
            px[3] = d2 >> 8;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint8_t* p = srow + 3 * (x + i);
                px[i] = i < n ? (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) : 0u;
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int xi = x + i;
            const u64 w = (xi >> 6) == (x >> 6) ? w0 : w1;
            o[i] = (px[i] & 0x00FFFFFFu) | (((w >> (xi & 63)) & 1ull) ? 0xFF000000u : 0u);
        }
        q = reinterpret_cast<uint32_t*>(out + od.off + (int64_t)oy * od.pitch) + ox;
    };
    auto put = [&](const uint32_t (&o)[4], int n, uint32_t* q) {
        if (n == 4 && ((reinterpret_cast<uintptr_t>(q) & 15u) == 0u)) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            // streaming store (-0.7 % against a plain one)
            __builtin_nontemporal_store(u32x4{o[0], o[1], o[2], o[3]}, reinterpret_cast<u32x4*>(q));
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (i < n) q[i] = o[i];
        }
    };
    for (int64_t it = (int64_t)rb * 256 + threadIdx.x; it < items; it += 2 * stride) {
        uint32_t oa[4], ob[4];
        int na, nb = 0;
        uint32_t *qa, *qb = nullptr;
        item(it, oa, na, qa);
        if (it + stride < items) item(it + stride, ob, nb, qb);
        put(oa, na, qa);
        if (nb) put(ob, nb, qb);
    }
}

// (b') k_ccl_crop_rows: the same crop-fit, one wave per crop row at a time.
//     The stream above is texture-path bound (TA busy 96 % of the launch,
//     profiles/r05/r05s9/prof_video4k): three unaligned dword loads plus the
//     mask-word loads per 4 pixels.  Here a wave loads its row's source span
//     with aligned 16-byte buffer loads (1 KB per instruction), stages it in
//     LDS, and every lane assembles its 4 pixels from there (two LDS reads and
//     v_alignbyte; the row's alignment is uniform), with the row's mask words
//     read once into LDS too: per 4 pixels 0.75 load and 1 store instruction
//     instead of ≈ 4.5 loads and 1 store.
#ifndef IPP_CCL_CROP_ROW_BLOCKS
#define IPP_CCL_CROP_ROW_BLOCKS 256
#endif
constexpr int CROP_ROW_BLOCKS = IPP_CCL_CROP_ROW_BLOCKS;  // blocks per image (4 waves each) striding over the crop rows
#ifndef IPP_CCL_CROP_PF
#define IPP_CCL_CROP_PF 1  // the next (row, segment)'s loads in flight during this one (0: after it, A/B)
#endif
constexpr int CROP_SEG = 4 * 256;            // output pixels per wave iteration (4 × 64 lanes × 4)
constexpr int CROP_CHUNKS = 3 * CROP_SEG / 16 + 1;  // 16-B source chunks one iteration may touch

struct CropRowsLds {
    uint32_t stage[WAVES][CROP_CHUNKS * 4];  // source span of the wave's iteration
    u64 words[WAVES][TW + 2];               // the row's mask words (tile columns tc0 ..), zero-padded
};

__global__ void __launch_bounds__(256)
k_ccl_crop_rows(const uint8_t* __restrict__ img, const ipp_image_desc* __restrict__ descs,
                const ipp_ccl_work* __restrict__ works, uint8_t* __restrict__ scratch,
                int32_t* __restrict__ bbox, uint8_t* __restrict__ out,
                const ipp_image_desc* __restrict__ out_descs) {
    __shared__ CropRowsLds L;
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = b / CROP_ROW_BLOCKS;
    const int rb = b - im * CROP_ROW_BLOCKS;
    const int bx0 = bbox[4 * im + 0], by0 = bbox[4 * im + 1], bx1 = bbox[4 * im + 2], by1 = bbox[4 * im + 3];
    if (bx1 <= bx0 || by1 <= by0) {  // no kept component (k_ccl_finish folded in, as in k_ccl_crop_stream)
        if (rb == 0 && threadIdx.x < 4) bbox[4 * im + threadIdx.x] = -1;
        return;
    }
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const ipp_image_desc d = descs[im];
    const ipp_image_desc od = out_descs[im];
    const Frame f = frame_of(d);
    const Work k = work_of(scratch, works[im]);
    const int cw = bx1 - bx0;
    const int tc0 = bx0 >> 6, ntc = ((bx1 - 1) >> 6) - tc0 + 1;  // ≤ 61 tile columns
    // The buffer starts at the 16-B aligned address at or below the frame
    // (fmis bytes before it, in the same aligned chunk) and ends with the
    // 4-aligned dword holding the frame's last byte: the range check works per
    // dword (a straddling one reads 0), and neither extension crosses a page.
    const uint8_t* fbase = img + d.off;
    const uint32_t fmis = (uint32_t)(reinterpret_cast<uintptr_t>(fbase) & 15u);
    const uint32_t fbytes = (uint32_t)((int64_t)d.h * d.pitch);
    const uint32_t nrec = (fmis + fbytes + 3u) & ~3u;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(fbase - fmis), (short)0, (int)nrec, 0x00020000);
    uint32_t* stage = L.stage[wave];
    u64* words = L.words[wave];
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    // The wave's (row, segment) units in order; each unit's chunk loads (and,
    // on a row's first segment, its mask words) are issued before the
    // previous unit is assembled and stored (IPP_CCL_CROP_PF), so their
    // latency overlaps that work instead of stalling the wave.
    struct Unit {
        int y, seg;
        uint32_t R, sh0;  // buffer byte of the row's first crop pixel; its offset in its 16-B chunk
        int c0, c1;       // the segment's chunks
    };
    const int ystep = CROP_ROW_BLOCKS * WAVES;
    auto unit_at = [&](int y, int seg) {
        Unit u;
        u.y = y;
        u.seg = seg;
        u.R = fmis + (uint32_t)y * (uint32_t)d.pitch + 3u * (uint32_t)bx0;
        u.sh0 = u.R & 15u;
        const int npx = min(CROP_SEG, cw - seg);
        u.c0 = (int)((u.sh0 + 3u * (uint32_t)seg) >> 4);
        u.c1 = (int)((u.sh0 + 3u * (uint32_t)(seg + npx) + 15u) >> 4);
        return u;
    };
    auto next = [&](const Unit& u) { return u.seg + CROP_SEG < cw ? unit_at(u.y, u.seg + CROP_SEG) : unit_at(u.y + ystep, 0); };
    auto load = [&](const Unit& u, u32x4 (&v)[4], u64& wd) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = u.c0 + lane + 64 * i;
            if (c < u.c1)
                v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, u.R - u.sh0 + 16u * (uint32_t)c, 0, 0));
        }
        // the row's kept-component words, restricted by k_ccl_inwords (lanes
        // past the row's tiles: zero), on its first segment
        if (u.seg == 0)
            wd = lane < ntc ? k.mask[((int64_t)(u.y >> 6) * f.tiles_x + tc0 + lane) * TH + (u.y & (TH - 1))] : 0ull;
    };
    Unit cur = unit_at(by0 + rb * WAVES + wave, 0);
    if (cur.y >= by1) return;
    u32x4 vc[4];
    u64 wc = 0ull;
    load(cur, vc, wc);
    for (;;) {
        const Unit nx = next(cur);
        const bool more = nx.y < by1;
        u32x4 vn[4];
        u64 wn = 0ull;
        if (IPP_CCL_CROP_PF && more) load(nx, vn, wn);
        wave_sync();  // (the previous unit's stage and word reads done)
        if (cur.seg == 0) {
            words[lane] = wc;
            if (lane < 2) words[TW + lane] = 0ull;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = cur.c0 + lane + 64 * i;
            if (c < cur.c1) *reinterpret_cast<u32x4*>(stage + 4 * (c - cur.c0)) = vc[i];
        }
        wave_sync();
        uint8_t* orow = out + od.off + (int64_t)(cur.y - by0) * od.pitch;
        // byte offset of pixel seg in the stage, and the row's dword alignment
        const uint32_t o0 = cur.sh0 + 3u * (uint32_t)cur.seg - 16u * (uint32_t)cur.c0;
        const uint32_t sh = o0 & 3u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int ox = cur.seg + 256 * u + 4 * lane;
            if (ox >= cw) continue;
            const uint32_t o = o0 + 3u * (uint32_t)(ox - cur.seg);  // ≡ sh (mod 4)
            const uint32_t* q = stage + (o >> 2);
            const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3];
            const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh),
                           w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
            const uint32_t px[4] = {w0, __builtin_amdgcn_alignbyte(w1, w0, 3), __builtin_amdgcn_alignbyte(w2, w1, 2),
                                    w2 >> 8};
            // the 4 pixels' bits: columns x .. x + 3 of the row's words
            const int x = bx0 + ox, t = (x >> 6) - tc0, bb = x & 63;
            const u64 lo = words[t] >> bb, hi = bb ? words[t + 1] << (64 - bb) : 0ull;
            const uint32_t fb = (uint32_t)(lo | hi);
            uint32_t o4[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) o4[i] = (px[i] & 0x00FFFFFFu) | (((fb >> i) & 1u) ? 0xFF000000u : 0u);
            uint32_t* qo = reinterpret_cast<uint32_t*>(orow) + ox;
            const int n = min(4, cw - ox);
            if (n == 4 && (reinterpret_cast<uintptr_t>(qo) & 15u) == 0u) {
                __builtin_nontemporal_store(u32x4{o4[0], o4[1], o4[2], o4[3]}, reinterpret_cast<u32x4*>(qo));
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (i < n) qo[i] = o4[i];
            }
        }
        if (!more) break;
        if (!IPP_CCL_CROP_PF) load(nx, vn, wn);
        cur = nx;
#pragma unroll
        for (int i = 0; i < 4; ++i) vc[i] = vn[i];
        if (cur.seg == 0) wc = wn;
    }
}

__global__ void k_ccl_prep(const ipp_ccl_work* __restrict__ works, uint8_t* __restrict__ scratch, int32_t* bbox,
                           unsigned long long* best, int32_t* counts, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        bbox[4 * i + 0] = INT32_MAX;
        bbox[4 * i + 1] = INT32_MAX;
        bbox[4 * i + 2] = -1;
        bbox[4 * i + 3] = -1;
        best[i] = 0ull;
        counts[i] = 0;
        ImgRec* rec = reinterpret_cast<ImgRec*>(scratch + works[i].img_off);
        rec->ckey = 0ull;
        rec->root = -1;
    }
}

__global__ void k_ccl_finish(int32_t* bbox, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && bbox[4 * i + 2] < 0) bbox[4 * i + 0] = bbox[4 * i + 1] = bbox[4 * i + 2] = bbox[4 * i + 3] = -1;
}

struct Launch {
    int tiles_x, tiles_y, groups_x, groups_per_img, chunks_per_img;
    dim3 group_grid, ent_grid, chunk_grid;
    bool ok;
};

Launch plan_launch(int n, int max_w, int max_h) {
    Launch L{};
    L.tiles_x = (max_w + TW - 1) / TW;
    L.tiles_y = (max_h + TH - 1) / TH;
    L.groups_x = (L.tiles_x + WAVES - 1) / WAVES;
    L.groups_per_img = L.groups_x * L.tiles_y;
    L.chunks_per_img = (L.tiles_x * L.tiles_y + 63) / 64;
    const int64_t gb = (int64_t)L.groups_per_img * n, eb = (int64_t)ENT_BLOCKS * n;
    const int64_t cb = ((int64_t)L.chunks_per_img * n + WAVES - 1) / WAVES;
    L.ok = gb < INT32_MAX && eb < INT32_MAX && cb < INT32_MAX;
    L.group_grid = dim3((uint32_t)gb);
    L.ent_grid = dim3((uint32_t)eb);
    L.chunk_grid = dim3((uint32_t)cb);
    return L;
}

template <int SRC, int NR, bool ZONES>
void launch_label(const Launch& L, hipStream_t s, const uint8_t* img, const ipp_image_desc* descs,
                  const ipp_ccl_work* works, uint8_t* scratch, int32_t* counts, const ipp_hsv_params& hp) {
    hipLaunchKernelGGL((k_ccl_label<SRC, NR, ZONES>), L.group_grid, dim3(64 * WAVES), 0, s, img, descs, works,
                       scratch, counts, L.groups_per_img, L.groups_x, hp);
}

// K1..K5 common to both entry points.
int run_labels(int src, const uint8_t* img, const ipp_image_desc* descs, int32_t n, int32_t max_w, int32_t max_h,
               const ipp_hsv_params* hsv, const ipp_ccl_work* works, uint8_t* scratch, int32_t* counts,
               unsigned long long* best, int32_t* bbox, hipStream_t s, Launch& L) {
    L = plan_launch(n, max_w, max_h);
    if (!L.ok) return IPP_E_ARG;
    const int nb = (n + 255) / 256;
    hipLaunchKernelGGL(k_ccl_prep, dim3(nb), dim3(256), 0, s, works, scratch, bbox, best, counts, n);
    if (src == SRC_ALPHA) {
        launch_label<SRC_ALPHA, 1, false>(L, s, img, descs, works, scratch, counts, ipp_hsv_params{});
    } else {
        const bool zones = hsv_has_zones(*hsv);
        const bool small = hsv->n_ranges <= 4;
        const ipp_hsv_params q = hsv_pad(*hsv, small ? 4 : IPP_MAX_HSV_RANGES);
        if (small && !zones) launch_label<SRC_HSV, 4, false>(L, s, img, descs, works, scratch, counts, q);
        else if (small) launch_label<SRC_HSV, 4, true>(L, s, img, descs, works, scratch, counts, q);
        else if (!zones) launch_label<SRC_HSV, IPP_MAX_HSV_RANGES, false>(L, s, img, descs, works, scratch, counts, q);
        else launch_label<SRC_HSV, IPP_MAX_HSV_RANGES, true>(L, s, img, descs, works, scratch, counts, q);
    }
    hipLaunchKernelGGL(k_ccl_border, L.chunk_grid, dim3(64 * WAVES), 0, s, descs, works, scratch, L.chunks_per_img,
                       n);
    hipLaunchKernelGGL(k_ccl_resolve, L.ent_grid, dim3(256), 0, s, works, scratch, counts);
    hipLaunchKernelGGL(k_ccl_best, L.ent_grid, dim3(256), 0, s, works, scratch, counts, best);
    hipLaunchKernelGGL(k_ccl_bbox, L.ent_grid, dim3(256), 0, s, descs, works, scratch, counts, best, bbox);
    return IPP_OK;
}

}  // namespace

extern "C" int64_t ipp_ccl_scratch_layout(int32_t w, int32_t h, ipp_ccl_work* work) {
    if (w <= 0 || h <= 0) return IPP_E_ARG;
    const int64_t wb = (w + 1) / 2, hb = (h + 1) / 2;
    const int64_t slots = 2 * wb * hb;
    if (slots >= INT32_MAX) return IPP_E_RANGE;
    const int64_t tiles = (int64_t)((w + TW - 1) / TW) * ((h + TH - 1) / TH);
    // open components only when closed keys fit (see CLOSED_SLOTS): each
    // touches the tile's ring of 252 edge pixels, and two of them are never
    // adjacent on it (≤ 126 per tile); else every component (≤ CMAX per tile)
    const int64_t cap = tiles * (slots <= CLOSED_SLOTS ? 128 : CMAX);
    auto al = [](int64_t v) { return (v + 255) & ~(int64_t)255; };
    ipp_ccl_work k{};
    k.img_off = 0;
    k.mask_off = 256;
    k.edge_off = k.mask_off + al(8 * TH * tiles);
    k.p_off = k.edge_off + al(4 * 4 * 64 * tiles);
    k.a_off = k.p_off + al(4 * slots);
    k.ent_off = k.a_off + al(4 * slots);
    k.ent_cap = cap;
    k.tile_off = k.ent_off + al(24 * cap);
    const int64_t total = k.tile_off + al((int64_t)sizeof(TileRec) * tiles);
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
    const int rc =
        run_labels(SRC_ALPHA, img, descs, n_images, max_w, max_h, nullptr, works, scratch, counts, best, bbox, s, L);
    if (rc != IPP_OK) return rc;
    hipLaunchKernelGGL(k_ccl_apply, L.group_grid, dim3(64 * WAVES), 0, s, img, descs, works, scratch,
                       L.groups_per_img, L.groups_x);
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
    const int rc =
        run_labels(SRC_HSV, frames, descs, n_images, max_w, max_h, hsv, works, scratch, counts, best, bbox, s, L);
    if (rc != IPP_OK) return rc;
    hipLaunchKernelGGL(k_ccl_inwords, L.group_grid, dim3(64 * WAVES), 0, s, descs, works, scratch, bbox,
                       L.groups_per_img, L.groups_x);
    if (IPP_CCL_CROP_ROWS)
        hipLaunchKernelGGL(k_ccl_crop_rows, dim3((uint32_t)((int64_t)CROP_ROW_BLOCKS * n_images)), dim3(256), 0, s,
                           frames, descs, works, scratch, bbox, out, out_descs);
    else
        hipLaunchKernelGGL(k_ccl_crop_stream, dim3((uint32_t)((int64_t)CROP_BLOCKS * n_images)), dim3(256), 0, s,
                           frames, descs, works, scratch, bbox, out, out_descs);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
