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
//
// Experiment switches left in this file are the live ones that DESIGN.md §3
// names (IPP_HP_BANDS, IPP_COPY_GROUP/SLABS, IPP_VB_WPE/DB/HOIST_MAX); the
// diagnostic builds of rounds 1-5 and the closed A/B switches were removed in
// round 6 (their numbers stay in DESIGN.md).
#include <algorithm>
#include <type_traits>

#include "ipp_hsv.h"
#include "ipp_sampler.h"

namespace {

constexpr int HR = 16;            // H-pass rows per band (4 per thread)
constexpr int RING = 512;         // window ring: M columns x live at x & (RING - 1)
// LDS bytes per plane row of the window ring.  544 ≡ 8 dwords mod 64 banks:
// the phase-2 ds_read_b128 (4 lane groups of 16, 4 dwords each) then covers
// 64 distinct banks per group, and the phase-1 ds_write_b32 rows pair up 2-way,
// which a dword store absorbs (MI355X_MICROARCH.md §LDS).
constexpr int WSTRIDE = 544;

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
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7FFFFFFF, 0x00020000);
}

// ---------------------------------------------------------------------------
// H pass (MFMA taps): per-pixel buffer-load gathers, table-driven HSV test.
//
// The M pixel is (R, G, B) of the source or black outside it (rotations.py
// fills with transparent black and filtres_liste.py:84 reads the file back
// with cv2.imread, which drops alpha, so fill and real black pixels are
// indistinguishable from the HSV step on).  Hence:
//   * gathers go through a buffer resource whose range check returns 0 for the
//     out-of-window offset 0xFFFFFFFF — no validity bits, no value masking;
//   * the inRange union is decided by three LDS mask tables instead of packed
//     compares: bit k of vm[v], sm[s], hm[h + 32] says range k holds on that
//     channel, so  excluded ⟺ vm[v] & sm[s] & hm[h + 32] (& zone bits) ≠ 0.
//
// Block = one 16-row band of one item, 4 waves.  It sweeps the item's output
// tiles in chunks of ≤ 4 tiles whose input window fits the 512-column
// channel-planar LDS ring.  Phase 1 gathers the chunk's new M columns into the
// ring (16 columns × 16 rows per wave and step; a lane takes 4 consecutive M
// columns of one row, i.e. the ring dword it writes); phase 2 runs the taps on
// the matrix cores.
// (An LDS-staged form — coalesced source spans, dense HSV — was bit-exact but
// 1.6× slower, VALU-bound: DESIGN.md §3, profiles/r03_staged/.)
// ---------------------------------------------------------------------------
typedef uint8_t WinRing[4][HR][WSTRIDE];   // planar window ring, bytes p ^ 0x80

template <int NR>
struct __attribute__((aligned(16))) Hpass2Lds {
    WinRing win;
    HsvTables<NR> T;                  // table-driven HSV test (ipp_hsv.h)
    int32_t zc[NR > 8 ? 2 * NR : 1];  // > 8 ranges with zones: column bounds here, not in registers
};

// M pixel → window byte quad (p | α 255) ^ 0x80 when kept, 0x80808080 (transparent black) when excluded.
template <int NR, bool ZONES>
__device__ __forceinline__ uint32_t hsv2_px(const HsvTables<NR>& T, uint32_t raw, uint32_t zbits) {
    uint32_t ex = hsv_tab_excl<NR, false>(T, raw);
    if (ZONES) ex &= zbits;
    const uint32_t t = (raw | 0xFF000000u) ^ 0x80808080u;
    return ex ? 0x80808080u : t;
}

// Per-block state.
struct Hp2Block {
    u32x4_t rsv;                // source window buffer resource
    uint32_t lim;               // CLAMP: last byte offset where a dword fits
    uint32_t rowx, rowy;        // 16.16 source position of column 0 of the lane's row
    int32_t b0, b3, pitch, in_w, in_h;
    int32_t xlo, xhi;           // band's valid M columns ⊆ [xlo, xhi] (conservative)
};

// 4 gathered pixels of a lane (raw dwords; 0 outside the window).  CLAMP:
// only the image's last pixel can have its dword cross the image end (bytes
// beyond it are out of range and would zero the whole dword); that pixel is
// loaded one byte early and shifted down, marked by bit 1 + k of fl.
struct Raw4 {
    uint32_t p[4];
    uint32_t fl;  // CLAMP: bit 1 + k = pixel k was loaded one byte early
    bool any;     // some pixel of the lane is inside the window
    bool live;    // the step's loads were issued (block-uniform)
};

// The gathers are issued by inline asm and waited for by hand.  The compiler
// then neither counts them (its vmcnt bookkeeping merges paths pessimistically,
// so a step skipped on some path made every later wait drain the gathers
// issued for the steps ahead) nor copies their registers (a copy of a register
// whose load is in flight would wait for it — or, worse, read it early: the
// hazard tests/test_asm_gather_hazard.py checks in the emitted ISA).  Dead
// steps issue nothing; a set is waited for with vmcnt(4 × live sets issued
// after it), which never exceeds the loads really issued after it
// (compiler-issued loads in between only make the wait stricter).  The wait
// names the four data registers as in/out operands, so no use of them can
// move above it.
__device__ __forceinline__ uint32_t asm_gather(u32x4_t rs, uint32_t off) {
    uint32_t v;
    asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(rs));
    return v;
}
// One asm statement on every path (newer = 8, 4, 0, or -1: the set was not
// issued, no wait): with a wait per path the compiler merged the paths through
// register copies, which read the data registers before their loads landed.
// (The leading comment names the four registers in the emitted ISA, for the
// static check in tools/asm_hazard.py.)
__device__ __forceinline__ void asm_wait(uint32_t (&p)[4], int32_t newer) {
    asm volatile(
        "; gather wait %0 %1 %2 %3\n\t"
        "s_cmp_eq_u32 %4, 8\n\t"
        "s_cbranch_scc0 1f\n\t"
        "s_waitcnt vmcnt(8)\n\t"
        "s_branch 4f\n"
        "1:\n\t"
        "s_cmp_eq_u32 %4, 4\n\t"
        "s_cbranch_scc0 2f\n\t"
        "s_waitcnt vmcnt(4)\n\t"
        "s_branch 4f\n"
        "2:\n\t"
        "s_cmp_eq_u32 %4, 0\n\t"
        "s_cbranch_scc0 4f\n\t"
        "s_waitcnt vmcnt(0)\n"
        "4:"
        : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3])
        : "s"(newer)
        : "scc");
}

// Gathers of one live step: xx/yy = 16.16 source position of the lane's
// first pixel (its next three are the following M columns).  Out-of-window
// pixels load offset 0xFFFFFFFF (the range check returns 0).  Two forms:
//   CLAMP (general): column and row tested, the records run to the image end,
//   and an offset past the last whole dword is clamped back (the pixel then
//   loaded one byte early, fl);
//   fast (the bench's crops): rows outside the window fail the buffer's range
//   check by themselves — the records end one byte past the window's last
//   pixel and row in_h starts at or past that byte — so only the column is
//   tested (H 8.79 -> 8.75 ms, round 5, profiles/r05/ab_gather_yrange_r05ar.txt);
//   hpass_block takes it only where that holds and no row offset can wrap
//   (yr_range_ok).
template <int CN, bool CLAMP>
__device__ __forceinline__ void hp2_issue(const Hp2Block& B, uint32_t xx, uint32_t yy, Raw4& o) {
    bool any = false;
    uint32_t off[4];
    if (CLAMP) o.fl = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int xin = (int32_t)xx >> 16, yin = (int32_t)yy >> 16;
        const bool ok = CLAMP ? ((uint32_t)xin < (uint32_t)B.in_w) & ((uint32_t)yin < (uint32_t)B.in_h)
                              : (uint32_t)xin < (uint32_t)B.in_w;
        uint32_t o1 = (uint32_t)__mul24(yin, B.pitch) + (uint32_t)__umul24((uint32_t)xin, (uint32_t)CN);
        if (CLAMP) {
            const uint32_t offc = min(o1, B.lim);
            o.fl |= (uint32_t)(o1 != offc) << (1 + k);
            o1 = offc;
        }
        off[k] = ok ? o1 : 0xFFFFFFFFu;
        any |= ok;
        xx += (uint32_t)B.b0;
        yy += (uint32_t)B.b3;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) o.p[k] = asm_gather(B.rsv, off[k]);
    o.any = any;
    o.live = true;
}

constexpr int HP_NW = 4;              // waves per block
constexpr int HP_STEPC = 16 * HP_NW;  // M columns per block-wide phase-1 step

// Sticky status of the pipe kernels (ipp_pipe_status): bit 0 = an H-pass
// output tile's input window was wider than the LDS ring (the plan violated
// the ring limit of ipp.h; that tile's T columns are wrong).
__device__ int32_t g_pipe_status;

// One chunk of ≤ 4 output tiles whose input window fits the ring.
struct Hp2Chunk {
    int s0, s1;   // tiles [s0, s1)
    int c0;       // first M column not yet in the ring
    int ng4;      // new 4-column groups
    int nsteps;   // this wave's phase-1 steps (16 groups per step over the block)
};

// The chunk's four candidate headers are read at once (scalar loads of 64
// B; reading up to three headers past the table stays inside the tap buffer
// — the tile biases follow it): per chunk one load round trip instead of a
// chain of dependent ones.
__device__ __forceinline__ Hp2Chunk hp2_chunk(const int4* hdr, int s0, int ntiles, int& filled, int wave) {
    Hp2Chunk c;
    c.s0 = s0;
    int4 hh[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) hh[k] = hdr[s0 + k];
    const int W0 = hh[0].x;
    int W1 = hh[0].x + 64 * hh[0].y, s1 = s0 + 1;
    if (W1 - W0 > RING && threadIdx.x == 0) atomicOr(&g_pipe_status, 1);  // single tile beyond the ring
    bool grow = true;
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        const int e = max(W1, hh[k].x + 64 * hh[k].y);
        grow = grow && s0 + k < ntiles && e - W0 <= RING;  // the longest prefix of ≤ 4 tiles that fits
        if (grow) {
            W1 = e;
            s1 = s0 + k + 1;
        }
    }
    c.s1 = s1;
    c.c0 = max(filled, W0);
    c.ng4 = max(0, (W1 - c.c0) >> 2);
    c.nsteps = c.ng4 > wave * 4 ? (c.ng4 - wave * 4 + 4 * HP_NW - 1) / (4 * HP_NW) : 0;
    filled = max(filled, W1);
    return c;
}

// (Round 6: a block walking 2-4 bands chunk-outer, band-inner — each chunk's
// taps loaded once for its bands, its window re-gathered per band — measured
// slower than this one-band block: the taps, meta and bias held across the
// next band's phase 1 cost more than the tap loads they save; DESIGN.md §3
// "Round 6, multi-band H blocks".)
template <int NR, bool ZONES, int CN, bool CLAMP>
__device__ __forceinline__ void hpass2_body(const HsvTables<NR>& T, WinRing& win, int wave, const Hp2Block& B,
                                            uint8_t* __restrict__ tmp, const int32_t* __restrict__ coefs,
                                            const ipp_resample_desc& h, int row0, int nrows, const int32_t* zc0,
                                            const int32_t* zcw, uint32_t zrow) {
    const int lane = threadIdx.x & 63;
    const int r = 2 * (lane >> 3) + ((lane >> 1) & 1);  // the lane's window row
    const int ntiles = (h.out_len + 15) >> 4;
    const int4* hdr = reinterpret_cast<const int4*>(coefs + h.coef_off);
    const int32_t* tbias = coefs + h.coef_off + 4 * (int64_t)ntiles;
    const uint4* tblk = reinterpret_cast<const uint4*>(coefs + h.coef_off + 20 * (int64_t)ntiles);
    const uint32_t sx = (uint32_t)HP_STEPC * (uint32_t)B.b0, sy = (uint32_t)HP_STEPC * (uint32_t)B.b3;  // per-step advance

    int filled = hdr[0].x;  // ring holds M columns [.., filled)
    Hp2Chunk ck = hp2_chunk(hdr, 0, ntiles, filled, wave);
    // Lane's first column of step 0 and its source position.
    auto lane_x = [&](const Hp2Chunk& c) { return c.c0 + 16 * wave + 8 * ((lane >> 2) & 1) + 4 * (lane & 1); };
    // (24-bit products: columns < 2^15 and |b| ≤ 2^16; a 32-bit product made
    // the compiler use a 64-bit mad whose unused high addend was a register
    // that can still be in flight)
    int xl = lane_x(ck);
    uint32_t xxl = B.rowx + (uint32_t)__mul24(xl, B.b0), yyl = B.rowy + (uint32_t)__mul24(xl, B.b3);
    Raw4 RA, RB, RC;
    RA.live = RB.live = RC.live = false;
    RA.fl = RB.fl = RC.fl = 0u;
    // A step = 16 columns of 16 rows per wave; steps past the chunk or wholly
    // outside the band's valid columns are dead: no gathers, no HSV, constant
    // window bytes.
    auto issue = [&](const Hp2Chunk& c, int st, uint32_t xx, uint32_t yy, Raw4& o) {
        const int xs = c.c0 + 16 * wave + HP_STEPC * st;
        const bool live = st < c.nsteps && xs + 15 >= B.xlo && xs <= B.xhi;
        if (!live) {
            o.any = false;
            o.live = false;
            return;
        }
        hp2_issue<CN, CLAMP>(B, xx, yy, o);
    };
    issue(ck, 0, xxl, yyl, RA);
    issue(ck, 1, xxl + sx, yyl + sy, RB);
    // The block's first gathers fly across the table barrier (r06k A/B:
    // −0.01 ms per headline step).
    __syncthreads();  // tables visible
    // Fill value (raw 0): uniform over the block except for zone bits.
    const uint32_t fill = __builtin_amdgcn_readfirstlane(hsv2_px<NR, ZONES>(T, 0u, ~0u));  // (in an SGPR)

    for (;;) {
        // This wave's tile taps for the first K step, in flight during phase 1.
        const int t = ck.s0 + wave;
        const bool has_tile = t < ck.s1 && nrows > 0;
        int4 th = make_int4(0, 0, 0, 0);
        uint4 bn[3];
        int32_t meta = 0;  // compact tiles: g0 | len << 8 | base << 16 of the lane's output
        int32_t bias = 0;  // the lane's output column bias, in flight with the taps
        {
            // Loaded unconditionally (a valid tile stands in when the wave
            // has none), so the loads in flight do not depend on the path.
            const int te = min(t, ntiles - 1);
            th = hdr[te];
            // wave-uniform: kept in SGPRs
            th.x = __builtin_amdgcn_readfirstlane(th.x);
            th.y = __builtin_amdgcn_readfirstlane(th.y);
            th.z = __builtin_amdgcn_readfirstlane(th.z);
            th.w = __builtin_amdgcn_readfirstlane(th.w);
            // Compact tiles (th.w, ipp.h): meta[16] then one 64-block array
            // per plane — one load per plane for every K step.  Dense tiles:
            // the first K step's blocks (meta then reads tap bytes, unused).
#pragma unroll
            for (int p = 0; p < 3; ++p) bn[p] = tblk[th.z + (th.w ? 4 : 0) + lane + p * 64];
            if (!has_tile) th.y = 0;
        }
        const int te = min(t, ntiles - 1);

        // Phase 1: new M columns → planar LDS ring.  Three register sets
        // rotate so that each step's gathers have two steps of HSV work to land.
        const int c0 = ck.c0, ng4 = ck.ng4, nsteps = ck.nsteps;
        // newer = gather loads issued after P's (4 per live later set)
        auto process = [&](Raw4& P, int st, int newer) {
            asm_wait(P.p, P.live ? newer : -1);
            // lane holds columns 8gc + 4dx .. +3 of its row
            const int cg = wave * 4 + 4 * HP_NW * st + 2 * ((lane >> 2) & 1) + (lane & 1);
            const int x = c0 + 4 * cg;
            const bool active = (cg < ng4) && (r < nrows);
            uint32_t px[4], zb[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                zb[k] = ~0u;
                if (ZONES) {
                    const int xk = x + k;
                    zb[k] = 0;
#pragma unroll
                    for (int q = 0; q < NR; ++q) zb[k] |= (uint32_t)((uint32_t)(xk - zc0[q]) < (uint32_t)zcw[q]) << q;
                    zb[k] &= zrow;
                }
            }
            // One branch per step (not per pixel) so the four pixels' table
            // reads and arithmetic interleave in one basic block.
            uint32_t ch[4];
            if (__builtin_amdgcn_ballot_w64(P.any) != 0ull) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    uint32_t raw = P.p[k];
                    if (CLAMP) raw >>= ((P.fl >> (1 + k)) & 1u) << 3;
                    px[k] = hsv2_px<NR, ZONES>(T, raw, zb[k]);
                }
                transpose4(px[0], px[1], px[2], px[3], ch);
            } else if (ZONES) {
#pragma unroll
                for (int k = 0; k < 4; ++k) px[k] = hsv2_px<NR, ZONES>(T, 0u, zb[k]);
                transpose4(px[0], px[1], px[2], px[3], ch);
            } else {
#pragma unroll
                for (int c = 0; c < 4; ++c) ch[c] = ((fill >> (8 * c)) & 0xFFu) * 0x01010101u;
            }
            if (active) {
                const int pos = x & (RING - 1);
#pragma unroll
                for (int c = 0; c < 4; ++c) *reinterpret_cast<uint32_t*>(&win[c][r][pos]) = ch[c];
            }
        };
        auto iss = [&](int st2, Raw4& o) { issue(ck, st2, xxl + st2 * sx, yyl + st2 * sy, o); };
        // The loop runs whole register-set rotations (a trailing step past
        // nsteps is dead).  With no early exit each set keeps its registers;
        // an exit mid-rotation made the compiler shuffle the sets through
        // copies, and copying a register whose load is in flight waits for it.
        //
        // The phase-2 column bias and (compact tiles) the lane's group meta
        // are issued at the start of the last rotation: in flight during all
        // of phase 1 they cost the registers phase 1 needs; issued after it,
        // their latency sat exposed before the barrier (r06j/r06k A/B: −0.075
        // ms per headline step).  (Reading the next chunk's headers there too
        // spilled SGPRs to scratch.)  The gathers issued before them wait a
        // little longer than needed (vmcnt counts the two loads as newer).
        bool mb = false;
        for (int st = 0; st < nsteps; st += 3) {
            iss(st + 2, RC);
            if (st + 3 >= nsteps) {
                meta = reinterpret_cast<const int32_t*>(tblk + th.z)[lane & 15];
                bias = tbias[min(16 * te + (lane & 15), h.out_len - 1)];
                mb = true;
            }
            process(RA, st, 4 * (RB.live + RC.live));
            iss(st + 3, RA);
            process(RB, st + 1, 4 * (RC.live + RA.live));
            iss(st + 4, RB);
            process(RC, st + 2, 4 * (RA.live + RB.live));
        }

        // The chunk's first tap loads (issued before its gathers) and the bias
        // and meta loads below are waited for on every path before the next
        // chunk's gathers: a compiler wait for them after those asm gathers
        // would drain the gathers as well.
        if (!mb) {  // (a wave with no phase-1 steps)
            meta = reinterpret_cast<const int32_t*>(tblk + th.z)[lane & 15];
            bias = tbias[min(16 * te + (lane & 15), h.out_len - 1)];
        }
        const int s1 = ck.s1;
        const bool more = s1 < ntiles;
        if (more) {
            ck = hp2_chunk(hdr, s1, ntiles, filled, wave);
            xl = lane_x(ck);
            xxl = B.rowx + (uint32_t)__mul24(xl, B.b0);
            yyl = B.rowy + (uint32_t)__mul24(xl, B.b3);
        } else {
            ck.nsteps = 0;  // no loads
        }
        asm volatile("" ::"v"(bn[0].x), "v"(bn[1].x), "v"(bn[2].x), "v"(bias), "v"(meta));
        // Next chunk's first steps, issued now so they fly during phase 2
        // (whose K-step tap loads, issued after them, then wait for them too:
        // vmcnt retires in order).  (Issuing them after the MFMAs, with the
        // accumulators live, let the compiler move the in-flight gather
        // registers and broke parity.)
        issue(ck, 0, xxl, yyl, RA);
        issue(ck, 1, xxl + sx, yyl + sy, RB);
        __syncthreads();

        // Phase 2 (mfma): wave w takes tile s0 + w; A = 16 window rows × 64
        // columns of one channel (lane l: row l&15, bytes 16(l>>4)..+15),
        // B = 64 columns × 16 outputs of one tap byte plane.  D lane l =
        // output l&15, rows 4(l>>4)..+3 = exactly one 16-B T group.  The
        // column bias (lowered by 128 << 22, so that the signed saturation
        // below yields clip8 ^ 0x80) rides in the first byte plane's initial
        // accumulator.
        if (has_tile) {
            i32x4 acc[4][3];
            const int32_t b0 = bias - (128 << 22);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                acc[c][0] = i32x4{b0, b0, b0, b0};
                acc[c][1] = i32x4{0, 0, 0, 0};
                acc[c][2] = i32x4{0, 0, 0, 0};
            }
            const int arow = lane & 15, akoff = 16 * (lane >> 4);
            if (th.w) {
                // Compact tile: the B operand of lane (output n, group kg) for
                // K step ks is block base + g - g0 of the lane holding it
                // (ds_bpermute), zeros outside g0 .. g0 + len - 1; one plane
                // at a time, so only 4 operand registers are live.
#pragma unroll 1
                for (int ks = 0; ks < th.y; ++ks) {
                    const int rel = 4 * ks + (lane >> 4) - (meta & 0xFF);
                    const bool ok = (unsigned)rel < (unsigned)((meta >> 8) & 0xFF);
                    const int src = ((meta >> 16) + rel) << 2;
                    const int pos = (th.x + 64 * ks + akoff) & (RING - 1);
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        const uint32_t w[4] = {bn[p].x, bn[p].y, bn[p].z, bn[p].w};
                        i32x4 bq;
#pragma unroll
                        for (int d = 0; d < 4; ++d) {
                            const int v = __builtin_amdgcn_ds_bpermute(src, (int)w[d]);
                            bq[d] = ok ? v : 0;
                        }
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            const i32x4 av = *reinterpret_cast<const i32x4*>(&win[c][arow][pos]);
                            acc[c][p] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bq, acc[c][p], 0, 0, 0);
                        }
                    }
                }
            } else {
                // Dense tile (nK = 1, identity axes, or more than 64 nonzero
                // groups): each K step's blocks loaded in turn.
#pragma unroll 1
                for (int ks = 0; ks < th.y; ++ks) {
                    if (ks > 0) {
#pragma unroll
                        for (int p = 0; p < 3; ++p) bn[p] = tblk[th.z + lane + (ks * 3 + p) * 64];
                    }
                    const int pos = (th.x + 64 * ks + akoff) & (RING - 1);
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const i32x4 av = *reinterpret_cast<const i32x4*>(&win[c][arow][pos]);
#pragma unroll
                        for (int p = 0; p < 3; ++p)
                            acc[c][p] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, __builtin_bit_cast(i32x4, bn[p]),
                                                                            acc[c][p], 0, 0, 0);
                    }
                }
            }
            const int xo = 16 * t + (lane & 15);
            if (xo < h.out_len) {
                // T bytes = clip8 ^ 0x80 (the MFMA's signed form), from the
                // signed saturation of the bias-lowered sums
                uint32_t outc[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    int32_t ss[4];
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) ss[rr] = planes3(acc[c][0][rr], acc[c][1][rr], acc[c][2][rr]);
                    outc[c] = clip8x4_x80(ss[0], ss[1], ss[2], ss[3]);
                }
                // (an opaque lane copy: hoisted out of the chunk loop, this
                // 64-bit row address was live through phase 1 and spilled)
                int ln = lane;
                asm volatile("" : "+v"(ln));
                const int grp = (row0 >> 2) + (ln >> 4);
                uint4* dst = reinterpret_cast<uint4*>(tmp + h.dst_off + (int64_t)grp * h.dst_pitch) + xo;
                const uint32_t w[4] = {outc[0], outc[1], outc[2], outc[3]};
                // Nontemporal: T is read back only after the whole launch
                // (-0.8 % against plain stores; nontemporal T loads in the V
                // pass measured +15 %).
                store16<2>(reinterpret_cast<uint8_t*>(dst), 16, true, w);
            }
        }
        // The next chunk's first sets are waited for here, at the end of
        // phase 2 (which hid their latency): from this point on the compiler
        // may copy their registers (it does, at the loop's back edge).
        asm_wait(RA.p, RA.live ? 4 * RB.live : -1);
        asm_wait(RB.p, RB.live ? 0 : -1);
        if (!more) break;
        __syncthreads();
    }
}

// Composite rows outside the overlay's 16-row bands [vb0, vb1) are plain
// copies of the background (Paste.c leaves them untouched).  The H-pass
// launch's copy blocks write them (and, column split, the band rows' groups
// outside the overlay), so ipp_pipe_vblend_bands only visits the overlay.
__device__ __forceinline__ void paste_bands(const ipp_paste_desc& p, int& vb0, int& vb1) {
    vb0 = (p.y >> 4) << 4;
    vb1 = min(p.bg_h, ((p.y + p.ov_h + 15) >> 4) << 4);
    vb1 = max(vb1, vb0);
}

// Column split of the band rows [vb0, vb1): on dense, 16-B aligned images
// whose width is a multiple of 16, the H pass's copy blocks also write the
// band rows' 16-pixel groups outside [gx0, gx1) (the groups the overlay
// touches) and the V pass visits only [gx0, gx1).  Both kernels decide it
// with this one predicate (ipp_plan.cpp counts the bytes the same way).
__device__ __forceinline__ bool band_cols_split(const ipp_paste_desc& p, const uint8_t* bg, const uint8_t* dst,
                                                int& gx0, int& gx1) {
    const int rb = 3 * p.bg_w;
    gx0 = max(p.x, 0) >> 4;
    gx1 = min((p.x + p.ov_w + 15) >> 4, p.bg_w >> 4);
    const int64_t lr = 3 * (p.bg_w >> 4);  // ≥ the split's vectors per band row
    return (p.bg_w & 15) == 0 && p.bg_pitch == rb && p.dst_pitch == rb && gx0 < gx1 &&
           (int64_t)p.bg_h * lr * lr < (1ll << 32) &&  // (the H copy's umulhi division stays exact)
           ((reinterpret_cast<uintptr_t>(bg + p.bg_off) | reinterpret_cast<uintptr_t>(dst + p.dst_off)) & 15u) == 0;
}

// 16-B vectors per thread in flight in the per-item background copy.  A copy
// block holds one of the CU's four H-pass block slots for as long as it
// streams, so bytes in flight per block set how much H-pass time the copy
// displaces.
constexpr int kCopyU = 16;
template <int NT = 256, int U = kCopyU>
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
        // Two flat byte ranges [0, vb0·rb) and [vb1·rb, bg_h·rb) in 16-B
        // vectors, then (column split) each band row's L vectors left of the
        // overlay's groups and R right of them.
        int gx0, gx1;
        const bool split = band_cols_split(p, bg, dst, gx0, gx1);
        const int L = split ? 3 * gx0 : 0, LR = split ? 3 * ((p.bg_w >> 4) - gx1) + L : 0;
        const int rv = rb / 16, rgt = 3 * gx1 - L;       // vectors per row; right part's column shift
        const uint32_t mag = LR > 0 ? (uint32_t)((0x100000000ull + LR - 1) / LR) : 0u;  // j / LR = umulhi(j, mag)
        const int64_t n0 = (int64_t)vb0 * rb / 16, n1 = (int64_t)(p.bg_h - vb1) * rb / 16;
        const int64_t n2 = (int64_t)(vb1 - vb0) * LR, V = n0 + n1 + n2;
        const int64_t a = V * share / nshare, e = V * (share + 1) / nshare;
        const int64_t skip = (int64_t)vb1 * rb / 16 - n0;  // vector index gap over the bands
        auto vec_of = [&](int64_t i) -> int64_t {
            if (i < n0) return i;
            if (i < n0 + n1) return i + skip;
            // j < n2 ≤ bg_h·LR, so j·LR < 2^32 (band_cols_split) and umulhi is exact
            const uint32_t j = (uint32_t)(i - n0 - n1);
            const uint32_t r = __umulhi(j, mag), c = j - r * (uint32_t)LR;
            return (int64_t)(vb0 + (int)r) * rv + (int)c + ((int)c < L ? 0 : rgt);
        };
        const u32x4_t* s4 = reinterpret_cast<const u32x4_t*>(sb);
        u32x4_t* d4 = reinterpret_cast<u32x4_t*>(db);
        for (int64_t i0 = a + threadIdx.x; i0 < e; i0 += U * NT) {
            u32x4_t v[U];
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int64_t i = i0 + NT * j;
                if (i < e) v[j] = s4[vec_of(i)];
            }
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int64_t i = i0 + NT * j;
                if (i < e) __builtin_nontemporal_store(v[j], d4 + vec_of(i));
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

// Grouped background copy (round 5).  Items are background-sorted, so runs
// of consecutive items paste onto the same background.  A copy block takes
// one row slab of a group of kCopyGroup consecutive items: each thread loads a
// 16-B background vector once and stores it to every item of the run whose
// composite takes it — outside the item's overlay bands [vb0, vb1), or (column
// split) outside the overlay's 16-pixel groups [gx0, gx1) in a band row.  The
// copy's load instructions, which queue on the same texture path as the H
// pass's gathers, drop by the run length (its stores stay: they are most of
// the ≈ 1.4 ms the copy still adds to the H launch).  Items
// whose composite is not flat (pitches, alignment) take bg_copy_outside_bands
// with share = slab.
#ifndef IPP_COPY_GROUP
#define IPP_COPY_GROUP IPP_PIPE_COPY_GROUP  // (ipp.h; experiment builds may override it)
#endif
// Copy blocks per group: one per item (A/B, B = 4096, alternating runs on
// one box: H launch 8.78-8.87 ms at 8 slabs per 8 items, 8.76-8.83 at 6, 8.80-8.88
// at 4, 8.94 at 16, 9.08-9.10 at 32; per-item copy blocks of round 4: 9.07-9.20;
// groups of 4 / 12 / 16 items: 8.89-8.90 / 8.84-8.92 / 9.10).
#ifndef IPP_COPY_SLABS
#define IPP_COPY_SLABS IPP_COPY_GROUP
#endif
// 16-B vectors per thread in flight in the grouped copy (8 made the kernel
// spill inside the H pass's 128-VGPR budget; 2 measured 0.5 % slower than 4).
// Stores: buffer stores with the nt bit (global nt stores 9.02-9.03, plain
// 9.35, sc1 9.41 ms for the H launch; round 5, one box).
constexpr int kCopyGU = 4;
constexpr int kCopyGroup = IPP_COPY_GROUP;  // items per copy group (≤ 64: one lane per item)
constexpr int kCopySlabs = IPP_COPY_SLABS;  // copy blocks (row slabs) per group
static_assert(kCopyGroup >= 1 && kCopyGroup <= 64, "one lane per item of a copy group");

// Item j of a copy group: its composite's flat-copy parameters (lane j).
struct CopyItem {
    uint32_t dlo, dhi;        // dst + dst_off
    uint32_t blo, bhi;        // bg + bg_off
    int32_t dims;             // bg_w | bg_h << 16 (the run key with the bg pointer)
    int32_t vb0, vb1;         // overlay bands
    int32_t c0, c1;           // band-row vectors [c0, c1) left to the V pass
    int32_t flat;             // composite is a flat 16-B aligned copy of bg
};

template <int NT = 256, int U = kCopyGU>
__device__ __forceinline__ void bg_copy_group(const ipp_pipe_desc* __restrict__ descs, int n, int i0, int slab,
                                              const uint8_t* __restrict__ bg, uint8_t* __restrict__ dst) {
    const int cnt = min(kCopyGroup, n - i0);
    if (cnt <= 0) return;
    const int lane = threadIdx.x & 63;
    CopyItem ci = {0u, 0u, 0u, 0u, -1, 0, 0, 0, 0, 0};
    if (lane < cnt) {
        const ipp_paste_desc& p = descs[i0 + lane].p;
        const int rb = 3 * p.bg_w;
        const uint8_t* sb = bg + p.bg_off;
        uint8_t* db = dst + p.dst_off;
        const uint64_t du = reinterpret_cast<uint64_t>(db), bu = reinterpret_cast<uint64_t>(sb);
        ci.dlo = (uint32_t)du;
        ci.dhi = (uint32_t)(du >> 32);
        ci.blo = (uint32_t)bu;
        ci.bhi = (uint32_t)(bu >> 32);
        ci.dims = p.bg_w | (p.bg_h << 16);
        int vb0, vb1, gx0, gx1;
        paste_bands(p, vb0, vb1);
        ci.vb0 = vb0;
        ci.vb1 = vb1;
        const bool split = band_cols_split(p, bg, dst, gx0, gx1);
        ci.c0 = split ? 3 * gx0 : 0;
        ci.c1 = split ? 3 * gx1 : rb / 16;
        // The slab's vector index i is split into (row, column) by umulhi(i,
        // ⌈2^32 / rv⌉), exact while i·rv < 2^32: the slab's vector count times
        // rv must stay below 2^32 (and row / column fit 16 bits each).
        const int64_t rv = rb / 16, slab_rows = (p.bg_h + kCopySlabs - 1) / kCopySlabs;
        ci.flat = p.bg_pitch == rb && p.dst_pitch == rb && (rb & 15) == 0 && ((du | bu) & 15u) == 0 &&
                  p.bg_w < 65536 && p.bg_h < 32768 && slab_rows * rv * rv < (1ll << 32);
    }
    auto rl = [](int32_t v, int j) { return __builtin_amdgcn_readlane(v, j); };
    auto rlu = [](uint32_t v, int j) { return (uint32_t)__builtin_amdgcn_readlane((int32_t)v, j); };
    int j0 = 0;
    while (j0 < cnt) {
        // run [j0, j1): consecutive items on one background (same pointer and dims)
        const uint32_t blo = rlu(ci.blo, j0), bhi = rlu(ci.bhi, j0);
        const int32_t dims = rl(ci.dims, j0);
        int j1 = j0 + 1;
        while (j1 < cnt && rlu(ci.blo, j1) == blo && rlu(ci.bhi, j1) == bhi && rl(ci.dims, j1) == dims) ++j1;
        // flat items of the run: one shared load per vector
        uint64_t fm = 0;
        for (int j = j0; j < j1; ++j) fm |= (uint64_t)(rl(ci.flat, j) != 0) << j;
        if (fm) {
            const int bw = dims & 0xFFFF, bh = dims >> 16;
            const int rv = 3 * bw / 16;  // vectors per row
            const int ya = (int)((int64_t)bh * slab / kCopySlabs), ye = (int)((int64_t)bh * (slab + 1) / kCopySlabs);
            const uint32_t total = (uint32_t)((ye - ya) * rv);
            const uint32_t mag = (uint32_t)((0x100000000ull + rv - 1) / rv);  // i / rv = umulhi(i, mag) for i·rv < 2^32
            const u32x4_t* s4 = reinterpret_cast<const u32x4_t*>(((uint64_t)bhi << 32) | blo) + (int64_t)ya * rv;
            for (uint32_t ib = threadIdx.x; ib < total; ib += U * NT) {
                u32x4_t v[U];
                uint32_t rc[U];  // slab row << 16 | vector column (one register per vector)
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t i = ib + NT * u;
                    const uint32_t q = __umulhi(i, mag);
                    rc[u] = (q << 16) | (i - q * (uint32_t)rv);
                    if (i < total) v[u] = s4[i];
                }
                for (int j = j0; j < j1; ++j) {
                    if (!((fm >> j) & 1u)) continue;
                    // the item's band rows relative to the slab, its band-row vectors [c0, c1)
                    const int32_t r0 = rl(ci.vb0, j) - ya, rn = rl(ci.vb1, j) - rl(ci.vb0, j);
                    const int32_t c0 = rl(ci.c0, j), cn = rl(ci.c1, j) - c0;
                    u32x4_t* d4 = reinterpret_cast<u32x4_t*>(((uint64_t)rlu(ci.dhi, j) << 32) | rlu(ci.dlo, j)) +
                                  (int64_t)ya * rv;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t i = ib + NT * u;
                        const bool inside = (uint32_t)((int32_t)(rc[u] >> 16) - r0) < (uint32_t)rn &&
                                            (uint32_t)((int32_t)(rc[u] & 0xFFFFu) - c0) < (uint32_t)cn;
                        if (i < total && !inside) __builtin_amdgcn_raw_buffer_store_b128(v[u], rsrc_of(d4), i * 16u, 0, 2);
                    }
                }
            }
        }
        // the run's other items: their own copy, this block's slab of it
        for (int j = j0; j < j1; ++j)
            if (!((fm >> j) & 1u)) bg_copy_outside_bands<NT>(descs[i0 + j].p, bg, dst, slab, kCopySlabs);
        j0 = j1;
    }
}

// May an H-pass block of this window drop the gathers' row test (YR)?  Row
// in_h must start at or past the buffer's last record (need), and no row
// offset yin·pitch (|yin| ≤ 2^15: 16.16 positions) may wrap around 2^32 back
// into [0, need).  (A full-width crop of a dense 3-channel source, pitch =
// 3·in_w, has in_h·pitch = need - 1 and keeps the row test.)
__device__ __forceinline__ bool yr_range_ok(int in_h, int pitch, int need) {
    return (int64_t)in_h * pitch >= (int64_t)need && (int64_t)32768 * pitch + need <= (int64_t)1 << 32;
}

// One H-pass block: band tb of item im.
template <int NR, bool ZONES, int CN>
__device__ __forceinline__ void hpass_block(Hpass2Lds<NR>& L, const uint8_t* __restrict__ src,
                                            uint8_t* __restrict__ tmp, const int32_t* __restrict__ coefs,
                                            const ipp_pipe_desc* __restrict__ descs, int im, int tb,
                                            const ipp_hsv_params& hp) {
    const ipp_gather_desc g = descs[im].g;
    const ipp_resample_desc h = descs[im].h;
    const int row0 = tb * HR;
    if (row0 >= h.lines) return;  // block-uniform
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

    hsv_tables_init<NR>(L.T, hp);

    // Zones: per-lane row bits now, column bits per pixel.  With > 8 ranges
    // the column bounds live in LDS (in registers they spilled).
    int32_t zc0r[ZONES && NR <= 8 ? NR : 1], zcwr[ZONES && NR <= 8 ? NR : 1];
    int32_t* zc0 = zc0r;
    int32_t* zcw = zcwr;
    if (ZONES && NR > 8) {
        zc0 = L.zc;
        zcw = L.zc + NR;
    }
    uint32_t zrow = 0;
    const int lane = threadIdx.x & 63;
    const int y = h.line0 + row0 + 2 * (lane >> 3) + ((lane >> 1) & 1);
    if (ZONES) {
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            int a, bb, cc, dd;
            slice_indices(hp.r[k].zone[0], g.out_h - hp.r[k].zone[1], g.out_h, a, bb);
            slice_indices(hp.r[k].zone[2], g.out_w - hp.r[k].zone[3], g.out_w, cc, dd);
            zrow |= (uint32_t)(y >= a && y < bb) << k;
            if (NR <= 8 || threadIdx.x == 0) {
                zc0[k] = cc;
                zcw[k] = dd - cc;
            }
        }
    }

    // Source window as a buffer resource: every in-window dword read is in
    // range; out-of-window pixels use offset 0xFFFFFFFF (range check → 0).
    const Sampler S = make_sampler(src, g);
    // (32-bit scalar arithmetic: a 64-bit min would land in VGPRs and turn every
    // buffer load into a waterfall loop; items are < 2 GiB, checked on the host.)
    const int nrec = (g.src_h - g.in_y0) * g.src_pitch - g.in_x0 * g.src_cn;
    const int need = (g.in_h - 1) * g.src_pitch + g.in_w * CN + (CN == 3 ? 1 : 0);
    // The fast body needs no clamp (the last pixel's dword ends inside the
    // image) and a window whose rows the range check can reject; every other
    // block takes the general (CLAMP) body.  Block-uniform.
    const bool fast = need <= nrec && yr_range_ok(g.in_h, (int)S.pitch, need);
    const uint64_t sbu = reinterpret_cast<uint64_t>(S.base);
    Hp2Block B;
    // records: to the image end, or (fast) only to one byte past the window's
    // last pixel, so that a row above or below the window is out of range
    B.rsv = u32x4_t{(uint32_t)sbu, (uint32_t)(sbu >> 32) & 0xFFFFu, (uint32_t)(fast ? min(nrec, need) : nrec),
                    0x00020000u};
    B.lim = S.lim;
    B.rowx = (uint32_t)S.b2 + (uint32_t)y * (uint32_t)S.b1;
    B.rowy = (uint32_t)S.b5 + (uint32_t)y * (uint32_t)S.b4;
    B.b0 = S.b0;
    B.b3 = S.b3;
    B.pitch = (int32_t)S.pitch;
    B.in_w = S.in_w;
    B.in_h = S.in_h;
    {
        // Row y's valid columns: 0 <= xx(x) < in_w·2^16 and 0 <= yy(x) < in_h·2^16,
        // both linear in x; ±2 columns of slack absorb the rounding.  Union over
        // the block's 16 rows (lanes 8(r>>1) + 2(r&1) .. hold row r) by readlane.
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
        clip((float)(int32_t)B.rowx, (float)S.b0, 65536.0f * (float)S.in_w);
        clip((float)(int32_t)B.rowy, (float)S.b3, 65536.0f * (float)S.in_h);
        const int ilo = lo > hi ? 0x3FFFFFFF : (int)fmaxf(lo - 2.0f, -1e8f);
        const int ihi = lo > hi ? -0x3FFFFFFF : (int)fminf(hi + 2.0f, 1e8f);
        int blo = 0x3FFFFFFF, bhi = -0x3FFFFFFF;
#pragma unroll
        for (int rr = 0; rr < HR; ++rr) {
            const int lr = 8 * (rr >> 1) + 2 * (rr & 1);  // a lane of row rr
            blo = min(blo, __builtin_amdgcn_readlane(ilo, lr));
            bhi = max(bhi, __builtin_amdgcn_readlane(ihi, lr));
        }
        B.xlo = blo;
        B.xhi = bhi;
    }

    // (the table barrier is in the body, after the first gathers)
    const int nrows = min(HR, h.lines - row0);
    if (fast)
        hpass2_body<NR, ZONES, CN, false>(L.T, L.win, wave, B, tmp, coefs, h, row0, nrows, zc0, zcw, zrow);
    else
        hpass2_body<NR, ZONES, CN, true>(L.T, L.win, wave, B, tmp, coefs, h, row0, nrows, zc0, zcw, zrow);
}

// 4 waves per SIMD (≤ 128 VGPRs); the zone forms get 3 (their per-lane zone
// bounds spill at 128, and nothing may spill between an asm gather and its
// wait).
template <int NR, bool ZONES, int CN>
__global__ void __launch_bounds__(64 * HP_NW) __attribute__((amdgpu_waves_per_eu(ZONES ? 3 : 4)))
k_pipe_hpass2(const uint8_t* __restrict__ src, uint8_t* __restrict__ tmp, const int32_t* __restrict__ coefs,
              const ipp_pipe_desc* __restrict__ descs, int n, FastDiv tiles_y, FastDiv per_grp, ipp_hsv_params hp,
              const uint8_t* __restrict__ bg, uint8_t* __restrict__ dst) {
    __shared__ Hpass2Lds<NR> L;
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    // tiles_y = H-pass blocks per item (one per band).  Each group of
    // kCopyGroup items owns its items' H-pass blocks followed by kCopySlabs
    // background-copy blocks (per_grp = kCopyGroup·tiles_y + kCopySlabs), so
    // the copies run beside the H pass on every XCD.
    const int ty = (int)tiles_y.d;
    const int grp = (int)fdiv(b, per_grp);
    const int t = (int)(b - (uint32_t)grp * per_grp.d);
    if (t >= kCopyGroup * ty) {
        bg_copy_group<64 * HP_NW>(descs, n, grp * kCopyGroup, t - kCopyGroup * ty, bg, dst);
        return;
    }
    const int j = (int)fdiv((uint32_t)t, tiles_y);
    const int im = grp * kCopyGroup + j;
    if (im >= n) return;
    hpass_block<NR, ZONES, CN>(L, src, tmp, coefs, descs, im, t - j * ty, hp);
}

// V pass on MFMA (tap tiles aligned with 16-row background bands: the plan's
// phase = p.y mod 16) → unpremultiply → blend onto the background.  Block =
// 16 composite rows of one item.  A = taps of the band's 16 overlay rows (lane
// l: row l&15, T rows 16(l>>4)..+15 of the K step), B = 64 T rows × 16
// overlay columns of one channel (four 16-B T groups per lane give all four
// channels), D lane l = column l&15, rows 4(l>>4)..+3.
//
// Horner accumulation over the tap byte planes (round 6): one accumulator per
// channel instead of one per (channel, plane) — plane 2's products summed over
// every K step, shifted left by 8, plane 1's added, shifted again with the row
// bias added (v_lshl_add), then plane 0's: ((S2 << 8) + S1) << 8 + bias + S0
// equals planes3(bias + S0, S1, S2) in int32 wrap-around arithmetic.  It
// frees 32 VGPRs of the 48 the accumulators took.
constexpr int VBR = 16;
// V pass: column tiles with nK ≤ IPP_VB_DB double-buffer their T groups (the
// wave's next tile's loads fly during this tile's MFMAs).
#ifndef IPP_VB_DB
#define IPP_VB_DB 2
#endif
// V pass: the band's taps loaded once for all its column tiles (nK ≤
// IPP_VB_HOIST_MAX; larger nK load each K step's taps per column tile).  Of
// the bench's V tiles 7 % have nK 1, 74 % nK 2, 19 % nK 3.
#ifndef IPP_VB_HOIST_MAX
#define IPP_VB_HOIST_MAX 3
#endif
// V pass occupancy target (waves per SIMD).  Round 5 (three accumulators per
// channel): 3 fit 160 VGPRs with every nK ≤ 4 hoisted (the compiler's own
// choice, 168 VGPRs + 52 AGPRs, gave 2 waves): 1.49-1.52 -> 1.37-1.40 ms.
#ifndef IPP_VB_WPE
#define IPP_VB_WPE 3
#endif

// orow (the band's unpremultiplied overlay rows in LDS) is indexed by
// composite column - (p.x & ~15), so a 16-pixel composite group reads its 16
// overlay pixels with four aligned ds_read_b128; the ≤ 15 columns before the
// overlay and after it are zero (α 0: the background stays).
__host__ __device__ constexpr int orow_stride(int ov_w_max) { return (ov_w_max + 32 + 3) & ~3; }
// The widest overlay the V launch takes: its rows must fit 64 KB of LDS
// (IPP_PIPE_MAX_OV_W in ipp.h; the magic-divisor table is dropped for
// overlays too wide to hold it beside the rows).
static_assert((size_t)VBR * orow_stride(IPP_PIPE_MAX_OV_W) * 4 <= 64 * 1024, "V-pass rows in LDS");
static_assert((size_t)VBR * orow_stride(IPP_PIPE_MAX_OV_W + 1) * 4 > 64 * 1024, "IPP_PIPE_MAX_OV_W is the limit");

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Paste.c BLEND on two bytes at once (16-bit lanes): DIV255(bg·(255 - a) +
// ov·a), written as 255·bg + 128 + (ov - bg)·a (mod 2^16: the true value is
// in [0, 65153]) followed by DIV255's (t + (t >> 8)) >> 8.
__device__ __forceinline__ uint32_t blend_u16x2(uint32_t bg, uint32_t ov, uint32_t al) {
    const u16x2 b = __builtin_bit_cast(u16x2, bg), o = __builtin_bit_cast(u16x2, ov), a = __builtin_bit_cast(u16x2, al);
    const u16x2 c255 = {255, 255}, c128 = {128, 128}, c8 = {8, 8};
    const u16x2 t = (u16x2)(o - b) * a + (b * c255 + c128);
    return __builtin_bit_cast(uint32_t, (u16x2)((u16x2)(t + (t >> c8)) >> c8));
}

// 16 composite pixels (48 bytes, bg[0..11]) blended in place with 16 RGBA
// overlay pixels (ov[0..15]).  Byte j of the row segment is channel j mod 3
// of pixel j / 3; each output dword is done as two byte pairs (bytes 0, 2 and
// 1, 3) in 16-bit lanes, the overlay byte and its pixel's α gathered by v_perm.
__device__ __forceinline__ void blend48(uint32_t (&bg)[12], const uint32_t (&ov)[16]) {
#pragma unroll
    for (int d = 0; d < 12; ++d) {
        uint32_t r[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j0 = 4 * d + h, j1 = j0 + 2;                 // the pair's bytes
            const int p0 = j0 / 3, p1 = j1 / 3, c0 = j0 % 3, c1 = j1 % 3;
            // v_perm(hi, lo, sel): bytes 0-3 of lo = sel 0-3, of hi = 4-7; 0x0c = 0
            const uint32_t sel_ov = (uint32_t)c0 | 0x0c00u | ((uint32_t)(p1 == p0 ? c1 : 4 + c1) << 16) | 0x0c000000u;
            const uint32_t sel_al = 3u | 0x0c00u | ((uint32_t)(p1 == p0 ? 3 : 7) << 16) | 0x0c000000u;
            const uint32_t ovp = __builtin_amdgcn_perm(ov[p1], ov[p0], sel_ov);
            const uint32_t alp = __builtin_amdgcn_perm(ov[p1], ov[p0], sel_al);
            const uint32_t bgp = __builtin_amdgcn_perm(0u, bg[d], h ? 0x0c030c01u : 0x0c020c00u);
            r[h] = blend_u16x2(bgp, ovp, alp);
        }
        bg[d] = __builtin_amdgcn_perm(r[1], r[0], 0x06020400u);  // r0 b0, r1 b0, r0 b2, r1 b2
    }
}

// acc = (acc << 8) + (a0, a1, a2, a3) (Horner step; the compiler emits one
// v_lshl_add_u32 per dword.  Plain code, not inline asm: the MFMA results it
// reads need the wait states the compiler's hazard recognizer inserts, which
// it does not do for an asm operand.)
__device__ __forceinline__ void horner8(i32x4& acc, int32_t a0, int32_t a1, int32_t a2, int32_t a3) {
    acc = (acc << 8) + i32x4{a0, a1, a2, a3};
}

// Channel c's B operand of one K step: dword c of its four T groups (a
// register transpose the MFMA needs anyway: its source tuple must be four
// consecutive registers).
__device__ __forceinline__ i32x4 vb_bop(const u32x4_t (&g)[4], int c) {
    return i32x4{(int)g[0][c], (int)g[1][c], (int)g[2][c], (int)g[3][c]};
}

// One column tile's V sums, Horner over the tap byte planes (see above):
// plane 2's MFMAs over all NK K steps, << 8, plane 1's, << 8 with the row
// biases, plane 0's.  bq = the channel-major B operands (vb_bop) per K step.
template <int NK>
__device__ __forceinline__ void vb_mfma_tile(const i32x4 (&ta)[NK][3], const i32x4 (&bq)[NK][4], const int32_t (&rb)[4],
                                             i32x4 (&acc)[4]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = i32x4{0, 0, 0, 0};
#pragma unroll
    for (int q = 2; q >= 0; --q) {
#pragma unroll
        for (int ks = 0; ks < NK; ++ks)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ta[ks][q], bq[ks][c], acc[c], 0, 0, 0);
        if (q == 2) {
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[c] <<= 8;
        } else if (q == 1) {
#pragma unroll
            for (int c = 0; c < 4; ++c) horner8(acc[c], rb[0], rb[1], rb[2], rb[3]);
        }
    }
}

// One V-pass block: band ty of item im, counted from the first 16-row band
// the overlay touches (the rows outside those bands: ipp_pipe_hpass_bgcopy).
// MAGIC: unpremultiply by the per-block LDS table of magic divisors (exact,
// unpremultiply_magic) instead of a reciprocal and two fix-ups per channel:
// 1.340 -> 1.319 ms (round 5, profiles/r05/vpass/ab_unpremul_magic_r05al.txt);
// overlays too wide for the table beside their rows take the reciprocal.
template <bool MAGIC>
__device__ __forceinline__ void vblend_block(uint32_t* __restrict__ orow, const uint8_t* __restrict__ tmp,
                                             const uint8_t* __restrict__ bg, uint8_t* __restrict__ dst,
                                             const int32_t* __restrict__ coefs,
                                             const ipp_pipe_desc* __restrict__ descs, int im, int ty, int ov_w_max) {
    const ipp_paste_desc p = descs[im].p;
    int y0 = ty * VBR;
    {
        int vb0, vb1;
        paste_bands(p, vb0, vb1);
        y0 += vb0;
        if (y0 >= vb1) return;
    }
    if (y0 >= p.bg_h) return;
    const int nrows = min(VBR, p.bg_h - y0);
    const int oy_lo = max(0, y0 - p.y), oy_hi = min(p.ov_h, y0 + nrows - p.y);
    const bool any = oy_lo < oy_hi;  // block-uniform
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

    const int os = orow_stride(ov_w_max), xo = p.x & 15;  // orow column of overlay column 0
    const uint8_t* bgb = bg + p.bg_off + (int64_t)y0 * p.bg_pitch;
    uint8_t* dsb = dst + p.dst_off + (int64_t)y0 * p.dst_pitch;
    const bool groups = (p.bg_w & 15) == 0 && ((p.bg_pitch | p.dst_pitch) & 15) == 0 &&
                        ((reinterpret_cast<uintptr_t>(bgb) | reinterpret_cast<uintptr_t>(dsb)) & 15u) == 0;
    // groups per row visited: all of them, or (column split) the overlay's
    // [sx0, sx1) — the H pass's copy blocks wrote the rest of the band rows
    int sx0, sx1;
    const bool csplit = groups && band_cols_split(p, bg, dst, sx0, sx1);
    const int gc0 = csplit ? sx0 : 0;
    const int G = csplit ? sx1 - sx0 : p.bg_w >> 4, lg = 31 - __builtin_clz(max(G, 1));
    const bool pow2 = (G & (G - 1)) == 0;
    const int gtotal = nrows * G;
    auto gload = [&](int idx, uint4 (&v)[3]) {
        const int rr = pow2 ? idx >> lg : idx / G;
        const int gi = gc0 + idx - rr * G;
        const uint4* sp = reinterpret_cast<const uint4*>(bgb + (int64_t)rr * p.bg_pitch) + 3 * gi;
#pragma unroll
        for (int q = 0; q < 3; ++q) v[q] = sp[q];
    };
    uint4 gcur[3];
    if (any) {
        uint32_t* umag = orow + VBR * os;  // MAGIC: the unpremultiply divisors
        if (MAGIC) {
            umag[threadIdx.x] = unpremul_magic(threadIdx.x);
            __syncthreads();
        }
        // zero the ≤ 15 columns before the overlay and the 16 after it
        for (int e = threadIdx.x; e < VBR * 32; e += 256) {
            const int row = e >> 5, c = e & 31;
            if (c < xo) orow[row * os + c] = 0u;
            else if (c >= 16) orow[row * os + xo + p.ov_w + c - 16] = 0u;
        }
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
        // the row biases (added at the last Horner step)
        int32_t rb[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) rb[r] = tbias[16 * t + 4 * (lane >> 4) + r];
        const u32x4_t* tbase = reinterpret_cast<const u32x4_t*>(tmp + v.src_off);
        const int gbase = (th.x + 16 * (lane >> 4)) >> 2;
        // T groups of K step ks of column tile ct: rows th.x + 64 ks + 16 (lane >> 4) .. + 15
        auto tload = [&](int ct, int ks, u32x4_t (&g)[4]) {
            const int xs = min(16 * ct + x_l, p.ov_w - 1);
            const u32x4_t* tq = tbase + xs + (int64_t)(gbase + 16 * ks) * gstride;
#pragma unroll
            for (int j = 0; j < 4; ++j) g[j] = tq[j * gstride];
        };
        // the tile's unpremultiplied overlay pixels into the band's LDS rows
        // (s(c, r) = the sum of channel c, tile row r)
        auto epilogue = [&](int ct, auto s) {
            const int x = 16 * ct + x_l;
            if (x < p.ov_w) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 4 * (lane >> 4) + r;  // band row = tile row
                    const int o = y0 + row - p.y;         // overlay row
                    if (o >= oy_lo && o < oy_hi) {
                        const uint32_t px = clip8x4_mfma(s(0, r), s(1, r), s(2, r), s(3, r));
                        orow[row * os + xo + x] = MAGIC ? unpremultiply_magic(px, umag) : unpremultiply(px);
                    }
                }
            }
        };
        // The band's taps (the A operand) are the same for every column tile:
        // with nK ≤ IPP_VB_HOIST_MAX they are loaded once, before the column
        // tiles, and every tile's T groups for all its K steps are issued
        // before its MFMAs.
        auto tiles = [&](auto nkc) {
            constexpr int NK = decltype(nkc)::value;
            if constexpr (NK > 0) {
                i32x4 ta[NK][3];
#pragma unroll
                for (int ks = 0; ks < NK; ++ks)
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        ta[ks][q] = __builtin_bit_cast(i32x4, tblk[th.z + (ks * 3 + q) * 64 + lane]);
                // the loaded T groups of a tile, turned channel-major
                auto transpose = [&](const u32x4_t (&g)[NK][4], i32x4 (&bq)[NK][4]) {
#pragma unroll
                    for (int ks = 0; ks < NK; ++ks)
#pragma unroll
                        for (int c = 0; c < 4; ++c) bq[ks][c] = vb_bop(g[ks], c);
                };
                if constexpr (NK <= IPP_VB_DB) {
                    // double-buffered T groups: the wave's next column tile's
                    // loads are in flight during this tile's MFMAs and
                    // epilogue; the buffer carried to the next tile is the
                    // channel-major operands, so raw and transposed groups
                    // are never live together
                    i32x4 bc[NK][4];
                    u32x4_t gn[NK][4];
                    int ct = wave;
                    if (ct < ctiles) {
#pragma unroll
                        for (int ks = 0; ks < NK; ++ks) tload(ct, ks, gn[ks]);
                        transpose(gn, bc);
                    }
                    for (; ct < ctiles; ct += 4) {
                        const bool more = ct + 4 < ctiles;
                        if (more) {
#pragma unroll
                            for (int ks = 0; ks < NK; ++ks) tload(ct + 4, ks, gn[ks]);
                        }
                        i32x4 acc[4];
                        vb_mfma_tile<NK>(ta, bc, rb, acc);
                        epilogue(ct, [&](int c, int r) { return acc[c][r]; });
                        if (more) transpose(gn, bc);
                    }
                } else {
                    for (int ct = wave; ct < ctiles; ct += 4) {
                        u32x4_t g[NK][4];
#pragma unroll
                        for (int ks = 0; ks < NK; ++ks) tload(ct, ks, g[ks]);
                        i32x4 bq[NK][4];
                        transpose(g, bq);
                        i32x4 acc[4];
                        vb_mfma_tile<NK>(ta, bq, rb, acc);
                        epilogue(ct, [&](int c, int r) { return acc[c][r]; });
                    }
                }
            } else {
                // nK beyond the hoisted forms: each K step's taps and T groups
                // loaded in turn, one accumulator per (channel, plane)
                for (int ct = wave; ct < ctiles; ct += 4) {
                    i32x4 acc[4][3];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        acc[c][0] = i32x4{rb[0], rb[1], rb[2], rb[3]};
                        acc[c][1] = i32x4{0, 0, 0, 0};
                        acc[c][2] = i32x4{0, 0, 0, 0};
                    }
#pragma unroll 1
                    for (int ks = 0; ks < th.y; ++ks) {
                        i32x4 a[3];
#pragma unroll
                        for (int q = 0; q < 3; ++q) a[q] = __builtin_bit_cast(i32x4, tblk[th.z + (ks * 3 + q) * 64 + lane]);
                        u32x4_t g[4];
                        tload(ct, ks, g);
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            const i32x4 bq = vb_bop(g, c);
#pragma unroll
                            for (int q = 0; q < 3; ++q)
                                acc[c][q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[q], bq, acc[c][q], 0, 0, 0);
                        }
                    }
                    epilogue(ct, [&](int c, int r) { return planes3(acc[c][0][r], acc[c][1][r], acc[c][2][r]); });
                }
            }
        };
        // (a tile with more K steps than IPP_VB_HOIST_MAX takes the generic loop)
        switch (th.y <= IPP_VB_HOIST_MAX ? th.y : 0) {
            case 1: tiles(std::integral_constant<int, 1>{}); break;
#if IPP_VB_HOIST_MAX >= 2
            case 2: tiles(std::integral_constant<int, 2>{}); break;
#endif
#if IPP_VB_HOIST_MAX >= 3
            case 3: tiles(std::integral_constant<int, 3>{}); break;
#endif
#if IPP_VB_HOIST_MAX >= 4
            case 4: tiles(std::integral_constant<int, 4>{}); break;
#endif
            default: tiles(std::integral_constant<int, 0>{}); break;
        }
        __syncthreads();
    }

    // Phase 2: composite rows = background bytes, blended inside the footprint.
    const int row_bytes = 3 * p.bg_w;
    if (groups) {
        // 16-pixel groups: 48 bytes per thread and step (three 16-B loads in
        // flight; the next step's loads are issued before this step's blend
        // and stores), the overlay pixels from orow, blended in 16-bit lanes.
        const int gx0 = p.x >> 4, gx1 = (p.x + p.ov_w + 15) >> 4;  // groups the overlay touches
        if ((int)threadIdx.x < gtotal) gload(threadIdx.x, gcur);
        for (int idx = threadIdx.x; idx < gtotal; idx += 256) {
            uint4 gnxt[3];
            if (idx + 256 < gtotal) gload(idx + 256, gnxt);
            const int rr = pow2 ? idx >> lg : idx / G;
            const int gi = gc0 + idx - rr * G;
            uint32_t w[12];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                w[4 * q] = gcur[q].x;
                w[4 * q + 1] = gcur[q].y;
                w[4 * q + 2] = gcur[q].z;
                w[4 * q + 3] = gcur[q].w;
            }
            const int o = y0 + rr - p.y;
            if (any && o >= oy_lo && o < oy_hi && gi >= gx0 && gi < gx1) {
                const uint4* orw = reinterpret_cast<const uint4*>(orow + rr * os + 16 * (gi - gx0));
                uint32_t ov[16];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint4 v4 = orw[q];
                    ov[4 * q] = v4.x;
                    ov[4 * q + 1] = v4.y;
                    ov[4 * q + 2] = v4.z;
                    ov[4 * q + 3] = v4.w;
                }
                blend48(w, ov);
            }
            // plain stores (nt 1.356, sc1 1.581 against 1.335 ms; round 5,
            // profiles/r05/vpass/ab_vstore_policy_r05af.txt)
            uint8_t* dp = dsb + (int64_t)rr * p.dst_pitch + 48 * gi;
#pragma unroll
            for (int q = 0; q < 3; ++q) store16<0>(dp + 16 * q, 16, true, w + 4 * q);
#pragma unroll
            for (int q = 0; q < 3; ++q) gcur[q] = gnxt[q];
        }
        return;
    }
    // General layout: 16-B chunks, byte-wise blend.  Four chunks per thread are
    // loaded before any is stored, so each wave keeps four reads in flight.
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
                load16(bp, nb[u], nb[u] == 16 && (reinterpret_cast<uintptr_t>(bp) & 15u) == 0, w[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (nb[u] <= 0) continue;
            const int o = y0 + rr[u] - p.y;
            if (any && o >= oy_lo && o < oy_hi && c0[u] + nb[u] > 3 * p.x && c0[u] < 3 * (p.x + p.ov_w)) {
                const uint32_t* orw = orow + rr[u] * os + xo;
                blend16(w[u], c0[u], nb[u], p.x, p.ov_w, [&](int ox) { return orw[ox]; });
            }
            uint8_t* dp = dst + p.dst_off + (int64_t)(y0 + rr[u]) * p.dst_pitch + c0[u];
            store16<0>(dp, nb[u], nb[u] == 16 && (reinterpret_cast<uintptr_t>(dp) & 15u) == 0, w[u]);
        }
    }
}

#if IPP_VB_WPE > 0
#define IPP_VB_ATTR __attribute__((amdgpu_waves_per_eu(IPP_VB_WPE)))
#else
#define IPP_VB_ATTR
#endif
template <bool MAGIC>
__global__ void __launch_bounds__(256) IPP_VB_ATTR
k_pipe_vblend_mfma(const uint8_t* __restrict__ tmp, const uint8_t* __restrict__ bg, uint8_t* __restrict__ dst,
                   const int32_t* __restrict__ coefs, const ipp_pipe_desc* __restrict__ descs, FastDiv tiles_y,
                   int ov_w_max) {
    extern __shared__ __attribute__((aligned(16))) uint32_t orow[];  // [VBR][orow_stride(ov_w_max)] (+ 256 divisors)
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int im = (int)fdiv(b, tiles_y);
    const int ty = (int)(b - (uint32_t)im * tiles_y.d);
    vblend_block<MAGIC>(orow, tmp, bg, dst, coefs, descs, im, ty, ov_w_max);
}

template <int NR, bool ZONES, int CN>
void launch_hpass(int n, int ty, hipStream_t s, const uint8_t* src, uint8_t* tmp, const int32_t* coefs,
                  const ipp_pipe_desc* descs, const ipp_hsv_params& hp, const uint8_t* bg, uint8_t* dst) {
    // H pass + the background outside the overlays, per group of kCopyGroup items
    const int64_t groups = (n + kCopyGroup - 1) / kCopyGroup;
    const uint32_t per_grp = (uint32_t)(kCopyGroup * ty + kCopySlabs);
    hipLaunchKernelGGL((k_pipe_hpass2<NR, ZONES, CN>), dim3((uint32_t)(groups * per_grp)), dim3(64 * HP_NW), 0, s,
                       src, tmp, coefs, descs, n, fast_div((uint32_t)ty), fast_div(per_grp), hp, bg, dst);
}

template <int NR>
void launch_hpass_nr(bool zones, int cn, int n, int ty, hipStream_t s, const uint8_t* src, uint8_t* tmp,
                     const int32_t* coefs, const ipp_pipe_desc* descs, const ipp_hsv_params& hp, const uint8_t* bg,
                     uint8_t* dst) {
    if (zones) {
        if (cn == 4) launch_hpass<NR, true, 4>(n, ty, s, src, tmp, coefs, descs, hp, bg, dst);
        else launch_hpass<NR, true, 3>(n, ty, s, src, tmp, coefs, descs, hp, bg, dst);
    } else {
        if (cn == 4) launch_hpass<NR, false, 4>(n, ty, s, src, tmp, coefs, descs, hp, bg, dst);
        else launch_hpass<NR, false, 3>(n, ty, s, src, tmp, coefs, descs, hp, bg, dst);
    }
}

}  // namespace

extern "C" int ipp_pipe_hpass_bgcopy(const uint8_t* src, uint8_t* tmp, const int32_t* coefs,
                                     const ipp_pipe_desc* descs, int32_t n_images, int32_t max_out_w,
                                     int32_t max_rows, int32_t src_cn, const ipp_hsv_params* hsv,
                                     int32_t tap_format, const uint8_t* bg, uint8_t* dst, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !tmp || !coefs || !descs || !hsv || !bg || !dst || n_images < 0 || max_out_w <= 0 || max_rows <= 0)
        return IPP_E_ARG;
    if (src_cn != 3 && src_cn != 4) return IPP_E_ARG;
    if (tap_format != IPP_TAPS_MFMA) return IPP_E_ARG;
    const int ty = (max_rows + HR - 1) / HR;  // one block per 16-row band
    if ((int64_t)(kCopyGroup * ty + kCopySlabs) * ((n_images + kCopyGroup - 1) / kCopyGroup) >= INT32_MAX)
        return IPP_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    // Zones are needed unless every range's zone is the whole image (all
    // margins 0).  The source channel count is uniform over the batch.
    bool zones = false;
    for (int k = 0; k < hsv->n_ranges; ++k)
        for (int m = 0; m < 4; ++m) zones |= hsv->r[k].zone[m] != 0;
    const int cn = src_cn, n = n_images;
    // A range that never matches: lo_v = 1 > hi_v = 0 (cv::inRange's empty range).
    const ipp_hsv_range never = ipp_hsv_range{{0, 0, 1}, {180, 255, 0}, {0, 0, 0, 0}};
    switch (hsv->n_ranges) {
        case 1: launch_hpass_nr<1>(zones, cn, n, ty, s, src, tmp, coefs, descs, *hsv, bg, dst); break;
        case 2: launch_hpass_nr<2>(zones, cn, n, ty, s, src, tmp, coefs, descs, *hsv, bg, dst); break;
        case 3: launch_hpass_nr<3>(zones, cn, n, ty, s, src, tmp, coefs, descs, *hsv, bg, dst); break;
        case 4: launch_hpass_nr<4>(zones, cn, n, ty, s, src, tmp, coefs, descs, *hsv, bg, dst); break;
        case 5: case 6: {
            ipp_hsv_params q = *hsv;  // pad with never-matching ranges (lo > hi in v)
            for (int k = q.n_ranges; k < 6; ++k) q.r[k] = never;
            launch_hpass_nr<6>(zones, cn, n, ty, s, src, tmp, coefs, descs, q, bg, dst);
            break;
        }
        default: {
            if (hsv->n_ranges > IPP_MAX_HSV_RANGES) return IPP_E_ARG;
            ipp_hsv_params q = *hsv;
            for (int k = q.n_ranges; k < IPP_MAX_HSV_RANGES; ++k) q.r[k] = never;
            launch_hpass_nr<IPP_MAX_HSV_RANGES>(zones, cn, n, ty, s, src, tmp, coefs, descs, q, bg, dst);
            break;
        }
    }
    IPP_CHECK_LAUNCH();
    return IPP_OK;
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
    if (tap_format != IPP_TAPS_MFMA || max_ov_w <= 0 || max_ov_w > bg_w || max_ov_h <= 0 || max_ov_h > bg_h ||
        max_ov_w > IPP_PIPE_MAX_OV_W)
        return IPP_E_ARG;
    const size_t rows = (size_t)VBR * orow_stride(max_ov_w) * sizeof(uint32_t);
    const size_t magic = 256 * sizeof(uint32_t);  // the unpremultiply divisors, when they fit beside the rows
    const bool use_magic = rows + magic <= 64 * 1024;
    // an overlay of height H at any y spans at most ceil((15 + H) / 16) bands
    const int tyb = std::min((max_ov_h + 15 + VBR - 1) / VBR, (bg_h + VBR - 1) / VBR);
    const int64_t nb = (int64_t)tyb * n_images;
    if (nb >= INT32_MAX) return IPP_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    const FastDiv ftyb = fast_div((uint32_t)tyb);
    if (use_magic)
        hipLaunchKernelGGL(k_pipe_vblend_mfma<true>, dim3((uint32_t)nb), dim3(256), rows + magic, st, tmp, bg, dst,
                           coefs, descs, ftyb, max_ov_w);
    else
        hipLaunchKernelGGL(k_pipe_vblend_mfma<false>, dim3((uint32_t)nb), dim3(256), rows, st, tmp, bg, dst, coefs,
                           descs, ftyb, max_ov_w);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
