// ipp_gather.hip — K1..K5: margin crop → RGBA → NEAREST rotate (expand) →
// alpha-bbox crop → flip, as ONE gather per output pixel; plus the plain
// window copy/flip and the alpha bounding-box reduction.
//
// Reference call sites: recadrages.py:46 (slice), rotations.py:55 (convert
// RGBA), :96 (rotate, NEAREST, expand), :99-101 (getbbox/crop),
// symmetry.py:114-119 (cv2.flip 1/0/-1), pixels_isolés.py:77-81 (crop-fit).
// Library arithmetic reproduced: Pillow Geometry.c affine_fixed (16.16 int32
// accumulation, arithmetic >> 16, out-of-range → zero pixel).
//
// Layout: each thread owns 4 horizontally adjacent output pixels (16 bytes of
// RGBA) so a wave stores 1 KiB with dwordx4 stores; a 256-thread block covers a
// 64×16 output tile.  Blocks are remapped so the tiles of one image share an
// XCD (its source stays in that XCD's L2).
#include "ipp_device.h"
#include "ipp_sampler.h"

namespace {

constexpr int TILE_W = 64, TILE_H = 16, PX_PER_THREAD = 4;
constexpr int STAGE_W = 72;  // words per restaged row (dense map)

struct TileGrid {
    int tiles_x, tiles_y;
};

// One column of RT 64×16 output tiles per block (64 × 16·RT pixels),
// branch-free gathers, all RT tiles' loads issued before the first is used
// (RT gathers in flight per thread).  Two lane maps:
//   PATCH: wave w gathers the 16×16 patch at columns 16w.. (lane: row lane>>2,
//          4 pixels at 4·(lane&3)) — each load instruction's addresses fall in
//          a compact source patch — then each tile is restaged through LDS so
//          every wave stores 4 full rows (256 B per row per instruction);
//   ROWS:  wave w covers rows 4w..4w+3 directly (16 lanes × 4 pixels per row).
// Tiles per block: 1 / 2 / 4 measured 2.87 / 2.84 / 3.07 ms for config 2
// (round 4, nontemporal stores).
// Tiles per block 2 / 3 / 4 / 5: 2.44 / 2.41 / 2.42 / 2.45 ms for config 2
// (round 6, one box, profiles/r06/ab_rotflip_rt_r06o.txt).  A map without
// the LDS restage — wave w the 8 rows × 32 columns at (8(w>>1), 32(w&1)),
// 4 adjacent pixels per lane stored directly — measured 2.52 (r06n).
#ifndef IPP_ROT_RT
#define IPP_ROT_RT 3
#endif
constexpr int RT = IPP_ROT_RT;  // tiles per block (rows of 16)

template <int CN, bool PATCH, bool DENSE = false>
__device__ __forceinline__ void rotate_tiles(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                             const ipp_gather_desc& d, int tx, int tyb, uint4* stage) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int gy, gx;  // gathered pixel block (row, first column) of this thread within a tile
    if (DENSE) {  // pixels (gy, gx), (gy, gx + 8), (gy + 8, gx), (gy + 8, gx + 8)
        gy = lane >> 3;
        gx = 16 * wave + (lane & 7);
    } else if (PATCH) {
        gy = lane >> 2;
        gx = 16 * wave + 4 * (lane & 3);
    } else {
        gy = (int)(threadIdx.x >> 4);
        gx = 4 * (int)(threadIdx.x & 15);
    }
    const int ty0 = tyb * RT;
    if (ty0 * TILE_H >= d.out_h || tx * TILE_W >= d.out_w) return;  // block-uniform
    const int nt = min(RT, (d.out_h - ty0 * TILE_H + TILE_H - 1) / TILE_H);
    const Sampler S = make_sampler(src, d);
    const int x0 = tx * TILE_W + gx;
    Gather4<CN> G[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) {
        if (r < nt) {
            const int y = (ty0 + r) * TILE_H + gy;
            const uint32_t xx = (uint32_t)S.b2 + (uint32_t)y * (uint32_t)S.b1 + (uint32_t)x0 * (uint32_t)S.b0;
            const uint32_t yy = (uint32_t)S.b5 + (uint32_t)y * (uint32_t)S.b4 + (uint32_t)x0 * (uint32_t)S.b3;
            if (DENSE) gather4_issue_sq8<CN>(S, xx, yy, G[r]);
            else gather4_issue<CN>(S, xx, yy, G[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < RT; ++r) {
        if (r >= nt) break;  // block-uniform
        uint4 px;
        px.x = gather4_pixel<CN>(G[r], 0);
        px.y = gather4_pixel<CN>(G[r], 1);
        px.z = gather4_pixel<CN>(G[r], 2);
        px.w = gather4_pixel<CN>(G[r], 3);
        int sy = (ty0 + r) * TILE_H + gy, sx0 = x0;
        if (DENSE) {  // restage pixel by pixel: store pattern = ROWS map
            if (r > 0) __syncthreads();
            // rows STAGE_W words apart: the 4 rows × 8 columns of a half-wave's
            // dword writes land on 32 distinct banks (64 words: 4-way conflicts)
            uint32_t* st32 = reinterpret_cast<uint32_t*>(stage);
            st32[gy * STAGE_W + gx] = px.x;
            st32[gy * STAGE_W + gx + 8] = px.y;
            st32[(gy + 8) * STAGE_W + gx] = px.z;
            st32[(gy + 8) * STAGE_W + gx + 8] = px.w;
            __syncthreads();
            const int ry = (int)(threadIdx.x >> 4), rx = 4 * (int)(threadIdx.x & 15);
            px = stage[ry * (STAGE_W / 4) + (rx >> 2)];
            sy = (ty0 + r) * TILE_H + ry;
            sx0 = tx * TILE_W + rx;
        } else if (PATCH) {  // restage: store pattern = ROWS map
            if (r > 0) __syncthreads();  // previous tile's stage reads done
            stage[gy * 16 + (gx >> 2)] = px;
            __syncthreads();
            const int ry = (int)(threadIdx.x >> 4), rx = 4 * (int)(threadIdx.x & 15);
            px = stage[ry * 16 + (rx >> 2)];
            sy = (ty0 + r) * TILE_H + ry;
            sx0 = tx * TILE_W + rx;
        }
        if (sy >= d.out_h || sx0 >= d.out_w) continue;
        uint8_t* o = dst + d.dst_off + (int64_t)sy * d.dst_pitch + 4 * sx0;
        if (sx0 + 4 <= d.out_w && ((reinterpret_cast<uintptr_t>(o) & 15u) == 0)) {
            // streaming (nontemporal) store: the output is not re-read here, and
            // plain stores that allocate in L2 cost 25 % (3.55 vs 2.84 ms)
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(v4u{px.x, px.y, px.z, px.w}, reinterpret_cast<v4u*>(o));
        } else {
            const uint32_t pv[4] = {px.x, px.y, px.z, px.w};
            for (int k = 0; k < 4; ++k)
                if (sx0 + k < d.out_w) reinterpret_cast<uint32_t*>(o)[k] = pv[k];
        }
    }
}

// (the block index split by FastDiv: the two runtime divisions were ~60 of
// the kernel's ~350 scalar instructions)
template <bool PATCH, bool DENSE = false>
__global__ void __launch_bounds__(256)
k_rotate_flip_nearest(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                      const ipp_gather_desc* __restrict__ descs, FastDiv per_img, FastDiv tiles_x) {
    __shared__ uint4 stage[PATCH || DENSE ? TILE_H * (STAGE_W / 4) : 1];
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int img = (int)fdiv(b, per_img);
    const int t = (int)(b - (uint32_t)img * per_img.d);
    const int ty = (int)fdiv((uint32_t)t, tiles_x), tx = t - ty * (int)tiles_x.d;
    const ipp_gather_desc d = descs[img];
    if (d.src_cn == 4) rotate_tiles<4, PATCH, DENSE>(src, dst, d, tx, ty, stage);  // block-uniform
    else rotate_tiles<3, PATCH, DENSE>(src, dst, d, tx, ty, stage);
}

// Window copy with optional mirror, any bytes-per-pixel (1..4).  Each thread
// owns 16 bytes of one output row (a block covers 4 rows × 1 KiB): rows that
// are not mirrored in x are contiguous byte runs, copied with 4 unaligned
// dword loads and one 16-B store; mirrored rows take a per-byte path.  With
// FROM_BBOX the window is read from a device bbox array (x0, y0, x1, y1) per
// image — the crop-fit of pixels_isolés.py:74-81 without a host round trip;
// an empty bbox (x0 < 0) copies nothing.
template <bool FROM_BBOX>
__global__ void __launch_bounds__(256)
k_copy_rows(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, const ipp_copy_desc* __restrict__ descs,
            const int32_t* __restrict__ bbox, int tiles_x, int tiles_y) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int per_img = tiles_x * tiles_y;
    const int img = b / per_img;
    const int t = b - img * per_img;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const ipp_copy_desc d = descs[img];
    int x0 = d.x0, y0 = d.y0, w = d.w, h = d.h;
    if (FROM_BBOX) {
        x0 = bbox[4 * img + 0];
        y0 = bbox[4 * img + 1];
        w = bbox[4 * img + 2] - x0;
        h = bbox[4 * img + 3] - y0;
        if (x0 < 0) return;
    }
    const int y = ty * 4 + (int)(threadIdx.x >> 6);
    const int c0 = (tx * 64 + (int)(threadIdx.x & 63)) * 16;
    const int row_bytes = w * d.cn;
    if (y >= h || c0 >= row_bytes) return;
    const int sy = y0 + ((d.flip & 2) ? h - 1 - y : y);
    const uint8_t* s = src + d.src_off + (int64_t)sy * d.src_pitch + (int64_t)x0 * d.cn;
    uint8_t* o = dst + d.dst_off + (int64_t)y * d.dst_pitch + c0;
    const int n = min(16, row_bytes - c0);
    uint32_t wv[4] = {0u, 0u, 0u, 0u};
    if (!(d.flip & 1)) {
        if (n == 16) {
#pragma unroll
            for (int k = 0; k < 4; ++k) wv[k] = ld_u32_unaligned(s + c0 + 4 * k);
        } else {
            for (int j = 0; j < n; ++j) wv[j >> 2] |= (uint32_t)s[c0 + j] << (8 * (j & 3));
        }
    } else {
        for (int j = 0; j < n; ++j) {
            const int bi = c0 + j, px = bi / d.cn, ch = bi - px * d.cn;
            wv[j >> 2] |= (uint32_t)s[(int64_t)(w - 1 - px) * d.cn + ch] << (8 * (j & 3));
        }
    }
    const bool vec = n == 16 && (reinterpret_cast<uintptr_t>(o) & 15u) == 0;
    store16(o, n, vec, wv);
}

// Bounding box of non-zero pixels (Pillow getbbox(alpha_only=True): the alpha
// band for LA/RGBA, any band otherwise; also cv2.findNonZero+boundingRect on
// an alpha plane): per block min/max over its tile with wave reductions, then
// four device-scope atomics.  bbox is pre-set to (INT_MAX, INT_MAX, -1, -1).
__global__ void __launch_bounds__(256)
k_alpha_bbox(const uint8_t* __restrict__ img, const ipp_image_desc* __restrict__ descs,
             int tiles_x, int tiles_y, int32_t* __restrict__ bbox) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int per_img = tiles_x * tiles_y;
    const int im = b / per_img;
    const int t = b - im * per_img;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const ipp_image_desc d = descs[im];
    const int y = ty * TILE_H + (int)(threadIdx.x >> 4);
    const int x0 = tx * TILE_W + (int)(threadIdx.x & 15) * PX_PER_THREAD;
    int xmin = INT32_MAX, ymin = INT32_MAX, xmax = -1, ymax = -1;
    if (y < d.h) {
        const uint8_t* row = img + d.off + (int64_t)y * d.pitch;
        for (int k = 0; k < PX_PER_THREAD; ++k) {
            const int x = x0 + k;
            bool nz = false;
            if (x < d.w) {
                const uint8_t* px = row + (int64_t)x * d.cn;
                if (d.cn == 2 || d.cn == 4) {
                    nz = px[d.cn - 1] != 0;  // alpha band (Pillow getbbox alpha_only)
                } else {
                    for (int c = 0; c < d.cn; ++c) nz |= px[c] != 0;  // any band non-zero
                }
            }
            if (nz) {
                xmin = min(xmin, x);
                xmax = max(xmax, x);
                ymin = min(ymin, y);
                ymax = max(ymax, y);
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        xmin = min(xmin, __shfl_xor(xmin, off));
        ymin = min(ymin, __shfl_xor(ymin, off));
        xmax = max(xmax, __shfl_xor(xmax, off));
        ymax = max(ymax, __shfl_xor(ymax, off));
    }
    if ((threadIdx.x & 63) == 0 && xmax >= 0) {
        atomicMin(&bbox[4 * im + 0], xmin);
        atomicMin(&bbox[4 * im + 1], ymin);
        atomicMax(&bbox[4 * im + 2], xmax + 1);
        atomicMax(&bbox[4 * im + 3], ymax + 1);
    }
}

__global__ void k_bbox_init(int32_t* bbox, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        bbox[4 * i + 0] = INT32_MAX;
        bbox[4 * i + 1] = INT32_MAX;
        bbox[4 * i + 2] = -1;
        bbox[4 * i + 3] = -1;
    }
}

__global__ void k_bbox_finish(int32_t* bbox, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && bbox[4 * i + 2] < 0) {
        bbox[4 * i + 0] = bbox[4 * i + 1] = -1;
    }
}

inline bool grid_ok(int64_t blocks) { return blocks > 0 && blocks < (int64_t)INT32_MAX; }

}  // namespace

extern "C" int ipp_rotate_flip_nearest(const uint8_t* src, uint8_t* dst, const ipp_gather_desc* descs,
                                       int32_t n_images, int32_t max_out_w, int32_t max_out_h,
                                       void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !dst || !descs || n_images < 0 || max_out_w <= 0 || max_out_h <= 0) return IPP_E_ARG;
    const int tx = (max_out_w + TILE_W - 1) / TILE_W, ty = (max_out_h + TILE_H * RT - 1) / (TILE_H * RT);
    const int64_t blocks = (int64_t)tx * ty * n_images;
    if (!grid_ok(blocks)) return IPP_E_ARG;
    // the dense 8×8 gather map with the LDS restage (the row map and the
    // 16×16-patch map of rounds 1-2 measured slower)
    hipLaunchKernelGGL((k_rotate_flip_nearest<false, true>), dim3((uint32_t)blocks), dim3(256), 0,
                       (hipStream_t)stream, src, dst, descs, fast_div((uint32_t)(tx * ty)), fast_div((uint32_t)tx));
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_copy_window(const uint8_t* src, uint8_t* dst, const ipp_copy_desc* descs, int32_t n_images,
                               int32_t max_w, int32_t max_h, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !dst || !descs || n_images < 0 || max_w <= 0 || max_h <= 0) return IPP_E_ARG;
    // max_w is in pixels; size the grid for 4 bytes per pixel (threads past a
    // row's bytes exit)
    const int tx = (max_w * 4 + 1023) / 1024, ty = (max_h + 3) / 4;
    const int64_t blocks = (int64_t)tx * ty * n_images;
    if (!grid_ok(blocks)) return IPP_E_ARG;
    hipLaunchKernelGGL(k_copy_rows<false>, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, src, dst,
                       descs, nullptr, tx, ty);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_crop_to_bbox(const uint8_t* src, uint8_t* dst, const ipp_copy_desc* descs, const int32_t* bbox,
                                int32_t n_images, int32_t max_w, int32_t max_h, int32_t cn, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!src || !dst || !descs || !bbox || n_images < 0 || max_w <= 0 || max_h <= 0 || cn < 1 || cn > 4)
        return IPP_E_ARG;
    const int tx = (max_w * cn + 1023) / 1024, ty = (max_h + 3) / 4;
    const int64_t blocks = (int64_t)tx * ty * n_images;
    if (!grid_ok(blocks)) return IPP_E_ARG;
    hipLaunchKernelGGL(k_copy_rows<true>, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, src, dst, descs,
                       bbox, tx, ty);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}

extern "C" int ipp_alpha_bbox(const uint8_t* img, const ipp_image_desc* descs, int32_t n_images, int32_t max_w,
                              int32_t max_h, int32_t* bbox, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!img || !descs || !bbox || n_images < 0 || max_w <= 0 || max_h <= 0) return IPP_E_ARG;
    const int tx = (max_w + TILE_W - 1) / TILE_W, ty = (max_h + TILE_H - 1) / TILE_H;
    const int64_t blocks = (int64_t)tx * ty * n_images;
    if (!grid_ok(blocks)) return IPP_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    const int nb = (n_images + 255) / 256;
    hipLaunchKernelGGL(k_bbox_init, dim3(nb), dim3(256), 0, s, bbox, n_images);
    hipLaunchKernelGGL(k_alpha_bbox, dim3((uint32_t)blocks), dim3(256), 0, s, img, descs, tx, ty, bbox);
    hipLaunchKernelGGL(k_bbox_finish, dim3(nb), dim3(256), 0, s, bbox, n_images);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
