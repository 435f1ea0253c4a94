// ipp_ccl.hip — K10..K13: pixels_isolés.keep_largest_component.
//
// Reference: pixels_isolés.py:32 threshold(α, 1, 255, BINARY) → fg = α > 1;
// :35 connectedComponentsWithStats(fg, connectivity=8); :38-44 largest area,
// strict '>' so the lowest OpenCV label wins ties; :47-55 α := 0 outside it
// (when there is no foreground at all, label 0 — the background — is "kept"
// and α is left unchanged); :74-81 crop-fit to the bbox of α ≠ 0.
//
// Labels live in BLOCK-RASTER index space: pixel (x, y) ↦
//   L = ((y >> 1) * wb + (x >> 1)) * 4 + (y & 1) * 2 + (x & 1),  wb = ⌈w/2⌉.
// Union-find always links the larger index under the smaller, so a
// component's root is its minimum L, and root >> 2 is the first 2×2 scan block
// (in raster order of blocks) that touches it — the order in which OpenCV's
// block-based 8-connectivity labelling (Spaghetti/BBDT) numbers components.
// The tie rule is therefore "smallest root", restated (UNPINNED: OpenCV is
// absent here).  All four pixels of a 2×2 block are mutually 8-adjacent, so
// no two components share a block.
//
// Union: lock-free atomicMin linking (Playne–Hawick style); parents only
// decrease, so stale reads cost extra iterations, never a wrong answer.
#include "ipp_device.h"

namespace {

constexpr int CHUNK = 1024;  // index-space entries per block (4 per thread)

struct Geo {
    int w, h, wb, hb;
    int64_t size;  // 4 * wb * hb
};

__device__ __forceinline__ Geo geo_of(const ipp_image_desc& d) {
    Geo g;
    g.w = d.w;
    g.h = d.h;
    g.wb = (d.w + 1) >> 1;
    g.hb = (d.h + 1) >> 1;
    g.size = 4ll * g.wb * g.hb;
    return g;
}

__device__ __forceinline__ void decode(const Geo& g, int64_t L, int& x, int& y) {
    const int64_t blk = L >> 2;
    const int by = (int)(blk / g.wb), bx = (int)(blk - (int64_t)by * g.wb);
    x = 2 * bx + (int)(L & 1);
    y = 2 * by + (int)((L >> 1) & 1);
}

__device__ __forceinline__ int32_t encode(const Geo& g, int x, int y) {
    return (int32_t)((((int64_t)(y >> 1) * g.wb + (x >> 1)) << 2) + ((y & 1) << 1) + (x & 1));
}

__device__ __forceinline__ int32_t ld(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int32_t find_root(const int32_t* P, int32_t x) {
    int32_t p = ld(P + x);
    while (p != x) {
        x = p;
        p = ld(P + x);
    }
    return x;
}

__device__ __forceinline__ void unite(int32_t* P, int32_t a, int32_t b) {
    bool done;
    do {
        a = find_root(P, a);
        b = find_root(P, b);
        if (a < b) {
            const int32_t old = atomicMin(P + b, a);
            done = (old == b);
            b = old;
        } else if (b < a) {
            const int32_t old = atomicMin(P + a, b);
            done = (old == a);
            a = old;
        } else {
            done = true;
        }
    } while (!done);
}

struct Block {
    int im;
    int64_t base;
};

__device__ __forceinline__ Block block_of(int chunks_per_img) {
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    Block r;
    r.im = (int)(b / chunks_per_img);
    r.base = (int64_t)(b - (uint32_t)r.im * chunks_per_img) * CHUNK;
    return r;
}

__device__ __forceinline__ bool is_fg(const uint8_t* img, const ipp_image_desc& d, int x, int y) {
    return x < d.w && y < d.h && img[d.off + (int64_t)y * d.pitch + 4 * (int64_t)x + 3] > 1;
}

__global__ void __launch_bounds__(256)
k_ccl_init(const uint8_t* __restrict__ img, const ipp_image_desc* __restrict__ descs, int chunks,
           int32_t* __restrict__ labels, const int64_t* __restrict__ lab_off, uint32_t* __restrict__ area) {
    const Block bk = block_of(chunks);
    const ipp_image_desc d = descs[bk.im];
    const Geo g = geo_of(d);
    int32_t* P = labels + lab_off[bk.im];
    uint32_t* A = area + lab_off[bk.im];
    for (int k = 0; k < 4; ++k) {
        const int64_t L = bk.base + threadIdx.x + 256 * k;
        if (L >= g.size) break;
        int x, y;
        decode(g, L, x, y);
        P[L] = is_fg(img, d, x, y) ? (int32_t)L : -1;
        A[L] = 0u;
    }
}

__global__ void __launch_bounds__(256)
k_ccl_merge(const ipp_image_desc* __restrict__ descs, int chunks, int32_t* __restrict__ labels,
            const int64_t* __restrict__ lab_off) {
    const Block bk = block_of(chunks);
    const ipp_image_desc d = descs[bk.im];
    const Geo g = geo_of(d);
    int32_t* P = labels + lab_off[bk.im];
    for (int k = 0; k < 4; ++k) {
        const int64_t L = bk.base + threadIdx.x + 256 * k;
        if (L >= g.size) break;
        if (ld(P + L) < 0) continue;
        int x, y;
        decode(g, L, x, y);
        // 8-connectivity: left, up-left, up, up-right (each pair once)
        const int nx[4] = {x - 1, x - 1, x, x + 1};
        const int ny[4] = {y, y - 1, y - 1, y - 1};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (nx[j] < 0 || ny[j] < 0 || nx[j] >= g.w) continue;
            const int32_t q = encode(g, nx[j], ny[j]);
            if (ld(P + q) >= 0) unite(P, (int32_t)L, q);
        }
    }
}

__global__ void __launch_bounds__(256)
k_ccl_flatten_area(const ipp_image_desc* __restrict__ descs, int chunks, int32_t* __restrict__ labels,
                   const int64_t* __restrict__ lab_off, uint32_t* __restrict__ area) {
    const Block bk = block_of(chunks);
    const ipp_image_desc d = descs[bk.im];
    const Geo g = geo_of(d);
    int32_t* P = labels + lab_off[bk.im];
    uint32_t* A = area + lab_off[bk.im];
    for (int k = 0; k < 4; ++k) {
        const int64_t L = bk.base + threadIdx.x + 256 * k;
        int32_t root = -1;
        if (L < g.size && P[L] >= 0) {
            root = find_root(P, (int32_t)L);
            P[L] = root;
        }
        // wave-aggregated area histogram: one atomic per distinct root per wave
        uint64_t pending = __ballot(root >= 0);
        while (pending) {
            const int leader = __ffsll((unsigned long long)pending) - 1;
            const int32_t r = __shfl(root, leader);
            const uint64_t same = __ballot(root == r) & pending;
            if ((int)(threadIdx.x & 63) == leader) atomicAdd(A + r, (uint32_t)__popcll(same));
            pending &= ~same;
        }
    }
}

__global__ void __launch_bounds__(256)
k_ccl_best(const ipp_image_desc* __restrict__ descs, int chunks, const int32_t* __restrict__ labels,
           const int64_t* __restrict__ lab_off, const uint32_t* __restrict__ area,
           unsigned long long* __restrict__ best) {
    const Block bk = block_of(chunks);
    const ipp_image_desc d = descs[bk.im];
    const Geo g = geo_of(d);
    const int32_t* P = labels + lab_off[bk.im];
    const uint32_t* A = area + lab_off[bk.im];
    unsigned long long key = 0ull;
    for (int k = 0; k < 4; ++k) {
        const int64_t L = bk.base + threadIdx.x + 256 * k;
        if (L < g.size && P[L] == (int32_t)L) {
            const unsigned long long kk =
                ((unsigned long long)A[L] << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)L);
            key = kk > key ? kk : key;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(key, off);
        key = o > key ? o : key;
    }
    if ((threadIdx.x & 63) == 0 && key) atomicMax(best + bk.im, key);
}

__global__ void __launch_bounds__(256)
k_ccl_apply(uint8_t* __restrict__ img, const ipp_image_desc* __restrict__ descs, int chunks,
            const int32_t* __restrict__ labels, const int64_t* __restrict__ lab_off,
            const unsigned long long* __restrict__ best, int32_t* __restrict__ bbox) {
    const Block bk = block_of(chunks);
    const ipp_image_desc d = descs[bk.im];
    const Geo g = geo_of(d);
    const int32_t* P = labels + lab_off[bk.im];
    const unsigned long long bkey = best[bk.im];
    const int32_t broot = (int32_t)(0xFFFFFFFFu - (uint32_t)(bkey & 0xFFFFFFFFull));
    int xmin = INT32_MAX, ymin = INT32_MAX, xmax = -1, ymax = -1;
    for (int k = 0; k < 4; ++k) {
        const int64_t L = bk.base + threadIdx.x + 256 * k;
        if (L >= g.size) break;
        int x, y;
        decode(g, L, x, y);
        if (x >= g.w || y >= g.h) continue;
        uint8_t* a = img + d.off + (int64_t)y * d.pitch + 4 * (int64_t)x + 3;
        uint8_t av = *a;
        if (bkey != 0ull && P[L] != broot && av != 0) {
            av = 0;
            *a = 0;
        }
        if (av != 0) {
            xmin = min(xmin, x);
            xmax = max(xmax, x);
            ymin = min(ymin, y);
            ymax = max(ymax, y);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        xmin = min(xmin, __shfl_xor(xmin, off));
        ymin = min(ymin, __shfl_xor(ymin, off));
        xmax = max(xmax, __shfl_xor(xmax, off));
        ymax = max(ymax, __shfl_xor(ymax, off));
    }
    if ((threadIdx.x & 63) == 0 && xmax >= 0) {
        atomicMin(&bbox[4 * bk.im + 0], xmin);
        atomicMin(&bbox[4 * bk.im + 1], ymin);
        atomicMax(&bbox[4 * bk.im + 2], xmax + 1);
        atomicMax(&bbox[4 * bk.im + 3], ymax + 1);
    }
}

__global__ void k_ccl_prep(int32_t* bbox, unsigned long long* best, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        bbox[4 * i + 0] = INT32_MAX;
        bbox[4 * i + 1] = INT32_MAX;
        bbox[4 * i + 2] = -1;
        bbox[4 * i + 3] = -1;
        best[i] = 0ull;
    }
}

__global__ void k_ccl_finish(int32_t* bbox, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && bbox[4 * i + 2] < 0) bbox[4 * i + 0] = bbox[4 * i + 1] = -1;
}

}  // namespace

// stats: caller scratch of n_images 64-bit words (best key per image:
// area << 32 | ~root); labels/area: int32/uint32 scratch of
// 4*ceil(w/2)*ceil(h/2) entries per image starting at lab_off[i].
extern "C" int ipp_ccl_keep_largest(uint8_t* img, const ipp_image_desc* descs, int32_t n_images, int32_t max_w,
                                    int32_t max_h, int32_t* labels, const int64_t* lab_off, uint32_t* area,
                                    int64_t* stats, int32_t* bbox, void* stream) {
    if (n_images == 0) return IPP_OK;
    if (!img || !descs || !labels || !lab_off || !area || !stats || !bbox || n_images < 0 || max_w <= 0 ||
        max_h <= 0)
        return IPP_E_ARG;
    const int64_t size = 4ll * ((max_w + 1) / 2) * ((max_h + 1) / 2);
    if (size >= INT32_MAX) return IPP_E_RANGE;
    const int chunks = (int)((size + CHUNK - 1) / CHUNK);
    const int64_t blocks = (int64_t)chunks * n_images;
    if (blocks >= INT32_MAX) return IPP_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    unsigned long long* best = reinterpret_cast<unsigned long long*>(stats);
    const int nb = (n_images + 255) / 256;
    const dim3 grid((uint32_t)blocks), blk(256);
    hipLaunchKernelGGL(k_ccl_prep, dim3(nb), blk, 0, s, bbox, best, n_images);
    hipLaunchKernelGGL(k_ccl_init, grid, blk, 0, s, img, descs, chunks, labels, lab_off, area);
    hipLaunchKernelGGL(k_ccl_merge, grid, blk, 0, s, descs, chunks, labels, lab_off);
    hipLaunchKernelGGL(k_ccl_flatten_area, grid, blk, 0, s, descs, chunks, labels, lab_off, area);
    hipLaunchKernelGGL(k_ccl_best, grid, blk, 0, s, descs, chunks, labels, lab_off, area, best);
    hipLaunchKernelGGL(k_ccl_apply, grid, blk, 0, s, img, descs, chunks, labels, lab_off, best, bbox);
    hipLaunchKernelGGL(k_ccl_finish, dim3(nb), blk, 0, s, bbox, n_images);
    IPP_CHECK_LAUNCH();
    return IPP_OK;
}
