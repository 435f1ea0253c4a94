/*
 * ipp.h — C ABI of the MI355X-native image_processor_pipeline hot path.
 *
 * The reference (Tezahc/image_processor_pipeline) is pure Python: its pixel
 * arithmetic lives in Pillow's and OpenCV's C routines, called from the
 * transforms plugins.  Each entry point below replaces one of those library
 * calls (or a fused chain of them); the reference call site it stands in for
 * is cited on each declaration.  The Python host layer
 * (image_processor_pipeline_amd/) keeps the reference's plugin signatures and
 * binds these symbols with ctypes.
 *
 * Conventions
 *   - Images are HWC uint8 in caller-owned DEVICE memory; every pointer is a
 *     device pointer, every size is in bytes/pixels as named.
 *   - Batched calls take a DEVICE array of per-image descriptors, so one launch
 *     covers a ragged batch.  Nothing here allocates persistent memory: scratch
 *     is caller-provided.  All calls are asynchronous and stream-ordered on the
 *     given hipStream_t (passed as void*), reentrant, and graph-capturable.
 *   - Return value: 0 on success, a negative IPP_E* code otherwise (the Python
 *     wrappers map codes to the exceptions the reference raises).
 *   - Host-side planning helpers (ipp_plan_*) run on the CPU and fill
 *     descriptors / tap tables; they reproduce the library's host arithmetic
 *     bit-for-bit (double precision, same libm).
 */
#ifndef IPP_H
#define IPP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IPP_OK 0
#define IPP_E_ARG (-1)      /* invalid argument (null pointer, bad size)      */
#define IPP_E_LAUNCH (-2)   /* HIP launch / runtime error                     */
#define IPP_E_RANGE (-3)    /* geometry outside the supported fixed-point range */

#define IPP_MAX_HSV_RANGES 16

/* ------------------------------------------------------------------------ */
/* K1+K2+K3+K4+K5: crop → RGBA → NEAREST rotate (expand) → bbox crop → flip  */
/* ------------------------------------------------------------------------ */
/* One image of the ragged batch.  The rotated canvas pixel (X, Y) reads
 *   xin = (a2 + Y*a1 + X*a0) >> 16,  yin = (a5 + Y*a4 + X*a3) >> 16
 * (int32 arithmetic, exactly Pillow Geometry.c affine_fixed) from the crop
 * window [in_x0, in_x0+in_w) × [in_y0, in_y0+in_h) of the source, or writes
 * (0,0,0,0) when (xin, yin) falls outside it.  Output pixel (x, y) is canvas
 * pixel (off_x + fx, off_y + fy) with fx = flip&1 ? out_w-1-x : x and
 * fy = flip&2 ? out_h-1-y : y.  Pillow's 0/90/180/270 fast paths are encoded
 * with exact integer coefficients by ipp_plan_rotate.                        */
typedef struct ipp_gather_desc {
    int64_t src_off;   /* byte offset of this image's source in src         */
    int64_t dst_off;   /* byte offset of this image's output in dst         */
    int32_t src_pitch; /* bytes per source row                              */
    int32_t src_cn;    /* source channels: 3 (RGB) or 4 (RGBA)              */
    int32_t src_w, src_h; /* full source dims (bounds the wide loads)       */
    int32_t in_x0, in_y0, in_w, in_h; /* crop window = image seen by rotate */
    int32_t a0, a1, a2, a3, a4, a5;   /* 16.16 inverse affine               */
    int32_t out_w, out_h;             /* output dims (after the bbox crop)  */
    int32_t off_x, off_y;             /* bbox origin inside the canvas      */
    int32_t flip;                     /* bit0: mirror x ('h'), bit1: mirror y ('v') */
    int32_t dst_pitch;                /* bytes per output row (≥ 4*out_w)   */
    /* The sampler of the fields above, filled by ipp_gather_prepare
     * (prepared = 1) so that every block of the gather kernels reads it
     * instead of recomputing it; with prepared = 0 the kernels compute it. */
    int64_t base_off;                 /* src_off + in_y0*src_pitch + in_x0*src_cn */
    uint32_t lim;                     /* last byte offset from base where a 4-byte load fits */
    int32_t b[6];                     /* 16.16 map with the flip and bbox origin folded in:
                                         x_src = b2 + y*b1 + x*b0, y_src = b5 + y*b4 + x*b3 */
    int32_t prepared;
} ipp_gather_desc;

/* Fills the sampler fields of n host-side descriptors (same arithmetic as
 * the kernels' own, 32-bit wrap-around). */
int ipp_gather_prepare(ipp_gather_desc* descs, int32_t n);

/* rotations.py:55 convert('RGBA') + :96 rotate(angle, expand=True) + :99-101
 * getbbox()/crop(), recadrages.py:46 margin crop, symmetry.py:114-119 flip —
 * fused gather.  Writes RGBA. */
int ipp_rotate_flip_nearest(const uint8_t* src, uint8_t* dst,
                            const ipp_gather_desc* descs, int32_t n_images,
                            int32_t max_out_w, int32_t max_out_h, void* stream);

/* Opt-in BILINEAR rotation: Pillow rotate(angle, expand=True,
 * resample=BILINEAR) of an RGB/RGBA source through RGBa (PIL/Image.py:2978-
 * 2983, Geometry.c affine_transform + bilinear_filter32RGB).  The
 * reference's rotations.py:96 is NEAREST; north_star asks for "rotations.py
 * (bilinear)" — process_rotations(..., resample="bilinear").  Output: the
 * full RGBA canvas (out_w × out_h = the expanded size) with the flip bits
 * folded into the write (bit0 mirror x, bit1 mirror y); the caller crops it
 * to its alpha bbox (ipp_alpha_bbox + ipp_copy_window).  m = Pillow's double
 * inverse matrix. */
typedef struct ipp_affine_desc {
    int64_t src_off, dst_off;
    int32_t src_pitch, src_cn;        /* cn 3 (α = 255) or 4 (RGBA)          */
    int32_t in_x0, in_y0, in_w, in_h; /* source window seen by rotate        */
    int32_t out_w, out_h, dst_pitch;  /* canvas; dst_pitch multiple of 4     */
    int32_t flip;
    double m[6];
} ipp_affine_desc;

int ipp_rotate_bilinear(const uint8_t* src, uint8_t* dst, const ipp_affine_desc* descs,
                        int32_t n_images, int32_t max_out_w, int32_t max_out_h, void* stream);

/* ------------------------------------------------------------------------ */
/* Plain 2-D window copy / flip (recadrages.py:46 slice, crop_square.py:196  */
/* slice, symmetry.py:114-119 cv2.flip codes 1/0/-1, pixels_isolés.py:81).   */
/* ------------------------------------------------------------------------ */
typedef struct ipp_copy_desc {
    int64_t src_off, dst_off;
    int32_t src_pitch, dst_pitch;
    int32_t x0, y0, w, h;   /* window in the source (pixels)               */
    int32_t cn;             /* bytes per pixel (1..4)                       */
    int32_t flip;           /* bit0 mirror x, bit1 mirror y                 */
} ipp_copy_desc;

int ipp_copy_window(const uint8_t* src, uint8_t* dst, const ipp_copy_desc* descs,
                    int32_t n_images, int32_t max_w, int32_t max_h, void* stream);

/* Crop-fit with the window taken from a DEVICE bbox array (x0, y0, x1, y1 per
 * image, as ipp_alpha_bbox / ipp_ccl_keep_largest write it) — the
 * pixels_isolés.py:74-81 `_crop_fit` slice without a host round trip.  The
 * descriptor's x0/y0/w/h are ignored; images whose bbox is empty (x0 < 0) are
 * not written.  max_w/max_h bound the windows (pixels); cn = bytes per pixel. */
int ipp_crop_to_bbox(const uint8_t* src, uint8_t* dst, const ipp_copy_desc* descs,
                     const int32_t* bbox, int32_t n_images, int32_t max_w, int32_t max_h,
                     int32_t cn, void* stream);

/* ------------------------------------------------------------------------ */
/* K6+K7: OpenCV BGR2HSV (8-bit) + inRange × R + zone AND + OR + NOT → alpha */
/* filtres_liste.py:84 imread(BGR) :90 cvtColor :97-123 inRange/zone/OR/NOT  */
/* :132-134 merge(b, g, r, alpha).                                           */
/* ------------------------------------------------------------------------ */
typedef struct ipp_hsv_range {
    int32_t lo[3], hi[3];   /* inRange bounds already prepared like cv::inRange
                               (cvRound'ed, saturated; empty → lo=1, hi=0)   */
    int32_t zone[4];        /* (top, bottom, left, right) margins; NumPy slice
                               semantics rows[top:H-bottom], cols[left:W-right] */
} ipp_hsv_range;

typedef struct ipp_hsv_params {
    int32_t n_ranges;
    int32_t bgr;            /* 1: input channel order is B,G,R (cv2); 0: R,G,B */
    ipp_hsv_range r[IPP_MAX_HSV_RANGES];
} ipp_hsv_params;

typedef struct ipp_image_desc {
    int64_t off;            /* byte offset in the buffer                    */
    int32_t w, h, pitch;    /* dims, bytes per row                          */
    int32_t cn;             /* channels                                     */
} ipp_image_desc;

/* src: 3- or 4-channel images (an input alpha is dropped, as cv2.imread
 * IMREAD_COLOR does); dst: 4-channel (same channel order + new alpha). */
int ipp_hsv_mask(const uint8_t* src, const ipp_image_desc* src_descs,
                 uint8_t* dst, const ipp_image_desc* dst_descs, int32_t n_images,
                 int32_t max_w, int32_t max_h, const ipp_hsv_params* params, void* stream);

/* ------------------------------------------------------------------------ */
/* K8: Pillow resize(LANCZOS) of RGBA — separable 8bpc passes                */
/* overlays.py:129 (PIL Image.resize → RGBa convert → ImagingResample H,V →  */
/* RGBA convert).  Taps are int32 (22-bit fixed point) from ipp_plan_lanczos. */
/* ------------------------------------------------------------------------ */
typedef struct ipp_resample_desc {
    int64_t src_off, dst_off;
    int32_t src_pitch, dst_pitch;
    int32_t in_len;         /* H pass: input width;  V pass: input height     */
    int32_t out_len;        /* H pass: output width; V pass: output height    */
    int32_t lines;          /* H pass: rows processed; V pass: columns        */
    int32_t line0;          /* H pass: first source row (ybox_first)          */
    int32_t ksize;          /* taps per output sample                         */
    int32_t pad_;
    int64_t coef_off;       /* int32 index of this image's bounds in coefs:
                               bounds[2*out_len] (xmin, count) then
                               taps[out_len*ksize]                            */
} ipp_resample_desc;

/* flags */
#define IPP_RS_PREMULTIPLY 1   /* apply rgbA2rgba on the input (H pass)      */
#define IPP_RS_UNPREMULTIPLY 2 /* apply rgba2rgbA on the output (V pass)     */

int ipp_lanczos_h(const uint8_t* src, uint8_t* dst, const int32_t* coefs,
                  const ipp_resample_desc* descs, int32_t n_images,
                  int32_t max_out, int32_t max_lines, int32_t flags, void* stream);
int ipp_lanczos_v(const uint8_t* src, uint8_t* dst, const int32_t* coefs,
                  const ipp_resample_desc* descs, int32_t n_images,
                  int32_t max_out, int32_t max_lines, int32_t flags, void* stream);

/* ------------------------------------------------------------------------ */
/* K9: background.copy() + paste(ov, (x, y), ov) onto RGB                     */
/* overlays.py:138-139 (Paste.c paste_mask_RGBA, BLEND = DIV255).             */
/* ------------------------------------------------------------------------ */
typedef struct ipp_paste_desc {
    int64_t bg_off, ov_off, dst_off;
    int32_t bg_w, bg_h, bg_pitch, dst_pitch;
    int32_t ov_w, ov_h, ov_pitch;
    int32_t x, y;           /* paste position (must fit inside the bg)        */
    int32_t pad_;
} ipp_paste_desc;

int ipp_paste_blend(const uint8_t* bg, const uint8_t* ov, uint8_t* dst,
                    const ipp_paste_desc* descs, int32_t n_images,
                    int32_t bg_w, int32_t bg_h, void* stream);

/* ------------------------------------------------------------------------ */
/* Fused 5-stage pipe (configs 3/4): crop → rotate → flip → HSV mask →        */
/* LANCZOS H pass, all computed on the fly from the source (the RGBA cut-out  */
/* is never materialised); then LANCZOS V pass → unpremultiply → paste onto   */
/* the background, fused with the background copy.                           */
/* ------------------------------------------------------------------------ */
typedef struct ipp_pipe_desc {
    ipp_gather_desc g;      /* stage 1-3 (dst fields unused)                  */
    ipp_resample_desc h;    /* H pass: src = the virtual cut-out, dst = tmp   */
    ipp_resample_desc v;    /* V pass: src = tmp                              */
    ipp_paste_desc p;       /* paste: ov = V-pass result (never stored)        */
} ipp_pipe_desc;

/* Tap format of the pipe kernels (ipp_plan_pipe_axes format = 2 + phase).
 * The pipe kernels take IPP_TAPS_MFMA only; any other value returns
 * IPP_E_ARG. */
#define IPP_TAPS_MFMA 1   /* 16-output tiles, v_mfma_i32_16x16x64_i8          */

/* The batched 5-stage pipe as two launches (fused.PipeRunner.run, bench.py;
 * reference chain pipeline.py:526-541 → rotations.py:96, symmetry.py:114-119,
 * filtres_liste.py:84-134, overlays.py:129,138-139).  A composite's rows
 * outside the 16-row bands the overlay touches, [16⌊y/16⌋, 16⌈(y + ov_h)/16⌉),
 * are plain copies of the background (Paste.c leaves them untouched), and so
 * are, inside those bands, the 16-pixel groups outside the overlay's
 * [⌊x/16⌋, ⌈(x + ov_w)/16⌉) when the composite is dense and 16-B aligned with
 * a width that is a multiple of 16 (the "column split", one predicate in both
 * kernels):
 *   ipp_pipe_hpass_bgcopy: the LANCZOS H pass over the virtual cut-out (crop →
 *     rotate → flip → HSV α computed per pixel from the source, never stored)
 *     into the scratch `tmp`, plus the copy of those background bytes into
 *     `dst` by copy blocks that run beside the H-pass blocks: one block per
 *     row slab and group of IPP_PIPE_COPY_GROUP consecutive items, each
 *     background vector loaded once and stored to every item of the group on
 *     that background;
 *   ipp_pipe_vblend_bands: the V pass over the overlay bands, fused with the
 *     unpremultiply and the alpha blend; it writes the rest of each band: the
 *     overlay's 16-pixel groups under the column split, the whole band rows
 *     otherwise.
 * The two launches together write every composite byte exactly once: run
 * both, in this order, on the same dst (either alone leaves part of it
 * unwritten).
 * src_cn: channels of every source in the batch (3 or 4); hsv: HOST pointer;
 * tap_format: IPP_TAPS_MFMA (V axes planned with transposed = 2 + (p.y mod
 * 16), i.e. tap tiles aligned with 16-row background bands); max_ov_w /
 * max_ov_h bound the overlay sizes; ipp_pipe_vblend_bands takes overlays up
 * to IPP_PIPE_MAX_OV_W pixels wide (their 16 rows live in 64 KB of LDS;
 * fused.plan_pipe rejects wider ones before either launch runs).
 * Ring limit: the H pass keeps each 16-output tile's input window in a
 * 512-column LDS ring, so every H tile must satisfy 64·nK ≤ 512 (nK = its K
 * steps; ipp_plan_mfma_nk_bound(in, out, ksize) ≤ 8, i.e. LANCZOS downscales
 * of at most ≈ 23×; fused.plan_pipe refuses plans beyond it).  A violating
 * tile sets bit 0 of the sticky status read by ipp_pipe_status; its T columns
 * are then wrong. */
int ipp_pipe_hpass_bgcopy(const uint8_t* src, uint8_t* tmp, const int32_t* coefs,
                          const ipp_pipe_desc* descs, int32_t n_images,
                          int32_t max_out_w, int32_t max_rows, int32_t src_cn,
                          const ipp_hsv_params* hsv, int32_t tap_format,
                          const uint8_t* bg, uint8_t* dst, void* stream);
int ipp_pipe_vblend_bands(const uint8_t* tmp, const uint8_t* bg, uint8_t* dst,
                          const int32_t* coefs, const ipp_pipe_desc* descs, int32_t n_images,
                          int32_t bg_w, int32_t bg_h, int32_t max_ov_w, int32_t max_ov_h,
                          int32_t tap_format, void* stream);

/* Reads and clears the sticky status of the pipe kernels (bit 0: ring limit
 * violated, see above).  Synchronises `stream`. */
int ipp_pipe_status(int32_t* status, void* stream);

/* ------------------------------------------------------------------------ */
/* K10-K13: pixels_isolés.keep_largest_component                             */
/* :32 threshold(α,1,255) :35 connectedComponentsWithStats(8) :38-55 keep    */
/* largest :74-81 crop-fit (findNonZero + boundingRect).                     */
/* ------------------------------------------------------------------------ */
/* Scratch of one image inside a caller-provided byte buffer (offsets in
 * bytes, 256-B aligned; ipp_ccl_scratch_layout fills them for a w×h image
 * relative to 0 — add the image's base offset).  Per 64×64 tile: mask = 64
 * row words of fg bits (tile-major), edge = the global root of each edge
 * pixel (top, bottom, left, right × 64 int32), tile = (first entry, count).
 * P/A: int32/uint32 per run-start index (touched at component roots only);
 * ent: ent_cap {root, area, bbox} records of the components that touch a
 * tile edge (the others are final after the tile pass). */
typedef struct ipp_ccl_work {
    int64_t mask_off, edge_off, p_off, a_off, ent_off;
    int64_t ent_cap;
    int64_t tile_off;   /* per tile: component count, only root, edge flags */
    int64_t img_off;    /* per image: best closed component, kept root      */
} ipp_ccl_work;

/* Bytes of scratch for one w×h image; fills *work (may be NULL). */
int64_t ipp_ccl_scratch_layout(int32_t w, int32_t h, ipp_ccl_work* work);

/* α > 1 → 8-connected components → α := 0 outside the largest (lowest root on
 * ties) IN PLACE on 4-channel images; images without any component are left
 * unchanged.  works: device array of per-image scratch offsets into `scratch`;
 * max_ent = largest ent_cap; counts: int32[n] scratch; stats: int64[n]
 * scratch (best key = area << 32 | ~root); bbox[i] = (x0, y0, x1, y1) of the
 * kept component or (-1,-1,-1,-1) when there is none (the caller then takes
 * the α ≠ 0 bbox of the unchanged image, pixels_isolés.py:74-81). */
int ipp_ccl_keep_largest(uint8_t* img, const ipp_image_desc* descs, int32_t n_images,
                         int32_t max_w, int32_t max_h, const ipp_ccl_work* works,
                         uint8_t* scratch, int64_t max_ent, int32_t* counts, int64_t* stats,
                         int32_t* bbox, void* stream);

/* Fused config-5 chain on 3-channel BGR frames: filtres_liste's HSV mask
 * (filtres_liste.py:84-134, params as for ipp_hsv_mask with bgr = 1) → α > 1
 * components → keep the largest → crop-fit (pixels_isolés.py:29-81), written
 * as BGRA (α 255 inside the component, 0 elsewhere) at out_descs[i] (the
 * slot must hold the whole frame).  bbox as above; a frame with no kept pixel
 * gets bbox (-1,...) and no output (the reference raises there). */
int ipp_video_keep_largest(const uint8_t* frames, const ipp_image_desc* descs, int32_t n_images,
                           int32_t max_w, int32_t max_h, const ipp_hsv_params* hsv,
                           const ipp_ccl_work* works, uint8_t* scratch, int64_t max_ent,
                           int32_t* counts, int64_t* stats, int32_t* bbox, uint8_t* out,
                           const ipp_image_desc* out_descs, void* stream);

/* Bounding box of non-zero pixels, Pillow getbbox() rule (rotations.py:99,
 * recadrages.py:70): the alpha band for 2/4-channel images, any band for
 * 1/3-channel ones (also cv2.findNonZero+boundingRect, pixels_isolés.py:77-79).
 * bbox[i] = (x0, y0, x1, y1) or (-1,-1,-1,-1) when empty. */
int ipp_alpha_bbox(const uint8_t* img, const ipp_image_desc* descs, int32_t n_images,
                   int32_t max_w, int32_t max_h, int32_t* bbox, void* stream);

/* ------------------------------------------------------------------------ */
/* Host-side planning (CPU).                                                 */
/* ------------------------------------------------------------------------ */
/* Pillow Resample.c precompute_coeffs + normalize_coeffs_8bpc for LANCZOS
 * (support 3): writes bounds[2*out_size] (xmin, count) followed by
 * taps[out_size*ksize] into `out` (int32); returns ksize, or the required
 * int32 count when out == NULL (as -count), or IPP_E_ARG. */
int64_t ipp_plan_lanczos(int32_t in_size, double in0, double in1, int32_t out_size,
                         int32_t* out, int64_t out_capacity);
/* Batch form: n axes (in_sizes[i] → out_sizes[i], box = full axis), each
 * written at int32 offset offsets[i] of `out`; n_threads ≤ 0 = all cores. */
int ipp_plan_lanczos_batch(int32_t n, const int32_t* in_sizes, const int32_t* out_sizes,
                           const int64_t* offsets, int32_t* out, int64_t out_capacity,
                           int32_t n_threads);
/* Plan every axis of a pipe batch in the MFMA tile format (threaded);
 * identity[i] = no pass on that axis; shift_first[i] = shift bounds to
 * ybox_first; transposed[i] = 2 + tile phase (other values: IPP_E_ARG);
 * first_last receives (ybox_first, ybox_last). */
int ipp_plan_pipe_axes(int32_t n, const int32_t* in_sizes, const int32_t* out_sizes,
                       const int32_t* identity, const int32_t* shift_first,
                       const int32_t* transposed, const int64_t* offsets, int32_t* out,
                       int32_t* first_last, int32_t n_threads);
/* MFMA tile format of a pipe axis (v_mfma_i32_16x16x64_i8; see ipp_host.cpp):
 * size bound in int32 for (in, out, ksize), bound on K steps per tile, and the
 * conversion from standard Pillow taps (input indices minus `shift`, tiles
 * offset by `phase` outputs).  ipp_plan_pipe_axes writes this format for axes
 * with transposed[i] = 2 + phase. */
int64_t ipp_plan_mfma_size(int32_t in_size, int32_t out_size, int32_t ksize);
int32_t ipp_plan_mfma_nk_bound(int32_t in_size, int32_t out_size, int32_t ksize);
int ipp_plan_mfma_from_taps(int32_t in_size, int32_t out_size, int32_t ksize,
                            const int32_t* std_taps, int32_t shift, int32_t phase, int32_t* out);
/* ksize for (in_size, out_size) without computing taps. */
int32_t ipp_plan_lanczos_ksize(double in0, double in1, int32_t out_size);

/* Alpha bbox of the rotated canvas of a fully opaque in_w×in_h image under
 * the 16.16 affine (a0..a5) on an nw×nh canvas, computed analytically per
 * row with exact integer arithmetic.  bbox = (x0, y0, x1, y1) or all -1. */
int ipp_plan_opaque_bbox(int32_t in_w, int32_t in_h, const int32_t a[6],
                         int32_t nw, int32_t nh, int32_t bbox[4]);

/* ------------------------------------------------------------------------ */
/* Batch planner of the fused pipe (ipp_plan.cpp; replaces the per-item host  */
/* loop of fused.plan_pipe).  Draws every random parameter in the order of    */
/* the reference's chained file-mode pipeline with CPython's generator        */
/* (rotations.py:89, symmetry.py:122, pipeline.py:202, overlays.py:108,       */
/* :133-134), plans each item's geometry (rotations.py:96-109,                */
/* overlays.py:106-126) and fills the pipe descriptors (grouped by background) */
/* and the per-axis records of the device tap planner.                        */
/* ------------------------------------------------------------------------ */
typedef struct ipp_pipe_plan_cfg {
    int32_t src_h, src_w, src_pitch;          /* RGB u8 sources; pitch 0 = 3·src_w */
    int32_t crop_t, crop_b, crop_l, crop_r;   /* crop_from_border margins (px)     */
    int32_t bg_h, bg_w, n_bg;
    int32_t n_sym, sym_flip[4];               /* symmetry pool (flip code per entry) */
    int32_t n_global, start, stop;            /* plan items [start, stop) of n_global */
    int32_t given;                            /* 1: items[] hold angle, ratio, sym,
                                                 bg_index, x, y (nothing is drawn) */
    int32_t n_threads;                        /* ≤ 0: all cores                    */
    int32_t ring_cols;                        /* H-pass LDS ring (≤ 0: 512); an H tile
                                                 needing a wider window is refused */
    int32_t pad_;
    uint64_t seed;                            /* |n| of random.seed(n)             */
    double angle_min, angle_max, scale_min, scale_max;
} ipp_pipe_plan_cfg;

typedef struct ipp_pipe_item {
    double angle, ratio;
    int32_t sym, bg_index, x, y;              /* sym: index into the pool          */
    int32_t rot_w, rot_h;                     /* rotated canvas (expand=True)      */
    int32_t cut_x, cut_y, cut_w, cut_h;       /* its getbbox = the cut-out         */
    int32_t ov_w, ov_h;                       /* resized overlay                   */
} ipp_pipe_item;

/* One resampling axis (2 per item: H then V) for ipp_pipe_plan_taps. */
typedef struct ipp_tap_axis {
    int32_t in_size, out_size;
    int32_t identity;     /* 1: no pass on this axis (single 2^22 tap)        */
    int32_t shift;        /* subtracted from every xmin (V axis: ybox_first)  */
    int32_t phase;        /* tile phase (V axis: y mod 16)                    */
    int32_t nkb;          /* ipp_plan_mfma_nk_bound: K-step slots per tile     */
    int32_t compact;      /* 1: tiles may use the compact block layout (H
                             axis of the pipe, see ipp_plan_mfma_tile)         */
    int32_t n_tiles;      /* (out_size + phase + 15) / 16                     */
    int64_t coef_off;     /* int32 index of the axis block in coefs           */
} ipp_tap_axis;

/* totals[] slots of ipp_plan_pipe_batch */
#define IPP_PT_COEF_WORDS 0   /* int32 size of the coefs buffer               */
#define IPP_PT_TMP_BYTES 1
#define IPP_PT_MAX_OUT_W 2
#define IPP_PT_MAX_ROWS 3
#define IPP_PT_MAX_OV_W 4
#define IPP_PT_MAX_OV_H 5
#define IPP_PT_ALGO_H 6       /* algorithmic bytes, see fused.PipePlan        */
#define IPP_PT_ALGO_V 7
#define IPP_PT_COPY_BYTES 8   /* 2 x the composite bytes the H launch copies
                                 (read + write as the V pass would move them;
                                 dense 16-B aligned images assumed)            */
#define IPP_PT_MAX_TILES 9
#define IPP_PT_ERR_ITEM 10    /* on IPP_E_RANGE: global item index and reason: */
#define IPP_PT_ERR_CODE 11    /* 1 canvas beyond 16.16, 2 ScaleAffine table,
                                 3 degenerate overlay, 4 given parameters do not
                                 fit, 5 H window beyond the LDS ring, 6 empty
                                 randint range                                 */
#define IPP_PT_COPY_READS 12  /* background bytes the H launch's grouped copy
                                 loads: one background per run of
                                 same-background items in each group of
                                 IPP_PIPE_COPY_GROUP items                     */
#define IPP_PLAN_TOTALS 16

/* Items per background-copy group of ipp_pipe_hpass_bgcopy (one shared load
 * per background vector and run of same-background items in the group). */
#define IPP_PIPE_COPY_GROUP 8
/* Widest overlay (pixels) of the pipe's V launch (ipp_pipe_vblend_bands). */
#define IPP_PIPE_MAX_OV_W 992

/* items[stop - start]: outputs (inputs too when cfg->given); descs[n] (in
 * processing order), axes[2n]; totals[IPP_PLAN_TOTALS]. */
int ipp_plan_pipe_batch(const ipp_pipe_plan_cfg* cfg, ipp_pipe_item* items, ipp_pipe_desc* descs,
                        ipp_tap_axis* axes, int64_t* totals);

/* Device tap planner (ipp_taps.hip): builds the MFMA tile format of every
 * axis (what ipp_plan_mfma_from_taps writes from Pillow's taps: hdr, bias,
 * blocks; tile t's blocks at uint4 offset t·nkb·192 of the axis's block area)
 * directly in `coefs` (device, IPP_PT_COEF_WORDS int32).  The taps are
 * computed in fp64 on the device; any tile holding a tap whose rounding point
 * lies within 2^-22 of a quantisation boundary is recomputed on the host with
 * the libm sin Pillow uses and copied over, so the result is bit-exact with
 * Resample.c.  scratch: device, ipp_pipe_taps_scratch_bytes(n_axes).
 * Synchronises `stream`.  stats[0] = tiles recomputed on the host, stats[1] =
 * device status (bit 0: a tile needed more K steps than nkb). */
int64_t ipp_pipe_taps_scratch_bytes(int32_t n_axes);
int ipp_pipe_plan_taps(const ipp_tap_axis* axes, int32_t n_axes, int32_t* coefs, void* scratch,
                       int64_t* stats, void* stream);
/* ipp_pipe_plan_taps with the size cap of the one packed upload of the
 * host-rebuilt tiles given (0 <= pack_cap <= the scratch's pack region, 4 MiB;
 * ipp_pipe_plan_taps passes the region size).  Rebuilt tiles whose pack
 * exceeds the cap are copied tile by tile instead; the taps are the same byte
 * for byte (tests/test_gpu_taps.py forces that path with pack_cap = 0). */
int ipp_pipe_plan_taps_cap(const ipp_tap_axis* axes, int32_t n_axes, int32_t* coefs, void* scratch,
                           int64_t* stats, int64_t pack_cap, void* stream);
/* Host restatement of one tile of that format (Resample.c taps, libm sin):
 * hdr[4], bias[16], blocks (nK·3072 bytes, ≤ blocks_cap).
 * Compact layout (axis->compact, nK >= 2 and at most 64 nonzero 16-column
 * groups over the tile's 16 outputs; hdr[3] = 1): bytes 0..63 hold
 * meta[16], meta[n] = g0 | len << 8 | base << 16 (output n's taps lie in the
 * 16-column groups g0 .. g0 + len - 1 counted from K0; base = the sum of len
 * over the outputs before n); plane p's group block i (16 signed bytes) sits
 * at byte 64 + (64 p + i)·16, block base + j holding output n's group g0 + j;
 * everything else is zero.  The H pass loads one block per lane and plane and
 * builds each K step's B operand by ds_bpermute (ipp_pipe.hip), 3 loads per
 * tile instead of 3·nK. */
int ipp_plan_mfma_tile(const ipp_tap_axis* axis, int32_t t, int32_t hdr[4], int32_t bias[16],
                       uint8_t* blocks, int64_t blocks_cap);
/* Pieces of ipp_plan_pipe_batch exposed for the tests: the division-free
 * form of ipp_plan_opaque_bbox, CPython's math.hypot (vector_norm), the
 * rotation plan (out = nw, nh, a0..a5) and the first n random() values of
 * random.seed(seed). */
int ipp_plan_opaque_bbox_fast(int32_t in_w, int32_t in_h, const int32_t a[6],
                              int32_t nw, int32_t nh, int32_t bbox[4]);
double ipp_plan_py_hypot(double x, double y);
int ipp_plan_rotation(int32_t w, int32_t h, double angle, int32_t out[8]);
int ipp_plan_py_random(uint64_t seed, int32_t n, double* out);

/* ------------------------------------------------------------------------ */
/* tranfo.enhance_image (transforms/tranfo.py:37-53) on RGB images:           */
/* ImageEnhance Brightness/Contrast/Color (:38-40, Image.blend, Blend.c),     */
/* GaussianBlur (:42-44, BoxBlur.c) and the r/g/b point() LUTs (:46-51).      */
/* ------------------------------------------------------------------------ */
#define IPP_ENH_BLUR 1   /* a GaussianBlur follows (box passes, ipp_box_pass) */
#define IPP_ENH_LUT 2    /* apply the image's 3×256 LUT (after the blur)      */

typedef struct ipp_enhance_desc {
    int64_t src_off, dst_off;          /* RGB images, explicit pitches      */
    int32_t w, h, src_pitch, dst_pitch;
    float f_brightness, f_contrast, f_color;  /* float32(factor), Blend.c   */
    int32_t flags;                     /* IPP_ENH_*                          */
    int32_t box_r;                     /* box radius (int part), BoxBlur.c   */
    uint32_t box_ww, box_fw;           /* 8.24 weights of the box pass       */
    int32_t pad_;
    int64_t lut_off;                   /* byte offset of 3×256 LUT bytes     */
} ipp_enhance_desc;

/* Σ L of the brightened image per image into sums[n] (zeroed first). */
int ipp_enhance_lsum(const uint8_t* src, const ipp_enhance_desc* descs, int32_t n_images,
                     int64_t max_pixels, uint64_t* sums, void* stream);
/* brightness → contrast (mean = int(Σ/N + 0.5)) → color [→ LUT when the
 * image has IPP_ENH_LUT and no IPP_ENH_BLUR]; writes dst (dst_off/pitch). */
int ipp_enhance_color(const uint8_t* src, uint8_t* dst, const ipp_enhance_desc* descs,
                      int32_t n_images, int64_t max_pixels, const uint64_t* sums,
                      const uint8_t* luts, void* stream);
/* One BoxBlur.c pass along x (axis 0) or y (axis 1) of packed RGB planes at
 * byte offsets offs[i] (pitch 3w) in src → dst at the same offsets, or at the
 * descriptor's dst_off/dst_pitch when final_dst; luts != NULL applies the
 * LUTs (last pass).  A GaussianBlur is 3 x passes then 3 y passes. */
int ipp_box_pass(const uint8_t* src, uint8_t* dst, const ipp_enhance_desc* descs, int32_t n_images,
                 int64_t max_pixels, const int64_t* offs, int32_t axis, const uint8_t* luts,
                 int32_t final_dst, void* stream);

/* ------------------------------------------------------------------------ */
/* Measurement helper (the copy-kernel ceiling of the box).     */
/* ------------------------------------------------------------------------ */
/* dst[0, nbytes) = src[0, nbytes) with 16-B non-temporal loads/stores; both
 * pointers 16-B aligned.  Not a reference call site: bench.py times it to
 * report the roofline against the HBM rate a plain copy reaches here. */
int ipp_stream_copy(const uint8_t* src, uint8_t* dst, int64_t nbytes, void* stream);

/* Library version / build info string. */
const char* ipp_version(void);

#ifdef __cplusplus
}
#endif
#endif /* IPP_H */
