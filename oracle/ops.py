"""CPU oracle: NumPy restatements of the hot-path pixel routines.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Images are HWC uint8
NumPy arrays.  Pillow-mode images are RGB/RGBA; OpenCV-mode images are
BGR/BGRA exactly as ``cv2.imread`` would return them.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np

# ---------------------------------------------------------------------------
# A1. Pillow Image.rotate(angle, expand=True) with the default NEAREST filter.
#     Reference call site: transforms/rotations.py:96 (``img.rotate(angle,
#     expand=True)``; no ``resample`` → Resampling.NEAREST).
#     Library: PIL/Image.py:2475-2589 (Python geometry) and libImaging
#     Geometry.c ``affine_fixed`` (16.16 fixed-point nearest gather).
# ---------------------------------------------------------------------------


def rotate_geometry(w: int, h: int, angle: float) -> dict:
    """Return the transform Pillow applies for ``rotate(angle, expand=True)``.

    kind: 'copy' | 'rot90' | 'rot180' | 'rot270' | 'affine'.
    For 'affine' also returns the float matrix and the 16.16 coefficients.
    """
    angle = angle % 360.0
    if angle == 0:
        return {"kind": "copy", "nw": w, "nh": h}
    if angle == 180:
        return {"kind": "rot180", "nw": w, "nh": h}
    if angle in (90, 270):
        return {"kind": "rot90" if angle == 90 else "rot270", "nw": h, "nh": w}
    cx, cy = w / 2, h / 2
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0,
         round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]

    def T(x, y):
        return m[0] * x + m[1] * y + m[2], m[3] * x + m[4] * y + m[5]

    m[2], m[5] = T(-cx - 0, -cy - 0)
    m[2] += cx
    m[5] += cy
    xs, ys = [], []
    for x, y in ((0, 0), (w, 0), (w, h), (0, h)):
        tx, ty = T(x, y)
        xs.append(tx)
        ys.append(ty)
    nw = math.ceil(max(xs)) - math.floor(min(xs))
    nh = math.ceil(max(ys)) - math.floor(min(ys))
    m[2], m[5] = T(-(nw - w) / 2.0, -(nh - h) / 2.0)
    if m[1] == 0 and m[3] == 0:
        kind = "scale_affine"  # Geometry.c ImagingScaleAffine branch
    else:
        kind = "affine"
        for (x, y) in ((0, 0), (nw, nh), (0, nh), (nw, 0)):
            if not (abs(x * m[0] + y * m[1] + m[2]) < 32768.0
                    and abs(x * m[3] + y * m[4] + m[5]) < 32768.0):
                kind = "float_affine"
    fix = lambda v: math.floor(v * 65536.0 + 0.5)  # noqa: E731  (Geometry.c FIX)
    A = (fix(m[0]), fix(m[1]), fix(m[2] + m[0] * 0.5 + m[1] * 0.5),
         fix(m[3]), fix(m[4]), fix(m[5] + m[3] * 0.5 + m[4] * 0.5))
    return {"kind": kind, "nw": nw, "nh": nh, "matrix": tuple(m), "A": A}


def rotate_expand_nearest(img: np.ndarray, angle: float) -> np.ndarray:
    """Pillow ``img.rotate(angle, expand=True)`` (NEAREST) for an RGBA array."""
    h, w = img.shape[:2]
    g = rotate_geometry(w, h, angle)
    kind = g["kind"]
    if kind == "copy":
        return img.copy()
    if kind == "rot180":
        return img[::-1, ::-1].copy()
    if kind == "rot90":        # Transpose.ROTATE_90 (counter-clockwise)
        return np.rot90(img, 1).copy()
    if kind == "rot270":
        return np.rot90(img, -1).copy()
    if kind != "affine":
        raise NotImplementedError(f"Pillow {kind} branch not restated")
    a0, a1, a2, a3, a4, a5 = (np.int64(v) for v in g["A"])
    nw, nh = g["nw"], g["nh"]
    y = np.arange(nh, dtype=np.int64)[:, None]
    x = np.arange(nw, dtype=np.int64)[None, :]
    xin = (a2 + y * a1 + x * a0) >> 16
    yin = (a5 + y * a4 + x * a3) >> 16
    ok = (xin >= 0) & (xin < w) & (yin >= 0) & (yin < h)
    out = np.zeros((nh, nw, img.shape[2]), np.uint8)
    out[ok] = img[yin[ok], xin[ok]]
    return out


def rotate_expand_bilinear(img: np.ndarray, angle: float) -> np.ndarray:
    """Pillow ``img.rotate(angle, expand=True, resample=BILINEAR)`` for an RGBA
    array — the opt-in BILINEAR mode of process_rotations (north_star names
    "rotations.py (bilinear)"; the reference's own call, rotations.py:96, is
    NEAREST).  PIL/Image.py:2978-2983 runs RGBA through RGBa; Geometry.c
    ``affine_transform`` maps output (x, y) to ``a0(x+.5) + a1(y+.5) + a2``
    in double and ``bilinear_filter32RGB`` rejects points outside [0, w) ×
    [0, h), shifts by -0.5, clamps the x neighbours and the first row, falls
    back to row y when y+1 is out of range, lerps in double and truncates
    (SURVEY Appendix A9).  The 0/90/180/270 fast paths are transposes."""
    h, w = img.shape[:2]
    g = rotate_geometry(w, h, angle)
    if g["kind"] in ("copy", "rot90", "rot180", "rot270"):
        return rotate_expand_nearest(img, angle)
    m0, m1, m2, m3, m4, m5 = g["matrix"]
    nw, nh = g["nw"], g["nh"]
    src = premultiply(img).astype(np.float64)
    X = np.arange(nw, dtype=np.float64)[None, :] + 0.5
    Y = np.arange(nh, dtype=np.float64)[:, None] + 0.5
    xin = m0 * X + m1 * Y + m2
    yin = m3 * X + m4 * Y + m5
    ok = (xin >= 0.0) & (xin < w) & (yin >= 0.0) & (yin < h)
    xs, ys = xin - 0.5, yin - 0.5
    xi, yi = np.floor(xs), np.floor(ys)
    dx, dy = (xs - xi)[..., None], (ys - yi)[..., None]
    xi, yi = xi.astype(np.int64), yi.astype(np.int64)
    x0, x1 = np.clip(xi, 0, w - 1), np.clip(xi + 1, 0, w - 1)
    y0, y1 = np.clip(yi, 0, h - 1), np.clip(yi + 1, 0, h - 1)
    y1ok = ((yi + 1 >= 0) & (yi + 1 < h))[..., None]
    v1 = src[y0, x0] + (src[y0, x1] - src[y0, x0]) * dx
    v2 = np.where(y1ok, src[y1, x0] + (src[y1, x1] - src[y1, x0]) * dx, v1)
    v = v1 + (v2 - v1) * dy
    out = np.where(ok[..., None], v, 0.0).astype(np.uint8)
    return unpremultiply(out)


def getbbox_alpha(img: np.ndarray) -> Optional[Tuple[int, int, int, int]]:
    """Pillow ``getbbox()`` (alpha_only=True) on an RGBA array.

    PIL/Image.py:1480-1497; reference call site rotations.py:99.
    Returns (x0, y0, x1, y1) or None.
    """
    if img.shape[2] == 4:
        nz = img[:, :, 3] != 0
    else:
        nz = np.any(img != 0, axis=2)
    rows = np.flatnonzero(nz.any(axis=1))
    if rows.size == 0:
        return None
    cols = np.flatnonzero(nz.any(axis=0))
    return int(cols[0]), int(rows[0]), int(cols[-1]) + 1, int(rows[-1]) + 1


def rotate_and_crop(img_rgba: np.ndarray, angle: float, resample: str = "nearest") -> np.ndarray:
    """rotations.py:96-109: rotate, then crop to the alpha bbox (fallback:
    the uncropped canvas when the bbox is None or empty)."""
    rot = (rotate_expand_bilinear if resample == "bilinear" else rotate_expand_nearest)(img_rgba, angle)
    bb = getbbox_alpha(rot)
    if bb is None:
        return rot
    x0, y0, x1, y1 = bb
    crop = rot[y0:y1, x0:x1]
    if crop.shape[0] > 0 and crop.shape[1] > 0:
        return crop.copy()
    return rot


def to_rgba(img_rgb: np.ndarray) -> np.ndarray:
    """Pillow ``convert('RGBA')`` of an RGB array (rotations.py:55): α = 255."""
    if img_rgb.shape[2] == 4:
        return img_rgb.copy()
    h, w = img_rgb.shape[:2]
    out = np.empty((h, w, 4), np.uint8)
    out[..., :3] = img_rgb
    out[..., 3] = 255
    return out


# ---------------------------------------------------------------------------
# symmetry.py:114-119 — cv2.flip codes: 'h' → 1 (mirror x), 'v' → 0 (mirror
# y), 'hv' → -1 (both); 'o' → copy.
# ---------------------------------------------------------------------------

def flip(img: np.ndarray, sym: str) -> np.ndarray:
    if sym == "o":
        return img.copy()
    if sym == "h":
        return img[:, ::-1].copy()
    if sym == "v":
        return img[::-1, :].copy()
    if sym == "hv":
        return img[::-1, ::-1].copy()
    raise ValueError(sym)


# ---------------------------------------------------------------------------
# recadrages.py:7-10 and :37-46 — margin crop.
# ---------------------------------------------------------------------------

def compute_crop(value: float, total: int) -> int:
    if value < 0:
        raise ValueError("negative crop margin")
    return int(total * value) if 0 <= value < 1 else int(value)


def crop_from_border(img: np.ndarray, margins: Sequence[float]) -> np.ndarray:
    h, w = img.shape[:2]
    t, b, l, r = (compute_crop(margins[0], h), compute_crop(margins[1], h),
                  compute_crop(margins[2], w), compute_crop(margins[3], w))
    if t + b >= h or l + r >= w:
        raise ValueError("margins too large")
    return img[t:h - b, l:w - r].copy()


# ---------------------------------------------------------------------------
# A6/A7. OpenCV BGR→HSV (8-bit, H in [0,180)) + inRange + zone masks.
#   Reference: filtres_liste.py:90 (cvtColor), :97-134 (inRange×R, AND zone,
#   OR, NOT, merge).  Restated from OpenCV 4.x color_hsv RGB2HSV_b
#   (hsv_shift = 12, cvRound-built division tables) and core inRange
#   (scalar bounds → int32 via cvRound, impossible channel → empty range,
#   then saturate to uchar).  PARITY UNPINNED (OpenCV absent here).
# ---------------------------------------------------------------------------

_HSV_SHIFT = 12


def _hsv_tables():
    i = np.arange(256, dtype=np.float64)
    with np.errstate(divide="ignore"):
        sdiv = np.rint((255 << _HSV_SHIFT) / i)
        hdiv = np.rint((180 << _HSV_SHIFT) / (6.0 * i))
    sdiv[0] = 0
    hdiv[0] = 0
    return sdiv.astype(np.int64), hdiv.astype(np.int64)


SDIV_TABLE, HDIV_TABLE_180 = _hsv_tables()


def bgr_to_hsv(img_bgr: np.ndarray) -> np.ndarray:
    b = img_bgr[..., 0].astype(np.int64)
    g = img_bgr[..., 1].astype(np.int64)
    r = img_bgr[..., 2].astype(np.int64)
    v = np.maximum(np.maximum(b, g), r)
    vmin = np.minimum(np.minimum(b, g), r)
    diff = v - vmin
    s = (diff * SDIV_TABLE[v] + (1 << (_HSV_SHIFT - 1))) >> _HSV_SHIFT
    h = np.where(v == r, g - b, np.where(v == g, b - r + 2 * diff, r - g + 4 * diff))
    h = (h * HDIV_TABLE_180[diff] + (1 << (_HSV_SHIFT - 1))) >> _HSV_SHIFT
    h = np.where(h < 0, h + 180, h)
    return np.stack([np.clip(h, 0, 255), s, v], axis=-1).astype(np.uint8)


def rescale_filter(f, use_gimp_scale=False):
    """filtres_liste.py:8-39 (`_rescale_filter`)."""
    min_H, min_S, min_V, max_H, max_S, max_V = f
    if not use_gimp_scale:
        if any(hv > 180 for hv in [min_H, max_H]):
            raise ValueError("H out of OpenCV range")
        return f
    if any(sv > 100 for sv in [min_S, min_V, max_S, max_V]):
        raise ValueError("S/V out of GIMP range")
    return (min_H // 2, min_S * 2.55, min_V * 2.55, max_H // 2, max_S * 2.55, max_V * 2.55)


def inrange_bounds(lo: Sequence[float], hi: Sequence[float]) -> Tuple[List[int], List[int]]:
    """cv::inRange scalar-bound preparation for an 8U source."""
    ilo = [int(np.rint(v)) for v in lo]
    ihi = [int(np.rint(v)) for v in hi]
    for k in range(3):
        if ilo[k] > ihi[k] or ilo[k] > 255 or ihi[k] < 0:
            ilo[k], ihi[k] = 1, 0
    ilo = [min(max(v, 0), 255) for v in ilo]
    ihi = [min(max(v, 0), 255) for v in ihi]
    return ilo, ihi


def zone_rows_cols(zone, h: int, w: int) -> Tuple[int, int, int, int]:
    """Effective [r0,r1) × [c0,c1) of ``mask[t:h-b, l:w-r] = 255`` (NumPy slice
    semantics, filtres_liste.py:102-103)."""
    t, b, l, r = zone if zone else (0, 0, 0, 0)
    r0, r1, _ = slice(t, h - b).indices(h)
    c0, c1, _ = slice(l, w - r).indices(w)
    return r0, max(r0, r1), c0, max(c0, c1)


def hsv_alpha_mask(img_bgr: np.ndarray, ranges, zones=None, use_gimp_scale=False) -> np.ndarray:
    """α = NOT(OR_r(inRange_r AND zone_r)); returns uint8 HxW."""
    h, w = img_bgr.shape[:2]
    if zones and len(zones) != len(ranges):
        raise ValueError("zones/ranges length mismatch")
    zones = zones or [None] * len(ranges)
    hsv = bgr_to_hsv(img_bgr)
    excl = np.zeros((h, w), bool)
    for f, z in zip(ranges, zones):
        hmin, smin, vmin, hmax, smax, vmax = rescale_filter(f, use_gimp_scale)
        lo, hi = inrange_bounds((hmin, smin, vmin), (hmax, smax, vmax))
        m = np.ones((h, w), bool)
        for c in range(3):
            m &= (hsv[..., c] >= lo[c]) & (hsv[..., c] <= hi[c])
        r0, r1, c0, c1 = zone_rows_cols(z, h, w)
        zm = np.zeros((h, w), bool)
        zm[r0:r1, c0:c1] = True
        excl |= m & zm
    return np.where(excl, 0, 255).astype(np.uint8)


def color_mask_bgra(img_bgr: np.ndarray, ranges, zones=None, use_gimp_scale=False) -> np.ndarray:
    """process_images_with_color_masks pixel result (BGRA, filtres_liste.py:132-134)."""
    a = hsv_alpha_mask(img_bgr[..., :3], ranges, zones, use_gimp_scale)
    return np.concatenate([img_bgr[..., :3], a[..., None]], axis=-1)


# ---------------------------------------------------------------------------
# A3/A4. Pillow resize(LANCZOS) of an RGBA image via premultiplied RGBa.
#   Reference: overlays.py:129.  Library: PIL/Image.py:2328-2438 and
#   libImaging Resample.c (precompute_coeffs, normalize_coeffs_8bpc,
#   ImagingResampleHorizontal/Vertical_8bpc, PRECISION_BITS = 22) and
#   Convert.c rgbA2rgba / rgba2rgbA.
# ---------------------------------------------------------------------------

PRECISION_BITS = 32 - 8 - 2


def _sinc(x: float) -> float:
    if x == 0.0:
        return 1.0
    x = x * math.pi
    return math.sin(x) / x


def lanczos_filter(x: float) -> float:
    if -3.0 <= x < 3.0:
        return _sinc(x) * _sinc(x / 3)
    return 0.0


def precompute_coeffs(in_size: int, in0: float, in1: float, out_size: int):
    """Returns (ksize, bounds[out,2] (xmin, count), int32 taps[out, ksize])."""
    scale = (in1 - in0) / out_size
    filterscale = scale if scale >= 1.0 else 1.0
    support = 3.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        ww = 0.0
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        k = []
        for x in range(xmax):
            wv = lanczos_filter((x + xmin - center + 0.5) * ss)
            k.append(wv)
            ww += wv
        for x in range(xmax):
            v = k[x] / ww if ww != 0.0 else k[x]
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return ksize, bounds, kk


def _clip8(ss: np.ndarray) -> np.ndarray:
    return np.clip(ss >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resample_h(img: np.ndarray, out_w: int, bounds, kk, row0: int = 0, nrows: Optional[int] = None) -> np.ndarray:
    nrows = img.shape[0] - row0 if nrows is None else nrows
    src = img[row0:row0 + nrows].astype(np.int64)
    out = np.empty((nrows, out_w, img.shape[2]), np.uint8)
    for xx in range(out_w):
        xmin, cnt = bounds[xx]
        acc = np.full((nrows, img.shape[2]), 1 << (PRECISION_BITS - 1), np.int64)
        acc += np.einsum("rkc,k->rc", src[:, xmin:xmin + cnt], kk[xx, :cnt])
        out[:, xx] = _clip8(acc)
    return out


def resample_v(img: np.ndarray, out_h: int, bounds, kk) -> np.ndarray:
    src = img.astype(np.int64)
    out = np.empty((out_h, img.shape[1], img.shape[2]), np.uint8)
    for yy in range(out_h):
        ymin, cnt = bounds[yy]
        acc = np.full((img.shape[1], img.shape[2]), 1 << (PRECISION_BITS - 1), np.int64)
        acc += np.einsum("kxc,k->xc", src[ymin:ymin + cnt], kk[yy, :cnt])
        out[yy] = _clip8(acc)
    return out


def premultiply(img: np.ndarray) -> np.ndarray:
    """Convert.c rgbA2rgba: c' = MULDIV255(c, α)."""
    out = img.copy()
    a = img[..., 3].astype(np.int64)
    for c in range(3):
        t = img[..., c].astype(np.int64) * a + 128
        out[..., c] = (((t >> 8) + t) >> 8).astype(np.uint8)
    return out


def unpremultiply(img: np.ndarray) -> np.ndarray:
    """Convert.c rgba2rgbA: α∈{0,255} → unchanged, else min(255, 255c // α)."""
    out = img.copy()
    a = img[..., 3].astype(np.int64)
    keep = (a == 0) | (a == 255)
    safe = np.where(keep, 1, a)
    for c in range(3):
        v = np.minimum(255, (255 * img[..., c].astype(np.int64)) // safe)
        out[..., c] = np.where(keep, img[..., c], v).astype(np.uint8)
    return out


def resize_lanczos_rgba(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """Pillow ``Image.resize((out_w, out_h), LANCZOS)`` on an RGBA image."""
    in_h, in_w = img.shape[:2]
    if (in_w, in_h) == (out_w, out_h):
        return img.copy()  # Image.py:2400 — no RGBa round trip
    pm = premultiply(img)
    need_h = out_w != in_w
    need_v = out_h != in_h
    _, bh, kh = precompute_coeffs(in_w, 0.0, float(in_w), out_w)
    _, bv, kv = precompute_coeffs(in_h, 0.0, float(in_h), out_h)
    cur = pm
    if need_h:
        y0 = int(bv[0, 0])
        y1 = int(bv[-1, 0] + bv[-1, 1])
        bv = bv.copy()
        bv[:, 0] -= y0
        cur = resample_h(cur, out_w, bh, kh, y0, y1 - y0)
    if need_v:
        cur = resample_v(cur, out_h, bv, kv)
    return unpremultiply(cur)


# ---------------------------------------------------------------------------
# A5. Pillow ``background.paste(ov, (x, y), ov)`` onto RGB (overlays.py:138-139;
#   libImaging Paste.c paste_mask_RGBA, BLEND/DIV255).
# ---------------------------------------------------------------------------

def paste_rgba_onto_rgb(bg: np.ndarray, ov: np.ndarray, x: int, y: int) -> np.ndarray:
    out = bg.copy()
    oh, ow = ov.shape[:2]
    region = out[y:y + oh, x:x + ow].astype(np.int64)
    a = ov[..., 3:4].astype(np.int64)
    t = region * (255 - a) + ov[..., :3].astype(np.int64) * a + 128
    out[y:y + oh, x:x + ow] = (((t >> 8) + t) >> 8).astype(np.uint8)
    return out


def overlay_geometry(ov_w: int, ov_h: int, bg_w: int, bg_h: int, ratio: float) -> Tuple[int, int]:
    """overlays.py:106-126 — overlay target size from the diagonal ratio."""
    bg_diag = math.hypot(bg_w, bg_h)
    ov_diag_target = bg_diag * ratio
    if ov_h == 0:
        raise ValueError("invalid overlay dims")
    ar = ov_w / ov_h
    h_max = min(bg_w / ar, bg_h)
    max_ov_diag = math.hypot(ar * h_max, h_max)
    ov_diag = min(ov_diag_target, max_ov_diag)
    new_h = int(math.sqrt(ov_diag ** 2 / (ar ** 2 + 1)))
    new_w = int(ar * new_h)
    return new_w, new_h


def yolo_label(cls_id: int, x: int, y: int, w: int, h: int, bg_w: int, bg_h: int) -> str:
    """overlays.py:143-149 with ultralytics xyxy2xywhn restated."""
    x1, y1, x2, y2 = float(x), float(y), float(x + w), float(y + h)
    cx = ((x1 + x2) / 2) / bg_w
    cy = ((y1 + y2) / 2) / bg_h
    wn = (x2 - x1) / bg_w
    hn = (y2 - y1) / bg_h
    return f"{cls_id} {cx:.6f} {cy:.6f} {wn:.6f} {hn:.6f}"


# ---------------------------------------------------------------------------
# A8. pixels_isolés.keep_largest_component (pixels_isolés.py:29-61, 74-81):
#   fg = α > 1 (cv2.threshold(α,1,255,BINARY)); 8-connected components;
#   largest area wins, ties → lowest OpenCV label (block-raster order of the
#   2×2 scan blocks: the tie rule is restated, UNPINNED); α := 0 outside it;
#   crop to bbox(α ≠ 0).  Partition cross-checked with scipy.ndimage.label.
# ---------------------------------------------------------------------------

def keep_largest_component(img_bgra: np.ndarray) -> np.ndarray:
    from scipy import ndimage

    alpha = img_bgra[..., 3]
    fg = alpha > 1
    lab, n = ndimage.label(fg, structure=np.ones((3, 3), int))
    out = img_bgra.copy()
    if n > 0:
        areas = np.bincount(lab.ravel(), minlength=n + 1)
        areas[0] = 0
        h, w = fg.shape
        ys, xs = np.nonzero(fg)
        wb = (w + 1) // 2
        bkey = (ys // 2) * wb + (xs // 2)
        first = np.full(n + 1, np.iinfo(np.int64).max, np.int64)
        np.minimum.at(first, lab[ys, xs], bkey)
        best = max(range(1, n + 1), key=lambda L: (areas[L], -first[L]))
        out[..., 3] = np.where(lab == best, alpha, 0)
    a = out[..., 3]
    rows = np.flatnonzero((a != 0).any(axis=1))
    if rows.size == 0:
        raise ValueError("no non-transparent pixel (cv2.boundingRect(None))")
    cols = np.flatnonzero((a != 0).any(axis=0))
    return out[rows[0]:rows[-1] + 1, cols[0]:cols[-1] + 1].copy()


# ---------------------------------------------------------------------------
# tranfo.enhance_image (transforms/tranfo.py:37-53): ImageEnhance Brightness /
# Contrast / Color, ImageFilter.GaussianBlur, per-channel point() LUTs.
# Library: PIL/ImageEnhance.py (degenerate images + Image.blend), libImaging
# Blend.c (float32 blend, truncation; clipped extrapolation), Convert.c
# rgb2l (L = (19595 R + 38470 G + 7471 B + 0x8000) >> 16), ImageStat mean,
# BoxBlur.c (Gaussian = 3 box passes per axis, 8.24 fixed point).
# ---------------------------------------------------------------------------

def blend(im1: np.ndarray, im2: np.ndarray, factor: float) -> np.ndarray:
    """Image.blend(im1, im2, factor): Blend.c with alpha = float32(factor)."""
    a = np.float32(factor)
    if a == np.float32(0.0):
        return im1.copy()
    if a == np.float32(1.0):
        return im2.copy()
    i1 = im1.astype(np.float32)
    d = (im2.astype(np.int32) - im1.astype(np.int32)).astype(np.float32)
    t = i1 + a * d                      # two float32 roundings (no FMA)
    if np.float32(0.0) <= a <= np.float32(1.0):
        return t.astype(np.uint8)       # (UINT8) truncation
    out = np.where(t <= 0.0, 0, np.where(t >= 255.0, 255, t))
    return out.astype(np.uint8)


def rgb_to_l(img: np.ndarray) -> np.ndarray:
    """Convert.c rgb2l."""
    r, g, b = (img[..., k].astype(np.int64) for k in range(3))
    return ((r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16).astype(np.uint8)


def enhance_brightness(img: np.ndarray, f: float) -> np.ndarray:
    return blend(np.zeros_like(img), img, f)


def enhance_contrast(img: np.ndarray, f: float) -> np.ndarray:
    lum = rgb_to_l(img)
    s = float(np.sum(lum, dtype=np.int64))           # ImageStat sum (exact in double)
    mean = int(s / lum.size + 0.5)
    return blend(np.full_like(img, mean), img, f)


def enhance_color(img: np.ndarray, f: float) -> np.ndarray:
    lum = rgb_to_l(img)
    return blend(np.repeat(lum[..., None], 3, axis=2), img, f)


def gaussian_box_radius(radius: float, passes: int = 3) -> float:
    """BoxBlur.c _gaussian_blur_radius in float32 (sqrt/floor in double)."""
    r = np.float32(radius)
    sigma2 = np.float32(r * r / np.float32(passes))
    L = np.float32(math.sqrt(12.0 * float(sigma2) + 1.0))
    l = np.float32(math.floor((float(L) - 1.0) / 2.0))
    a = np.float32((np.float32(2) * l + np.float32(1)) * (l * (l + np.float32(1)) - np.float32(3) * sigma2))
    a = np.float32(a / (np.float32(6) * (sigma2 - (l + np.float32(1)) * (l + np.float32(1)))))
    return float(np.float32(l + a))


def box_blur_rows(img: np.ndarray, fradius: float) -> np.ndarray:
    """BoxBlur.c ImagingHorizontalBoxBlur on every row (uint32 fixed point):
    out[x] = (acc(x)·ww + (in[x-r-1] + in[x+r+1])·fw + 2^23) >> 24 with
    acc(x) = Σ in[clamp(i)], i ∈ [x-r, x+r], indices clamped to the row."""
    fr = np.float32(fradius)
    r = int(fr)
    ww = int(np.float32(1 << 24) / (fr * np.float32(2) + np.float32(1)))
    fw = ((1 << 24) - (2 * r + 1) * ww) // 2
    h, w = img.shape[:2]
    src = img.astype(np.int64)
    idx = np.arange(w)
    acc = np.zeros_like(src)
    for i in range(-r, r + 1):
        acc += src[:, np.clip(idx + i, 0, w - 1)]
    far = src[:, np.clip(idx - r - 1, 0, w - 1)] + src[:, np.clip(idx + r + 1, 0, w - 1)]
    bulk = (acc * ww + far * fw) & 0xFFFFFFFF
    return (((bulk + (1 << 23)) & 0xFFFFFFFF) >> 24).astype(np.uint8)


def gaussian_blur(img: np.ndarray, radius: float, passes: int = 3) -> np.ndarray:
    """ImageFilter.GaussianBlur(radius) (tranfo.py:44): BoxBlur.c
    ImagingGaussianBlur → ImagingBoxBlur with the same box radius on both axes."""
    br = gaussian_box_radius(radius, passes)
    out = img.copy()
    if br == 0.0:
        return out
    for _ in range(passes):
        out = box_blur_rows(out, br)
    t = np.ascontiguousarray(out.transpose(1, 0, 2))
    for _ in range(passes):
        t = box_blur_rows(t, br)
    return np.ascontiguousarray(t.transpose(1, 0, 2))


def point_luts(rng_uniform, lo: float = 0.75, hi: float = 1.25) -> np.ndarray:
    """tranfo.py:48-50: for r, g, b in turn, Image.point calls the lambda for
    p = 0..255 (one uniform draw each) and rounds: round(max(0, min(255, p·u)))."""
    luts = np.zeros((3, 256), np.uint8)
    for c in range(3):
        for p in range(256):
            luts[c, p] = round(max(0, min(255, p * rng_uniform(lo, hi))))
    return luts


def enhance_image(img_rgb: np.ndarray, apply_blur: bool, apply_rgb: bool, rnd) -> np.ndarray:
    """tranfo.enhance_image pixel chain with the draws taken from `rnd`
    (a random.Random or the random module) in the reference order."""
    out = enhance_brightness(img_rgb, rnd.uniform(0.7, 1.3))
    out = enhance_contrast(out, rnd.uniform(0.7, 1.3))
    out = enhance_color(out, rnd.uniform(0.7, 1.3))
    if apply_blur:
        out = gaussian_blur(out, rnd.uniform(0.5, 3))
    if apply_rgb:
        luts = point_luts(rnd.uniform)
        out = np.stack([luts[c][out[..., c]] for c in range(3)], axis=-1)
    return out
