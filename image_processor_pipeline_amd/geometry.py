"""Host-side geometry for the hot path (product code, CPU, per image).

Reproduces the *host* arithmetic of the library calls the reference makes, in
Python double precision exactly as those libraries compute it, so the device
kernels receive the integers Pillow/OpenCV would use:

* ``rotation_plan`` — PIL ``Image.rotate(angle, expand=True)`` geometry
  (Pillow 12.2.0 PIL/Image.py:2475-2589) and Geometry.c ``affine_fixed``'s
  16.16 coefficients; Pillow's 0/90/180/270 fast paths and the
  ``ImagingScaleAffine`` branch are encoded as exact integer maps.
  Reference call site: transforms/rotations.py:96.
* ``rotated_bbox`` — ``getbbox()`` after the rotation (rotations.py:99) for an
  opaque source, analytic (C helper ``ipp_plan_opaque_bbox``).
* ``overlay_size`` — transforms/overlays.py:106-126.
* ``crop_margins`` — transforms/recadrages.py:7-10, :37-43.
* ``hsv_params`` — filtres_liste.py:8-39 (``_rescale_filter``) plus
  cv::inRange's bound preparation (cvRound → int32, empty ranges, saturate).
"""
from __future__ import annotations

import ctypes
import math
import warnings
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N

FIX_ONE = 65536
HALF = 32768


@dataclass(frozen=True)
class RotationPlan:
    kind: str            # 'copy' | 'rot90' | 'rot180' | 'rot270' | 'affine' | 'scale_affine'
    nw: int              # canvas width  (expand=True)
    nh: int              # canvas height
    A: Tuple[int, int, int, int, int, int]  # 16.16 inverse map (a0..a5)
    M: Optional[Tuple[float, ...]] = None   # Pillow's double matrix ('affine' / 'scale_affine'; BILINEAR)


def _with_m(plan: "RotationPlan", m) -> "RotationPlan":
    return RotationPlan(plan.kind, plan.nw, plan.nh, plan.A, tuple(m))


def _fix(v: float) -> int:
    return math.floor(v * 65536.0 + 0.5)  # Geometry.c FIX()


def rotation_plan(w: int, h: int, angle: float) -> RotationPlan:
    """Pillow rotate(angle, expand=True) with NEAREST, as an int 16.16 map."""
    angle = angle % 360.0
    if angle == 0:
        return RotationPlan("copy", w, h, (FIX_ONE, 0, HALF, 0, FIX_ONE, HALF))
    if angle == 180:
        return RotationPlan("rot180", w, h, (-FIX_ONE, 0, (w - 1) * FIX_ONE + HALF,
                                             0, -FIX_ONE, (h - 1) * FIX_ONE + HALF))
    if angle == 90:   # Transpose.ROTATE_90: out[Y][X] = in[X][w-1-Y]
        return RotationPlan("rot90", h, w, (0, -FIX_ONE, (w - 1) * FIX_ONE + HALF, FIX_ONE, 0, HALF))
    if angle == 270:  # Transpose.ROTATE_270: out[Y][X] = in[h-1-X][Y]
        return RotationPlan("rot270", h, w, (0, FIX_ONE, HALF, -FIX_ONE, 0, (h - 1) * FIX_ONE + HALF))
    cx, cy = w / 2, h / 2
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0,
         round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]

    def tr(x, y):
        return m[0] * x + m[1] * y + m[2], m[3] * x + m[4] * y + m[5]

    m[2], m[5] = tr(-cx - 0, -cy - 0)
    m[2] += cx
    m[5] += cy
    xs, ys = zip(*(tr(x, y) for x, y in ((0, 0), (w, 0), (w, h), (0, h))))
    nw = math.ceil(max(xs)) - math.floor(min(xs))
    nh = math.ceil(max(ys)) - math.floor(min(ys))
    m[2], m[5] = tr(-(nw - w) / 2.0, -(nh - h) / 2.0)
    if m[1] == 0 and m[3] == 0:
        return _with_m(_scale_affine_plan(w, h, nw, nh, m), m)
    for x, y in ((0, 0), (nw, nh), (0, nh), (nw, 0)):
        if not (abs(x * m[0] + y * m[1] + m[2]) < 32768.0 and abs(x * m[3] + y * m[4] + m[5]) < 32768.0):
            raise NotImplementedError("rotation canvas beyond Pillow's 16.16 fixed-point range (>32767 px)")
    A = (_fix(m[0]), _fix(m[1]), _fix(m[2] + m[0] * 0.5 + m[1] * 0.5),
         _fix(m[3]), _fix(m[4]), _fix(m[5] + m[3] * 0.5 + m[4] * 0.5))
    return RotationPlan("affine", nw, nh, A, tuple(m))


def _scale_affine_plan(w, h, nw, nh, m) -> RotationPlan:
    """Geometry.c ImagingScaleAffine (taken when sin rounds to 0 at 15
    decimals): pretabulated COORD() in double.  Reachable only for angles
    within ~1e-13° of 0/180; encoded as an exact integer map."""
    def coords(o, step, n):
        out = []
        for _ in range(n):
            out.append(-1 if o < 0.0 else int(o))
            o += step
        return out
    xt = coords(m[2] + m[0] * 0.5, m[0], nw)
    yt = coords(m[5] + m[4] * 0.5, m[4], nh)
    for t in (xt, yt):
        if len(t) > 1 and any(t[i + 1] - t[i] != t[1] - t[0] for i in range(len(t) - 1)):
            raise NotImplementedError("non-affine ScaleAffine table")
        if len(t) > 1 and abs(t[1] - t[0]) != 1:
            raise NotImplementedError("ScaleAffine with non-unit step")
    sx = (xt[1] - xt[0]) if nw > 1 else 1
    sy = (yt[1] - yt[0]) if nh > 1 else 1
    return RotationPlan("scale_affine", nw, nh,
                        (sx * FIX_ONE, 0, xt[0] * FIX_ONE + HALF, 0, sy * FIX_ONE, yt[0] * FIX_ONE + HALF))


def rotated_bbox(in_w: int, in_h: int, plan: RotationPlan) -> Optional[Tuple[int, int, int, int]]:
    """getbbox() of the rotated canvas of an OPAQUE in_w×in_h image."""
    lib = N.load()
    a = (ctypes.c_int32 * 6)(*plan.A)
    bb = (ctypes.c_int32 * 4)()
    N.check(lib.ipp_plan_opaque_bbox(in_w, in_h, ctypes.addressof(a), plan.nw, plan.nh, ctypes.addressof(bb)),
            "ipp_plan_opaque_bbox")
    return None if bb[0] < 0 else (bb[0], bb[1], bb[2], bb[3])


def overlay_size(ov_w: int, ov_h: int, bg_w: int, bg_h: int, ratio: float) -> Tuple[int, int]:
    """overlays.py:106-126 (diagonal ratio, capped to fit, aspect kept)."""
    bg_diag = math.hypot(bg_w, bg_h)
    ov_diag_target = bg_diag * ratio
    if ov_h == 0:
        raise ValueError(f"dimensions de l'overlay invalides ({ov_w}x{ov_h}).")
    ar = ov_w / ov_h
    h_max = min(bg_w / ar, bg_h)
    max_ov_diag = math.hypot(ar * h_max, h_max)
    ov_diag = min(ov_diag_target, max_ov_diag)
    new_h = int(math.sqrt(ov_diag ** 2 / (ar ** 2 + 1)))
    new_w = int(ar * new_h)
    return new_w, new_h


def compute_crop(value: float, total: int) -> int:
    """recadrages.py:7-10."""
    if value < 0:
        raise ValueError("Les valeurs de rognage ne peuvent pas être négatives.")
    return int(total * value) if 0 <= value < 1 else int(value)


def crop_margins(h: int, w: int, margins: Sequence[float], name: str = "") -> Tuple[int, int, int, int]:
    """recadrages.py:37-43 → (top, bottom, left, right) in pixels."""
    t, b, l, r = margins
    tp, bp, lp, rp = compute_crop(t, h), compute_crop(b, h), compute_crop(l, w), compute_crop(r, w)
    if tp + bp >= h or lp + rp >= w:
        raise ValueError(f"Les marges de rognage sont trop grandes pour l'image {name}.")
    return tp, bp, lp, rp


def rescale_filter(f, use_gimp_scale: bool = False):
    """filtres_liste.py:8-39."""
    min_H, min_S, min_V, max_H, max_S, max_V = f
    if not use_gimp_scale:
        if any(hv > 180 for hv in [min_H, max_H]):
            raise ValueError(f"Valeur(s) H ({min_H} - {max_H}) du filtre HSV au format OpenCV non conforme")
        if all(val <= 100 for val in [min_S, min_V, max_S, max_V]):
            print(f"Warning : aucune des valeurs S et V du filtre HSV au dessus de 100. ({min_S}, {min_V}, "
                  f"{max_S}, {max_V}).Vérifiez que votre filtre est au format OpenCV (0-180, 0-255, 0-255)"
                  "Non-bloquant, poursuite du traitement...")
        return f
    if any(sv > 100 for sv in [min_S, min_V, max_S, max_V]):
        raise ValueError(f"Valeur(s) S et V ({min_S}, {min_V}, {max_S}, {max_V}) au delà des limites admises "
                         "par GIMP.Vérifiez que votre filtre est au format de GIMP (0-360, 0-100, 0-100)")
    min_H //= 2
    max_H //= 2
    return min_H, min_S * 2.55, min_V * 2.55, max_H, max_S * 2.55, max_V * 2.55


def _cv_round(v: float) -> int:
    return int(np.rint(float(v)))  # cvRound: round half to even


def hsv_params(ranges, zones=None, use_gimp_scale: bool = False, bgr: bool = True) -> np.ndarray:
    """Pack the reference's HSV exclusion ranges into an ``ipp_hsv_params``.

    Ranges that cv::inRange would turn empty (lo > hi, or wholly outside
    [0, 255] in a channel) can never match and are dropped here."""
    if not ranges:
        raise ValueError("`color_ranges_to_exclude_hsv` est requis pour traiter les données")
    if zones and len(zones) != len(ranges):
        raise ValueError(f"Les zones d'application des filtres colorimétriques ({len(zones)}) ne correspondent pas "
                         f"aux filtres ({len(ranges)}). Les 2 paramètres doivent être de même longueur !.")
    zones = zones or [None] * len(ranges)
    p = np.zeros((), N.HSV_PARAMS)
    p["bgr"] = 1 if bgr else 0
    n = 0
    for f, z in zip(ranges, zones):
        hmin, smin, vmin, hmax, smax, vmax = rescale_filter(f, use_gimp_scale)
        lo = [_cv_round(v) for v in (hmin, smin, vmin)]
        hi = [_cv_round(v) for v in (hmax, smax, vmax)]
        if any(lo[k] > hi[k] or lo[k] > 255 or hi[k] < 0 for k in range(3)):
            continue
        if n >= N.IPP_MAX_HSV_RANGES:
            raise NotImplementedError(f"more than {N.IPP_MAX_HSV_RANGES} HSV ranges")
        lo = [min(max(v, 0), 255) for v in lo]
        hi = [min(max(v, 0), 255) for v in hi]
        zt, zb, zl, zr = z if z else (0, 0, 0, 0)
        p["r"][n]["lo"] = lo
        p["r"][n]["hi"] = hi
        p["r"][n]["zone"] = (int(zt), int(zb), int(zl), int(zr))
        n += 1
    p["n_ranges"] = n
    return p


# The reference's own HSV exclusion list (filtres_liste.py:186-190) — the
# canonical filter config of the benchmark pipe.
REFERENCE_HSV_RANGES = [
    (0, 0, 0, 180, 255, 150),
    (15, 60, 200, 35, 255, 255),
    (15, 30 * 2.55, 55 * 2.55, 30, 60 * 2.55, 80 * 2.55),
    (15, 60 * 2.55, 60 * 2.55, 30, 75 * 2.55, 90 * 2.55),
]


def lanczos_taps(in_size: int, out_size: int) -> Tuple[int, np.ndarray]:
    """(ksize, int32[2*out + out*ksize]) via the C planner (Resample.c)."""
    lib = N.load()
    need = -lib.ipp_plan_lanczos(in_size, 0.0, float(in_size), out_size, None, 0)
    if need <= 0:
        raise ValueError(f"invalid resize {in_size}->{out_size}")
    buf = np.empty(need, np.int32)
    k = lib.ipp_plan_lanczos(in_size, 0.0, float(in_size), out_size, N.np_ptr(buf), need)
    N.check(0 if k > 0 else int(k), "ipp_plan_lanczos")
    return int(k), buf


def identity_taps(n: int) -> Tuple[int, np.ndarray]:
    """Taps that reproduce the input exactly: (2^21 + p·2^22) >> 22 = p."""
    buf = np.empty(3 * n, np.int32)
    buf[0:2 * n:2] = np.arange(n)
    buf[1:2 * n:2] = 1
    buf[2 * n:] = 1 << 22
    return 1, buf


def gaussian_box(radius: float, passes: int = 3) -> Tuple[int, int, int, float]:
    """ImageFilter.GaussianBlur(radius) (tranfo.py:44) → the box pass of
    libImaging BoxBlur.c: ``_gaussian_blur_radius`` in float32 (sqrt and
    floor in double), then ImagingHorizontalBoxBlur's integer radius and
    8.24 weights ww = (uint32)(2^24 / (2·r_f + 1)), fw = (2^24 - (2r+1)·ww) / 2.
    Returns (r, ww, fw, r_f); r_f == 0 means no blur."""
    f32 = np.float32
    r = f32(radius)
    sigma2 = f32(r * r / f32(passes))
    L = f32(math.sqrt(12.0 * float(sigma2) + 1.0))
    l = f32(math.floor((float(L) - 1.0) / 2.0))
    a = f32((f32(2) * l + f32(1)) * (l * (l + f32(1)) - f32(3) * sigma2))
    a = f32(a / (f32(6) * (sigma2 - (l + f32(1)) * (l + f32(1)))))
    fr = f32(l + a)
    ir = int(fr)
    ww = int(f32(1 << 24) / (fr * f32(2) + f32(1)))
    fw = ((1 << 24) - (2 * ir + 1) * ww) // 2
    return ir, ww, fw, float(fr)
