"""Tensor-level device ops: thin wrappers that plan on the host and launch the
gfx950 kernels of libipp.so on torch's current HIP stream.

Tensors are HWC ``torch.uint8`` on a ROCm device.  Every op calls the HIP
C-ABI; if the library (or the GPU) is missing the call raises — there is no
CPU fallback in the product path.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from . import geometry as G

SYM_FLIP = {"o": 0, "h": 1, "v": 2, "hv": 3}


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _to_dev(a: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(device)


def _keep(*tensors: torch.Tensor) -> None:
    """Tie small device buffers (descriptors, taps) to the current stream so
    the caching allocator cannot hand their memory to a later H2D copy before
    the kernels that read them have run."""
    for t in tensors:
        t.record_stream(torch.cuda.current_stream(t.device))


def _require_cuda(t: torch.Tensor, name: str) -> None:
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.uint8):
        raise N.NativeUnavailable(f"{name}: expected a uint8 tensor on a ROCm device (no CPU fallback)")


# ---------------------------------------------------------------------------
# Rotate (+ margin crop, bbox crop, flip): rotations.py / recadrages.py /
# symmetry.py in one gather.
# ---------------------------------------------------------------------------

@dataclass
class GatherPlan:
    descs: np.ndarray              # GATHER_DESC[n]
    shapes: List[Tuple[int, int]]  # output (h, w) per image
    offsets: np.ndarray            # byte offset per output (packed, 16-B aligned rows)
    pitches: np.ndarray
    total_bytes: int
    max_w: int
    max_h: int


def plan_rotate_flip(src_dims: Sequence[Tuple[int, int, int]], angles: Sequence[float],
                     flips: Sequence[int], windows: Optional[Sequence[Tuple[int, int, int, int]]] = None,
                     src_offsets: Optional[Sequence[int]] = None, src_pitches: Optional[Sequence[int]] = None,
                     crop_to_bbox: bool = True, row_align: int = 128) -> GatherPlan:
    """Plan the fused gather for opaque (3-channel) or alpha-free sources.

    src_dims: (h, w, cn) per source; windows: (x0, y0, w, h) crop window per
    source (default: whole image).  The rotated canvas is cropped to its
    alpha bbox analytically (opaque input ⇒ exact; rotations.py:99-109).
    row_align: output row pitch alignment in bytes (a multiple of 16)."""
    n = len(src_dims)
    d = np.zeros(n, N.GATHER_DESC)
    shapes, offs, pitches = [], np.zeros(n, np.int64), np.zeros(n, np.int64)
    off = 0
    max_w = max_h = 1
    for i, (h, w, cn) in enumerate(src_dims):
        x0, y0, iw, ih = windows[i] if windows is not None else (0, 0, w, h)
        plan = G.rotation_plan(iw, ih, float(angles[i]))
        ox, oy, ow, oh = 0, 0, plan.nw, plan.nh
        if crop_to_bbox:
            bb = G.rotated_bbox(iw, ih, plan)
            if bb is not None and bb[2] > bb[0] and bb[3] > bb[1]:
                ox, oy, ow, oh = bb[0], bb[1], bb[2] - bb[0], bb[3] - bb[1]
        # 128-B row pitch (the packed buffer is 256-B aligned): a tile row's
        # 256-B nontemporal store then covers whole 128-B lines, and only each
        # row's last line is written partially (16-B pitches split a line
        # between two tiles at every tile boundary: 12 % more HBM writes)
        pitch = (4 * ow + row_align - 1) // row_align * row_align
        d[i]["src_off"] = src_offsets[i] if src_offsets is not None else 0
        d[i]["src_pitch"] = src_pitches[i] if src_pitches is not None else w * cn
        d[i]["src_cn"] = cn
        d[i]["src_w"], d[i]["src_h"] = w, h
        d[i]["in_x0"], d[i]["in_y0"], d[i]["in_w"], d[i]["in_h"] = x0, y0, iw, ih
        for k in range(6):
            d[i][f"a{k}"] = plan.A[k]
        d[i]["out_w"], d[i]["out_h"] = ow, oh
        d[i]["off_x"], d[i]["off_y"] = ox, oy
        d[i]["flip"] = int(flips[i])
        d[i]["dst_off"] = off
        d[i]["dst_pitch"] = pitch
        shapes.append((oh, ow))
        offs[i] = off
        pitches[i] = pitch
        off += pitch * oh
        max_w, max_h = max(max_w, ow), max(max_h, oh)
    # the per-image sampler (flip and bbox origin folded into the affine),
    # once here instead of in every block of the kernel
    N.check(N.load().ipp_gather_prepare(N.np_ptr(d), n), "ipp_gather_prepare")
    return GatherPlan(d, shapes, offs, pitches, off, max_w, max_h)


def rotate_flip_nearest(src: torch.Tensor, plan: GatherPlan, out: Optional[torch.Tensor] = None,
                        descs_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Launch the gather over a flat source buffer; returns the packed output."""
    _require_cuda(src, "rotate_flip_nearest")
    lib = N.load()
    if out is None:
        out = torch.empty(max(plan.total_bytes, 16), dtype=torch.uint8, device=src.device)
    if descs_dev is None:
        descs_dev = _to_dev(plan.descs, src.device)
    N.check(lib.ipp_rotate_flip_nearest(src.data_ptr(), out.data_ptr(), descs_dev.data_ptr(), len(plan.descs),
                                        plan.max_w, plan.max_h, _stream(src.device)), "ipp_rotate_flip_nearest")
    return out


def unpack(buf: torch.Tensor, plan: GatherPlan, cn: int = 4) -> List[torch.Tensor]:
    """Views (h, w, cn) into a packed pitched buffer."""
    outs = []
    for (h, w), off, pitch in zip(plan.shapes, plan.offsets, plan.pitches):
        outs.append(torch.as_strided(buf, (h, w, cn), (int(pitch), cn, 1), int(off)))
    return outs


def rotate_crop_single(img: torch.Tensor, angle: float, flip: int = 0) -> torch.Tensor:
    """rotations.py:55,96-109 for one image (3- or 4-channel, HWC).

    Opaque sources use the analytic bbox; sources with an alpha channel are
    rotated onto the full canvas, their alpha bbox is reduced on the device
    and the window copied out (Pillow semantics incl. the None/empty-bbox
    fallback to the uncropped canvas)."""
    _require_cuda(img, "rotate_crop_single")
    img = img.contiguous()
    h, w, cn = img.shape
    if cn == 3:
        plan = plan_rotate_flip([(h, w, 3)], [angle], [flip])
        buf = rotate_flip_nearest(img.reshape(-1), plan)
        return unpack(buf, plan)[0].contiguous()
    plan = plan_rotate_flip([(h, w, 4)], [angle], [0], crop_to_bbox=False)
    canvas = unpack(rotate_flip_nearest(img.reshape(-1), plan), plan)[0].contiguous()
    bb = alpha_bbox([canvas])[0]
    if bb is None or bb[2] <= bb[0] or bb[3] <= bb[1]:
        x0, y0, x1, y1 = 0, 0, canvas.shape[1], canvas.shape[0]
    else:
        x0, y0, x1, y1 = bb
    return copy_window(canvas, (x0, y0, x1 - x0, y1 - y0), flip)


def rotate_bilinear_canvas(img: torch.Tensor, angle: float, flip: int = 0) -> torch.Tensor:
    """Pillow ``convert('RGBA').rotate(angle, expand=True, resample=BILINEAR)``
    canvas of an RGB/RGBA image (ipp_rotate_bilinear; fast-path angles are
    transposes and take the NEAREST gather), flip bits folded in."""
    _require_cuda(img, "rotate_bilinear_canvas")
    img = img.contiguous()
    h, w, cn = img.shape
    plan = G.rotation_plan(w, h, float(angle))
    if plan.M is None:   # 0/90/180/270: exact transposes, identical for every filter
        gp = plan_rotate_flip([(h, w, cn)], [angle], [flip], crop_to_bbox=False)
        return unpack(rotate_flip_nearest(img.reshape(-1), gp), gp)[0].contiguous()
    d = np.zeros(1, N.AFFINE_DESC)
    d[0]["src_pitch"], d[0]["src_cn"] = w * cn, cn
    d[0]["in_w"], d[0]["in_h"] = w, h
    d[0]["out_w"], d[0]["out_h"], d[0]["dst_pitch"], d[0]["flip"] = plan.nw, plan.nh, 4 * plan.nw, flip
    d[0]["m"] = plan.M
    out = torch.empty((plan.nh, plan.nw, 4), dtype=torch.uint8, device=img.device)
    dd = _to_dev(d, img.device)
    N.check(N.load().ipp_rotate_bilinear(img.data_ptr(), out.data_ptr(), dd.data_ptr(), 1, plan.nw, plan.nh,
                                         _stream(img.device)), "ipp_rotate_bilinear")
    _keep(dd)
    return out


def rotate_crop_bilinear(img: torch.Tensor, angle: float, flip: int = 0) -> torch.Tensor:
    """rotations.py:96-109 with resample=BILINEAR: canvas, then its alpha
    bbox (fallback: the uncropped canvas when None or empty)."""
    canvas = rotate_bilinear_canvas(img, angle, flip)
    bb = alpha_bbox([canvas])[0]
    if bb is None or bb[2] <= bb[0] or bb[3] <= bb[1]:
        return canvas
    x0, y0, x1, y1 = bb
    return copy_window(canvas, (x0, y0, x1 - x0, y1 - y0))


# ---------------------------------------------------------------------------
# Window copy / flip (recadrages.py:46, crop_square.py:196, symmetry.py:114-119)
# ---------------------------------------------------------------------------

def copy_window(img: torch.Tensor, window: Optional[Tuple[int, int, int, int]] = None,
                flip: int = 0) -> torch.Tensor:
    _require_cuda(img, "copy_window")
    img = img.contiguous()
    h, w, cn = img.shape
    x0, y0, ww, wh = window if window is not None else (0, 0, w, h)
    out = torch.empty((wh, ww, cn), dtype=torch.uint8, device=img.device)
    if ww == 0 or wh == 0:
        return out
    d = np.zeros(1, N.COPY_DESC)
    d[0]["src_pitch"], d[0]["dst_pitch"] = w * cn, ww * cn
    d[0]["x0"], d[0]["y0"], d[0]["w"], d[0]["h"], d[0]["cn"], d[0]["flip"] = x0, y0, ww, wh, cn, flip
    dd = _to_dev(d, img.device)
    N.check(N.load().ipp_copy_window(img.data_ptr(), out.data_ptr(), dd.data_ptr(), 1, ww, wh,
                                     _stream(img.device)), "ipp_copy_window")
    _keep(dd)
    return out


def flip(img: torch.Tensor, sym: str) -> torch.Tensor:
    """cv2.flip for symmetry.py's keys ('o' = copy)."""
    return copy_window(img, None, SYM_FLIP[sym])


# ---------------------------------------------------------------------------
# Alpha bbox (Pillow getbbox alpha_only / cv2.findNonZero + boundingRect)
# ---------------------------------------------------------------------------

def alpha_bbox(imgs: Sequence[torch.Tensor]) -> List[Optional[Tuple[int, int, int, int]]]:
    dev = imgs[0].device
    n = len(imgs)
    d = np.zeros(n, N.IMAGE_DESC)
    flat = []
    off = 0
    for i, im in enumerate(imgs):
        _require_cuda(im, "alpha_bbox")
        h, w, cn = im.shape
        d[i]["off"], d[i]["w"], d[i]["h"], d[i]["pitch"], d[i]["cn"] = off, w, h, w * cn, cn
        flat.append(im.contiguous().reshape(-1))
        off += h * w * cn
    buf = torch.cat(flat) if n > 1 else flat[0]
    bbox = torch.empty(4 * n, dtype=torch.int32, device=dev)
    mw = max(int(im.shape[1]) for im in imgs)
    mh = max(int(im.shape[0]) for im in imgs)
    dd = _to_dev(d, dev)
    N.check(N.load().ipp_alpha_bbox(buf.data_ptr(), dd.data_ptr(), n, mw, mh, bbox.data_ptr(),
                                    _stream(dev)), "ipp_alpha_bbox")
    bb = bbox.cpu().numpy().reshape(n, 4)
    return [None if r[0] < 0 else tuple(int(v) for v in r) for r in bb]


# ---------------------------------------------------------------------------
# HSV range mask (filtres_liste.py:84-134)
# ---------------------------------------------------------------------------

def hsv_mask(img: torch.Tensor, params: np.ndarray) -> torch.Tensor:
    """img: (H, W, 3|4) in the channel order params['bgr'] names → (H, W, 4)."""
    _require_cuda(img, "hsv_mask")
    img = img.contiguous()
    h, w, cn = img.shape
    out = torch.empty((h, w, 4), dtype=torch.uint8, device=img.device)
    sd = np.zeros(1, N.IMAGE_DESC)
    sd[0]["w"], sd[0]["h"], sd[0]["pitch"], sd[0]["cn"] = w, h, w * cn, cn
    dd = np.zeros(1, N.IMAGE_DESC)
    dd[0]["w"], dd[0]["h"], dd[0]["pitch"], dd[0]["cn"] = w, h, 4 * w, 4
    p = np.ascontiguousarray(params)
    sdd, ddd = _to_dev(sd, img.device), _to_dev(dd, img.device)
    N.check(N.load().ipp_hsv_mask(img.data_ptr(), sdd.data_ptr(), out.data_ptr(), ddd.data_ptr(), 1, w, h,
                                  N.np_ptr(p), _stream(img.device)), "ipp_hsv_mask")
    _keep(sdd, ddd)
    return out


# ---------------------------------------------------------------------------
# LANCZOS resize of RGBA (overlays.py:129) and paste (overlays.py:138-139)
# ---------------------------------------------------------------------------

def resize_lanczos_rgba(img: torch.Tensor, out_w: int, out_h: int) -> torch.Tensor:
    """Pillow ``Image.resize((out_w, out_h), LANCZOS)`` of an RGBA image."""
    _require_cuda(img, "resize_lanczos_rgba")
    img = img.contiguous()
    in_h, in_w, cn = img.shape
    if cn != 4:
        raise ValueError("resize_lanczos_rgba expects RGBA")
    if (in_w, in_h) == (out_w, out_h):
        return img.clone()  # Image.py:2400: plain copy, no RGBa round trip
    lib = N.load()
    dev = img.device
    need_h, need_v = out_w != in_w, out_h != in_h
    kh, th = G.lanczos_taps(in_w, out_w)
    kv, tv = G.lanczos_taps(in_h, out_h)
    cur = img
    if need_h:
        y0 = int(tv[0])
        y1 = int(tv[2 * out_h - 2] + tv[2 * out_h - 1])
        tv = tv.copy()
        tv[0:2 * out_h:2] -= y0
        rows = y1 - y0
        tmp = torch.empty((rows, out_w, 4), dtype=torch.uint8, device=dev)
        d = np.zeros(1, N.RESAMPLE_DESC)
        d[0]["src_pitch"], d[0]["dst_pitch"] = 4 * in_w, 4 * out_w
        d[0]["in_len"], d[0]["out_len"], d[0]["lines"], d[0]["line0"], d[0]["ksize"] = in_w, out_w, rows, y0, kh
        flags = N.IPP_RS_PREMULTIPLY | (0 if need_v else N.IPP_RS_UNPREMULTIPLY)
        thd, dd = _to_dev(th, dev), _to_dev(d, dev)
        N.check(lib.ipp_lanczos_h(cur.data_ptr(), tmp.data_ptr(), thd.data_ptr(), dd.data_ptr(), 1, out_w, rows,
                                  flags, _stream(dev)), "ipp_lanczos_h")
        _keep(thd, dd)
        cur = tmp
    if need_v:
        out = torch.empty((out_h, out_w, 4), dtype=torch.uint8, device=dev)
        d = np.zeros(1, N.RESAMPLE_DESC)
        d[0]["src_pitch"], d[0]["dst_pitch"] = 4 * out_w, 4 * out_w
        d[0]["in_len"], d[0]["out_len"], d[0]["lines"], d[0]["ksize"] = cur.shape[0], out_h, out_w, kv
        flags = N.IPP_RS_UNPREMULTIPLY | (0 if need_h else N.IPP_RS_PREMULTIPLY)
        tvd, dd = _to_dev(tv, dev), _to_dev(d, dev)
        N.check(lib.ipp_lanczos_v(cur.data_ptr(), out.data_ptr(), tvd.data_ptr(), dd.data_ptr(), 1, out_h, out_w,
                                  flags, _stream(dev)), "ipp_lanczos_v")
        _keep(tvd, dd)
        cur = out
    return cur


def paste_blend(bg: torch.Tensor, ov: torch.Tensor, x: int, y: int) -> torch.Tensor:
    """``bg.copy(); bg.paste(ov, (x, y), ov)`` for RGB bg and RGBA ov."""
    _require_cuda(bg, "paste_blend")
    _require_cuda(ov, "paste_blend")
    bg = bg.contiguous()
    ov = ov.contiguous()
    bh, bw, _ = bg.shape
    oh, ow, _ = ov.shape
    if x < 0 or y < 0 or x + ow > bw or y + oh > bh:
        raise ValueError("overlay must lie inside the background")
    out = torch.empty_like(bg)
    d = np.zeros(1, N.PASTE_DESC)
    d[0]["bg_w"], d[0]["bg_h"], d[0]["bg_pitch"], d[0]["dst_pitch"] = bw, bh, 3 * bw, 3 * bw
    d[0]["ov_w"], d[0]["ov_h"], d[0]["ov_pitch"], d[0]["x"], d[0]["y"] = ow, oh, 4 * ow, x, y
    dd = _to_dev(d, bg.device)
    N.check(N.load().ipp_paste_blend(bg.data_ptr(), ov.data_ptr(), out.data_ptr(), dd.data_ptr(), 1, bw, bh,
                                     _stream(bg.device)), "ipp_paste_blend")
    _keep(dd)
    return out


# ---------------------------------------------------------------------------
# tranfo.enhance_image (tranfo.py:37-53): brightness / contrast / color
# blends, GaussianBlur box passes, per-channel LUTs
# ---------------------------------------------------------------------------

@dataclass
class EnhanceParams:
    brightness: float
    contrast: float
    color: float
    blur_radius: Optional[float] = None        # GaussianBlur radius, None = no blur
    luts: Optional[np.ndarray] = None           # uint8 (3, 256) r/g/b tables, None = no point()


def enhance_rgb(imgs: Sequence[torch.Tensor], params: Sequence[EnhanceParams]) -> List[torch.Tensor]:
    """Batched tranfo.enhance_image pixel chain on (H, W, 3) RGB tensors:
    one ipp_enhance_lsum + one ipp_enhance_color launch for the whole batch,
    plus 6 ipp_box_pass launches when any image is blurred."""
    n = len(imgs)
    if n == 0:
        return []
    dev = imgs[0].device
    lib = N.load()
    d = np.zeros(n, N.ENHANCE_DESC)
    luts = np.zeros((n, 3, 256), np.uint8)
    src_parts, off = [], 0
    max_px = 1
    any_blur = any_lut = False
    for i, (im, p) in enumerate(zip(imgs, params)):
        _require_cuda(im, "enhance_rgb")
        h, w, cn = im.shape
        if cn != 3:
            raise ValueError("enhance_rgb expects RGB images (tranfo.py:37 converts to RGB)")
        d[i]["src_off"] = d[i]["dst_off"] = off
        d[i]["w"], d[i]["h"], d[i]["src_pitch"], d[i]["dst_pitch"] = w, h, 3 * w, 3 * w
        d[i]["f_brightness"], d[i]["f_contrast"], d[i]["f_color"] = p.brightness, p.contrast, p.color
        flags = 0
        if p.blur_radius is not None:
            r, ww, fw, fr = G.gaussian_box(p.blur_radius)
            if fr != 0.0:
                flags |= N.IPP_ENH_BLUR
                d[i]["box_r"], d[i]["box_ww"], d[i]["box_fw"] = r, ww, fw
                any_blur = True
        if p.luts is not None:
            flags |= N.IPP_ENH_LUT
            luts[i] = p.luts
            any_lut = True
        d[i]["flags"] = flags
        d[i]["lut_off"] = i * 768
        src_parts.append(im.contiguous().reshape(-1))
        off += h * w * 3
        max_px = max(max_px, h * w)
    src = torch.cat(src_parts) if n > 1 else src_parts[0]
    out = torch.empty_like(src)
    dd = _to_dev(d, dev)
    ld = _to_dev(luts, dev) if any_lut else None
    sums = torch.empty(n, dtype=torch.int64, device=dev)
    st = _stream(dev)
    N.check(lib.ipp_enhance_lsum(src.data_ptr(), dd.data_ptr(), n, max_px, sums.data_ptr(), st), "ipp_enhance_lsum")
    N.check(lib.ipp_enhance_color(src.data_ptr(), out.data_ptr(), dd.data_ptr(), n, max_px, sums.data_ptr(),
                                  ld.data_ptr() if ld is not None else None, st), "ipp_enhance_color")
    keep = [dd, sums] + ([ld] if ld is not None else [])
    if any_blur:
        # blurred images only: 3 row passes then 3 column passes, ping-pong
        bi = [i for i in range(n) if d[i]["flags"] & N.IPP_ENH_BLUR]
        bd = d[bi].copy()
        offs = np.array([int(d[i]["src_off"]) for i in bi], np.int64)
        bdd, od = _to_dev(bd, dev), _to_dev(offs, dev)
        tmp = torch.empty_like(src)
        a, b = out, tmp
        bmax = max(int(bd[k]["w"]) * int(bd[k]["h"]) for k in range(len(bi)))
        for k in range(6):
            last = k == 5
            N.check(lib.ipp_box_pass(a.data_ptr(), (out if last else b).data_ptr(), bdd.data_ptr(), len(bi), bmax,
                                     od.data_ptr(), 0 if k < 3 else 1,
                                     ld.data_ptr() if (last and ld is not None) else None, 0, st), "ipp_box_pass")
            if not last:
                a, b = b, a
        keep += [bdd, od, tmp]
    _keep(*keep)
    res = []
    for i, im in enumerate(imgs):
        h, w, _ = im.shape
        o = int(d[i]["src_off"])
        res.append(out[o:o + h * w * 3].view(h, w, 3))
    return res
