"""Host-in / host-out batched device ops for the plugins' ``.batch`` hooks
(the codec boundary).

A ProcessingStep hands a plugin a chunk of argument tuples; the plugin
decodes them on host threads, calls ONE of these functions for the whole
chunk, and encodes on host threads.  Each function packs the chunk's images
into one pinned host buffer, makes one H2D copy, one launch (or one launch
per pass), and one D2H copy — instead of a synchronous H2D/launch/D2H round
trip per file.  Pixels are those of the per-file device ops (same kernels).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from . import _rt
from . import geometry as G
from .device import _keep, _stream, _to_dev


def _pack(imgs: Sequence[np.ndarray], align: int = 16) -> Tuple[torch.Tensor, List[int]]:
    """One device buffer holding every image (16-B aligned offsets)."""
    offs, total = [], 0
    for im in imgs:
        offs.append(total)
        total += (im.nbytes + align - 1) // align * align
    host = torch.empty(max(total, align), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
    hv = host.numpy()
    for im, o in zip(imgs, offs):
        hv[o:o + im.nbytes] = np.ascontiguousarray(im).reshape(-1).view(np.uint8)
    return host.to(_rt.device(), non_blocking=True), offs


def _unpack(buf: torch.Tensor, offs: Sequence[int], shapes: Sequence[Tuple[int, ...]]) -> List[np.ndarray]:
    host = buf.cpu().numpy()
    return [host[o:o + int(np.prod(s))].reshape(s).copy() for o, s in zip(offs, shapes)]


def _layout(shapes: Sequence[Tuple[int, ...]], align: int = 16) -> Tuple[List[int], int]:
    offs, total = [], 0
    for s in shapes:
        offs.append(total)
        total += (int(np.prod(s)) + align - 1) // align * align
    return offs, max(total, align)


def copy_windows(imgs: Sequence[np.ndarray], jobs: Sequence[Tuple[int, Tuple[int, int, int, int], int]]
                 ) -> List[np.ndarray]:
    """jobs: (image index, (x0, y0, w, h), flip bits) → one ipp_copy_window
    launch for all of them (recadrages.py:46 crops, symmetry.py:114-119
    flips).  Images are (H, W) or (H, W, cn) uint8, cn ≤ 4."""
    if not jobs:
        return []
    src, soffs = _pack(imgs)
    cns = [1 if im.ndim == 2 else im.shape[2] for im in imgs]
    shapes = [(j[1][3], j[1][2], cns[j[0]]) for j in jobs]
    doffs, total = _layout(shapes)
    out = torch.empty(total, dtype=torch.uint8, device=src.device)
    d = np.zeros(len(jobs), N.COPY_DESC)
    for k, (i, (x0, y0, w, h), fl) in enumerate(jobs):
        cn = cns[i]
        d[k]["src_off"], d[k]["dst_off"] = soffs[i], doffs[k]
        d[k]["src_pitch"], d[k]["dst_pitch"] = imgs[i].shape[1] * cn, w * cn
        d[k]["x0"], d[k]["y0"], d[k]["w"], d[k]["h"], d[k]["cn"], d[k]["flip"] = x0, y0, w, h, cn, fl
    mw = max(max(j[1][2] for j in jobs), 1)
    mh = max(max(j[1][3] for j in jobs), 1)
    dd = _to_dev(d, src.device)
    N.check(N.load().ipp_copy_window(src.data_ptr(), out.data_ptr(), dd.data_ptr(), len(jobs), mw, mh,
                                     _stream(src.device)), "ipp_copy_window")
    _keep(dd, src)
    res = _unpack(out, doffs, shapes)
    return [r[..., 0] if imgs[j[0]].ndim == 2 else r for r, j in zip(res, jobs)]


def hsv_masks(imgs: Sequence[np.ndarray], params: np.ndarray) -> List[np.ndarray]:
    """filtres_liste.py:84-134 for a chunk: BGR(A) → BGRA, one ipp_hsv_mask."""
    if not imgs:
        return []
    src, soffs = _pack(imgs)
    shapes = [(im.shape[0], im.shape[1], 4) for im in imgs]
    doffs, total = _layout(shapes)
    out = torch.empty(total, dtype=torch.uint8, device=src.device)
    sd = np.zeros(len(imgs), N.IMAGE_DESC)
    dd = np.zeros(len(imgs), N.IMAGE_DESC)
    for i, im in enumerate(imgs):
        h, w = im.shape[:2]
        cn = im.shape[2]
        sd[i]["off"], sd[i]["w"], sd[i]["h"], sd[i]["pitch"], sd[i]["cn"] = soffs[i], w, h, w * cn, cn
        dd[i]["off"], dd[i]["w"], dd[i]["h"], dd[i]["pitch"], dd[i]["cn"] = doffs[i], w, h, 4 * w, 4
    p = np.ascontiguousarray(params)
    sdd, ddd = _to_dev(sd, src.device), _to_dev(dd, src.device)
    N.check(N.load().ipp_hsv_mask(src.data_ptr(), sdd.data_ptr(), out.data_ptr(), ddd.data_ptr(), len(imgs),
                                  max(im.shape[1] for im in imgs), max(im.shape[0] for im in imgs), N.np_ptr(p),
                                  _stream(src.device)), "ipp_hsv_mask")
    _keep(sdd, ddd, src)
    return _unpack(out, doffs, shapes)


def keep_largest(imgs: Sequence[np.ndarray]) -> List[Optional[np.ndarray]]:
    """pixels_isolés.py:29-81 for a chunk of BGRA images: one
    ipp_ccl_keep_largest launch, then one crop launch; None where no pixel
    is left (the reference's boundingRect(None) raises there)."""
    from .device_ccl import keep_largest_packed
    if not imgs:
        return []
    src, soffs = _pack(imgs)
    # in place on the packed chunk (no second device copy of the images)
    bbs = keep_largest_packed(src, soffs, [(im.shape[0], im.shape[1]) for im in imgs])
    jobs = [(i, (b[0], b[1], b[2] - b[0], b[3] - b[1]), 0) for i, b in enumerate(bbs) if b is not None]
    if not jobs:
        return [None] * len(imgs)
    # crop straight from the cleaned device buffer
    shapes = [(j[1][3], j[1][2], 4) for j in jobs]
    doffs, total = _layout(shapes)
    out = torch.empty(total, dtype=torch.uint8, device=src.device)
    d = np.zeros(len(jobs), N.COPY_DESC)
    for k, (i, (x0, y0, w, h), _) in enumerate(jobs):
        d[k]["src_off"], d[k]["dst_off"] = soffs[i], doffs[k]
        d[k]["src_pitch"], d[k]["dst_pitch"] = imgs[i].shape[1] * 4, w * 4
        d[k]["x0"], d[k]["y0"], d[k]["w"], d[k]["h"], d[k]["cn"] = x0, y0, w, h, 4
    dd = _to_dev(d, src.device)
    N.check(N.load().ipp_copy_window(src.data_ptr(), out.data_ptr(), dd.data_ptr(), len(jobs),
                                     max(j[1][2] for j in jobs), max(j[1][3] for j in jobs), _stream(src.device)),
            "ipp_copy_window")
    _keep(dd, src)
    crops = iter(_unpack(out, doffs, shapes))
    return [next(crops) if b is not None else None for b in bbs]


def overlays(ovs: Sequence[np.ndarray], bgs: Sequence[np.ndarray], sizes: Sequence[Tuple[int, int]],
             pos: Sequence[Tuple[int, int]]) -> List[np.ndarray]:
    """overlays.py:129-139 for a chunk: LANCZOS resize of each RGBA overlay
    to sizes[i] = (w, h) (RGBa round trip) and paste onto its RGB background
    at pos[i] — ipp_lanczos_h + ipp_lanczos_v + ipp_paste_blend, one launch
    each for the items resized on both axes; one-axis and identity resizes
    (rare) take the per-image device path."""
    from .device import paste_blend, resize_lanczos_rgba
    n = len(ovs)
    if n == 0:
        return []
    lib = N.load()
    both = [i for i in range(n) if sizes[i][0] != ovs[i].shape[1] and sizes[i][1] != ovs[i].shape[0]]
    res: List[Optional[np.ndarray]] = [None] * n
    for i in sorted(set(range(n)) - set(both)):
        rs = resize_lanczos_rgba(_rt.h2d(ovs[i]), *sizes[i])
        res[i] = _rt.d2h(paste_blend(_rt.h2d(bgs[i]), rs, *pos[i]))
    if not both:
        return res
    ov_buf, ooffs = _pack([ovs[i] for i in both])
    bg_buf, boffs = _pack([bgs[i] for i in both])
    dev = ov_buf.device
    hd = np.zeros(len(both), N.RESAMPLE_DESC)
    vd = np.zeros(len(both), N.RESAMPLE_DESC)
    pd = np.zeros(len(both), N.PASTE_DESC)
    th_all, tv_all, th_off, tv_off = [], [], 0, 0
    tmp_shapes, rs_shapes = [], []
    for k, i in enumerate(both):
        in_h, in_w = ovs[i].shape[:2]
        ow, oh = sizes[i]
        kh, th = G.lanczos_taps(in_w, ow)
        kv, tv = G.lanczos_taps(in_h, oh)
        y0 = int(tv[0])
        y1 = int(tv[2 * oh - 2] + tv[2 * oh - 1])
        tv = tv.copy()
        tv[0:2 * oh:2] -= y0
        rows = y1 - y0
        tmp_shapes.append((rows, ow, 4))
        rs_shapes.append((oh, ow, 4))
        hd[k]["src_off"], hd[k]["src_pitch"], hd[k]["dst_pitch"] = ooffs[k], 4 * in_w, 4 * ow
        hd[k]["in_len"], hd[k]["out_len"], hd[k]["lines"], hd[k]["line0"], hd[k]["ksize"] = in_w, ow, rows, y0, kh
        hd[k]["coef_off"] = th_off
        vd[k]["src_pitch"], vd[k]["dst_pitch"] = 4 * ow, 4 * ow
        vd[k]["in_len"], vd[k]["out_len"], vd[k]["lines"], vd[k]["ksize"] = rows, oh, ow, kv
        vd[k]["coef_off"] = tv_off
        th_all.append(th)
        tv_all.append(tv)
        th_off += th.size
        tv_off += tv.size
    toffs, ttotal = _layout(tmp_shapes)
    roffs, rtotal = _layout(rs_shapes)
    for k in range(len(both)):
        hd[k]["dst_off"] = toffs[k]
        vd[k]["src_off"], vd[k]["dst_off"] = toffs[k], roffs[k]
    tmp = torch.empty(ttotal, dtype=torch.uint8, device=dev)
    rsb = torch.empty(rtotal, dtype=torch.uint8, device=dev)
    out_shapes = [bgs[i].shape for i in both]
    coffs, ctotal = _layout(out_shapes)
    out = torch.empty(ctotal, dtype=torch.uint8, device=dev)
    for k, i in enumerate(both):
        bh, bw = bgs[i].shape[:2]
        ow, oh = sizes[i]
        p = pd[k]
        p["bg_off"], p["ov_off"], p["dst_off"] = boffs[k], roffs[k], coffs[k]
        p["bg_w"], p["bg_h"], p["bg_pitch"], p["dst_pitch"] = bw, bh, 3 * bw, 3 * bw
        p["ov_w"], p["ov_h"], p["ov_pitch"], p["x"], p["y"] = ow, oh, 4 * ow, pos[i][0], pos[i][1]
    thd = _to_dev(np.concatenate(th_all), dev)
    tvd = _to_dev(np.concatenate(tv_all), dev)
    hdd, vdd, pdd = _to_dev(hd, dev), _to_dev(vd, dev), _to_dev(pd, dev)
    st = _stream(dev)
    N.check(lib.ipp_lanczos_h(ov_buf.data_ptr(), tmp.data_ptr(), thd.data_ptr(), hdd.data_ptr(), len(both),
                              max(s[1] for s in tmp_shapes), max(s[0] for s in tmp_shapes), N.IPP_RS_PREMULTIPLY, st),
            "ipp_lanczos_h")
    N.check(lib.ipp_lanczos_v(tmp.data_ptr(), rsb.data_ptr(), tvd.data_ptr(), vdd.data_ptr(), len(both),
                              max(s[0] for s in rs_shapes), max(s[1] for s in rs_shapes), N.IPP_RS_UNPREMULTIPLY, st),
            "ipp_lanczos_v")
    N.check(lib.ipp_paste_blend(bg_buf.data_ptr(), rsb.data_ptr(), out.data_ptr(), pdd.data_ptr(), len(both),
                                max(s[1] for s in out_shapes), max(s[0] for s in out_shapes), st), "ipp_paste_blend")
    _keep(thd, tvd, hdd, vdd, pdd, tmp, rsb, ov_buf, bg_buf)
    for i, c in zip(both, _unpack(out, coffs, out_shapes)):
        res[i] = c
    return res
