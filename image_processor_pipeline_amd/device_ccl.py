"""Device op for pixels_isolés.keep_largest_component (K10–K13).

Reference: transforms/pixels_isolés.py:29-61 (threshold α > 1, 8-connected
components, keep the largest — lowest label on ties —, α := 0 elsewhere) and
:74-81 (crop to the bbox of α ≠ 0; cv2.boundingRect(None) raises when no pixel
is left).  All work runs in libipp.so (ipp_ccl_keep_largest: bit-plane run
labelling per 64×64 tile + border merge, csrc/ipp_ccl.hip); the host reads back four ints per
image for the crop window.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from .device import _keep, _require_cuda, _stream, _to_dev, alpha_bbox, copy_window


class CclScratch:
    """Per-image scratch layout (ipp_ccl_scratch_layout) for a batch of
    (h, w) images, packed into one device byte buffer."""

    def __init__(self, dims: Sequence[Tuple[int, int]], device):
        lib = N.load()
        n = len(dims)
        self.works = np.zeros(n, N.CCL_WORK)
        one = np.zeros(1, N.CCL_WORK)
        base = 0
        self.max_ent = 1
        for i, (h, w) in enumerate(dims):
            size = lib.ipp_ccl_scratch_layout(int(w), int(h), N.np_ptr(one))
            if size < 0:
                N.check(int(size), "ipp_ccl_scratch_layout")
            for f in (f for f in N.CCL_WORK.names if f.endswith("_off")):
                self.works[i][f] = one[0][f] + base
            self.works[i]["ent_cap"] = one[0]["ent_cap"]
            self.max_ent = max(self.max_ent, int(one[0]["ent_cap"]))
            base += (int(size) + 255) // 256 * 256
        self.bytes = base
        self.scratch = torch.empty(max(base, 256), dtype=torch.uint8, device=device)
        self.works_dev = _to_dev(self.works, device)
        self.counts = torch.empty(n, dtype=torch.int32, device=device)
        self.stats = torch.empty(n, dtype=torch.int64, device=device)
        self.bbox = torch.empty(4 * n, dtype=torch.int32, device=device)


def keep_largest_packed(buf: torch.Tensor, offs: Sequence[int],
                        dims: Sequence[Tuple[int, int]]) -> List[Optional[Tuple[int, int, int, int]]]:
    """In place on (H, W, 4) images packed in one contiguous device byte
    buffer at byte offsets `offs` (dims = (H, W) each): α zeroed outside the
    largest component.  Returns the α ≠ 0 bbox (x0, y0, x1, y1) per image or
    None (no pixel left)."""
    if not dims:
        return []
    _require_cuda(buf, "keep_largest_component")
    if buf.dtype != torch.uint8 or not buf.is_contiguous():
        raise ValueError("keep_largest_packed expects a contiguous uint8 buffer")
    dev = buf.device
    n = len(dims)
    d = np.zeros(n, N.IMAGE_DESC)
    for i, ((h, w), off) in enumerate(zip(dims, offs)):
        if off < 0 or off + 4 * h * w > buf.numel():
            raise ValueError(f"image {i} ({h}x{w}x4 at {off}) outside the buffer")
        d[i]["off"], d[i]["w"], d[i]["h"], d[i]["pitch"], d[i]["cn"] = off, w, h, 4 * w, 4
    sc = CclScratch([(int(h), int(w)) for h, w in dims], dev)
    mw = max(int(w) for _, w in dims)
    mh = max(int(h) for h, _ in dims)
    dd = _to_dev(d, dev)
    N.check(N.load().ipp_ccl_keep_largest(buf.data_ptr(), dd.data_ptr(), n, mw, mh, sc.works_dev.data_ptr(),
                                          sc.scratch.data_ptr(), sc.max_ent, sc.counts.data_ptr(),
                                          sc.stats.data_ptr(), sc.bbox.data_ptr(), _stream(dev)),
            "ipp_ccl_keep_largest")
    _keep(dd)
    bb = sc.bbox.cpu().numpy().reshape(n, 4)
    out: List[Optional[Tuple[int, int, int, int]]] = []
    for i, r in enumerate(bb):
        if r[0] >= 0:
            out.append(tuple(int(v) for v in r))
        else:
            # no component (no α > 1): label 0 is kept and α left unchanged
            # (pixels_isolés.py:38-47) — crop to its α ≠ 0 pixels (:77-81)
            h, w = dims[i]
            out.append(alpha_bbox([buf[offs[i]:offs[i] + 4 * h * w].view(h, w, 4)])[0])
    return out


def keep_largest_masks(imgs: Sequence[torch.Tensor]) -> List[Optional[Tuple[int, int, int, int]]]:
    """In place on each (H, W, 4) image: α zeroed outside the largest
    component.  Returns the α ≠ 0 bbox (x0, y0, x1, y1) per image or None."""
    if not imgs:
        return []
    for im in imgs:
        _require_cuda(im, "keep_largest_component")
        if im.dim() != 3 or im.shape[2] != 4:
            raise ValueError("keep_largest_component expects (H, W, 4) images")
    n = len(imgs)
    if n == 1 and imgs[0].is_contiguous() and imgs[0].dtype == torch.uint8:
        im = imgs[0]
        return keep_largest_packed(im.view(-1), [0], [(int(im.shape[0]), int(im.shape[1]))])
    offs, off = [], 0
    for im in imgs:
        offs.append(off)
        off += im.numel()
    buf = torch.cat([im.contiguous().reshape(-1) for im in imgs])
    res = keep_largest_packed(buf, offs, [(int(im.shape[0]), int(im.shape[1])) for im in imgs])
    for im, o in zip(imgs, offs):
        im.copy_(buf[o:o + im.numel()].view(im.shape))
    return res


def keep_largest_component(img: torch.Tensor) -> torch.Tensor:
    """(H, W, 4) BGRA → cleaned and crop-fitted copy (pixels_isolés.py:29-61)."""
    work = img.contiguous().clone()
    bb = keep_largest_masks([work])[0]
    if bb is None:
        raise ValueError("aucun pixel non transparent (cv2.boundingRect(None))")
    x0, y0, x1, y1 = bb
    return copy_window(work, (x0, y0, x1 - x0, y1 - y0))
