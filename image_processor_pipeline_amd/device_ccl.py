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


def keep_largest_masks(imgs: Sequence[torch.Tensor]) -> List[Optional[Tuple[int, int, int, int]]]:
    """In place on each (H, W, 4) image: α zeroed outside the largest
    component.  Returns the α ≠ 0 bbox (x0, y0, x1, y1) per image or None."""
    if not imgs:
        return []
    dev = imgs[0].device
    n = len(imgs)
    d = np.zeros(n, N.IMAGE_DESC)
    off = 0
    flat = []
    for i, im in enumerate(imgs):
        _require_cuda(im, "keep_largest_component")
        if im.dim() != 3 or im.shape[2] != 4:
            raise ValueError("keep_largest_component expects (H, W, 4) images")
        h, w, _ = im.shape
        d[i]["off"], d[i]["w"], d[i]["h"], d[i]["pitch"], d[i]["cn"] = off, w, h, 4 * w, 4
        off += h * w * 4
        flat.append(im.contiguous().reshape(-1))
    buf = torch.cat(flat) if n > 1 else flat[0]
    sc = CclScratch([(int(im.shape[0]), int(im.shape[1])) for im in imgs], dev)
    mw = max(int(im.shape[1]) for im in imgs)
    mh = max(int(im.shape[0]) for im in imgs)
    dd = _to_dev(d, dev)
    N.check(N.load().ipp_ccl_keep_largest(buf.data_ptr(), dd.data_ptr(), n, mw, mh, sc.works_dev.data_ptr(),
                                          sc.scratch.data_ptr(), sc.max_ent, sc.counts.data_ptr(),
                                          sc.stats.data_ptr(), sc.bbox.data_ptr(), _stream(dev)),
            "ipp_ccl_keep_largest")
    _keep(dd)
    off = 0
    for im in imgs:  # write back when the inputs were not contiguous views of buf
        sz = im.numel()
        if n > 1 or not im.is_contiguous() or im.data_ptr() != buf.data_ptr():
            im.copy_(buf[off:off + sz].view(im.shape))
        off += sz
    bb = sc.bbox.cpu().numpy().reshape(n, 4)
    out: List[Optional[Tuple[int, int, int, int]]] = []
    for i, r in enumerate(bb):
        if r[0] >= 0:
            out.append(tuple(int(v) for v in r))
        else:
            # no component: α was left unchanged (label 0 kept) — crop to its α ≠ 0 pixels
            out.append(alpha_bbox([imgs[i]])[0])
    return out


def keep_largest_component(img: torch.Tensor) -> torch.Tensor:
    """(H, W, 4) BGRA → cleaned and crop-fitted copy (pixels_isolés.py:29-61)."""
    work = img.contiguous().clone()
    bb = keep_largest_masks([work])[0]
    if bb is None:
        raise ValueError("aucun pixel non transparent (cv2.boundingRect(None))")
    x0, y0, x1, y1 = bb
    return copy_window(work, (x0, y0, x1 - x0, y1 - y0))
