"""Device op for pixels_isolés.keep_largest_component (K10–K13).

Reference: transforms/pixels_isolés.py:29-61 (threshold α > 1, 8-connected
components, keep the largest — lowest label on ties —, α := 0 elsewhere) and
:74-81 (crop to the bbox of α ≠ 0; cv2.boundingRect(None) raises when no pixel
is left).  All work runs in libipp.so (ipp_ccl_keep_largest); the host only
reads back four ints per image for the crop window.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from .device import _require_cuda, _stream, _to_dev, copy_window


def _label_slots(h: int, w: int) -> int:
    return 4 * ((w + 1) // 2) * ((h + 1) // 2)


def keep_largest_masks(imgs: Sequence[torch.Tensor]) -> List[Optional[Tuple[int, int, int, int]]]:
    """In place on each (H, W, 4) image: α zeroed outside the largest
    component.  Returns the α ≠ 0 bbox (x0, y0, x1, y1) per image or None."""
    if not imgs:
        return []
    dev = imgs[0].device
    n = len(imgs)
    d = np.zeros(n, N.IMAGE_DESC)
    lab_off = np.zeros(n, np.int64)
    off = 0
    loff = 0
    flat = []
    for i, im in enumerate(imgs):
        _require_cuda(im, "keep_largest_component")
        if im.dim() != 3 or im.shape[2] != 4:
            raise ValueError("keep_largest_component expects (H, W, 4) images")
        h, w, _ = im.shape
        d[i]["off"], d[i]["w"], d[i]["h"], d[i]["pitch"], d[i]["cn"] = off, w, h, 4 * w, 4
        lab_off[i] = loff
        loff += _label_slots(h, w)
        off += h * w * 4
        flat.append(im.contiguous().reshape(-1))
    buf = torch.cat(flat) if n > 1 else flat[0]
    labels = torch.empty(max(loff, 1), dtype=torch.int32, device=dev)
    area = torch.empty(max(loff, 1), dtype=torch.int32, device=dev)
    stats = torch.empty(n, dtype=torch.int64, device=dev)
    bbox = torch.empty(4 * n, dtype=torch.int32, device=dev)
    mw = max(int(im.shape[1]) for im in imgs)
    mh = max(int(im.shape[0]) for im in imgs)
    dd, lo = _to_dev(d, dev), _to_dev(lab_off, dev)
    N.check(N.load().ipp_ccl_keep_largest(buf.data_ptr(), dd.data_ptr(), n, mw, mh, labels.data_ptr(),
                                          lo.data_ptr(), area.data_ptr(), stats.data_ptr(), bbox.data_ptr(),
                                          _stream(dev)), "ipp_ccl_keep_largest")
    off = 0
    for im in imgs:  # write back when the inputs were not contiguous views of buf
        sz = im.numel()
        if n > 1 or not im.is_contiguous():
            im.copy_(buf[off:off + sz].view(im.shape))
        off += sz
    bb = bbox.cpu().numpy().reshape(n, 4)
    return [None if r[0] < 0 else tuple(int(v) for v in r) for r in bb]


def keep_largest_component(img: torch.Tensor) -> torch.Tensor:
    """(H, W, 4) BGRA → cleaned and crop-fitted copy (pixels_isolés.py:29-61)."""
    work = img.contiguous().clone()
    bb = keep_largest_masks([work])[0]
    if bb is None:
        raise ValueError("aucun pixel non transparent (cv2.boundingRect(None))")
    x0, y0, x1, y1 = bb
    return copy_window(work, (x0, y0, x1 - x0, y1 - y0))
