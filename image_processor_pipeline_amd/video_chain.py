"""Batched device mode of BASELINE config 5: 4K frames through
filtres_liste's HSV mask then pixels_isolés' keep-largest + crop-fit.

Per frame (reference call chain, files between steps):
  filtres_liste.py:84-134   imread BGR → HSV → OR of inRange(×R) → NOT → BGRA
  pixels_isolés.py:29-61    α > 1 → 8-connected components → keep largest
  pixels_isolés.py:74-81    crop to the bbox of α ≠ 0
Here a batch of F frames resident in HBM runs as ONE library call,
ipp_video_keep_largest: the HSV mask is evaluated inside the tile-labelling
kernel (the BGRA mask is never stored), components are merged across tiles,
and the crop-fit writes BGRA straight from the BGR frame — no host round trip;
crop windows stay on the device until `results()` reads them back.  The staged
form (ipp_hsv_mask → ipp_ccl_keep_largest → ipp_crop_to_bbox) is kept for
checking (`run_staged`).
Frames are independent: multi-GPU runs are replicas.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native as N
from . import geometry as G
from .device import _stream, _to_dev
from .device_ccl import CclScratch


class VideoChain:
    """Device-resident buffers and descriptors for F frames of H×W BGR."""

    def __init__(self, n: int, h: int, w: int, device, ranges: Optional[Sequence] = None, zones=None,
                 use_gimp_scale: bool = False):
        self.n, self.h, self.w = n, h, w
        self.device = torch.device(device)
        self.lib = N.load()
        self.hsv = G.hsv_params(ranges if ranges is not None else G.REFERENCE_HSV_RANGES, zones, use_gimp_scale,
                                bgr=True)
        dev = self.device
        self.out = torch.empty((n, h, w, 4), dtype=torch.uint8, device=dev)
        self.sc = CclScratch([(h, w)] * n, dev)
        self.bbox = self.sc.bbox
        self._bgra = None
        sd = np.zeros(n, N.IMAGE_DESC)
        dd = np.zeros(n, N.IMAGE_DESC)
        cd = np.zeros(n, N.COPY_DESC)
        for i in range(n):
            sd[i]["off"], sd[i]["w"], sd[i]["h"], sd[i]["pitch"], sd[i]["cn"] = i * h * w * 3, w, h, 3 * w, 3
            dd[i]["off"], dd[i]["w"], dd[i]["h"], dd[i]["pitch"], dd[i]["cn"] = i * h * w * 4, w, h, 4 * w, 4
            cd[i]["src_off"] = cd[i]["dst_off"] = i * h * w * 4
            cd[i]["src_pitch"] = cd[i]["dst_pitch"] = 4 * w
            cd[i]["cn"] = 4
        self.src_descs = _to_dev(sd, dev)
        self.dst_descs = _to_dev(dd, dev)
        self.copy_descs = _to_dev(cd, dev)

    def _check(self, frames: torch.Tensor) -> None:
        if frames.shape != (self.n, self.h, self.w, 3) or frames.dtype != torch.uint8 or not frames.is_contiguous():
            raise ValueError(f"frames must be contiguous uint8 {(self.n, self.h, self.w, 3)}")
        if frames.device != self.device:
            raise ValueError(f"frames must live on {self.device}")

    def run(self, frames: torch.Tensor) -> None:
        """Fused chain: frames (F, H, W, 3) BGR → crops in self.out, bbox in self.bbox."""
        self._check(frames)
        sc = self.sc
        N.check(self.lib.ipp_video_keep_largest(frames.data_ptr(), self.src_descs.data_ptr(), self.n, self.w, self.h,
                                                N.np_ptr(self.hsv), sc.works_dev.data_ptr(), sc.scratch.data_ptr(),
                                                sc.max_ent, sc.counts.data_ptr(), sc.stats.data_ptr(),
                                                sc.bbox.data_ptr(), self.out.data_ptr(), self.dst_descs.data_ptr(),
                                                _stream(self.device)), "ipp_video_keep_largest")

    # -- staged form (the three plugin-level ops in sequence) ---------------
    @property
    def bgra(self) -> torch.Tensor:
        if self._bgra is None:
            self._bgra = torch.empty((self.n, self.h, self.w, 4), dtype=torch.uint8, device=self.device)
        return self._bgra

    def mask(self, frames: torch.Tensor) -> None:
        """filtres_liste's pass alone: (F, H, W, 3) BGR → self.bgra."""
        self._check(frames)
        N.check(self.lib.ipp_hsv_mask(frames.data_ptr(), self.src_descs.data_ptr(), self.bgra.data_ptr(),
                                      self.dst_descs.data_ptr(), self.n, self.w, self.h, N.np_ptr(self.hsv),
                                      _stream(self.device)), "ipp_hsv_mask")

    def keep_largest(self) -> None:
        """pixels_isolés' components on self.bgra (in place) → self.bbox."""
        sc = self.sc
        N.check(self.lib.ipp_ccl_keep_largest(self.bgra.data_ptr(), self.dst_descs.data_ptr(), self.n, self.w,
                                              self.h, sc.works_dev.data_ptr(), sc.scratch.data_ptr(), sc.max_ent,
                                              sc.counts.data_ptr(), sc.stats.data_ptr(), sc.bbox.data_ptr(),
                                              _stream(self.device)), "ipp_ccl_keep_largest")

    def crop(self) -> None:
        """Crop-fit of self.bgra into self.out (row pitch 4·W)."""
        N.check(self.lib.ipp_crop_to_bbox(self.bgra.data_ptr(), self.out.data_ptr(), self.copy_descs.data_ptr(),
                                          self.bbox.data_ptr(), self.n, self.w, self.h, 4, _stream(self.device)),
                "ipp_crop_to_bbox")

    def run_staged(self, frames: torch.Tensor) -> None:
        self.mask(frames)
        self.keep_largest()
        self.crop()

    def results(self) -> List[Optional[np.ndarray]]:
        """Host copies of the cropped BGRA frames (None where no pixel is
        left: the reference's cv2.boundingRect(None) raises there)."""
        bb = self.bbox.cpu().numpy().reshape(self.n, 4)
        res = []
        for i, (x0, y0, x1, y1) in enumerate(bb):
            res.append(None if x0 < 0 else self.out[i, :y1 - y0, :x1 - x0].cpu().numpy())
        return res


def synthetic_frames(n: int, h: int, w: int, seed: int, device, start: int = 0, noise: int = 0) -> torch.Tensor:
    """Structured BGR frames: dark background (inside
    the first reference exclusion range, v <= 150), one large elliptic blob of
    a kept colour (~20 % of the area) and salt specks of random colour at
    0.5 % density.  Frame i is drawn from its own generator (seed, start + i).
    ``noise`` > 0 adds uniform ±noise LSB per channel to the background and
    the blob (camera-like content: no 64-pixel run of one colour, so the CCL
    mask pass's uniform-slot shortcut never applies); the classes stay the
    same for noise ≤ 8."""
    dev = torch.device(device)
    out = torch.empty((n, h, w, 3), dtype=torch.uint8, device=dev)
    yy = torch.arange(h, device=dev, dtype=torch.float32)[:, None]
    xx = torch.arange(w, device=dev, dtype=torch.float32)[None, :]
    for i in range(n):
        g = torch.Generator(device=dev)
        g.manual_seed(seed * 1000003 + start + i)
        u = torch.rand(6, generator=g, device=dev).tolist()
        frame = out[i]
        frame[..., 0], frame[..., 1], frame[..., 2] = 24, 18, 30          # background, v = 30
        cx, cy = w * (0.3 + 0.4 * u[0]), h * (0.3 + 0.4 * u[1])
        ax, ay = w * (0.22 + 0.08 * u[2]), h * (0.22 + 0.08 * u[3])
        blob = ((xx - cx) / ax) ** 2 + ((yy - cy) / ay) ** 2 <= 1.0
        colour = torch.tensor([220, 120 + int(40 * u[4]), 40], dtype=torch.uint8, device=dev)  # blue-ish, kept
        frame[blob] = colour
        if noise > 0:
            d = torch.randint(-noise, noise + 1, (h, w, 3), generator=g, device=dev, dtype=torch.int16)
            frame.copy_((frame.to(torch.int16) + d).clamp_(0, 255).to(torch.uint8))
        speck = torch.rand((h, w), generator=g, device=dev) < 0.005
        k = int(speck.sum())
        frame[speck] = torch.randint(0, 256, (k, 3), generator=g, device=dev, dtype=torch.uint8)
    return out


def keep_largest_from_video(video_path, batch: int = 32, device="cuda", ranges=None, zones=None,
                            use_gimp_scale: bool = False) -> List[Optional[np.ndarray]]:
    """video.frame_extraction → filtres_liste → pixels_isolés for one video,
    frames decoded on the host (transforms.video.open_video) and run through
    the fused device chain in batches of `batch` frames, without the JPEG
    files between the steps.  Returns one BGRA crop (or None) per frame."""
    from .transforms.video import iter_frame_batches
    out: List[Optional[np.ndarray]] = []
    chain = None
    for fr in iter_frame_batches(video_path, batch):
        n, h, w, _ = fr.shape
        if chain is None or (chain.n, chain.h, chain.w) != (n, h, w):
            chain = VideoChain(n, h, w, device, ranges, zones, use_gimp_scale)
        t = torch.from_numpy(fr).to(chain.device)
        chain.run(t)
        out.extend(chain.results())
    return out
