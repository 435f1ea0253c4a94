"""Batched device mode of the 5-stage pipe (BASELINE configs 3 and 4).

The reference runs five ``ProcessingStep``s chained through files
(pipeline.py:526-541), each calling one transform per item:

  1. recadrages.crop_from_border      (margin crop,          recadrages.py:13-61)
  2. rotations.process_rotations      (RGBA, NEAREST rotate, bbox crop, rotations.py:6-133)
  3. symmetry.generate_symmetries     (flip,                 symmetry.py:11-149)
  4. filtres_liste.process_images_with_color_masks (HSV α,   filtres_liste.py:41-149)
  5. overlays.paste_overlay_onto_background ('modulo' pairing with a cycled
     background set, LANCZOS resize + alpha paste,           overlays.py:24-187)

Here one host planning pass draws every random parameter in the reference's
draw order (``draw_params``) and fills one ``ipp_pipe_desc`` per item; the
device work is two launches for the whole batch (``ipp_pipe_hpass``,
``ipp_pipe_vblend``).  Intermediate cut-outs never touch HBM.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from . import geometry as G
from .device import SYM_FLIP, _stream, _to_dev

ALL_SYMS = ("o", "h", "v", "hv")
H_RING_COLUMNS = 512   # ipp_pipe.hip RING


@dataclass
class PipeConfig:
    margins: Tuple[float, float, float, float] = (64, 64, 64, 64)   # crop_from_border crop_margins
    angle_min: float = 1.0                                          # process_rotations defaults
    angle_max: float = 359.0
    sym_pool: Tuple[str, ...] = ALL_SYMS                             # generate_symmetries pool
    hsv_ranges: list = field(default_factory=lambda: list(G.REFERENCE_HSV_RANGES))
    zones: Optional[list] = None
    use_gimp_scale: bool = False
    scale_min: float = 0.15                                         # paste_overlay_onto_background
    scale_max: float = 0.30


@dataclass
class ItemParams:
    angle: float
    sym: str
    bg_index: int
    ratio: float
    x: int = 0
    y: int = 0


@dataclass
class PipePlan:
    descs: np.ndarray            # PIPE_DESC[n]
    coefs: np.ndarray            # int32 taps for all items
    hsv: np.ndarray              # HSV_PARAMS
    params: List[ItemParams]
    cut_dims: List[Tuple[int, int]]       # (h, w) of the cut-out M
    ov_dims: List[Tuple[int, int]]        # (h, w) of the resized overlay
    tmp_bytes: int
    max_out_w: int
    max_rows: int
    bg_w: int
    bg_h: int
    algo_bytes_hpass: int = 0
    algo_bytes_vblend: int = 0
    tap_format: int = 1                   # IPP_TAPS_MFMA (the only device format)
    max_ov_w: int = 1
    max_ov_h: int = 1
    # split form (ipp_pipe_hpass_bgcopy + ipp_pipe_vblend_bands): the
    # background rows outside the overlay bands move with the H pass
    algo_bytes_hpass_bgcopy: int = 0
    algo_bytes_vblend_bands: int = 0


def draw_params(n_global: int, stop: int, src_hw: Tuple[int, int], bg_hw: Tuple[int, int], n_bg: int,
                cfg: PipeConfig, seed: int):
    """Every random draw of the 5-step pipeline, consumed from ONE stream in
    the order a chained ``ProcessingPipeline`` of the five reference steps
    consumes it (step-major: each step runs over all its files, in sorted
    order, before the next step starts; pipeline.py:555-566):

      1. crop_from_border          — no draw;
      2. process_rotations         — one ``uniform(angle_min, angle_max)`` per
                                     file (rotations.py:89; num_rotations=1,
                                     include_original=False), all n_global files;
      3. generate_symmetries       — one ``sample(pool, 1)`` per file
                                     (symmetry.py:122; choose_random=1,
                                     include_original=False), all n_global files;
      4. process_images_with_color_masks — no draw;
      5. paste_overlay_onto_background, 'modulo' pairing — ``shuffle`` of the
         background list (pipeline.py:202), then per item ``uniform`` ratio
         (overlays.py:108) and two ``randint`` (overlays.py:133-134), whose
         ranges depend on the item's geometry, for items 0 .. stop-1.

    Returns (angles, syms, order, per-item (ratio, x, y, geometry)) for
    items 0 .. stop-1; items ≥ stop only consume their steps-2/3 draws."""
    H, W = src_hw
    bh, bw = bg_hw
    rng = random.Random(seed)
    pool = list(cfg.sym_pool)
    angles = [rng.uniform(cfg.angle_min, cfg.angle_max) for _ in range(n_global)]
    syms = [rng.sample(pool, 1)[0] for _ in range(n_global)]
    order = list(range(n_bg))
    rng.shuffle(order)
    t, b, l, r = G.crop_margins(H, W, cfg.margins)
    wc, hc = W - l - r, H - t - b
    per_item = []
    for gi in range(stop):
        ratio = rng.uniform(cfg.scale_min, cfg.scale_max)
        plan, box, (nw_, nh_) = item_geometry(wc, hc, angles[gi], ratio, bw, bh, gi)
        x = rng.randint(0, bw - nw_)
        y = rng.randint(0, bh - nh_)
        per_item.append((ratio, x, y, plan, box, (nw_, nh_)))
    return angles, syms, order, per_item


def item_geometry(wc: int, hc: int, angle: float, ratio: float, bw: int, bh: int, gi: int = 0):
    """One item's host geometry: the rotation plan of the wc×hc crop
    (rotations.py:96), its bbox (x, y, w, h) (rotations.py:99-109, fallback
    to the whole canvas) and the resized overlay (w, h) (overlays.py:106-126)."""
    plan = G.rotation_plan(wc, hc, angle)
    bb = G.rotated_bbox(wc, hc, plan)
    if bb is not None and bb[2] > bb[0] and bb[3] > bb[1]:
        box = (bb[0], bb[1], bb[2] - bb[0], bb[3] - bb[1])
    else:
        box = (0, 0, plan.nw, plan.nh)
    nw_, nh_ = G.overlay_size(box[2], box[3], bw, bh, ratio)
    if nw_ <= 0 or nh_ <= 0:
        raise ValueError(f"item {gi}: degenerate overlay size {nw_}x{nh_}")
    return plan, box, (nw_, nh_)


def shard_range(n_global: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block of the global item list owned by `rank`:
    sizes differ by at most one, lower ranks take the remainder."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    q, rem = divmod(n_global, world)
    start = rank * q + min(rank, rem)
    return start, start + q + (1 if rank < rem else 0)


def plan_pipe(src_hw: Tuple[int, int], n: int, bg_hw: Tuple[int, int], n_bg: int, cfg: PipeConfig,
              seed: int = 0, src_pitch: Optional[int] = None, item_range: Optional[Tuple[int, int]] = None,
              n_global: Optional[int] = None, params: Optional[Sequence[ItemParams]] = None) -> PipePlan:
    """Plan `n` items.  The random stream is the one a chained file-mode
    ``ProcessingPipeline`` of the five reference steps over ``n_global``
    sources would consume under ``random.seed(seed)`` (``draw_params``).
    With ``item_range=(start, stop)`` only items [start, stop) of that global
    batch are planned (stop - start must equal n): every rank of a sharded run
    sees exactly the parameters a single process would give those items, so
    outputs do not depend on the number of GPUs.  ``n_global`` defaults to
    ``stop``.  With ``params`` (one ItemParams per item) nothing is drawn:
    the caller's angles, symmetries, backgrounds, ratios and positions are
    planned as given (positions must keep the overlay inside the background)."""
    H, W = src_hw
    bh, bw = bg_hw
    start, stop = item_range if item_range is not None else (0, n)
    if stop - start != n or start < 0:
        raise ValueError(f"item_range {item_range} does not hold {n} items")
    n_global = stop if n_global is None else n_global
    if n_global < stop:
        raise ValueError(f"n_global {n_global} < item_range stop {stop}")
    t, b, l, r = G.crop_margins(H, W, cfg.margins)
    wc, hc = W - l - r, H - t - b
    if params is None:
        angles, syms, order, drawn = draw_params(n_global, stop, src_hw, bg_hw, n_bg, cfg, seed)
        given = None
    else:
        if len(params) != n:
            raise ValueError(f"{len(params)} ItemParams for {n} items")
        given = list(params)
    d = np.zeros(n, N.PIPE_DESC)
    params: List[ItemParams] = []
    cut_dims, ov_dims = [], []
    # axis list for the batch tap planner: (in, out) pairs, H then V per item
    axes_in, axes_out, identity = [], [], []
    for gi in range(start, stop):
        i = gi - start
        if given is None:
            ratio, x, y, plan, (ox, oy, rw, rh), (nw_, nh_) = drawn[gi]
            angle, sym, bgi = angles[gi], syms[gi], order[gi % n_bg]
        else:
            it = given[i]
            angle, sym, bgi, ratio, x, y = it.angle, it.sym, it.bg_index, it.ratio, it.x, it.y
            plan, (ox, oy, rw, rh), (nw_, nh_) = item_geometry(wc, hc, angle, ratio, bw, bh, gi)
            if not (0 <= x <= bw - nw_ and 0 <= y <= bh - nh_ and 0 <= bgi < n_bg and sym in SYM_FLIP):
                raise ValueError(f"item {gi}: parameters {it} do not fit a {bw}x{bh} background")
        params.append(ItemParams(angle, sym, bgi, ratio, x, y))
        cut_dims.append((rh, rw))
        ov_dims.append((nh_, nw_))
        g = d[i]["g"]
        g["src_off"] = i * H * (src_pitch or 3 * W)
        g["src_pitch"] = src_pitch or 3 * W
        g["src_cn"] = 3
        g["src_w"], g["src_h"] = W, H
        g["in_x0"], g["in_y0"], g["in_w"], g["in_h"] = l, t, wc, hc
        for k in range(6):
            g[f"a{k}"] = plan.A[k]
        g["out_w"], g["out_h"] = rw, rh
        g["off_x"], g["off_y"] = ox, oy
        g["flip"] = SYM_FLIP[sym]
        same = (nw_, nh_) == (rw, rh)
        identity.append((same or nw_ == rw, same or nh_ == rh))
        axes_in += [rw, rh]
        axes_out += [nw_, nh_]

    # ---- taps (C planner, threaded; MFMA tile format, see ipp_host.cpp) -----
    lib = N.load()
    m = 2 * n
    a_in = np.asarray(axes_in, np.int32)
    a_out = np.asarray(axes_out, np.int32)
    ident = np.array([identity[j // 2][j % 2] for j in range(m)], np.int32)
    # V axes are shifted to ybox_first whenever Pillow runs the H pass
    shift = np.array([(j % 2 == 1) and not identity[j // 2][0] for j in range(m)], np.int32)
    ks = np.array([1 if ident[j] else lib.ipp_plan_lanczos_ksize(0.0, float(a_in[j]), int(a_out[j]))
                   for j in range(m)], np.int64)
    # The H pass keeps each output tile's input window in a 512-column LDS ring
    # (ipp_pipe.hip RING): 64·nK columns must fit.
    for j in range(0, m, 2):
        if ident[j]:
            continue
        cols = 64 * lib.ipp_plan_mfma_nk_bound(int(a_in[j]), int(a_out[j]), int(ks[j]))
        if cols > H_RING_COLUMNS:
            raise ValueError(f"item {j // 2}: LANCZOS downscale {a_in[j]} -> {a_out[j]} needs a {cols}-column "
                             f"window, more than the fused H pass holds ({H_RING_COLUMNS}); use the plugin path")
    # H axes (even j): tiles of 16 outputs; V axes: tiles aligned with 16-row
    # background bands (phase = y mod 16)
    transp = np.array([2 if j % 2 == 0 else 2 + params[j // 2].y % 16 for j in range(m)], np.int32)
    sizes = np.array([lib.ipp_plan_mfma_size(int(a_in[j]), int(a_out[j]), int(ks[j])) for j in range(m)],
                     np.int64)
    sizes = (sizes + 3) // 4 * 4          # 16-B aligned axis blocks
    offs = np.zeros(m, np.int64)
    offs[1:] = np.cumsum(sizes)[:-1]
    coefs = np.zeros(int(sizes.sum()), np.int32)
    first_last = np.zeros(2 * m, np.int32)
    N.check(lib.ipp_plan_pipe_axes(m, N.np_ptr(a_in), N.np_ptr(a_out), N.np_ptr(ident), N.np_ptr(shift),
                                   N.np_ptr(transp), N.np_ptr(offs), N.np_ptr(coefs), N.np_ptr(first_last), 0),
            "ipp_plan_pipe_axes")

    # ---- descriptors ----------------------------------------------------
    tmp_off = 0
    max_out_w = max_rows = 1
    algo_h = algo_v = copy_rows = 0
    for i in range(n):
        rh, rw = cut_dims[i]
        nh_, nw_ = ov_dims[i]
        jh, jv = 2 * i, 2 * i + 1
        if not identity[i][0]:
            y0, y1 = int(first_last[2 * jv]), int(first_last[2 * jv + 1])
        else:
            y0, y1 = 0, rh
        rows = y1 - y0
        # V tiles read up to 64·nK rows past their 16-aligned start
        nkb = lib.ipp_plan_mfma_nk_bound(int(a_in[jv]), int(a_out[jv]), int(ks[jv]))
        groups = (((rows + 15) // 16) * 16 + 64 * nkb + 16) // 4
        pitch = 16 * nw_
        h = d[i]["h"]
        h["dst_off"] = tmp_off
        h["dst_pitch"] = pitch
        h["in_len"], h["out_len"], h["lines"], h["line0"], h["ksize"] = rw, nw_, rows, y0, ks[jh]
        h["coef_off"] = offs[jh]
        v = d[i]["v"]
        v["src_off"] = tmp_off
        v["src_pitch"] = pitch
        v["in_len"], v["out_len"], v["lines"], v["ksize"] = rows, nh_, nw_, ks[jv]
        v["coef_off"] = offs[jv]
        p = d[i]["p"]
        it = params[i]
        p["bg_off"] = it.bg_index * bh * bw * 3
        p["dst_off"] = i * bh * bw * 3
        p["bg_w"], p["bg_h"], p["bg_pitch"], p["dst_pitch"] = bw, bh, 3 * bw, 3 * bw
        p["ov_w"], p["ov_h"], p["ov_pitch"], p["x"], p["y"] = nw_, nh_, 4 * nw_, it.x, it.y
        tmp_off += pitch * groups
        tmp_off = (tmp_off + 255) // 256 * 256
        max_out_w = max(max_out_w, nw_)
        max_rows = max(max_rows, rows)
        t_bytes = pitch * ((rows + 3) // 4)
        algo_h += 3 * hc * wc + t_bytes
        algo_v += t_bytes + 3 * bh * bw + 3 * bh * bw
        vb0 = (it.y // 16) * 16                      # overlay bands (ipp.h, ipp_pipe_vblend_bands)
        vb1 = max(vb0, min(bh, -(-(it.y + nh_) // 16) * 16))
        copy_rows += bh - (vb1 - vb0)
    # Processing order: group items by background so that the items pasting
    # onto one background run back to back (and, through the XCD-aware block
    # mapping, on one XCD): the 3 MB background then stays in L2/L3 instead of
    # being re-read from HBM per item.  Outputs keep their item offsets.
    order = np.argsort(np.array([it.bg_index for it in params]), kind="stable")
    d = d[order]
    hsv = G.hsv_params(cfg.hsv_ranges, cfg.zones, cfg.use_gimp_scale, bgr=False)
    copy_bytes = 2 * 3 * bw * copy_rows           # read + write of the rows outside the bands
    return PipePlan(d, coefs, hsv, params, cut_dims, ov_dims, max(tmp_off, 256), max_out_w, max_rows, bw, bh,
                    algo_h, algo_v, N.IPP_TAPS_MFMA,
                    max(w for _, w in ov_dims), max(h for h, _ in ov_dims),
                    algo_h + copy_bytes, algo_v - copy_bytes)


class PipeRunner:
    """Device-resident plan + scratch for repeated runs of one batch."""

    def __init__(self, plan: PipePlan, device):
        self.plan = plan
        self.device = torch.device(device)
        self.descs = _to_dev(plan.descs, self.device)
        self.coefs = torch.from_numpy(plan.coefs).to(self.device)
        self.tmp = torch.empty(plan.tmp_bytes, dtype=torch.uint8, device=self.device)
        self.lib = N.load()
        nb = self.lib.ipp_pipe_sync_bytes(len(plan.descs), plan.bg_h, plan.max_ov_h)
        if nb < 0:
            raise N.NativeError(f"ipp_pipe_sync_bytes({len(plan.descs)}, {plan.bg_h}, {plan.max_ov_h}) failed")
        self.sync = torch.empty(max(int(nb), 4), dtype=torch.uint8, device=self.device)

    def hpass(self, src: torch.Tensor) -> None:
        p = self.plan
        N.check(self.lib.ipp_pipe_hpass(src.data_ptr(), self.tmp.data_ptr(), self.coefs.data_ptr(),
                                        self.descs.data_ptr(), len(p.descs), p.max_out_w, p.max_rows, 3,
                                        N.np_ptr(p.hsv), p.tap_format, _stream(self.device)), "ipp_pipe_hpass")

    def vblend(self, bgs: torch.Tensor, out: torch.Tensor) -> None:
        p = self.plan
        N.check(self.lib.ipp_pipe_vblend(self.tmp.data_ptr(), bgs.data_ptr(), out.data_ptr(), self.coefs.data_ptr(),
                                         self.descs.data_ptr(), len(p.descs), p.bg_w, p.bg_h, p.max_ov_w,
                                         p.tap_format, _stream(self.device)), "ipp_pipe_vblend")

    def hpass_bgcopy(self, src: torch.Tensor, bgs: torch.Tensor, out: torch.Tensor) -> None:
        """H pass + the composite rows outside the overlay bands (split form)."""
        p = self.plan
        N.check(self.lib.ipp_pipe_hpass_bgcopy(src.data_ptr(), self.tmp.data_ptr(), self.coefs.data_ptr(),
                                               self.descs.data_ptr(), len(p.descs), p.max_out_w, p.max_rows, 3,
                                               N.np_ptr(p.hsv), p.tap_format, bgs.data_ptr(), out.data_ptr(),
                                               _stream(self.device)), "ipp_pipe_hpass_bgcopy")

    def vblend_bands(self, bgs: torch.Tensor, out: torch.Tensor) -> None:
        """V pass + paste over the 16-row bands the overlay touches (split form)."""
        p = self.plan
        N.check(self.lib.ipp_pipe_vblend_bands(self.tmp.data_ptr(), bgs.data_ptr(), out.data_ptr(),
                                               self.coefs.data_ptr(), self.descs.data_ptr(), len(p.descs), p.bg_w,
                                               p.bg_h, p.max_ov_w, p.max_ov_h, p.tap_format,
                                               _stream(self.device)), "ipp_pipe_vblend_bands")

    def fused(self, src: torch.Tensor, bgs: torch.Tensor, out: torch.Tensor) -> None:
        """The whole pipe in one launch (+ the queued-band launch): H pass,
        background copy and V pass with paste (ipp_pipe_fused)."""
        p = self.plan
        N.check(self.lib.ipp_pipe_fused(src.data_ptr(), self.tmp.data_ptr(), self.coefs.data_ptr(),
                                        self.descs.data_ptr(), len(p.descs), p.max_out_w, p.max_rows, 3,
                                        N.np_ptr(p.hsv), p.tap_format, bgs.data_ptr(), out.data_ptr(), p.bg_w,
                                        p.bg_h, p.max_ov_w, p.max_ov_h, self.sync.data_ptr(),
                                        _stream(self.device)), "ipp_pipe_fused")

    def queued_bands(self) -> int:
        """Bands the last fused launch queued for its second launch (not
        ready when their block started).  Synchronises."""
        torch.cuda.synchronize(self.device)
        return int(self.sync[4 * len(self.plan.descs):4 * len(self.plan.descs) + 4].view(torch.int32).item())

    def status(self) -> int:
        """Sticky status of the pipe kernels since the last call (ipp_pipe_status;
        bit 0: an H tile's window exceeded the LDS ring).  Synchronises."""
        st = np.zeros(1, np.int32)
        N.check(self.lib.ipp_pipe_status(N.np_ptr(st), _stream(self.device)), "ipp_pipe_status")
        return int(st[0])

    @property
    def split(self) -> bool:
        return self.plan.tap_format == N.IPP_TAPS_MFMA

    def run(self, src: torch.Tensor, bgs: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        for t, name in ((src, "src"), (bgs, "bgs"), (out, "out")):
            if not (t.is_cuda and t.dtype == torch.uint8 and t.is_contiguous()):
                raise N.NativeUnavailable(f"PipeRunner.run: {name} must be a contiguous uint8 ROCm tensor")
        if self.split:
            self.fused(src, bgs, out)
        else:
            self.hpass(src)
            self.vblend(bgs, out)
        return out
