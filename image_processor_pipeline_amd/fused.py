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
device work is two launches for the whole batch (``ipp_pipe_hpass_bgcopy``,
``ipp_pipe_vblend_bands``).  Intermediate cut-outs never touch HBM.
"""
from __future__ import annotations

import math
import os
import random
import time
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
    descs: np.ndarray            # PIPE_DESC[n], processing order (grouped by background)
    axes: np.ndarray             # TAP_AXIS[2n]: H then V axis of each item (device tap planner)
    coef_words: int              # int32 size of the device tap buffer
    hsv: np.ndarray              # HSV_PARAMS
    items: np.ndarray            # PIPE_ITEM[n]: drawn parameters and geometry, item order
    sym_pool: Tuple[str, ...]    # items["sym"] indexes this pool
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
    # composite outside the overlay's 16-pixel groups of its bands moves with
    # the H pass.  Algorithmic bytes follow SURVEY §8(d)'s fixed blend formula
    # (the background read once per item, the composite written once);
    # copy_read_bytes is what the grouped copy actually loads (one background
    # per run of same-background items in a copy group, IPP_PT_COPY_READS).
    algo_bytes_hpass_bgcopy: int = 0
    algo_bytes_vblend_bands: int = 0
    copy_read_bytes: int = 0

    @property
    def params(self) -> List[ItemParams]:
        it = self.items
        return [ItemParams(float(a), self.sym_pool[s], int(b), float(r), int(x), int(y))
                for a, s, b, r, x, y in zip(it["angle"], it["sym"], it["bg_index"], it["ratio"], it["x"], it["y"])]

    @property
    def cut_dims(self) -> List[Tuple[int, int]]:
        """(h, w) of each item's cut-out M."""
        return list(zip(self.items["cut_h"].tolist(), self.items["cut_w"].tolist()))

    @property
    def ov_dims(self) -> List[Tuple[int, int]]:
        """(h, w) of each item's resized overlay."""
        return list(zip(self.items["ov_h"].tolist(), self.items["ov_w"].tolist()))


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


def plan_threads() -> int:
    """Host threads for the batch planner: the job's CPU share
    (OMP_NUM_THREADS when set, else the CPUs this process may run on)."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    if n <= 0:
        n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(n, 32))


_PLAN_ERRORS = {
    1: (NotImplementedError, "rotation canvas beyond Pillow's 16.16 fixed-point range (>32767 px)"),
    2: (NotImplementedError, "non-affine ScaleAffine table"),
    3: (ValueError, "degenerate overlay size"),
    4: (ValueError, "parameters do not fit the background (position, background index or symmetry)"),
    5: (ValueError, "LANCZOS downscale needs a tap window wider than the fused H pass's 512-column LDS ring; "
                    "use the plugin path"),
    6: (ValueError, "empty range for randrange() (overlay larger than the background)"),
}


def plan_pipe(src_hw: Tuple[int, int], n: int, bg_hw: Tuple[int, int], n_bg: int, cfg: PipeConfig,
              seed: int = 0, src_pitch: Optional[int] = None, item_range: Optional[Tuple[int, int]] = None,
              n_global: Optional[int] = None, params: Optional[Sequence[ItemParams]] = None,
              n_threads: int = 0) -> PipePlan:
    """Plan `n` items.  The random stream is the one a chained file-mode
    ``ProcessingPipeline`` of the five reference steps over ``n_global``
    sources would consume under ``random.seed(seed)`` (``draw_params``).
    With ``item_range=(start, stop)`` only items [start, stop) of that global
    batch are planned (stop - start must equal n): every rank of a sharded run
    sees exactly the parameters a single process would give those items, so
    outputs do not depend on the number of GPUs.  ``n_global`` defaults to
    ``stop``.  With ``params`` (one ItemParams per item) nothing is drawn:
    the caller's angles, symmetries, backgrounds, ratios and positions are
    planned as given (positions must keep the overlay inside the background).

    The whole plan is one call of the threaded C planner
    (``ipp_plan_pipe_batch``: CPython's MT19937 draws, Pillow's rotate
    geometry, the opaque getbbox, the overlay size, the descriptors); the
    LANCZOS taps are built later on the device (``PipeRunner``)."""
    H, W = src_hw
    bh, bw = bg_hw
    start, stop = item_range if item_range is not None else (0, n)
    if stop - start != n or start < 0 or n <= 0:
        raise ValueError(f"item_range {item_range} does not hold {n} items")
    n_global = stop if n_global is None else n_global
    if n_global < stop:
        raise ValueError(f"n_global {n_global} < item_range stop {stop}")
    t, b, l, r = G.crop_margins(H, W, cfg.margins)
    items = np.zeros(n, N.PIPE_ITEM)
    c = np.zeros((), N.PIPE_PLAN_CFG)
    pool = tuple(cfg.sym_pool)
    given = params
    if given is None and not (isinstance(seed, int) and abs(seed) < 1 << 64):
        # seeds the C generator does not take (floats, strings, > 64 bits):
        # draw in Python, plan the draws as given parameters
        angles, syms, order, drawn = draw_params(n_global, stop, src_hw, bg_hw, n_bg, cfg, seed)
        given = [ItemParams(angles[g], syms[g], order[g % n_bg], drawn[g][0], drawn[g][1], drawn[g][2])
                 for g in range(start, stop)]
    if given is not None:
        if len(given) != n:
            raise ValueError(f"{len(given)} ItemParams for {n} items")
        pool = ALL_SYMS
        for i, it in enumerate(given):
            if it.sym not in SYM_FLIP:
                raise ValueError(f"item {start + i}: parameters {it} do not fit a {bw}x{bh} background")
        items["angle"] = [it.angle for it in given]
        items["ratio"] = [it.ratio for it in given]
        items["sym"] = [ALL_SYMS.index(it.sym) for it in given]
        items["bg_index"] = [it.bg_index for it in given]
        items["x"] = [it.x for it in given]
        items["y"] = [it.y for it in given]
        c["given"] = 1
    else:
        if not 1 <= len(pool) <= 4 or any(p not in SYM_FLIP for p in pool):
            raise ValueError(f"symmetry pool {pool}: 1 to 4 of {ALL_SYMS}")
        c["seed"] = abs(seed)
    c["src_h"], c["src_w"], c["src_pitch"] = H, W, src_pitch or 0
    c["crop_t"], c["crop_b"], c["crop_l"], c["crop_r"] = t, b, l, r
    c["bg_h"], c["bg_w"], c["n_bg"] = bh, bw, n_bg
    c["n_sym"] = len(pool)
    c["sym_flip"][:len(pool)] = [SYM_FLIP[p] for p in pool]
    c["n_global"], c["start"], c["stop"] = n_global, start, stop
    c["angle_min"], c["angle_max"] = cfg.angle_min, cfg.angle_max
    c["scale_min"], c["scale_max"] = cfg.scale_min, cfg.scale_max
    c["n_threads"] = n_threads or plan_threads()
    c["ring_cols"] = H_RING_COLUMNS
    descs = np.zeros(n, N.PIPE_DESC)
    axes = np.zeros(2 * n, N.TAP_AXIS)
    tot = np.zeros(N.IPP_PLAN_TOTALS, np.int64)
    lib = N.load()
    rc = lib.ipp_plan_pipe_batch(N.np_ptr(c), N.np_ptr(items), N.np_ptr(descs), N.np_ptr(axes), N.np_ptr(tot))
    if rc == N.IPP_E_RANGE and int(tot[N.PT["err_code"]]) in _PLAN_ERRORS:
        exc, msg = _PLAN_ERRORS[int(tot[N.PT["err_code"]])]
        raise exc(f"item {int(tot[N.PT['err_item']])}: {msg}")
    N.check(rc, "ipp_plan_pipe_batch")
    T = {k: int(tot[v]) for k, v in N.PT.items()}
    if T["max_ov_w"] > N.IPP_PIPE_MAX_OV_W:
        # refused here, before either launch: the V launch holds an overlay's
        # 16 rows in 64 KB of LDS (ipp.h IPP_PIPE_MAX_OV_W)
        raise ValueError(f"overlay width {T['max_ov_w']} px exceeds the fused pipe's limit of "
                         f"{N.IPP_PIPE_MAX_OV_W} px (ipp_pipe_vblend_bands); use the file-mode plugins")
    hsv = G.hsv_params(cfg.hsv_ranges, cfg.zones, cfg.use_gimp_scale, bgr=False)
    return PipePlan(descs, axes, T["coef_words"], hsv, items, pool, T["tmp_bytes"], T["max_out_w"], T["max_rows"],
                    bw, bh, T["algo_h"], T["algo_v"], N.IPP_TAPS_MFMA, T["max_ov_w"], T["max_ov_h"],
                    T["algo_h"] + T["copy_bytes"], T["algo_v"] - T["copy_bytes"], T["copy_reads"])


def plan_taps(plan: PipePlan, device, stream=None) -> Tuple[torch.Tensor, int]:
    """The plan's LANCZOS taps, built on the device (ipp_pipe_plan_taps):
    returns (int32 tensor of plan.coef_words (+ slack), tiles rebuilt on the
    host).  Synchronises the stream."""
    lib = N.load()
    device = torch.device(device)
    coefs = torch.empty(plan.coef_words + 4096, dtype=torch.int32, device=device)
    nb = lib.ipp_pipe_taps_scratch_bytes(len(plan.axes))
    scratch = torch.empty(int(nb), dtype=torch.uint8, device=device)
    stats = np.zeros(2, np.int64)
    N.check(lib.ipp_pipe_plan_taps(N.np_ptr(plan.axes), len(plan.axes), coefs.data_ptr(), scratch.data_ptr(),
                                   N.np_ptr(stats), stream if stream is not None else _stream(device)),
            "ipp_pipe_plan_taps")
    if stats[1]:
        raise N.NativeError(f"ipp_pipe_plan_taps: device status {int(stats[1])} (tile beyond its K-step bound)")
    return coefs, int(stats[0])


def overlap_bounds(n: int, parts: int, ratio: float = 1.0, group: int = N.IPP_PIPE_COPY_GROUP) -> List[int]:
    """Item-range bounds of PipeRunner.run_overlapped: `parts` ranges of whole
    copy groups, range k holding a share proportional to ratio**k; bounds[0]
    = 0, bounds[-1] = n, non-decreasing (a range may be empty)."""
    if n < 0 or parts < 1 or ratio <= 0:
        raise ValueError(f"overlap_bounds: n={n} parts={parts} ratio={ratio}")
    groups = (n + group - 1) // group
    w = [ratio ** k for k in range(parts)]
    cum = [sum(w[:k]) / sum(w) for k in range(parts + 1)]
    b = [min(n, group * int(round(groups * c))) for c in cum]
    b[-1] = n
    return b


class PipeRunner:
    """Device-resident plan + scratch for repeated runs of one batch."""

    def __init__(self, plan: PipePlan, device):
        self.plan = plan
        self.device = torch.device(device)
        self.descs = _to_dev(plan.descs, self.device)
        self.coefs, self.host_tiles = plan_taps(plan, self.device)
        self.tmp = torch.empty(plan.tmp_bytes, dtype=torch.uint8, device=self.device)
        self.lib = N.load()

    def hpass_bgcopy(self, src: torch.Tensor, bgs: torch.Tensor, out: torch.Tensor, items=None) -> None:
        """H pass + the composite rows outside the overlay bands (split form);
        `items` = (first, count) of the descriptors in processing order."""
        p = self.plan
        i0, n = items if items is not None else (0, len(p.descs))
        N.check(self.lib.ipp_pipe_hpass_bgcopy(src.data_ptr(), self.tmp.data_ptr(), self.coefs.data_ptr(),
                                               self.descs.data_ptr() + i0 * p.descs.itemsize, n, p.max_out_w,
                                               p.max_rows, 3, N.np_ptr(p.hsv), p.tap_format, bgs.data_ptr(),
                                               out.data_ptr(), _stream(self.device)), "ipp_pipe_hpass_bgcopy")

    def vblend_bands(self, bgs: torch.Tensor, out: torch.Tensor, items=None) -> None:
        """V pass + paste over the 16-row bands the overlay touches (split form)."""
        p = self.plan
        i0, n = items if items is not None else (0, len(p.descs))
        N.check(self.lib.ipp_pipe_vblend_bands(self.tmp.data_ptr(), bgs.data_ptr(), out.data_ptr(),
                                               self.coefs.data_ptr(), self.descs.data_ptr() + i0 * p.descs.itemsize,
                                               n, p.bg_w, p.bg_h, p.max_ov_w, p.max_ov_h, p.tap_format,
                                               _stream(self.device)), "ipp_pipe_vblend_bands")

    def run_overlapped(self, src: torch.Tensor, bgs: torch.Tensor, out: torch.Tensor, parts: int,
                       ratio: float = 1.0) -> None:
        """The batch in `parts` consecutive item ranges: the H launch of range k+1
        runs on the caller's stream while the V launch of range k runs on a
        side stream (event-ordered after its own H launch), so the V pass's
        HBM streaming overlaps the texture-bound H pass.  The ranges are whole
        copy groups of the H launch; the caller's stream waits for the last V
        launch."""
        bounds = overlap_bounds(len(self.plan.descs), parts, ratio)
        main = torch.cuda.current_stream(self.device)
        if getattr(self, "_vstream", None) is None:
            self._vstream = torch.cuda.Stream(self.device)
            self._events = []
        side = self._vstream
        while len(self._events) < parts:
            self._events.append(torch.cuda.Event())
        side.wait_stream(main)  # inputs and tmp reuse ordered after the caller's work
        for k in range(parts):
            i0, i1 = bounds[k], bounds[k + 1]
            if i1 <= i0:
                continue
            self.hpass_bgcopy(src, bgs, out, items=(i0, i1 - i0))
            ev = self._events[k]
            ev.record(main)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                self.vblend_bands(bgs, out, items=(i0, i1 - i0))
        main.wait_stream(side)

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
        if not self.split:
            raise N.NativeError(f"PipeRunner.run: tap format {self.plan.tap_format} (the pipe takes IPP_TAPS_MFMA)")
        self.hpass_bgcopy(src, bgs, out)
        self.vblend_bands(bgs, out)
        return out


class PipeStream:
    """Streaming form of PipeRunner (bench.py --stream): every batch has its
    own plan, built while earlier batches run.  Worker threads run the host
    plans (ipp_plan_pipe_batch; ctypes drops the GIL) and device taps
    (ipp_pipe_plan_taps, one side stream per slot) of batches k+1 ..
    k+lookahead while batch k's two launches run on the pipe stream.  Device
    buffers live in `slots` (≥ lookahead + 1) sets used in turn; a set is
    refilled only after the batch that last used it has completed (its HIP
    event)."""

    def __init__(self, device, plan_fn, slots: int = 3, priority: bool = True, lookahead: int = 2):
        self.device = torch.device(device)
        self.plan_fn = plan_fn                  # batch index -> PipePlan
        self.lib = N.load()
        # batches k+1 .. k+lookahead are being planned while batch k runs
        # (each on its own worker thread and side stream): the tap planner of
        # one batch then has `lookahead` batch times to get its share of the
        # GPU beside the pipe
        self.lookahead = max(1, int(lookahead))
        slots = max(slots, self.lookahead + 1)
        # The pipe launches go to a high-priority stream (the hardware queue
        # dispatches its blocks first): the tap planner of the next batch, on
        # the default-priority side stream, then fills the CU slots the pipe
        # leaves free instead of displacing H-pass blocks.
        self.main = torch.cuda.Stream(self.device, priority=-1) if priority else None
        self.slots = [{"done": torch.cuda.Event(), "bufs": {}, "side": torch.cuda.Stream(self.device)}
                      for _ in range(max(2, slots))]
        self.timing: List[Tuple[float, float, int]] = []   # per batch: host plan ms, taps ms, host tiles
        self.events: List[Tuple[torch.cuda.Event, torch.cuda.Event]] = []

    def _buf(self, slot, name: str, nbytes: int) -> torch.Tensor:
        b = slot["bufs"].get(name)
        if b is None or b.numel() < nbytes:
            slot["bufs"][name] = None
            b = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.device)
            slot["bufs"][name] = b
        return b

    def _prepare(self, k: int, slot):
        t0 = time.perf_counter()
        plan = self.plan_fn(k)
        t1 = time.perf_counter()
        slot["done"].synchronize()              # the batch that used these buffers has finished
        bufs = {"descs": self._buf(slot, "descs", plan.descs.nbytes),
                "coefs": self._buf(slot, "coefs", 4 * (plan.coef_words + 4096)),
                "tmp": self._buf(slot, "tmp", plan.tmp_bytes),
                "scratch": self._buf(slot, "scratch", self.lib.ipp_pipe_taps_scratch_bytes(len(plan.axes)))}
        stats = np.zeros(2, np.int64)
        side = slot["side"]
        with torch.cuda.stream(side):
            bufs["descs"][:plan.descs.nbytes].copy_(torch.from_numpy(plan.descs.view(np.uint8)))
            N.check(self.lib.ipp_pipe_plan_taps(N.np_ptr(plan.axes), len(plan.axes), bufs["coefs"].data_ptr(),
                                                bufs["scratch"].data_ptr(), N.np_ptr(stats),
                                                side.cuda_stream), "ipp_pipe_plan_taps")
        if stats[1]:
            raise N.NativeError(f"ipp_pipe_plan_taps: device status {int(stats[1])}")
        t2 = time.perf_counter()
        return plan, bufs, ((t1 - t0) * 1e3, (t2 - t1) * 1e3, int(stats[0]))

    def run(self, n_batches: int, src: torch.Tensor, bgs: torch.Tensor, out: torch.Tensor, mark=None,
            record: bool = False) -> None:
        """Run batches 0 .. n_batches-1 (plan_fn(k) plans batch k).  `mark`
        (optional callable) is called right before batch `mark.at` is
        launched, with the pipeline primed (its plan ready, the following
        lookahead-1 plans in flight) — bench.py starts its clock there."""
        from concurrent.futures import ThreadPoolExecutor
        main = self.main if self.main is not None else torch.cuda.current_stream(self.device)
        if self.main is not None:
            self.main.wait_stream(torch.cuda.current_stream(self.device))  # inputs written on the caller's stream
        L, ns = self.lookahead, len(self.slots)
        with ThreadPoolExecutor(L) as ex:
            futs = {j: ex.submit(self._prepare, j, self.slots[j % ns]) for j in range(min(L, n_batches))}
            for k in range(n_batches):
                plan, b, tm = futs.pop(k).result()
                if mark is not None and k == mark.at:
                    mark()
                slot = self.slots[k % ns]
                if k + L < n_batches:
                    # its slot was last used by batch k + L - ns <= k - 1, whose
                    # completion event is already recorded
                    futs[k + L] = ex.submit(self._prepare, k + L, self.slots[(k + L) % ns])
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if record else None
                if ev:
                    ev[0].record(main)
                N.check(self.lib.ipp_pipe_hpass_bgcopy(src.data_ptr(), b["tmp"].data_ptr(), b["coefs"].data_ptr(),
                                                       b["descs"].data_ptr(), len(plan.descs), plan.max_out_w,
                                                       plan.max_rows, 3, N.np_ptr(plan.hsv), plan.tap_format,
                                                       bgs.data_ptr(), out.data_ptr(), main.cuda_stream),
                        "ipp_pipe_hpass_bgcopy")
                N.check(self.lib.ipp_pipe_vblend_bands(b["tmp"].data_ptr(), bgs.data_ptr(), out.data_ptr(),
                                                       b["coefs"].data_ptr(), b["descs"].data_ptr(),
                                                       len(plan.descs), plan.bg_w, plan.bg_h, plan.max_ov_w,
                                                       plan.max_ov_h, plan.tap_format, main.cuda_stream),
                        "ipp_pipe_vblend_bands")
                if ev:
                    ev[1].record(main)
                    self.events.append(ev)
                slot["done"].record(main)
                self.timing.append(tm)
        if self.main is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.main)  # outputs visible to the caller's stream
