"""GPU parity: the HIP C-ABI kernels vs the CPU oracle / Pillow goldens.

Bit-exact for every op (integer/byte work).  Sizes are chosen so the oracle
finishes in seconds; full-size configs are covered through a few items at
1024² plus size-independent properties.
"""
import random

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import ops
from oracle import pipe as opipe
from tests.conftest import unpack

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def D():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from image_processor_pipeline_amd import device
    return device


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


# --------------------------------------------------------------------------- rotate

def test_rotate_crop_matches_pillow_goldens(D, golden):
    g = golden("rotate_pillow.npz")
    srcs = unpack(g["src_flat"], g["src_shapes"])
    outs = unpack(g["out_flat"], g["out_shapes"])
    for out, si, a, bb in zip(outs, g["src_index"], g["angles"], g["bboxes"]):
        src = srcs[si]
        exp = out if bb[0] < 0 else out[bb[1]:bb[3], bb[0]:bb[2]]
        if exp.shape[0] == 0 or exp.shape[1] == 0:
            exp = out
        got = D.rotate_crop_single(_t(src), float(a)).cpu().numpy()
        assert got.shape == exp.shape, (si, a)
        assert np.array_equal(got, exp), (si, a)


def test_rotations_reference_stream(D, golden):
    g = golden("rotations_ref.npz")
    outs = unpack(g["out_flat"], g["out_shapes"])
    random.seed(int(g["seed"]))
    for out in outs[1:]:
        a = random.uniform(1.0, 359.0)
        got = D.rotate_crop_single(_t(g["src"]), a).cpu().numpy()
        assert np.array_equal(got, out)


@pytest.mark.parametrize("shape", [(257, 300), (64, 64), (1, 7), (13, 2)])
def test_rotate_flip_batch_vs_oracle(D, shape):
    rng = np.random.default_rng(1)
    n = 12
    h, w = shape
    src = rng.integers(0, 256, (n, h, w, 3), np.uint8)
    angles = [0.0, 90.0, 180.0, 270.0] + [float(a) for a in rng.uniform(-720, 720, n - 4)]
    syms = [["o", "h", "v", "hv"][i % 4] for i in range(n)]
    flips = [D.SYM_FLIP[s] for s in syms]
    plan = D.plan_rotate_flip([(h, w, 3)] * n, angles, flips, src_offsets=[i * h * w * 3 for i in range(n)])
    buf = D.rotate_flip_nearest(_t(src).reshape(-1), plan)
    got = [v.cpu().numpy() for v in D.unpack(buf, plan)]
    for i in range(n):
        exp = ops.flip(ops.rotate_and_crop(ops.to_rgba(src[i]), angles[i]), syms[i])
        assert np.array_equal(got[i], exp), (i, angles[i], syms[i])


def test_rotate_flip_unprepared_descriptors_match(D):
    """Descriptors without the host-precomputed sampler (prepared = 0, the
    kernel computes it per block) give the same bytes as prepared ones
    (ipp_gather_prepare), margin windows and every flip included."""
    rng = np.random.default_rng(9)
    n, h, w = 8, 97, 131
    src = rng.integers(0, 256, (n, h, w, 3), np.uint8)
    angles = [float(a) for a in rng.uniform(-360, 360, n)]
    flips = [i % 4 for i in range(n)]
    wins = [(3 * i % 7, i % 5, w - 11, h - 9) for i in range(n)]
    plan = D.plan_rotate_flip([(h, w, 3)] * n, angles, flips, windows=wins, src_offsets=[i * h * w * 3 for i in range(n)])
    assert (plan.descs["prepared"] == 1).all()
    a = D.rotate_flip_nearest(_t(src).reshape(-1), plan).cpu().numpy()
    plan.descs["prepared"] = 0
    plan.descs["b"] = 0          # (garbage the kernel must not read)
    b = D.rotate_flip_nearest(_t(src).reshape(-1), plan).cpu().numpy()
    assert np.array_equal(a, b)


def test_rotate_with_margin_window(D):
    rng = np.random.default_rng(2)
    h, w = 120, 90
    src = rng.integers(0, 256, (h, w, 3), np.uint8)
    margins = (0.1, 5, 7, 0.25)
    crop = ops.crop_from_border(src, margins)
    t = ops.compute_crop(margins[0], h)
    l = ops.compute_crop(margins[2], w)
    plan = D.plan_rotate_flip([(h, w, 3)], [33.3], [3], windows=[(l, t, crop.shape[1], crop.shape[0])])
    got = D.unpack(D.rotate_flip_nearest(_t(src).reshape(-1), plan), plan)[0].cpu().numpy()
    exp = ops.flip(ops.rotate_and_crop(ops.to_rgba(crop), 33.3), "hv")
    assert np.array_equal(got, exp)


def test_rgba_source_alpha_bbox_path(D):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (50, 70, 4), np.uint8)
    img[..., 3] = 0
    img[10:30, 20:45, 3] = rng.integers(1, 256, (20, 25))
    for a in (17.0, 90.0, 200.5):
        got = D.rotate_crop_single(_t(img), a).cpu().numpy()
        assert np.array_equal(got, ops.rotate_and_crop(img, a)), a
    empty = np.zeros((9, 11, 4), np.uint8)
    got = D.rotate_crop_single(_t(empty), 45.0).cpu().numpy()
    assert np.array_equal(got, ops.rotate_and_crop(empty, 45.0))


# --------------------------------------------------------------------------- flip / crop

@pytest.mark.parametrize("cn", [1, 3, 4])
def test_flip_and_window(D, cn):
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (37, 29, cn), np.uint8)
    for s in ("o", "h", "v", "hv"):
        assert np.array_equal(D.flip(_t(img), s).cpu().numpy(), ops.flip(img, s))
    got = D.copy_window(_t(img), (3, 5, 20, 11)).cpu().numpy()
    assert np.array_equal(got, img[5:16, 3:23])


# --------------------------------------------------------------------------- HSV

def test_hsv_mask_vs_oracle(D):
    from image_processor_pipeline_amd import geometry as G
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (123, 77, 3), np.uint8)
    img[:10] = 0
    img[10:20, :, :] = img[10:20, :, :1]  # greys
    cases = [
        (G.REFERENCE_HSV_RANGES, None, False),
        ([(20, 100, 180, 40, 255, 255), (0, 0, 0, 180, 50, 100)], [(5, 10, 3, 7), None], False),
        ([(30, 20, 30, 90, 80, 90), (300, 10, 10, 360, 100, 60)], [(0, 0, 0, 0), (-5, 200, 10, -3)], True),
        ([(50, 0, 0, 10, 255, 255), (0, 0, 0, 180, 255, 255)], None, False),   # first empty
    ]
    for ranges, zones, gimp in cases:
        p = G.hsv_params(ranges, zones, gimp, bgr=True)
        got = D.hsv_mask(_t(img), p).cpu().numpy()
        exp = ops.color_mask_bgra(img, ranges, zones, gimp)
        assert np.array_equal(got, exp), (ranges, zones, gimp)


def test_hsv_all_pixel_values(D):
    """Exhaustive-ish: every (b, g, r) on a 4096×1024 lattice of 8-bit values."""
    from image_processor_pipeline_amd import geometry as G
    v = np.arange(256, dtype=np.uint8)
    b, g = np.meshgrid(v, v, indexing="ij")
    img = np.stack([b.ravel(), g.ravel(), np.zeros(65536, np.uint8)], -1)
    img = np.concatenate([img.copy() for _ in range(16)])
    img[:, 2] = np.repeat(np.arange(0, 256, 16, dtype=np.uint8), 65536)
    img = img.reshape(1024, 1024, 3)
    ranges = [(0, 0, 0, 180, 255, 150), (15, 60, 200, 35, 255, 255), (100, 3, 9, 170, 254, 254)]
    p = G.hsv_params(ranges, None, False, bgr=True)
    got = D.hsv_mask(_t(img), p).cpu().numpy()
    exp = ops.color_mask_bgra(img, ranges)
    assert np.array_equal(got, exp)


# --------------------------------------------------------------------------- LANCZOS / paste

def test_resize_matches_pillow_goldens(D, golden):
    g = golden("resize_pillow.npz")
    srcs = unpack(g["src_flat"], g["src_shapes"])
    outs = unpack(g["out_flat"], g["out_shapes"])
    for s, o, (ow, oh) in zip(srcs, outs, g["sizes"]):
        got = D.resize_lanczos_rgba(_t(s), int(ow), int(oh)).cpu().numpy()
        assert np.array_equal(got, o), (s.shape, ow, oh)


def test_resize_vs_oracle_random(D):
    rng = np.random.default_rng(6)
    for (h, w), (oh, ow) in [((300, 411), (61, 87)), ((97, 33), (211, 400)), ((512, 512), (100, 512))]:
        s = rng.integers(0, 256, (h, w, 4), np.uint8)
        s[..., 3] = np.where(rng.random((h, w)) < 0.5, 255, s[..., 3])
        got = D.resize_lanczos_rgba(_t(s), ow, oh).cpu().numpy()
        assert np.array_equal(got, ops.resize_lanczos_rgba(s, ow, oh))


def test_paste_matches_pillow_goldens(D, golden):
    g = golden("paste_pillow.npz")
    for (x, y), out in zip(g["pos"], g["outs"]):
        got = D.paste_blend(_t(g["bg"]), _t(g["ov"]), int(x), int(y)).cpu().numpy()
        assert np.array_equal(got, out[..., :3])


def test_overlay_reference_chain(D, golden):
    from image_processor_pipeline_amd import geometry as G
    g = golden("overlays_ref.npz")
    ovs = unpack(g["ov_flat"], g["ov_shapes"])
    bgs = unpack(g["bg_flat"], g["bg_shapes"])
    comps = unpack(g["comp_flat"], g["comp_shapes"])
    for ov, bg, comp, seed in zip(ovs, bgs, comps, g["seeds"]):
        random.seed(int(seed))
        ratio = random.uniform(0.15, 0.30)
        bh, bw = bg.shape[:2]
        nw, nh = G.overlay_size(ov.shape[1], ov.shape[0], bw, bh, ratio)
        x = random.randint(0, bw - nw)
        y = random.randint(0, bh - nh)
        rs = D.resize_lanczos_rgba(_t(ov), nw, nh)
        got = D.paste_blend(_t(bg), rs, x, y).cpu().numpy()
        assert np.array_equal(got, comp)


# --------------------------------------------------------------------------- batched pipe

def _run_pipe(n, H, W, K, bh, bw, cfg, seed):
    from image_processor_pipeline_amd import fused
    rng = np.random.default_rng(seed)
    src = rng.integers(0, 256, (n, H, W, 3), np.uint8)
    bgs = rng.integers(0, 256, (K, bh, bw, 3), np.uint8)
    plan = fused.plan_pipe((H, W), n, (bh, bw), K, cfg, seed=seed)
    runner = fused.PipeRunner(plan, DEV)
    out = torch.empty((n, bh, bw, 3), dtype=torch.uint8, device=DEV)
    runner.run(_t(src), _t(bgs), out)
    return src, bgs, plan, out.cpu().numpy()


def test_pipe_small_vs_oracle(D):
    from image_processor_pipeline_amd import fused
    cfg = fused.PipeConfig(margins=(0.05, 9, 0.1, 3))
    src, bgs, plan, got = _run_pipe(10, 150, 170, 3, 128, 160, cfg, seed=7)
    for i in range(len(got)):
        exp = opipe.pipe_item(src[i], bgs, plan.params[i], cfg)
        assert np.array_equal(got[i], exp), i


def test_pipe_full_width_crop_vs_oracle(D):
    """A crop that keeps the source's full width but not its last rows
    (margins top 3, bottom 5, left/right 0) on a dense source: pitch = 3·in_w,
    so the gather of pixel (0, in_h) would start inside the window's buffer
    records — these blocks must keep the row test (ipp_pipe.hip yr_range_ok;
    round-5 advisor finding).  Random source bytes: a real pixel sampled
    below the window in place of black would break parity."""
    from image_processor_pipeline_amd import fused
    cfg = fused.PipeConfig(margins=(3, 5, 0, 0))
    src, bgs, plan, got = _run_pipe(12, 150, 170, 3, 128, 160, cfg, seed=31)
    for i in range(len(got)):
        exp = opipe.pipe_item(src[i], bgs, plan.params[i], cfg)
        assert np.array_equal(got[i], exp), i


def test_pipe_structured_content_vs_oracle(D):
    """Content that exercises the HSV ranges (dark/yellow/grey regions)."""
    from image_processor_pipeline_amd import fused
    cfg = fused.PipeConfig(margins=(4, 4, 4, 4), zones=[None, (10, 0, 0, 5), None, (0, 0, 20, 0)])
    n, H, W = 6, 140, 120
    rng = np.random.default_rng(8)
    src = np.zeros((n, H, W, 3), np.uint8)
    src[:, :, :40] = (230, 200, 40)           # yellow (RGB)
    src[:, :, 40:80] = (20, 20, 20)           # dark
    src[:, :, 80:] = rng.integers(0, 256, (n, H, 40, 3))
    bgs = rng.integers(0, 256, (2, 96, 128, 3), np.uint8)
    plan = fused.plan_pipe((H, W), n, (96, 128), 2, cfg, seed=8)
    runner = fused.PipeRunner(plan, DEV)
    out = torch.empty((n, 96, 128, 3), dtype=torch.uint8, device=DEV)
    runner.run(_t(src), _t(bgs), out)
    got = out.cpu().numpy()
    for i in range(n):
        assert np.array_equal(got[i], opipe.pipe_item(src[i], bgs, plan.params[i], cfg)), i


def test_pipe_odd_background_widths_vs_oracle(D):
    """ipp_pipe_hpass_bgcopy + ipp_pipe_vblend_bands on backgrounds whose row
    bytes are not a multiple of 16 (the row-wise copy and blend paths) and on
    aligned ones, output buffers pre-filled with junk: every composite byte
    is written, and equals the oracle."""
    from image_processor_pipeline_amd import fused
    cfg = fused.PipeConfig(margins=(3, 5, 2, 7), scale_min=0.2, scale_max=0.6)
    for (bh, bw) in [(97, 125), (64, 96)]:
        n, H, W = 8, 90, 110
        rng = np.random.default_rng(bw)
        src = rng.integers(0, 256, (n, H, W, 3), np.uint8)
        bgs = rng.integers(0, 256, (3, bh, bw, 3), np.uint8)
        plan = fused.plan_pipe((H, W), n, (bh, bw), 3, cfg, seed=bw)
        runner = fused.PipeRunner(plan, DEV)
        assert runner.split
        a = torch.full((n, bh, bw, 3), 7, dtype=torch.uint8, device=DEV)
        runner.hpass_bgcopy(_t(src), _t(bgs), a)
        runner.vblend_bands(_t(bgs), a)
        torch.cuda.synchronize()
        got = a.cpu().numpy()
        for i in range(n):
            assert np.array_equal(got[i], opipe.pipe_item(src[i], bgs, plan.params[i], cfg)), (bw, i)


def test_pipe_copy_groups_straddling_backgrounds(D):
    """The H launch's grouped background copy (ipp_pipe.hip bg_copy_group,
    IPP_PIPE_COPY_GROUP = 8 items per group): 21 items on 4 backgrounds in
    background-sorted runs of 5-6 items, so groups straddle background
    changes and the last group holds 5 items; 16-px-multiple background widths
    (the column split of the band rows) and one that is not; outputs
    pre-filled with junk, every composite byte equal to the oracle's."""
    from image_processor_pipeline_amd import fused
    cfg = fused.PipeConfig(margins=(3, 5, 2, 7), scale_min=0.2, scale_max=0.6)
    for (bh, bw) in [(70, 256), (66, 200), (40, 125)]:
        n, K, H, W = 21, 4, 90, 110
        rng = np.random.default_rng(bh + bw)
        src = rng.integers(0, 256, (n, H, W, 3), np.uint8)
        bgs = rng.integers(0, 256, (K, bh, bw, 3), np.uint8)
        plan = fused.plan_pipe((H, W), n, (bh, bw), K, cfg, seed=bw)
        runs = np.bincount(plan.items["bg_index"], minlength=K)
        assert sorted(runs) == [5, 5, 5, 6], runs
        assert any(e % 8 for e in np.cumsum(runs)[:-1])  # a group of 8 straddles a background change
        runner = fused.PipeRunner(plan, DEV)
        a = torch.full((n, bh, bw, 3), 7, dtype=torch.uint8, device=DEV)
        runner.hpass_bgcopy(_t(src), _t(bgs), a)
        runner.vblend_bands(_t(bgs), a)
        torch.cuda.synchronize()
        got = a.cpu().numpy()
        for i in range(n):
            assert np.array_equal(got[i], opipe.pipe_item(src[i], bgs, plan.params[i], cfg)), (bw, i)


def test_pipe_wide_overlays_vs_oracle(D):
    """Overlays wider than 560 px (the V pass's overlay rows take most of its
    64 KB of LDS) on an 800-px background."""
    from image_processor_pipeline_amd import fused
    cfg = fused.PipeConfig(margins=(4, 4, 4, 4), scale_min=0.75, scale_max=0.8)
    n, H, W, bh, bw = 2, 300, 260, 760, 800
    rng = np.random.default_rng(11)
    src = rng.integers(0, 256, (n, H, W, 3), np.uint8)
    bgs = rng.integers(0, 256, (2, bh, bw, 3), np.uint8)
    plan = fused.plan_pipe((H, W), n, (bh, bw), 2, cfg, seed=4)
    assert plan.max_ov_w > 560
    runner = fused.PipeRunner(plan, DEV)
    a = torch.full((n, bh, bw, 3), 7, dtype=torch.uint8, device=DEV)
    runner.run(_t(src), _t(bgs), a)
    got = a.cpu().numpy()
    for i in range(n):
        assert np.array_equal(got[i], opipe.pipe_item(src[i], bgs, plan.params[i], cfg)), i


def test_pipe_stream_equals_runner(D):
    """fused.PipeStream (the bench's streaming leg) on a high-priority and on
    the default-priority stream: every batch has its own plan; the last
    batch's output equals a PipeRunner run of the same plan."""
    from image_processor_pipeline_amd import fused
    cfg = fused.PipeConfig(margins=(3, 5, 2, 7), scale_min=0.2, scale_max=0.6)
    n, H, W, bh, bw = 6, 90, 110, 120, 160
    rng = np.random.default_rng(21)
    src = _t(rng.integers(0, 256, (n, H, W, 3), np.uint8))
    bgs = _t(rng.integers(0, 256, (3, bh, bw, 3), np.uint8))
    plan_fn = lambda k: fused.plan_pipe((H, W), n, (bh, bw), 3, cfg, seed=100 + k)
    for prio in (True, False):
        out = torch.empty((n, bh, bw, 3), dtype=torch.uint8, device=DEV)
        fused.PipeStream(DEV, plan_fn, priority=prio).run(3, src, bgs, out, record=True)
        ref = torch.empty_like(out)
        fused.PipeRunner(plan_fn(2), DEV).run(src, bgs, ref)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), prio


def test_pipe_crop_reaching_source_end(D):
    """Zero bottom/right margins: the crop window ends at the source's last
    byte, so the last pixel's 4-byte gather would cross the image (and, for
    the last item, the allocation) end — the H pass takes its clamped path."""
    from image_processor_pipeline_amd import fused
    for margins in [(3, 0, 5, 0), (0, 0, 0, 0)]:
        cfg = fused.PipeConfig(margins=margins, scale_min=0.3, scale_max=0.7)
        src, bgs, plan, got = _run_pipe(5, 70, 90, 2, 80, 96, cfg, seed=21)
        for i in range(len(got)):
            assert np.array_equal(got[i], opipe.pipe_item(src[i], bgs, plan.params[i], cfg)), (margins, i)


def test_pipe_random_geometry_stress(D):
    """Many small items of random shapes, margins (zero margins included:
    the CLAMP path), angles and overlay ratios.  The H pass issues its source
    gathers by inline asm with hand-placed vmcnt waits (gather
    waits); a compiler copy of a register whose gather is still in flight would
    read stale bytes, which bit-exact comparisons on varied geometry expose."""
    from image_processor_pipeline_amd import fused
    rng = np.random.default_rng(77)
    for trial in range(6):
        H, W = int(rng.integers(40, 200)), int(rng.integers(40, 200))
        bh, bw = int(rng.integers(64, 160)), int(rng.integers(64, 160))
        m = [int(v) for v in rng.integers(0, 6, 4)]
        if trial % 2 == 0:
            m[1], m[3] = 0, 0
        cfg = fused.PipeConfig(margins=tuple(m), scale_min=0.3, scale_max=0.8)
        src, bgs, plan, got = _run_pipe(8, H, W, 2, bh, bw, cfg, seed=100 + trial)
        for i in range(len(got)):
            exp = opipe.pipe_item(src[i], bgs, plan.params[i], cfg)
            assert np.array_equal(got[i], exp), (trial, H, W, m, i, plan.params[i])


def test_pipe_edge_parameters_vs_oracle(D):
    """Explicit item parameters at the edges of their ranges: Pillow's
    right-angle fast paths (0/90/180/270 and their wraps) under every flip,
    overlays pasted flush with each background border, the smallest and the
    largest overlay ratios (the largest capped by the background height,
    overlays.py:106-126), and items sharing one background."""
    from image_processor_pipeline_amd import fused
    from image_processor_pipeline_amd import geometry as G
    cfg = fused.PipeConfig(margins=(6, 4, 2, 8))
    H, W, bh, bw, K = 96, 130, 120, 150, 2
    rng = np.random.default_rng(41)
    angles = [0.0, 90.0, 180.0, 270.0, 450.0, -90.0, 1.0, 359.0, 45.0, 135.0]
    syms = ["o", "h", "v", "hv", "hv", "v", "h", "o", "v", "h"]
    ratios = [0.05, 1.0, 0.5, 0.3, 0.9, 0.15, 0.7, 0.2, 1.0, 0.1]
    n = len(angles)
    src = rng.integers(0, 256, (n, H, W, 3), np.uint8)
    bgs = rng.integers(0, 256, (K, bh, bw, 3), np.uint8)
    params = []
    for i in range(n):
        p = fused.ItemParams(angle=angles[i], sym=syms[i], bg_index=i % K, ratio=ratios[i])
        mt, mb, ml, mr = G.crop_margins(H, W, cfg.margins)
        _, _, (nw, nh) = fused.item_geometry(W - ml - mr, H - mt - mb, angles[i], ratios[i], bw, bh, i)
        corner = i % 4  # flush with the left/top, right/top, left/bottom, right/bottom borders
        p.x = 0 if corner in (0, 2) else bw - nw
        p.y = 0 if corner in (0, 1) else bh - nh
        params.append(p)
    plan = fused.plan_pipe((H, W), n, (bh, bw), K, cfg, params=params)
    runner = fused.PipeRunner(plan, DEV)
    out = torch.empty((n, bh, bw, 3), dtype=torch.uint8, device=DEV)
    runner.run(_t(src), _t(bgs), out)
    got = out.cpu().numpy()
    for i in range(n):
        assert np.array_equal(got[i], opipe.pipe_item(src[i], bgs, plan.params[i], cfg)), (i, angles[i], syms[i])


def test_pipe_fullsize_items_vs_oracle(D):
    """BASELINE config 3 geometry (1024² sources, 64-px margins, 1024² bgs)."""
    from image_processor_pipeline_amd import fused
    cfg = fused.PipeConfig()
    src, bgs, plan, got = _run_pipe(3, 1024, 1024, 2, 1024, 1024, cfg, seed=11)
    for i in range(3):
        assert np.array_equal(got[i], opipe.pipe_item(src[i], bgs, plan.params[i], cfg)), i


# --------------------------------------------------------------------------- CCL

def test_keep_largest_component_vs_oracle(D):
    from image_processor_pipeline_amd import device_ccl
    rng = np.random.default_rng(9)
    imgs = []
    for (h, w) in [(64, 80), (101, 57), (33, 33), (7, 5)]:
        im = rng.integers(0, 256, (h, w, 4), np.uint8)
        im[..., 3] = np.where(rng.random((h, w)) < 0.45, rng.integers(0, 256, (h, w)), 0)
        imgs.append(im)
    blob = np.zeros((90, 120, 4), np.uint8)
    blob[..., :3] = 50
    blob[20:60, 30:90, 3] = 255
    blob[(rng.random((90, 120)) < 0.02), 3] = 200
    imgs.append(blob)
    tie = np.zeros((10, 12, 4), np.uint8)
    tie[1, 5, 3] = 9
    tie[0, 9, 3] = 9      # two single-pixel components of equal area
    imgs.append(tie)
    for im in imgs:
        got = device_ccl.keep_largest_component(_t(im)).cpu().numpy()
        exp = ops.keep_largest_component(im)
        assert np.array_equal(got, exp), im.shape


def _ccl_stress_masks(rng):
    """Foreground patterns for the bit-plane run labelling (64×64 tiles, lane =
    row): densities around the 8-connected percolation threshold, the maximum
    component count per tile (isolated pixels on the even grid: 1024 per
    tile, many LDS stats passes, mixed tiles in the emit), a serpentine that
    crosses every tile border many times (deep union-find chains), full rows
    (runs reaching column 63), equal-area components in different tiles (tie
    rule across tiles), and sizes off the tile grid."""
    out = []
    for (h, w), dens in [((130, 200), 0.3), ((129, 193), 0.42), ((200, 131), 0.6), ((64, 64), 0.5),
                         ((65, 127), 0.45)]:
        out.append(rng.random((h, w)) < dens)
    grid = np.zeros((128, 192), bool)
    grid[::2, ::2] = True
    grid[100, 101] = grid[101, 102] = True          # one 3-pixel component wins
    out.append(grid)
    snake = np.zeros((300, 260), bool)
    for c in range(0, 260, 3):
        snake[:, c] = True
        snake[0 if (c // 3) % 2 else 299, c:c + 3] = True
    snake[150, 1] = False                            # notch: still one component
    out.append(snake)
    full = np.zeros((70, 190), bool)
    full[3:9, :] = True
    full[40, 5:70] = True
    out.append(full)
    tie = np.zeros((140, 150), bool)
    tie[70:72, 100:103] = True                       # area 6, later block
    tie[5:7, 130:133] = True                         # area 6, first block: wins
    out.append(tie)
    for (h, w) in [(1, 1), (1, 77), (77, 1), (2, 65)]:
        out.append(rng.random((h, w)) < 0.6)
    return out


def test_keep_largest_component_stress(D):
    from image_processor_pipeline_amd import device_ccl
    rng = np.random.default_rng(31)
    for fg in _ccl_stress_masks(rng):
        if not fg.any():
            continue
        h, w = fg.shape
        im = rng.integers(0, 256, (h, w, 4), np.uint8)
        im[..., 3] = np.where(fg, rng.integers(2, 256, (h, w)), rng.integers(0, 2, (h, w)))
        got = device_ccl.keep_largest_component(_t(im)).cpu().numpy()
        exp = ops.keep_largest_component(im)
        assert np.array_equal(got, exp), (h, w)


def test_video_chain_noise_frames_vs_oracle(D):
    """Fused config-5 chain on frames whose HSV mask is dense noise (many
    components per tile, mixed tiles in the crop) and off-grid sizes."""
    from image_processor_pipeline_amd import geometry as G
    from image_processor_pipeline_amd.video_chain import VideoChain
    rng = np.random.default_rng(5)
    for (h, w, dens) in [(257, 389, 0.45), (130, 200, 0.6), (64, 128, 0.3)]:
        n = 2
        keep = np.array([220, 140, 40], np.uint8)        # kept colour (blue-ish)
        drop = np.array([24, 18, 30], np.uint8)          # excluded (dark)
        fr = np.where((rng.random((n, h, w)) < dens)[..., None], keep, drop).astype(np.uint8)
        chain = VideoChain(n, h, w, DEV)
        chain.run(_t(fr))
        res = chain.results()
        for i in range(n):
            exp = ops.keep_largest_component(ops.color_mask_bgra(fr[i], G.REFERENCE_HSV_RANGES))
            assert res[i] is not None and np.array_equal(res[i], exp), (h, w, i)


def test_video_chain_random_colour_frames_vs_oracle(D):
    """Uniform random BGR frames: every HSV path (v alone decides, full
    saturation / hue test) on every pixel position of the 4-pixels-per-lane
    loader, with heights that are multiples of 64 (the last tile row takes
    that loader too) and off-grid ones.  The kept share percolates, so the
    largest component spans the frame and the crop's α checks almost every
    foreground bit."""
    from image_processor_pipeline_amd import geometry as G
    from image_processor_pipeline_amd.video_chain import VideoChain
    rng = np.random.default_rng(8)
    for (h, w) in [(256, 320), (192, 448), (200, 330)]:
        n = 2
        fr = rng.integers(0, 256, (n, h, w, 3), np.uint8)
        chain = VideoChain(n, h, w, DEV)
        chain.run(_t(fr))
        res = chain.results()
        for i in range(n):
            exp = ops.keep_largest_component(ops.color_mask_bgra(fr[i], G.REFERENCE_HSV_RANGES))
            assert res[i] is not None and np.array_equal(res[i], exp), (h, w, i)
            assert res[i].shape[0] * res[i].shape[1] > 0.5 * h * w


def test_video_chain_uniform_colour_slots_vs_oracle(D):
    """The mask pass's reference-colour shortcut (ipp_ccl.hip
    IPP_CCL_UNIFORM: a pixel slot whose 64 pixels all have lane 0's colour
    takes that colour's cached result): flat kept and flat excluded
    backgrounds, single odd pixels in every slot of a lane's 4 pixels and
    on the reference pixel itself (column 64k, row 4j), a colour change
    between row groups (the cache refreshes), and a pixel one bit away from
    the reference colour next to it (the comparison is over its 24 bits, not
    the loaded dword's fourth byte, which belongs to the next pixel)."""
    from image_processor_pipeline_amd import geometry as G
    from image_processor_pipeline_amd.video_chain import VideoChain
    rng = np.random.default_rng(12)
    keep = np.array([220, 140, 40], np.uint8)
    drop = np.array([24, 18, 30], np.uint8)
    h, w, n = 192, 256, 4
    fr = np.empty((n, h, w, 3), np.uint8)
    fr[0], fr[1] = keep, drop
    fr[2, :96], fr[2, 96:] = keep, drop                     # colour change between row groups
    fr[3] = drop
    fr[3, 40:150, 30:200] = keep                            # a kept blob on a dark background
    for i in range(n):
        for x in (0, 1, 2, 3, 64, 127, 128, 255):           # slots 0-3, the reference pixel
            for y in (0, 4, 5, 63, 64, 100, 191):
                fr[i, y, x] = rng.integers(0, 256, 3)
        fr[i, 8, 65] = fr[i, 8, 64] ^ np.array([0, 0, 1], np.uint8)
    chain = VideoChain(n, h, w, DEV)
    chain.run(_t(fr))
    res = chain.results()
    for i in range(n):
        try:
            exp = ops.keep_largest_component(ops.color_mask_bgra(fr[i], G.REFERENCE_HSV_RANGES))
        except ValueError:  # no foreground: the reference raises, the chain gives no crop
            exp = None
        if exp is None:
            assert res[i] is None, i
        else:
            assert res[i] is not None and np.array_equal(res[i], exp), i


# --------------------------------------------------------------------------- config 5: 4K video chain

def test_video_chain_4k_vs_oracle(D):
    """BASELINE config 5 at full size: HSV mask → keep-largest → crop-fit on
    structured 3840×2160 frames, bit-exact vs the oracle; a frame with no
    foreground yields no crop (the reference raises there)."""
    from image_processor_pipeline_amd import geometry as G
    from image_processor_pipeline_amd.video_chain import VideoChain, synthetic_frames
    frames = synthetic_frames(3, 2160, 3840, 2, DEV)
    frames[2, ..., 0], frames[2, ..., 1], frames[2, ..., 2] = 24, 18, 30      # background only
    chain = VideoChain(3, 2160, 3840, DEV)
    chain.run(frames)
    res = chain.results()
    host = frames.cpu().numpy()
    for i in range(2):
        exp = ops.keep_largest_component(ops.color_mask_bgra(host[i], G.REFERENCE_HSV_RANGES))
        assert res[i] is not None and np.array_equal(res[i], exp), i
    assert res[2] is None
    # the staged form (mask → keep-largest → crop) gives the same crops, and
    # its mask stage alone matches the oracle
    chain.out.zero_()
    chain.run_staged(frames)
    staged = chain.results()
    assert all(np.array_equal(a, b) for a, b in zip(staged[:2], res[:2])) and staged[2] is None
    chain.mask(frames)
    torch.cuda.synchronize()
    assert np.array_equal(chain.bgra[0].cpu().numpy(), ops.color_mask_bgra(host[0], G.REFERENCE_HSV_RANGES))


def test_video_chain_4k_noisy_frames_vs_oracle(D):
    """Config 5 on camera-like frames (bench.py --frame-noise): ±2 LSB of
    noise on background and blob, so no 64-pixel slot is one colour and the
    mask pass never takes its uniform-slot shortcut; bit-exact vs the oracle."""
    from image_processor_pipeline_amd import geometry as G
    from image_processor_pipeline_amd.video_chain import VideoChain, synthetic_frames
    frames = synthetic_frames(2, 2160, 3840, 5, DEV, noise=2)
    host = frames.cpu().numpy()
    assert (host[:, :64, :64] != host[:, :1, :1]).any()   # the background is not flat
    chain = VideoChain(2, 2160, 3840, DEV)
    chain.run(frames)
    res = chain.results()
    for i in range(2):
        exp = ops.keep_largest_component(ops.color_mask_bgra(host[i], G.REFERENCE_HSV_RANGES))
        assert res[i] is not None and np.array_equal(res[i], exp), i


def test_crop_to_bbox_and_vector_copy(D):
    from image_processor_pipeline_amd import _native as N
    rng = np.random.default_rng(21)
    for cn in (1, 3, 4):
        img = rng.integers(0, 256, (37, 53, cn), np.uint8)
        for win in [(0, 0, 53, 37), (5, 3, 17, 9), (1, 2, 52, 35), (50, 36, 3, 1)]:
            for fl in (0, 1, 2, 3):
                x0, y0, w, h = win
                exp = img[y0:y0 + h, x0:x0 + w]
                exp = exp[:, ::-1] if fl & 1 else exp
                exp = exp[::-1] if fl & 2 else exp
                got = D.copy_window(_t(img), win, flip=fl).cpu().numpy()
                assert np.array_equal(got, exp), (cn, win, fl)
    n, h, w = 3, 31, 45
    imgs = rng.integers(0, 256, (n, h, w, 4), np.uint8)
    bbox = np.array([[3, 4, 40, 30], [-1, -1, -1, -1], [0, 0, 45, 31]], np.int32)
    cd = np.zeros(n, N.COPY_DESC)
    for i in range(n):
        cd[i]["src_off"] = cd[i]["dst_off"] = i * h * w * 4
        cd[i]["src_pitch"] = cd[i]["dst_pitch"] = 4 * w
        cd[i]["cn"] = 4
    src = _t(imgs)
    dst = torch.zeros_like(src)
    bb = _t(bbox.reshape(-1))
    cdd = D._to_dev(cd, src.device)
    N.check(N.load().ipp_crop_to_bbox(src.data_ptr(), dst.data_ptr(), cdd.data_ptr(), bb.data_ptr(), n, w, h, 4,
                                      D._stream(src.device)), "ipp_crop_to_bbox")
    out = dst.cpu().numpy()
    assert np.array_equal(out[0, :26, :37], imgs[0, 4:30, 3:40])
    assert not out[1].any()
    assert np.array_equal(out[2], imgs[2])


# --------------------------------------------------------------------------- round 2: Pillow pins at real geometry

def test_rotate_bilinear_matches_pillow_goldens(D, golden):
    """Opt-in BILINEAR rotate (ipp_rotate_bilinear, fp64 as Pillow): canvases
    bit-exact with Pillow, bbox crops too, flips folded into the write."""
    g = golden("rotate_bilinear_pillow.npz")
    srcs = unpack(g["src_flat"], g["src_shapes"])
    outs = unpack(g["out_flat"], g["out_shapes"])
    for k, (out, si, a, bb) in enumerate(zip(outs, g["src_index"], g["angles"], g["bboxes"])):
        fl = k % 4
        got = D.rotate_bilinear_canvas(_t(srcs[si]), float(a), fl).cpu().numpy()
        exp = out[:, ::-1] if fl & 1 else out
        exp = exp[::-1] if fl & 2 else exp
        assert got.shape == exp.shape and np.array_equal(got, exp), (si, a, fl)
        crop = D.rotate_crop_bilinear(_t(srcs[si]), float(a)).cpu().numpy()
        want = out if bb[0] < 0 else out[bb[1]:bb[3], bb[0]:bb[2]]
        if want.shape[0] == 0 or want.shape[1] == 0:
            want = out
        assert np.array_equal(crop, want), (si, a)


def test_rotate_bilinear_large_vs_oracle(D):
    rng = np.random.default_rng(31)
    img = rng.integers(0, 256, (300, 420, 4), np.uint8)
    img[..., 3] = np.where(rng.random((300, 420)) < 0.2, 0, 255)
    for a in (12.5, 45.0, 200.3):
        got = D.rotate_crop_bilinear(_t(img), a).cpu().numpy()
        assert np.array_equal(got, ops.rotate_and_crop(img, a, "bilinear")), a


@pytest.mark.parametrize("i", range(6))
def test_pipe_config3_alpha_zero_matches_pillow(D, golden, i):
    """The fused pipe's α = 0 path at config-3 geometry against Pillow alone
    (pipe_config3_black_pillow.npz): black planted in the 1024² source, the
    one exclusion range holding exactly the black pixels (fill included), so
    the cut-out has α = 0 regions of every size and the overlay partial α."""
    from image_processor_pipeline_amd import fused
    from tests.conftest import BLACK_RANGE, config3_black_source, sha256
    g = golden("pipe_config3_black_pillow.npz")
    src = config3_black_source(i)
    bgs = np.stack([np.random.default_rng(int(g["bg_seed"]) + k).integers(0, 256, (1024, 1024, 3), np.uint8)
                    for k in range(2)])
    x, y = (int(v) for v in g["xy"][i])
    cfg = fused.PipeConfig(hsv_ranges=[BLACK_RANGE])
    plan = fused.plan_pipe((1024, 1024), 1, (1024, 1024), 2, cfg,
                           params=[fused.ItemParams(float(g["angles"][i]), str(g["syms"][i]), int(g["bg_index"][i]),
                                                    float(g["ratios"][i]), x, y)])
    assert plan.ov_dims[0] == tuple(int(v) for v in g["ov_wh"][i])[::-1]
    runner = fused.PipeRunner(plan, DEV)
    out = torch.empty((1, 1024, 1024, 3), dtype=torch.uint8, device=DEV)
    runner.run(_t(src[None]), _t(bgs), out)
    assert sha256(out[0].cpu().numpy()) == str(g["comp_sha"][i])


@pytest.mark.parametrize("i", range(6))
def test_pipe_config3_geometry_matches_pillow(D, golden, i):
    """The fused pipe (MFMA tap tiles at the ≈5× downscale of config 3) on a
    1024² source, 896² crop, 1024² background, against the Pillow-only chain
    (α = 255 everywhere through an HSV range that never matches)."""
    from image_processor_pipeline_amd import fused
    from tests.conftest import NEVER_RANGE, config3_item, sha256
    g = golden("pipe_config3_pillow.npz")
    src, bgs, (angle, sym, bgi, ratio, x, y) = config3_item(g, i)
    cfg = fused.PipeConfig(hsv_ranges=[NEVER_RANGE])
    plan = fused.plan_pipe((1024, 1024), 1, (1024, 1024), 2, cfg,
                           params=[fused.ItemParams(angle, sym, bgi, ratio, x, y)])
    assert plan.ov_dims[0] == tuple(int(v) for v in g["ov_wh"][i])[::-1]
    runner = fused.PipeRunner(plan, DEV)
    out = torch.empty((1, 1024, 1024, 3), dtype=torch.uint8, device=DEV)
    runner.run(_t(src[None]), _t(bgs), out)
    assert sha256(out[0].cpu().numpy()) == str(g["comp_sha"][i])


@pytest.mark.parametrize("i", range(6))
def test_pipe_config3_vs_ranges_match_pillow(D, golden, i):
    """The pipe's HSV stage with several ranges OR-ed and zone masks, at
    config-3 geometry on a structured scene (pipe_config3_vs_pillow.npz): the
    ranges are fixed by V or by S = 0 alone, so the exclusion mask — and the
    partial-α edges it leaves after the ≈5× LANCZOS downscale — is exact
    without OpenCV, and the composite is Pillow's."""
    from image_processor_pipeline_amd import fused
    from tests.conftest import VS_RANGES, VS_ZONES, config3_vs_source, sha256
    g = golden("pipe_config3_vs_pillow.npz")
    src = config3_vs_source(i)
    bgs = np.stack([np.random.default_rng(int(g["bg_seed"]) + k).integers(0, 256, (1024, 1024, 3), np.uint8)
                    for k in range(2)])
    x, y = (int(v) for v in g["xy"][i])
    cfg = fused.PipeConfig(hsv_ranges=list(VS_RANGES), zones=list(VS_ZONES))
    plan = fused.plan_pipe((1024, 1024), 1, (1024, 1024), 2, cfg,
                           params=[fused.ItemParams(float(g["angles"][i]), str(g["syms"][i]), int(g["bg_index"][i]),
                                                    float(g["ratios"][i]), x, y)])
    assert plan.ov_dims[0] == tuple(int(v) for v in g["ov_wh"][i])[::-1]
    runner = fused.PipeRunner(plan, DEV)
    out = torch.empty((1, 1024, 1024, 3), dtype=torch.uint8, device=DEV)
    runner.run(_t(src[None]), _t(bgs), out)
    assert runner.status() == 0
    assert sha256(out[0].cpu().numpy()) == str(g["comp_sha"][i])

