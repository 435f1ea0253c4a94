"""Pin the CPU oracle against golden vectors from Pillow 12.2.0 and the
reference's own rotations.py / overlays.py (tools/make_goldens.py)."""
import random

import numpy as np
import pytest

from oracle import ops
from tests.conftest import unpack


def test_rotate_canvas_and_bbox_match_pillow(golden):
    g = golden("rotate_pillow.npz")
    srcs = unpack(g["src_flat"], g["src_shapes"])
    outs = unpack(g["out_flat"], g["out_shapes"])
    assert len(outs) == len(g["angles"]) > 100
    for out, si, a, bb in zip(outs, g["src_index"], g["angles"], g["bboxes"]):
        src = ops.to_rgba(srcs[si])
        got = ops.rotate_expand_nearest(src, float(a))
        assert got.shape == out.shape, (si, a)
        assert np.array_equal(got, out), (si, a)
        gbb = ops.getbbox_alpha(got)
        assert (gbb if gbb is not None else (-1, -1, -1, -1)) == tuple(bb)


def test_process_rotations_reference_outputs(golden):
    g = golden("rotations_ref.npz")
    outs = unpack(g["out_flat"], g["out_shapes"])
    names = list(g["names"])
    src = ops.to_rgba(g["src"])
    # r000 = original (rotations.py:77-85), then one file per angle draw (:88-119)
    assert names[0].endswith("_r000.png") and np.array_equal(outs[0], src)
    random.seed(int(g["seed"]))
    for i, out in enumerate(outs[1:], start=1):
        a = random.uniform(1.0, 359.0)
        assert a == g["angles"][i - 1]
        assert names[i].endswith(f"_r{i:03d}.png")
        assert np.array_equal(ops.rotate_and_crop(src, a), out)


def test_lanczos_resize_matches_pillow(golden):
    g = golden("resize_pillow.npz")
    srcs = unpack(g["src_flat"], g["src_shapes"])
    outs = unpack(g["out_flat"], g["out_shapes"])
    for s, o, (ow, oh) in zip(srcs, outs, g["sizes"]):
        got = ops.resize_lanczos_rgba(s, int(ow), int(oh))
        assert np.array_equal(got, o), (s.shape, ow, oh)


def test_paste_matches_pillow(golden):
    g = golden("paste_pillow.npz")
    for (x, y), out in zip(g["pos"], g["outs"]):
        got = ops.paste_rgba_onto_rgb(g["bg"], g["ov"], int(x), int(y))
        assert np.array_equal(got, out[..., :3])


def test_overlay_reference_composite_and_label(golden):
    g = golden("overlays_ref.npz")
    ovs = unpack(g["ov_flat"], g["ov_shapes"])
    bgs = unpack(g["bg_flat"], g["bg_shapes"])
    comps = unpack(g["comp_flat"], g["comp_shapes"])
    for ov, bg, comp, label, seed in zip(ovs, bgs, comps, g["labels"], g["seeds"]):
        random.seed(int(seed))
        ratio = random.uniform(0.15, 0.30)
        bh, bw = bg.shape[:2]
        nw, nh = ops.overlay_geometry(ov.shape[1], ov.shape[0], bw, bh, ratio)
        x = random.randint(0, bw - nw)
        y = random.randint(0, bh - nh)
        rs = ops.resize_lanczos_rgba(ov, nw, nh)
        got = ops.paste_rgba_onto_rgb(bg, rs, x, y)
        assert np.array_equal(got, comp)
        assert ops.yolo_label(0, x, y, nw, nh, bw, bh) == str(label)


def test_bilinear_rotate_matches_pillow(golden):
    """Opt-in BILINEAR mode: the oracle equals Pillow
    rotate(..., resample=BILINEAR) canvases (RGB and RGBA) and their bbox."""
    g = golden("rotate_bilinear_pillow.npz")
    srcs = unpack(g["src_flat"], g["src_shapes"])
    outs = unpack(g["out_flat"], g["out_shapes"])
    for out, si, a, bb in zip(outs, g["src_index"], g["angles"], g["bboxes"]):
        got = ops.rotate_expand_bilinear(ops.to_rgba(srcs[si]), float(a))
        assert got.shape == out.shape and np.array_equal(got, out), (si, a)
        gbb = ops.getbbox_alpha(got)
        assert (gbb if gbb is not None else (-1, -1, -1, -1)) == tuple(bb)


@pytest.mark.parametrize("i", [0, 3])
def test_oracle_pipe_at_config3_geometry_matches_pillow(golden, i):
    """BASELINE config-3 geometry (1024² source, 896² crop, ≈1266² rotated
    cut-out, ≈5× LANCZOS downscale, paste on 1024²): the oracle's stages hash
    to the Pillow chain's."""
    from tests.conftest import config3_item, sha256
    g = golden("pipe_config3_pillow.npz")
    src, bgs, (angle, sym, bgi, ratio, x, y) = config3_item(g, i)
    crop = ops.crop_from_border(src, (64, 64, 64, 64))
    cut = ops.flip(ops.rotate_and_crop(ops.to_rgba(crop), angle), sym)
    assert sha256(cut) == str(g["cut_sha"][i])
    ov = ops.to_rgba(cut[..., :3])
    nw, nh = ops.overlay_geometry(ov.shape[1], ov.shape[0], 1024, 1024, ratio)
    assert (nw, nh) == tuple(int(v) for v in g["ov_wh"][i])
    ovr = ops.resize_lanczos_rgba(ov, nw, nh)
    assert sha256(ovr) == str(g["ov_sha"][i])
    assert sha256(ops.paste_rgba_onto_rgb(bgs[bgi], ovr, x, y)) == str(g["comp_sha"][i])


@pytest.mark.parametrize("i", [1, 4])
def test_oracle_pipe_alpha_zero_matches_pillow(golden, i):
    """The α = 0 path at config-3 geometry (pipe_config3_black_pillow.npz):
    black planted in the source and the exclusion range that holds exactly
    the black pixels, so the oracle's own HSV mask, LANCZOS over premultiplied
    α = 0 pixels, unpremultiply and paste are pinned by Pillow alone."""
    from image_processor_pipeline_amd import fused
    from oracle import pipe as opipe
    from tests.conftest import BLACK_RANGE, config3_black_source, sha256
    g = golden("pipe_config3_black_pillow.npz")
    assert int(g["alpha_zero"][i]) > 1000 and int(g["alpha_partial"][i]) > 1000
    src = config3_black_source(i)
    bgs = np.stack([np.random.default_rng(int(g["bg_seed"]) + k).integers(0, 256, (1024, 1024, 3), np.uint8)
                    for k in range(2)])
    x, y = (int(v) for v in g["xy"][i])
    cfg = fused.PipeConfig(hsv_ranges=[BLACK_RANGE])
    p = fused.ItemParams(float(g["angles"][i]), str(g["syms"][i]), int(g["bg_index"][i]), float(g["ratios"][i]),
                         x, y)
    assert sha256(opipe.pipe_item(src, bgs, p, cfg)) == str(g["comp_sha"][i])


@pytest.mark.parametrize("i", [0, 3])
def test_oracle_pipe_vs_ranges_match_pillow(golden, i):
    """Multi-range OR with zones at config-3 geometry
    (pipe_config3_vs_pillow.npz): ranges fixed by V or by S = 0 alone, so the
    oracle's restated OpenCV HSV + inRange + zone masks are pinned by an
    OpenCV-free mask, and the whole chain by Pillow."""
    from image_processor_pipeline_amd import fused
    from oracle import pipe as opipe
    from tests.conftest import VS_RANGES, VS_ZONES, config3_vs_source, sha256, vs_alpha
    g = golden("pipe_config3_vs_pillow.npz")
    assert int(g["alpha_zero"][i]) > 1000 and int(g["alpha_partial"][i]) > 1000
    src = config3_vs_source(i)
    angle, sym = float(g["angles"][i]), str(g["syms"][i])
    cut = ops.flip(ops.rotate_and_crop(ops.to_rgba(ops.crop_from_border(src, (64, 64, 64, 64))), angle), sym)
    bgr = np.ascontiguousarray(cut[..., 2::-1])
    assert np.array_equal(ops.hsv_alpha_mask(bgr, VS_RANGES, VS_ZONES), vs_alpha(cut[..., :3]))
    bgs = np.stack([np.random.default_rng(int(g["bg_seed"]) + k).integers(0, 256, (1024, 1024, 3), np.uint8)
                    for k in range(2)])
    x, y = (int(v) for v in g["xy"][i])
    cfg = fused.PipeConfig(hsv_ranges=list(VS_RANGES), zones=list(VS_ZONES))
    p = fused.ItemParams(angle, sym, int(g["bg_index"][i]), float(g["ratios"][i]), x, y)
    assert sha256(opipe.pipe_item(src, bgs, p, cfg)) == str(g["comp_sha"][i])


def test_enhance_image_reference_outputs(golden):
    """tranfo.enhance_image: the oracle (Blend.c / rgb2l / ImageStat /
    BoxBlur.c / point() restated) with the draws taken in the reference order
    reproduces the reference's own outputs (tests/golden/tranfo_ref.npz)."""
    g = golden("tranfo_ref.npz")
    srcs = unpack(g["src_flat"], g["src_shapes"])
    outs = unpack(g["out_flat"], g["out_shapes"])
    for s, o, (blur, rgb), seed in zip(srcs, outs, g["flags"], g["seeds"]):
        rnd = random.Random(int(seed))
        got = ops.enhance_image(s[..., :3].copy(), bool(blur), bool(rgb), rnd)
        assert np.array_equal(got, o), (s.shape, blur, rgb)
