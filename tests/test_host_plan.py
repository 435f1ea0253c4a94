"""Host-side planning (CPU): the C planner and the Python geometry reproduce
the library host arithmetic exactly (checked against the oracle)."""
import math
import random

import numpy as np
import pytest

from image_processor_pipeline_amd import _native as N
from image_processor_pipeline_amd import geometry as G
from oracle import ops


@pytest.mark.parametrize("io", [(1024, 200), (1268, 307), (57, 20), (30, 45), (9, 3), (1, 1), (5, 9),
                                (896, 896), (1500, 151)])
def test_lanczos_taps_match_oracle(io):
    i, o = io
    k, buf = G.lanczos_taps(i, o)
    kk, bounds, taps = ops.precompute_coeffs(i, 0.0, float(i), o)
    assert k == kk
    assert np.array_equal(buf[:2 * o].reshape(o, 2), bounds)
    assert np.array_equal(buf[2 * o:].reshape(o, k), taps)


@pytest.mark.parametrize("wh", [(896, 896), (53, 37), (2, 3), (1, 9), (640, 480)])
def test_opaque_bbox_matches_bruteforce(wh):
    w, h = wh
    rng = random.Random(3)
    angles = [0.0, 90.0, 180.0, 270.0, 45.0, 1.0, 359.0, 89.9999] + [rng.uniform(0, 360) for _ in range(6)]
    img = np.full((h, w, 4), 255, np.uint8)
    for a in angles:
        plan = G.rotation_plan(w, h, a)
        g = ops.rotate_geometry(w, h, a)
        assert (plan.nw, plan.nh) == (g["nw"], g["nh"])
        if g["kind"] == "affine":
            assert plan.A == g["A"]
        if w * h <= 640 * 480 and (a in (45.0, 1.0) or w < 100):
            exp = ops.getbbox_alpha(ops.rotate_expand_nearest(img, a))
            assert G.rotated_bbox(w, h, plan) == exp, a


def test_fast_path_maps_are_exact_transposes():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (7, 11, 4), np.uint8)
    h, w = img.shape[:2]
    for a in (0.0, 90.0, 180.0, 270.0):
        plan = G.rotation_plan(w, h, a)
        a0, a1, a2, a3, a4, a5 = plan.A
        Y, X = np.mgrid[0:plan.nh, 0:plan.nw]
        xin = (a2 + Y * a1 + X * a0) >> 16
        yin = (a5 + Y * a4 + X * a3) >> 16
        got = img[yin, xin]
        assert np.array_equal(got, ops.rotate_expand_nearest(img, a)), a


def test_scale_affine_branch_reduces_to_integer_map():
    plan = G.rotation_plan(40, 30, 1e-14)
    assert plan.kind == "scale_affine" and (plan.nw, plan.nh) == (40, 30)
    assert plan.A == (65536, 0, 32768, 0, 65536, 32768)


def test_overlay_size_and_hsv_params():
    assert G.overlay_size(1000, 800, 1024, 1024, 0.2) == ops.overlay_geometry(1000, 800, 1024, 1024, 0.2)
    p = G.hsv_params(G.REFERENCE_HSV_RANGES, None, False)
    assert p["n_ranges"] == 4
    lo, hi = ops.inrange_bounds((15, 30 * 2.55, 55 * 2.55), (30, 60 * 2.55, 80 * 2.55))
    assert list(p["r"][2]["lo"]) == lo and list(p["r"][2]["hi"]) == hi
    p2 = G.hsv_params([(50, 0, 0, 10, 255, 255), (0, 0, 0, 180, 255, 255)])
    assert p2["n_ranges"] == 1            # the empty range is dropped
    with pytest.raises(ValueError):
        G.hsv_params([(0, 0, 0, 200, 255, 255)])
    with pytest.raises(ValueError):
        G.hsv_params([])


@pytest.mark.parametrize("io,shift,phase", [((1100, 230), 0, 0), ((1268, 150), 0, 7), ((896, 896), 0, 0),
                                            ((40, 13), 0, 3), ((1, 1), 0, 0), ((300, 299), 0, 15), ((57, 20), 0, 0),
                                            ((1150, 240), 9, 5)])
def test_mfma_tile_format_is_exact(io, shift, phase):
    """Emulate v_mfma_i32_16x16x64_i8 on the planned B blocks: for every
    output, bias + Σ_p 2^(8p) Σ_s Σ_k (pix[K0+64s+k] ^ 0x80) · B_p[k][col]
    == 2^21 + Σ p·k (the identity the MFMA H pass relies on)."""
    lib = N.load()
    i, o = io
    k, std = G.lanczos_taps(i, o)
    if shift:
        std[0:2 * o:2] += shift   # pretend the axis starts `shift` rows later
    size = lib.ipp_plan_mfma_size(i, o, k)
    out = np.zeros(size, np.int32)
    assert lib.ipp_plan_mfma_from_taps(i, o, k, N.np_ptr(std), shift, phase, N.np_ptr(out)) == 0
    T = (o + phase + 15) // 16
    hdr = out[:4 * T].reshape(T, 4)
    bias = out[4 * T:20 * T]
    nblk = int(max(hdr[:, 2] // 64 + hdr[:, 1] * 3))
    blocks = out[20 * T:20 * T + nblk * 256].view(np.uint8).view(np.int8).reshape(-1, 64, 16)
    rng = np.random.default_rng(5)
    pix = rng.integers(0, 256, i + 256, np.uint8)
    sp = (pix ^ 0x80).view(np.int8).astype(np.int64)
    for t in range(T):
        K0, nK, boff = int(hdr[t, 0]), int(hdr[t, 1]), int(hdr[t, 2])
        assert K0 % 16 == 0 and boff % 64 == 0
        acc = np.zeros((3, 16), np.int64)
        for s in range(nK):
            for p in range(3):
                blk = blocks[boff // 64 + s * 3 + p].astype(np.int64)  # [lane][j]
                Bm = np.zeros((64, 16), np.int64)                     # B[k][col]
                for lane in range(64):
                    Bm[16 * (lane >> 4):16 * (lane >> 4) + 16, lane & 15] = blk[lane]
                a = sp[K0 + 64 * s:K0 + 64 * s + 64]
                a = np.pad(a, (0, 64 - len(a)))
                acc[p] += a @ Bm
        for col in range(16):
            oo = 16 * t - phase + col
            if oo < 0 or oo >= o:
                assert bias[16 * t + col] == 0
                continue
            xmin, cnt = std[2 * oo] - shift, std[2 * oo + 1]
            ref = (1 << 21) + int((pix[xmin:xmin + cnt].astype(np.int64) * std[2 * o + oo * k:2 * o + oo * k + cnt]).sum())
            got = int(bias[16 * t + col]) + int(acc[0, col]) + (int(acc[1, col]) << 8) + (int(acc[2, col]) << 16)
            assert got == ref, (t, col)


def test_pipe_plan_rejects_windows_wider_than_the_ring():
    """A downscale whose tap window exceeds the H pass's 512-column LDS ring is
    refused at planning time (no silent window overrun on the device)."""
    from image_processor_pipeline_amd import fused
    with pytest.raises(ValueError, match="window"):
        fused.plan_pipe((1024, 1024), 2, (1024, 1024), 1, fused.PipeConfig(scale_min=0.01, scale_max=0.012), seed=0)
    plan = fused.plan_pipe((1024, 1024), 2, (1024, 1024), 1, fused.PipeConfig(), seed=0)
    assert plan.max_ov_h >= 1 and plan.algo_bytes_hpass_bgcopy > plan.algo_bytes_hpass


def test_pipe_plan_copy_read_bytes_follow_the_copy_groups():
    """IPP_PT_COPY_READS (fused.PipePlan.copy_read_bytes): the H launch's
    grouped copy loads one background per run of same-background items in
    each group of 8 consecutive items of the processing order (ipp_pipe.hip
    bg_copy_group) — recomputed here from the planned items."""
    from image_processor_pipeline_amd import fused
    for n, K, (bh, bw) in [(21, 4, (70, 256)), (64, 16, (96, 128)), (9, 1, (64, 80)), (40, 40, (32, 48))]:
        plan = fused.plan_pipe((90, 110), n, (bh, bw), K, fused.PipeConfig(margins=(3, 5, 2, 7)), seed=n)
        order = plan.items["bg_index"][np.argsort(plan.items["bg_index"], kind="stable")]
        runs = sum(1 for i in range(n) if i % 8 == 0 or order[i] != order[i - 1])
        assert plan.copy_read_bytes == runs * 3 * bw * bh, (n, K)
        assert plan.algo_bytes_hpass_bgcopy > plan.algo_bytes_hpass


def test_unpremultiply_magic_table_is_exact():
    """ipp_device.h unpremultiply_magic: floor(255·c / a) = (510·c · M[a]) >> 32
    with M[a] = floor(2^31 / a) + 1, for every α 1..255 and channel 0..255
    (the V pass's unpremultiply, Pillow's RGBa → RGBA integer division)."""
    c = np.arange(256, dtype=np.uint64)
    for a in range(1, 256):
        m = (1 << 31) // a + 1
        assert m < 1 << 32
        q = ((np.uint64(510) * c) * np.uint64(m)) >> np.uint64(32)
        assert np.array_equal(q, (255 * c) // a), a
