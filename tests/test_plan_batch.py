"""The C batch planner (ipp_plan.cpp, CPU): each piece against the Python
statement of the same arithmetic, then whole plans against the Python
planner (fused.draw_params / item_geometry / geometry.py — the restatement
that tests/test_draw_order.py pins to the reference's file-mode pipeline
and tests/test_host_plan.py to the oracle).

* CPython's generator: ``random.Random(seed).random()`` sequences.
* ``math.hypot`` (vector_norm) on overlay-like arguments.
* Pillow's rotate(expand=True) plan, incl. the 0/90/180/270 fast paths, the
  ScaleAffine branch and negative / > 360° angles.
* The division-free opaque bbox against the per-row division form.
* Per-item parameters, geometry and every descriptor field, for plans with
  and without item ranges, given parameters, non-square sizes.
* The per-tile host tap builder (ipp_plan_mfma_tile, the fix-up path of the
  device tap planner) against ipp_plan_mfma_from_taps.
"""
import ctypes
import math
import random

import numpy as np
import pytest

from image_processor_pipeline_amd import _native as N
from image_processor_pipeline_amd import fused as F
from image_processor_pipeline_amd import geometry as G
from image_processor_pipeline_amd.device import SYM_FLIP


@pytest.mark.parametrize("seed", [0, 1, 7919, 123456789, 2 ** 32 + 5, 2 ** 63 + 11, 2 ** 64 - 1])
def test_cpython_generator(seed):
    lib = N.load()
    out = np.zeros(2000, np.float64)
    assert lib.ipp_plan_py_random(seed, out.size, N.np_ptr(out)) == 0
    r = random.Random(seed)
    assert out.tolist() == [r.random() for _ in range(out.size)]


def test_cpython_hypot():
    lib = N.load()
    rng = random.Random(2)
    cases = [(1024, 1024), (1920, 1080), (3, 4), (0, 5), (7, 0), (1e-300, 1e-300), (1e300, 1e300)]
    for _ in range(100000):
        ar = rng.uniform(0.05, 20.0)
        h = rng.uniform(1, 5000)
        cases.append((ar * h, h))
        cases.append((rng.randint(1, 10 ** 5), rng.randint(1, 10 ** 5)))
    for x, y in cases:
        assert lib.ipp_plan_py_hypot(float(x), float(y)) == math.hypot(x, y), (x, y)


def test_rotation_plan():
    lib = N.load()
    rng = random.Random(4)
    angles = [0.0, 90.0, 180.0, 270.0, 360.0, -90.0, 450.0, 1e-14, 180 + 1e-13, 360 - 1e-12, 45.0, 1.0, 359.0,
              -30.5, 719.25]
    angles += [rng.uniform(0, 360) for _ in range(3000)]
    out = (ctypes.c_int32 * 8)()
    for w, h in ((896, 896), (53, 37), (1, 9), (2, 3), (1920, 1080)):
        for a in angles:
            p = G.rotation_plan(w, h, a)
            assert lib.ipp_plan_rotation(w, h, a, out) == 0
            assert (out[0], out[1]) == (p.nw, p.nh), (w, h, a)
            assert tuple(out[2:8]) == p.A, (w, h, a)


def test_opaque_bbox_division_free_form():
    lib = N.load()
    rng = random.Random(5)
    a = (ctypes.c_int32 * 6)()
    b1, b2 = (ctypes.c_int32 * 4)(), (ctypes.c_int32 * 4)()
    for k in range(1500):
        w, h = rng.randint(1, 700), rng.randint(1, 700)
        ang = rng.choice([0.0, 90.0, 180.0, 270.0, rng.uniform(0, 360), rng.uniform(-1e-3, 1e-3)])
        p = G.rotation_plan(w, h, ang)
        a[:] = list(p.A)
        assert lib.ipp_plan_opaque_bbox(w, h, a, p.nw, p.nh, b1) == 0
        assert lib.ipp_plan_opaque_bbox_fast(w, h, a, p.nw, p.nh, b2) == 0
        assert list(b1) == list(b2), (w, h, ang)
    # a map that misses the source entirely
    a[:] = [65536, 0, -(10 << 16), 0, 65536, 32768]
    assert lib.ipp_plan_opaque_bbox_fast(4, 4, a, 5, 5, b2) == 0 and list(b2) == [-1] * 4


def _python_plan(src_hw, n, bg_hw, n_bg, cfg, seed, item_range=None, n_global=None):
    """The Python statement of the plan (draw_params + item_geometry +
    the descriptor arithmetic of ipp_plan_pipe_batch) for the comparison."""
    lib = N.load()
    H, W = src_hw
    bh, bw = bg_hw
    start, stop = item_range or (0, n)
    n_global = n_global or stop
    angles, syms, order, drawn = F.draw_params(n_global, stop, src_hw, bg_hw, n_bg, cfg, seed)
    t, b, l, r = G.crop_margins(H, W, cfg.margins)
    rows = []
    for gi in range(start, stop):
        ratio, x, y, plan, (ox, oy, rw, rh), (nw, nh) = drawn[gi]
        same = (nw, nh) == (rw, rh)
        id_h, id_v = same or nw == rw, same or nh == rh
        ks_h = 1 if id_h else lib.ipp_plan_lanczos_ksize(0.0, float(rw), nw)
        ks_v = 1 if id_v else lib.ipp_plan_lanczos_ksize(0.0, float(rh), nh)
        y0, y1 = 0, rh
        if not id_h and not id_v:
            _, bnd = G.lanczos_taps(rh, nh)
            y0, y1 = int(bnd[0]), int(bnd[2 * (nh - 1)] + bnd[2 * (nh - 1) + 1])
        rows.append(dict(angle=angles[gi], sym=syms[gi], bg=order[gi % n_bg], ratio=ratio, x=x, y=y, A=plan.A,
                         box=(ox, oy, rw, rh), ov=(nw, nh), ks=(ks_h, ks_v), y0=y0, y1=y1, crop=(t, b, l, r),
                         flip=SYM_FLIP[syms[gi]]))
    return rows


CASES = [
    ((1024, 1024), 300, (1024, 1024), 16, F.PipeConfig(), 0, None, None),
    ((96, 80), 40, (64, 72), 5, F.PipeConfig(margins=(8, 8, 8, 8)), 1246, None, None),
    ((300, 200), 40, (256, 300), 3, F.PipeConfig(margins=(0.1, 5, 0.2, 0)), 77, (10, 50), 57),
    ((480, 640), 25, (720, 1280), 7, F.PipeConfig(margins=(0, 0, 0, 0), sym_pool=("h", "v"), scale_min=0.4,
                                                   scale_max=0.9, angle_min=-30, angle_max=30), 2 ** 40 + 3,
     None, None),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_batch_plan_matches_python_statement(case):
    src_hw, n, bg_hw, n_bg, cfg, seed, rng, ng = CASES[case]
    if rng:
        n = rng[1] - rng[0]
    plan = F.plan_pipe(src_hw, n, bg_hw, n_bg, cfg, seed=seed, item_range=rng, n_global=ng, n_threads=3)
    rows = _python_plan(src_hw, n, bg_hw, n_bg, cfg, seed, rng, ng)
    H, W = src_hw
    bh, bw = bg_hw
    it = plan.items
    order = np.argsort(it["bg_index"], kind="stable")
    assert [d["g"]["src_off"] for d in plan.descs] == [i * H * 3 * W for i in order]
    tmp_off = 0
    tmp_offs = []
    for i, e in enumerate(rows):
        p = plan.params[i]
        assert (p.angle, p.sym, p.bg_index, p.ratio, p.x, p.y) == (e["angle"], e["sym"], e["bg"], e["ratio"], e["x"],
                                                                    e["y"]), i
        assert (int(it["cut_x"][i]), int(it["cut_y"][i]), int(it["cut_w"][i]), int(it["cut_h"][i])) == e["box"]
        assert (int(it["ov_w"][i]), int(it["ov_h"][i])) == e["ov"]
        d = plan.descs[int(np.nonzero(order == i)[0][0])]
        g, h, v, pp = d["g"], d["h"], d["v"], d["p"]
        t, b, l, r = e["crop"]
        rw, rh = e["box"][2:]
        nw, nh = e["ov"]
        assert tuple(int(g[f"a{k}"]) for k in range(6)) == e["A"]
        assert (g["in_x0"], g["in_y0"], g["in_w"], g["in_h"]) == (l, t, W - l - r, H - t - b)
        assert (g["out_w"], g["out_h"], g["off_x"], g["off_y"], g["flip"]) == (rw, rh, e["box"][0], e["box"][1],
                                                                              e["flip"])
        rows_ = e["y1"] - e["y0"]
        assert (h["in_len"], h["out_len"], h["lines"], h["line0"], h["ksize"]) == (rw, nw, rows_, e["y0"], e["ks"][0])
        assert (v["in_len"], v["out_len"], v["lines"], v["ksize"]) == (rows_, nh, nw, e["ks"][1])
        assert (pp["bg_off"], pp["dst_off"], pp["x"], pp["y"], pp["ov_w"], pp["ov_h"]) == (
            e["bg"] * bh * bw * 3, i * bh * bw * 3, e["x"], e["y"], nw, nh)
        ah, av = plan.axes[2 * i], plan.axes[2 * i + 1]
        assert h["coef_off"] == ah["coef_off"] and v["coef_off"] == av["coef_off"]
        assert (ah["in_size"], ah["out_size"], ah["phase"], ah["shift"]) == (rw, nw, 0, 0)
        # V taps are shifted to ybox_first (0 unless both axes resample)
        assert (av["in_size"], av["out_size"], av["phase"], av["shift"]) == (rh, nh, e["y"] % 16, e["y0"])
        nkb = lib_nkb(rh, nh, e["ks"][1])
        groups = (((rows_ + 15) // 16) * 16 + 64 * nkb + 16) // 4
        assert h["dst_off"] == tmp_off and v["src_off"] == tmp_off
        tmp_offs.append(tmp_off)
        tmp_off = (tmp_off + 16 * nw * groups + 255) // 256 * 256
    assert plan.tmp_bytes == max(tmp_off, 256)


def lib_nkb(i, o, k):
    return N.load().ipp_plan_mfma_nk_bound(i, o, k)


def test_batch_plan_given_params_and_errors():
    cfg = F.PipeConfig()
    drawn = F.plan_pipe((512, 512), 20, (600, 500), 4, cfg, seed=9)
    again = F.plan_pipe((512, 512), 20, (600, 500), 4, cfg, params=drawn.params)
    assert again.descs.tobytes() == drawn.descs.tobytes()
    assert again.params == drawn.params
    bad = list(drawn.params)
    bad[3] = F.ItemParams(bad[3].angle, bad[3].sym, bad[3].bg_index, bad[3].ratio, 10 ** 6, bad[3].y)
    with pytest.raises(ValueError, match="item 3"):
        F.plan_pipe((512, 512), 20, (600, 500), 4, cfg, params=bad)
    bad[3] = F.ItemParams(drawn.params[3].angle, "x", 0, 0.2, 0, 0)
    with pytest.raises(ValueError):
        F.plan_pipe((512, 512), 20, (600, 500), 4, cfg, params=bad)
    # seeds beyond 64 bits and non-int seeds take the Python draws
    for seed in (2 ** 70 + 1, "abc"):
        p = F.plan_pipe((256, 256), 6, (300, 300), 2, cfg, seed=seed)
        angles, syms, order, per = F.draw_params(6, 6, (256, 256), (300, 300), 2, cfg, seed)
        assert [q.angle for q in p.params] == angles and [q.x for q in p.params] == [e[1] for e in per]


@pytest.mark.parametrize("io,shift,phase,ident", [((1100, 230), 0, 0, 0), ((1268, 150), 0, 7, 0),
                                                  ((896, 896), 0, 0, 1), ((40, 13), 0, 3, 0), ((1, 1), 0, 0, 1),
                                                  ((300, 299), 0, 15, 0), ((1150, 240), 9, 5, 0),
                                                  ((2000, 90), 3, 11, 0)])
def test_mfma_tile_matches_axis_planner(io, shift, phase, ident):
    lib = N.load()
    i, o = io
    if ident:
        k, std = G.identity_taps(o)
    else:
        k, std = G.lanczos_taps(i, o)
    if shift:
        std[0:2 * o:2] += shift
    out = np.zeros(lib.ipp_plan_mfma_size(i, o, k), np.int32)
    assert lib.ipp_plan_mfma_from_taps(i, o, k, N.np_ptr(std), shift, phase, N.np_ptr(out)) == 0
    T = (o + phase + 15) // 16
    ax = np.zeros(1, N.TAP_AXIS)
    ax["in_size"], ax["out_size"], ax["identity"], ax["shift"], ax["phase"] = i, o, ident, shift, phase
    ax["nkb"], ax["n_tiles"] = lib.ipp_plan_mfma_nk_bound(i, o, k), T
    hdr = out[:4 * T].reshape(T, 4)
    blocks = out[20 * T:].view(np.uint8)
    for t in range(T):
        h4, b16 = np.zeros(4, np.int32), np.zeros(16, np.int32)
        blk = np.zeros(int(ax["nkb"][0]) * 3072, np.uint8)
        # the axis planner got Pillow's bounds moved by +shift and subtracts
        # shift again: the tile builder sees the plain axis
        ax2 = ax.copy()
        ax2["shift"] = 0
        assert lib.ipp_plan_mfma_tile(N.np_ptr(ax2), t, N.np_ptr(h4), N.np_ptr(b16), N.np_ptr(blk), blk.size) == 0
        assert (h4[0], h4[1]) == (hdr[t, 0], hdr[t, 1]), t
        assert np.array_equal(b16, out[4 * T + 16 * t:4 * T + 16 * t + 16]), t
        nk = int(h4[1])
        assert np.array_equal(blk[:nk * 3072], blocks[hdr[t, 2] * 16:hdr[t, 2] * 16 + nk * 3072]), t
        assert h4[2] == t * int(ax["nkb"][0]) * 192


def test_plan_rejects_overlays_wider_than_the_v_launch():
    """Overlays wider than IPP_PIPE_MAX_OV_W are refused by the planner,
    before ipp_pipe_hpass_bgcopy could write part of the composites (round-5
    advisor finding); one just inside the limit plans."""
    from image_processor_pipeline_amd import fused
    from image_processor_pipeline_amd import _native as N
    # a 4096² background at ratio 0.30: overlays of ≈ 1229 px
    cfg = fused.PipeConfig(scale_min=0.30, scale_max=0.30)
    with pytest.raises(ValueError, match="overlay width"):
        fused.plan_pipe((256, 256), 4, (4096, 4096), 1, cfg, seed=3)
    cfg = fused.PipeConfig(scale_min=0.15, scale_max=0.15)   # ≈ 614 px
    plan = fused.plan_pipe((256, 256), 4, (4096, 4096), 1, cfg, seed=3)
    assert plan.max_ov_w <= N.IPP_PIPE_MAX_OV_W
