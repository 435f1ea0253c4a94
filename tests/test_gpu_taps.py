"""Device tap planner (ipp_taps.hip, ipp_pipe_plan_taps) against the host
restatement of Pillow's taps (ipp_plan_mfma_tile: Resample.c
precompute_coeffs + normalize_coeffs_8bpc with libm sin, reference call site
overlays.py:129), tile by tile: header, biases and every byte of the i8
blocks, bit-exact.  The host builder itself is pinned to the axis planner
(tests/test_plan_batch.py) and that to the oracle (tests/test_host_plan.py).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from image_processor_pipeline_amd import _native as N
from image_processor_pipeline_amd import fused as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _check_axes(plan, coefs, axes_idx):
    lib = N.load()
    c = coefs.cpu().numpy()
    bad = []
    for j in axes_idx:
        a = plan.axes[j:j + 1]
        T, off, nkb = int(a["n_tiles"][0]), int(a["coef_off"][0]), int(a["nkb"][0])
        hdr = c[off:off + 4 * T].reshape(T, 4)
        bias = c[off + 4 * T:off + 20 * T]
        blocks = c[off + 20 * T:].view(np.uint8)
        for t in range(T):
            h4, b16 = np.zeros(4, np.int32), np.zeros(16, np.int32)
            blk = np.zeros(nkb * 3072, np.uint8)
            assert lib.ipp_plan_mfma_tile(N.np_ptr(a), t, N.np_ptr(h4), N.np_ptr(b16), N.np_ptr(blk), blk.size) == 0
            nk = int(h4[1])
            ok = (np.array_equal(hdr[t], h4) and np.array_equal(bias[16 * t:16 * t + 16], b16)
                  and np.array_equal(blocks[h4[2] * 16:h4[2] * 16 + nk * 3072], blk[:nk * 3072]))
            if not ok:
                bad.append((j, t))
    return bad


@pytest.mark.parametrize("case", [
    ((1024, 1024), 300, (1024, 1024), 16, F.PipeConfig(), 0),
    ((96, 80), 40, (64, 72), 5, F.PipeConfig(margins=(8, 8, 8, 8)), 1246),
    ((480, 640), 25, (720, 1280), 7, F.PipeConfig(margins=(0, 0, 0, 0), scale_min=0.4, scale_max=0.9), 3),
    # upscales (ratio > source) and near-identity axes
    ((200, 160), 30, (1024, 1024), 2, F.PipeConfig(margins=(0, 0, 0, 0), scale_min=0.5, scale_max=0.9), 11),
    # long filters: ratios 11-19, up to ~117 taps per output (past the
    # planner's 64 register-held taps), 7 K steps (several staging windows)
    ((1024, 1024), 20, (640, 640), 3, F.PipeConfig(scale_min=0.1, scale_max=0.15), 5),
])
def test_device_taps_equal_host_taps(case):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    src_hw, n, bg_hw, n_bg, cfg, seed = case
    plan = F.plan_pipe(src_hw, n, bg_hw, n_bg, cfg, seed=seed)
    coefs, fixed = F.plan_taps(plan, DEV)
    torch.cuda.synchronize()
    bad = _check_axes(plan, coefs, range(len(plan.axes)))
    print(f"host-rebuilt tiles: {fixed}")
    assert not bad, bad[:10]


def test_device_taps_bench_plan():
    """The bench's B = 4096 plan: a seeded sample of 600 axes (every tile of
    each), plus the count of host-rebuilt tiles stays small."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    plan = F.plan_pipe((1024, 1024), 4096, (1024, 1024), 16, F.PipeConfig(), seed=0)
    coefs, fixed = F.plan_taps(plan, DEV)
    torch.cuda.synchronize()
    idx = np.random.default_rng(0).choice(len(plan.axes), 600, replace=False)
    bad = _check_axes(plan, coefs, sorted(idx.tolist()) + [0, 1, len(plan.axes) - 2, len(plan.axes) - 1])
    print(f"host-rebuilt tiles: {fixed}")
    assert not bad, bad[:10]
    assert fixed < 2000


class _Axes:
    """A tap plan of hand-made axes (the fields plan_taps reads)."""

    def __init__(self, pairs, compact=1):
        lib = N.load()
        self.axes = np.zeros(len(pairs), N.TAP_AXIS)
        off = 0
        for j, (n_in, n_out) in enumerate(pairs):
            ks = lib.ipp_plan_lanczos_ksize(0.0, float(n_in), n_out)
            a = self.axes[j]
            a["in_size"], a["out_size"], a["compact"] = n_in, n_out, compact
            a["nkb"] = lib.ipp_plan_mfma_nk_bound(n_in, n_out, ks)
            a["n_tiles"] = (n_out + 15) // 16
            a["coef_off"] = off
            off += (lib.ipp_plan_mfma_size(n_in, n_out, ks) + 3) // 4 * 4
        self.coef_words = off


def test_device_taps_long_filter_compact_last_tile():
    """Ratios of 10.6-12 (more taps per output than the planner's 64
    register-held ones) with 1-8 outputs in the last tile: that tile keeps
    <= 64 nonzero 16-column groups over >= 2 K steps, so it is compact and
    its taps past the register set go through stage_byte's compact layout
    (ipp_taps.hip).  Every tile equals the host restatement."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lib = N.load()
    pairs = [(n_out * r // 10, n_out) for n_out in (97, 99, 101, 104, 113, 120) for r in (106, 115, 120)]
    plan = _Axes(pairs)
    coefs, _ = F.plan_taps(plan, DEV)
    torch.cuda.synchronize()
    assert not _check_axes(plan, coefs, range(len(plan.axes)))
    c = coefs.cpu().numpy()
    hits = 0
    for j, (n_in, n_out) in enumerate(pairs):
        a = plan.axes[j]
        T, off = int(a["n_tiles"]), int(a["coef_off"])
        hdr = c[off:off + 4 * T].reshape(T, 4)
        ks = lib.ipp_plan_lanczos_ksize(0.0, float(n_in), n_out)
        hits += int(ks > 64 and n_out % 16 and hdr[T - 1][3] == 1 and hdr[T - 1][1] >= 2)
    assert hits > 0


def test_device_taps_per_tile_copies_equal_packed_upload():
    """The host-rebuilt tiles' fallback upload (one copy pair per tile, taken
    when their pack exceeds the scratch's pack region; forced here with
    pack_cap = 0 through ipp_pipe_plan_taps_cap) writes the same taps byte for
    byte as the packed upload + k_put_tiles of ipp_pipe_plan_taps."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lib = N.load()
    plan = F.plan_pipe((1024, 1024), 2048, (1024, 1024), 16, F.PipeConfig(), seed=3)
    scratch = torch.empty(int(lib.ipp_pipe_taps_scratch_bytes(len(plan.axes))), dtype=torch.uint8, device=DEV)
    st = torch.cuda.current_stream(DEV).cuda_stream
    outs, fixed = [], []
    for cap in (4 << 20, 0):
        # the same junk in both buffers: bytes the planner leaves alone compare equal
        coefs = torch.full((plan.coef_words + 4096,), 0x5A5A5A5A, dtype=torch.int32, device=DEV)
        stats = np.zeros(2, np.int64)
        N.check(lib.ipp_pipe_plan_taps_cap(N.np_ptr(plan.axes), len(plan.axes), coefs.data_ptr(),
                                           scratch.data_ptr(), N.np_ptr(stats), cap, st), "ipp_pipe_plan_taps_cap")
        torch.cuda.synchronize()
        assert int(stats[1]) == 0
        outs.append(coefs)
        fixed.append(int(stats[0]))
    assert fixed[0] == fixed[1] > 0
    assert torch.equal(outs[0], outs[1])
    stats = np.zeros(2, np.int64)
    assert lib.ipp_pipe_plan_taps_cap(N.np_ptr(plan.axes), len(plan.axes), outs[0].data_ptr(), scratch.data_ptr(),
                                      N.np_ptr(stats), -1, st) == N.IPP_E_ARG
