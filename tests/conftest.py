"""Shared pytest configuration.

`-m gpu` tests need a real MI355X (they call the HIP C-ABI library);
everything else runs on the CPU container.
"""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X GPU (HIP C-ABI library)")


def unpack(flat, shapes):
    """Inverse of tools/make_goldens.py::_pack."""
    out, off = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(flat[off:off + n].reshape(tuple(int(v) for v in s)))
        off += n
    return out


@pytest.fixture(scope="session")
def golden():
    def _load(name):
        return np.load(GOLDEN / name, allow_pickle=False)
    return _load


def config3_item(g, i):
    """Inputs of item i of tests/golden/pipe_config3_pillow.npz (regenerated
    from the seeds stored in the fixture, as tools/make_goldens.py made them):
    (1024² RGB source, the two 1024² backgrounds, ItemParams fields)."""
    src = np.random.default_rng(int(g["src_seed"]) + i).integers(0, 256, (1024, 1024, 3), np.uint8)
    bgs = np.stack([np.random.default_rng(int(g["bg_seed"]) + k).integers(0, 256, (1024, 1024, 3), np.uint8)
                    for k in range(2)])
    x, y = (int(v) for v in g["xy"][i])
    return src, bgs, (float(g["angles"][i]), str(g["syms"][i]), int(g["bg_index"][i]), float(g["ratios"][i]), x, y)


def sha256(a) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# HSV exclusion range that never matches (OpenCV 8-bit hue < 180): α = 255
# everywhere, so the pipe chain is Pillow-only (pipe_config3_pillow.npz).
NEVER_RANGE = (180, 0, 0, 180, 255, 255)


# HSV exclusion range holding exactly the pure-black pixels (V = max(r, g, b)
# = 0): the α = 0 path of the pipe pinned by Pillow alone
# (pipe_config3_black_pillow.npz, tools/make_goldens.py).
BLACK_RANGE = (0, 0, 0, 180, 255, 0)
CONFIG3_BLACK_SEED = 5000


def config3_black_source(i: int) -> np.ndarray:
    """Item i's 1024² source for pipe_config3_black_pillow.npz: random bytes
    with planted black (0, 0, 0) rectangles, stripes and 3 % scattered black
    pixels, so the cut-out has α = 0 regions of every size."""
    src = np.random.default_rng(CONFIG3_BLACK_SEED + i).integers(0, 256, (1024, 1024, 3), np.uint8)
    r = np.random.default_rng(CONFIG3_BLACK_SEED + 100 + i)
    for _ in range(8):
        y0, x0 = (int(v) for v in r.integers(0, 1000, 2))
        hh, ww = (int(v) for v in r.integers(8, 260, 2))
        src[y0:y0 + hh, x0:x0 + ww] = 0
    src[:, 300 + 37 * i:304 + 37 * i] = 0
    src[500 + 11 * i:503 + 11 * i, :] = 0
    src[r.random((1024, 1024)) < 0.03] = 0
    return src

# V / S-only exclusion ranges (pipe_config3_vs_pillow.npz): every range is
# fixed by V = max(r, g, b) alone or by S = 0 (r = g = b: diff 0 gives s = 0
# in any HSV conversion, and diff ≥ 1 gives s ≥ 1 with OpenCV's tables), with
# H and the other channel unconstrained, so the exclusion mask is exact
# without OpenCV.  Zones restrict two of them to windows of the cut-out M.
VS_RANGES = [(0, 0, 0, 180, 255, 40),       # dark (fill included)
             (0, 0, 96, 180, 255, 112),     # a band of V
             (0, 0, 0, 180, 0, 255)]        # grey (S = 0)
VS_ZONES = [None, (150, 40, 90, 260), (60, 200, 0, 120)]
CONFIG3_VS_SEED = 6000


def config3_vs_source(i: int) -> np.ndarray:
    """Item i's 1024² source for pipe_config3_vs_pillow.npz: a structured
    scene — colour gradients, exact greys (S = 0) at several levels (some dark,
    some inside the V band), near-greys (r = g = b + 1, S > 0), dark and
    V-band coloured shapes, thin grey lines and a noise patch — so the cut-out
    gets α edges from every range, their OR and the zone borders."""
    r = np.random.default_rng(CONFIG3_VS_SEED + i)
    yy, xx = np.mgrid[0:1024, 0:1024].astype(np.float64)
    src = np.empty((1024, 1024, 3), np.uint8)
    src[..., 0] = (xx / 4 + 30 * i) % 256
    src[..., 1] = (yy / 4 + 50 * np.sin(xx / 97.0 + i)) % 256
    src[..., 2] = 128 + 100 * np.sin((xx + yy) / 151.0 + 0.7 * i)
    for _ in range(14):
        y0, x0 = (int(v) for v in r.integers(0, 960, 2))
        hh, ww = (int(v) for v in r.integers(20, 240, 2))
        kind = int(r.integers(0, 5))
        lvl = int(r.choice([20, 38, 100, 104, 111, 150, 200, 255]))
        if kind == 0:                                    # exact grey rectangle
            src[y0:y0 + hh, x0:x0 + ww] = lvl
        elif kind == 1:                                  # near grey (S > 0)
            src[y0:y0 + hh, x0:x0 + ww] = (lvl, lvl, max(lvl - 1, 0))
        elif kind == 2:                                  # grey disc
            m = (yy - y0) ** 2 + (xx - x0) ** 2 < (hh / 2) ** 2
            src[m] = lvl
        elif kind == 3:                                  # coloured shape of V = lvl
            src[y0:y0 + hh, x0:x0 + ww] = (lvl, lvl // 3, (2 * lvl) // 5)
        else:                                            # noise patch
            src[y0:y0 + hh, x0:x0 + ww] = r.integers(0, 256, src[y0:y0 + hh, x0:x0 + ww].shape)
    for k in range(6):                                   # thin grey lines, 1-3 px
        c = 180 + 90 * k + 13 * i
        src[:, c:c + 1 + k % 3] = 60 + 30 * k
        src[c:c + 1 + (k + 1) % 3, :] = 104 if k % 2 else 255
    return src


def vs_alpha(rgb: np.ndarray) -> np.ndarray:
    """filtres_liste.py:97-134 α for VS_RANGES / VS_ZONES on the cut-out's RGB
    (any channel order): 0 where some range holds inside its zone."""
    h, w = rgb.shape[:2]
    v = rgb.max(axis=2).astype(np.int32)
    grey = rgb.min(axis=2).astype(np.int32) == v
    holds = [v <= 40, (v >= 96) & (v <= 112), grey]
    excl = np.zeros((h, w), bool)
    for hold, zone in zip(holds, VS_ZONES):
        zt, zb, zl, zr = zone if zone else (0, 0, 0, 0)
        zm = np.zeros((h, w), bool)
        zm[zt:h - zb, zl:w - zr] = True      # numpy slice, as zone_mask[...] = 255
        excl |= hold & zm
    return np.where(excl, 0, 255).astype(np.uint8)
