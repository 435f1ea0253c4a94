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
