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
