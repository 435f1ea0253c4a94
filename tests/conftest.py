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
