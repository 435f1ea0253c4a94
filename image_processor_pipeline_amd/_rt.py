"""Device runtime helpers for the file-mode transforms: one ROCm device per
process (the GPU-owning process of the pipeline), H2D/D2H of HWC uint8
arrays.  No CPU fallback: without a GPU or libipp.so the transforms raise
NativeUnavailable."""
from __future__ import annotations

import os
import threading

import numpy as np
import torch

from . import _native as N

_DEVICE = None
_LOCK = threading.Lock()


def device() -> torch.device:
    """The process's ROCm device, initialised once (thread-safe: GPU plugins
    may run on a ProcessingStep thread pool)."""
    global _DEVICE
    if _DEVICE is None:
        with _LOCK:
            if _DEVICE is None:
                N.load()
                if not torch.cuda.is_available():
                    raise N.NativeUnavailable("no ROCm GPU visible: the image_processor_pipeline_amd transforms run "
                                              "on MI355X only (there is no CPU fallback)")
                torch.cuda.init()
                n = torch.cuda.device_count()
                if n <= 0:
                    raise N.NativeUnavailable("no ROCm GPU visible")
                idx = int(os.environ.get("LOCAL_RANK", "0")) % n
                torch.cuda.set_device(idx)
                _DEVICE = torch.device("cuda", idx)
    return _DEVICE


def h2d(a: np.ndarray) -> torch.Tensor:
    if a.ndim == 2:
        a = a[..., None]
    return torch.from_numpy(np.require(a, requirements=["C", "W"])).to(device())


def d2h(t: torch.Tensor) -> np.ndarray:
    return t.contiguous().cpu().numpy()
