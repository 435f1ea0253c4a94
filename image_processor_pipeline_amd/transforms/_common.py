"""Shared helpers for the device transforms."""
from __future__ import annotations

import concurrent.futures
from typing import Callable, Iterable, List


def device_transform(fn: Callable) -> Callable:
    """Flag a plugin as GPU-driving: ProcessingStep runs it in the
    device-owning process (threads, never forked children)."""
    fn.__ipp_device__ = True
    return fn


def thread_map(fn: Callable, items: Iterable, threads: int) -> List:
    """Ordered map on a thread pool (codec work releases the GIL); each
    result is the value or the raised Exception."""
    items = list(items)

    def guarded(x):
        try:
            return fn(x)
        except Exception as e:   # returned, not raised: per-item error handling
            return e

    if threads <= 1 or len(items) <= 1:
        return [guarded(x) for x in items]
    with concurrent.futures.ThreadPoolExecutor(max_workers=threads) as ex:
        return list(ex.map(guarded, items))
