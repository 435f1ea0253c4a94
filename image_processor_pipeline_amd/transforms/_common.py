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


def batch_run(arg_tuples, threads: int, load: Callable, compute: Callable, save: Callable) -> List:
    """The codec-boundary pattern of the plugins' ``.batch`` hooks: ``load``
    (validation + decode, one call per tuple) on host threads; ``compute``
    once for the chunk with the loaded items in input order (random draws
    happen there, in the per-file order; one batched device call); ``save``
    (encode) on host threads.  An exception raised by ``load`` or ``save`` for
    one tuple becomes that tuple's result, as a per-file call would raise it."""
    loaded = thread_map(load, arg_tuples, threads)
    ok = [i for i, x in enumerate(loaded) if not isinstance(x, Exception)]
    outs = compute([loaded[i] for i in ok], [arg_tuples[i] for i in ok]) if ok else []
    by = dict(zip(ok, outs))

    def fin(i):
        if isinstance(loaded[i], Exception):
            raise loaded[i]
        return save(arg_tuples[i], loaded[i], by[i])

    return thread_map(fin, range(len(arg_tuples)), threads)
