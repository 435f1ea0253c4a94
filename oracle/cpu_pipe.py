"""CPU baseline for bench.py (TEST/REPORTING INFRASTRUCTURE ONLY).

Times the reference's own CPU path for one pipe item, in memory (no codecs):
the same library calls the reference's transforms make — NumPy slicing for
crop_from_border (recadrages.py:46), Pillow ``convert('RGBA')`` / ``rotate``
/ ``getbbox`` / ``crop`` (rotations.py:55, 96-101), NumPy flips for cv2.flip
(symmetry.py:114-119), the oracle's NumPy restatement of cvtColor+inRange
(filtres_liste.py:90-134; OpenCV is not installed), Pillow ``resize(LANCZOS)``
+ ``paste`` (overlays.py:129-139).  Item-level parallelism mirrors
ProcessingStep(workers=-1) → ProcessPoolExecutor (pipeline.py:84-90, 372),
capped to this job's CPU share.
"""
from __future__ import annotations

import math
import multiprocessing as mp
import os
import platform
import random
import time

import numpy as np

from oracle import ops

REF_RANGES = [
    (0, 0, 0, 180, 255, 150),
    (15, 60, 200, 35, 255, 255),
    (15, 30 * 2.55, 55 * 2.55, 30, 60 * 2.55, 80 * 2.55),
    (15, 60 * 2.55, 60 * 2.55, 30, 75 * 2.55, 90 * 2.55),
]


def _item_pipe5(src, bg, rng):
    from PIL import Image
    crop = src[64:-64, 64:-64]
    im = Image.fromarray(crop, "RGB").convert("RGBA")
    rot = im.rotate(rng.uniform(1.0, 359.0), expand=True)
    bb = rot.getbbox()
    if bb:
        rot = rot.crop(bb)
    arr = np.asarray(rot)
    sym = rng.sample(["o", "h", "v", "hv"], 1)[0]
    arr = ops.flip(arr, sym)
    bgr = arr[..., 2::-1]
    alpha = ops.hsv_alpha_mask(bgr, REF_RANGES)
    ov = Image.fromarray(np.concatenate([arr[..., :3], alpha[..., None]], -1), "RGBA")
    ratio = rng.uniform(0.15, 0.30)
    nw, nh = ops.overlay_geometry(ov.width, ov.height, bg.shape[1], bg.shape[0], ratio)
    ovr = ov.resize((nw, nh), Image.Resampling.LANCZOS)
    comp = Image.fromarray(bg, "RGB").copy()
    comp.paste(ovr, (rng.randint(0, bg.shape[1] - nw), rng.randint(0, bg.shape[0] - nh)), ovr)
    return comp


def _item_rotflip(src, bg, rng):
    from PIL import Image
    im = Image.fromarray(src, "RGB").convert("RGBA")
    rot = im.rotate(rng.uniform(1.0, 359.0), expand=True)
    bb = rot.getbbox()
    if bb:
        rot = rot.crop(bb)
    return ops.flip(np.asarray(rot), rng.sample(["o", "h", "v", "hv"], 1)[0])


def _item_video4k(src, bg, rng):
    """filtres_liste mask (NumPy restatement of cvtColor+inRange) then
    pixels_isolés keep-largest + crop-fit (SciPy labelling for cv2 CCL)."""
    return ops.keep_largest_component(ops.color_mask_bgra(src, REF_RANGES))


def _video_frame(nrng, h=2160, w=3840):
    f = np.empty((h, w, 3), np.uint8)
    f[...] = (24, 18, 30)
    yy, xx = np.mgrid[0:h, 0:w]
    u = nrng.random(4)
    cx, cy, ax, ay = w * (0.3 + 0.4 * u[0]), h * (0.3 + 0.4 * u[1]), w * (0.22 + 0.08 * u[2]), h * (0.22 + 0.08 * u[3])
    f[((xx - cx) / ax) ** 2 + ((yy - cy) / ay) ** 2 <= 1.0] = (220, 140, 40)
    sp = nrng.random((h, w)) < 0.005
    f[sp] = nrng.integers(0, 256, (int(sp.sum()), 3), np.uint8)
    return f


def _worker(task):
    seed, count, size, workload = task
    nrng = np.random.default_rng(seed)
    if workload == "video4k":
        srcs = [_video_frame(nrng) for _ in range(count)]
        bg = None
    else:
        srcs = [nrng.integers(0, 256, (size, size, 3), np.uint8) for _ in range(count)]
        bg = nrng.integers(0, 256, (size, size, 3), np.uint8)
    rng = random.Random(seed)
    fn = {"pipe5": _item_pipe5, "rotflip": _item_rotflip, "video4k": _item_video4k}[workload]
    fn(srcs[0], bg, rng)  # warm imports / allocator
    t0 = time.perf_counter()
    for s in srcs:
        fn(s, bg, rng)
    return time.perf_counter() - t0, count


def cpu_share() -> int:
    n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    cap = int(env) if env and env.isdigit() else 16
    return max(1, min(n, cap, 16))


def measure(sample: int = 192, size: int = 1024, workload: str = "pipe5") -> dict:
    workers = cpu_share()
    per = max(1, math.ceil(sample / workers))
    tasks = [(1000 + w, per, size, workload) for w in range(workers)]
    ctx = mp.get_context("spawn")
    # close + join, not the context manager: Pool.__exit__ terminates the
    # workers (SIGTERM), which a profiler wrapping the bench logs as aborts
    pool = ctx.Pool(workers)
    try:
        res = pool.map(_worker, tasks)
    finally:
        pool.close()
        pool.join()
    wall = max(t for t, _ in res)
    items = sum(c for _, c in res)
    px = 3840 * 2160 if workload == "video4k" else size * size
    mpix = items * px / 1e6
    per_item = sum(t for t, _ in res) / items
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(mpix / wall, 2),
        "unit": "Mpix/s",
        "cores": workers,
        "kind": "port",
        "sample": (f"{items} items of {'3840x2160' if workload == 'video4k' else f'{size}x{size}'}x3 ({workload}), "
                   f"{workers} worker processes, in-memory, Pillow {__import__('PIL').__version__} + NumPy "
                   f"(cv2 ops via the NumPy/SciPy restatement)"),
        "value_1core": round(px / 1e6 / per_item, 2),
        "cpu_model": model,
        # BASELINE.md asks for Pool(os.cpu_count()); the GPU box gives one
        # GPU's job a 16-CPU share of a larger machine, so the pool is capped
        # there and the all-core figure is the 1-core rate scaled linearly
        "host_cpus": os.cpu_count(),
        "value_host_cpus_linear": round(px / 1e6 / per_item * (os.cpu_count() or 1), 2),
    }


if __name__ == "__main__":
    import json
    print(json.dumps(measure(16, 1024)))
