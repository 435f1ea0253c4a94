#!/usr/bin/env python3
"""File-mode throughput of the reference's dataset chain (SURVEY §8(f) rank 1,
the codec boundary) — reported apart from bench.py's kernel metric.

Runs the five steps of the benchmark pipe through ProcessingPipeline on N
synthetic JPG sources (size S) and K PNG backgrounds, files between steps as
in the reference (crop_from_border JPG → rotations PNG → symmetries PNG →
colour mask PNG → overlays), twice:
  * batched: every plugin's .batch hook (threaded decode, one batched launch
    per chunk, threaded encode), `--threads` host threads;
  * per-file: the same plugins called one file at a time (the reference's
    sequential loop), device ops per file.
Prints one JSON line: items/s of each mode, host thread count, and the
share of wall time spent outside the device (codecs + file system).

  python tools/bench_filemode.py [--items 64] [--size 1024] [--threads 16]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import shutil
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def build(root: Path, threads: int, batch: int, per_file: bool):
    from image_processor_pipeline_amd import geometry as G
    from image_processor_pipeline_amd.pipeline import ProcessingPipeline, ProcessingStep
    from image_processor_pipeline_amd.transforms import filtres_liste, overlays, recadrages, rotations, symmetry
    fns = [recadrages.crop_from_border, rotations.process_rotations, symmetry.generate_symmetries,
           filtres_liste.process_images_with_color_masks, overlays.paste_overlay_onto_background]
    saved = {f: f.batch for f in fns}
    if per_file:
        for f in fns:
            del f.batch
    w = 1 if per_file else threads
    pipe = ProcessingPipeline(root_dir=root)
    pipe.add_step(ProcessingStep("crop", fns[0], root / "src", "c", workers=w, batch_size=batch,
                                 options={"crop_margins": (64, 64, 64, 64)}))
    pipe.add_step(ProcessingStep("rot", fns[1], output_dirs="r", workers=w, batch_size=batch,
                                 options={"num_rotations": 1, "include_original": False}))
    pipe.add_step(ProcessingStep("sym", fns[2], output_dirs="s", workers=w, batch_size=batch,
                                 options={"choose_random": 1, "include_original": False}))
    pipe.add_step(ProcessingStep("mask", fns[3], output_dirs="m", workers=w, batch_size=batch,
                                 options={"color_ranges_to_exclude_hsv": G.REFERENCE_HSV_RANGES}))
    pipe.add_step(ProcessingStep("ovl", fns[4], ["m", root / "bg"], ["oi", "ol"], pairing_method="modulo",
                                 fixed_input=True, workers=w, batch_size=batch))
    return pipe, (lambda: [setattr(f, "batch", b) for f, b in saved.items()])


def run(mode: str, base: Path, args) -> float:
    import numpy as np
    from PIL import Image
    root = base / mode
    (root / "src").mkdir(parents=True)
    (root / "bg").mkdir()
    rng = np.random.default_rng(0)
    for i in range(args.items):
        Image.fromarray(rng.integers(0, 256, (args.size, args.size, 3), np.uint8)).save(
            root / "src" / f"s{i:05d}.jpg", quality=95)
    for k in range(args.backgrounds):
        Image.fromarray(rng.integers(0, 256, (args.size, args.size, 3), np.uint8)).save(root / "bg" / f"b{k:02d}.png")
    pipe, restore = build(root, args.threads, args.batch, mode == "per_file")
    random.seed(0)
    t0 = time.perf_counter()
    try:
        pipe.run()
    finally:
        restore()
    dt = time.perf_counter() - t0
    n = len(list((root / "oi").iterdir()))
    if n != args.items:
        raise SystemExit(f"{mode}: {n} composites for {args.items} items")
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=64)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--backgrounds", type=int, default=4)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--batch", type=int, default=32)
    args = ap.parse_args()
    import contextlib
    import io
    base = Path(tempfile.mkdtemp(prefix="ipp_filemode_"))
    try:
        res = {}
        for mode in ("batched", "per_file"):
            with contextlib.redirect_stdout(io.StringIO()):
                res[mode] = run(mode, base, args)
        print(json.dumps({"metric": "file-mode items/s through the 5-step pipe (files between steps)",
                          "items": args.items, "image": f"{args.size}x{args.size}x3 JPG sources",
                          "batched_items_per_s": round(args.items / res["batched"], 2),
                          "per_file_items_per_s": round(args.items / res["per_file"], 2),
                          "batched_s": round(res["batched"], 2), "per_file_s": round(res["per_file"], 2),
                          "host_threads": args.threads, "batch_size": args.batch,
                          "note": "codec-bound (PNG/JPEG encode+decode on host threads); the kernel metric is "
                                  "bench.py's"}), flush=True)
    finally:
        shutil.rmtree(base, ignore_errors=True)


if __name__ == "__main__":
    main()
