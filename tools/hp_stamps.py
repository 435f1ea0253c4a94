#!/usr/bin/env python3
"""Where the H pass's wave time goes: runs the benchmark pipe's H pass with a
diagnostic library built with `make variant NAME=stamps "VFLAGS=-DIPP_DIAG
-DIPP_HP_STAMPS"` (IPP_LIB_PATH=variants/stamps/libipp.so) and prints the
per-wave shader-clock split: phase 1 (gathers + HSV + ring), barrier before
phase 2, phase 2 (MFMA + T stores), barrier after.  The stamps themselves cost
cycles (MI355X_MICROARCH.md: ≈+11 %), so read the split, not the total.

  IPP_LIB_PATH=$PWD/variants/stamps/libipp.so python tools/hp_stamps.py [--batch 1024] [--copy]
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--copy", action="store_true", help="the bgcopy form (copy blocks in the launch)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from image_processor_pipeline_amd import _native as N, fused
    dev = torch.device("cuda:0")
    S, K, B = 1024, 16, args.batch
    src = bench.make_sources(0, B, S, 0, dev)
    g0 = torch.Generator(device=dev)
    g0.manual_seed(1)
    bgs = torch.randint(0, 256, (K, S, S, 3), dtype=torch.uint8, device=dev, generator=g0)
    out = torch.empty((B, S, S, 3), dtype=torch.uint8, device=dev)
    plan = fused.plan_pipe((S, S), B, (S, S), K, fused.PipeConfig(), seed=0)
    runner = fused.PipeRunner(plan, dev)
    lib = N.load()
    fn = lib.ipp_diag_hp_stamps
    fn.argtypes = [ctypes.c_void_p]
    fn.restype = ctypes.c_int
    buf = np.zeros(8, np.uint64)
    run = (lambda: runner.hpass_bgcopy(src, bgs, out)) if args.copy else (lambda: runner.hpass(src))
    run()
    torch.cuda.synchronize()
    fn(buf.ctypes.data)
    for _ in range(args.reps):
        run()
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data) == 0
    p1, b1, p2, b2, waves, chunks, body = (int(v) for v in buf[:7])
    tot = p1 + b1 + p2 + b2
    print(json.dumps({"waves": waves // args.reps, "chunks_per_wave": round(chunks / max(waves, 1), 2),
                      "cycles_per_wave": round(body / max(waves, 1)),
                      "split": {"phase1": round(p1 / tot, 3), "barrier_before_p2": round(b1 / tot, 3),
                                "phase2": round(p2 / tot, 3), "barrier_after_p2": round(b2 / tot, 3)},
                      "cycles_per_chunk": {"phase1": round(p1 / chunks), "barrier1": round(b1 / chunks),
                                           "phase2": round(p2 / chunks), "barrier2": round(b2 / chunks)}}))


if __name__ == "__main__":
    main()
