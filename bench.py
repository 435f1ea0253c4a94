#!/usr/bin/env python3
"""Benchmark of the MI355X-native hot path (BASELINE.json metric).

Default workload = BASELINE config 3: the 5-stage pipe
(crop_from_border → process_rotations → generate_symmetries →
process_images_with_color_masks → paste_overlay_onto_background) over a batch
of B = 4096 synthetic 1024×1024×3 uint8 sources per GPU, pasted onto 16 shared
1024×1024 backgrounds.  One "step" = one pass of the pipe over the batch with
inputs resident in HBM.  N > 1: one process per GPU (torchrun), items sharded
(weak scaling, no data-path collective); the backgrounds are generated on rank
0 and broadcast once over RCCL.  Rank 0 prints ONE JSON line.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
                  [--workload pipe5|rotflip] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "Mpixels/sec through 5-stage pipe, 1024×1024 uint8; achieved HBM GB/s"
METRICS = {"pipe5": METRIC,
           "rotflip": "Mpixels/sec through rotations+symmetry fused gather, 1024×1024 uint8; achieved HBM GB/s",
           "video4k": "Mpixels/sec through the 4K despeckle chain (filtres_liste -> pixels_isolés), 3840×2160 uint8"}
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="items per GPU")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--backgrounds", type=int, default=16)
    ap.add_argument("--workload", choices=["pipe5", "rotflip", "video4k"], default="pipe5")
    ap.add_argument("--frames", type=int, default=256, help="video4k: 3840x2160 frames per GPU")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=192)
    ap.add_argument("--unsplit", action="store_true", help="pipe5: ipp_pipe_hpass + full-frame ipp_pipe_vblend")
    return ap.parse_args()


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, world, torch.device("cuda", local)


def barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def load_pmc_traffic(workload: str, kernel: str, batch: int):
    """Per-launch HBM bytes of the dominant kernel from the committed rocprofv3
    PMC summary (profiles/pmc_traffic.json, produced by tools/pmc_traffic.py
    from separate FETCH_SIZE / WRITE_SIZE passes of this bench at the default
    batch, gfx950 FETCH_SIZE ×2 correction applied).  None when absent or
    measured at another batch."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    try:
        d = json.loads(f.read_text())[workload]
        if d.get("_batch") not in (None, batch):
            return None
        return int(d[kernel]["hbm_bytes"])
    except Exception:
        return None


def make_sources(start: int, stop: int, size: int, seed: int, dev) -> torch.Tensor:
    """Synthetic sources, item i drawn from its own generator (seed, i): the
    bytes of an item do not depend on how the batch is sharded."""
    src = torch.empty((stop - start, size, size, 3), dtype=torch.uint8, device=dev)
    gen = torch.Generator(device=dev)
    for i in range(start, stop):
        gen.manual_seed(seed * 1000003 + i)
        src[i - start].random_(0, 256, generator=gen)
    return src


def cpu_baseline(args):
    from oracle import cpu_pipe
    sample = min(args.cpu_sample, 32) if args.workload == "video4k" else args.cpu_sample
    return cpu_pipe.measure(sample, size=args.size, workload=args.workload)


def main():
    args = parse()
    rank, world, dev = init_dist(args)
    from image_processor_pipeline_amd import fused, device as D

    B, S, K = args.batch, args.size, args.backgrounds
    scratch_bytes = None
    if args.workload == "video4k":
        B, FH, FW = args.frames, 2160, 3840
    # weak scaling: B items per GPU; rank r owns global items [r*B, (r+1)*B)
    start, stop = fused.shard_range(world * B, rank, world)
    if args.workload != "video4k":
        src = make_sources(start, stop, S, args.seed, dev)

    t_plan = time.perf_counter()
    if args.workload == "pipe5":
        bgs = torch.empty((K, S, S, 3), dtype=torch.uint8, device=dev)
        if rank == 0:
            g0 = torch.Generator(device=dev)
            g0.manual_seed(1)
            bgs.copy_(torch.randint(0, 256, (K, S, S, 3), dtype=torch.uint8, device=dev, generator=g0))
        if world > 1:
            dist.broadcast(bgs, src=0)  # the one exchange step: shared assets over xGMI
        cfg = fused.PipeConfig()
        plan = fused.plan_pipe((S, S), B, (S, S), K, cfg, seed=args.seed * 7919, item_range=(start, stop))
        runner = fused.PipeRunner(plan, dev)
        out = torch.empty((B, S, S, 3), dtype=torch.uint8, device=dev)
        if runner.split and not args.unsplit:
            # the H pass also copies the background rows outside the overlay bands
            algo = {"ipp_pipe_hpass_bgcopy": plan.algo_bytes_hpass_bgcopy,
                    "ipp_pipe_vblend_bands": plan.algo_bytes_vblend_bands}
            launches = [("ipp_pipe_hpass_bgcopy", lambda: runner.hpass_bgcopy(src, bgs, out)),
                        ("ipp_pipe_vblend_bands", lambda: runner.vblend_bands(bgs, out))]
        else:
            algo = {"ipp_pipe_hpass": plan.algo_bytes_hpass, "ipp_pipe_vblend": plan.algo_bytes_vblend}
            launches = [("ipp_pipe_hpass", lambda: runner.hpass(src)),
                        ("ipp_pipe_vblend", lambda: runner.vblend(bgs, out))]
        workload = "5-stage pipe: crop(64px)->rotate(NEAREST,expand,bbox)->flip->HSV mask(4 ref ranges)->LANCZOS+paste"
    elif args.workload == "video4k":
        from image_processor_pipeline_amd import video_chain
        frames = video_chain.synthetic_frames(B, FH, FW, args.seed + 2, dev, start=start)
        chain = video_chain.VideoChain(B, FH, FW, dev)
        chain.run(frames)
        torch.cuda.synchronize()
        bb = chain.bbox.cpu().numpy().reshape(B, 4)
        a_crop = int(sum(max(0, x1 - x0) * max(0, y1 - y0) for x0, y0, x1, y1 in bb))
        hw = B * FH * FW
        # compulsory bytes: read each BGR frame once, write the BGRA crop once
        # (the uint16 label plane and per-component scratch are reported apart)
        algo = {"ipp_video_keep_largest": 3 * hw + 4 * a_crop}
        scratch_bytes = B * (2 * FH * FW)
        launches = [("ipp_video_keep_largest", lambda: chain.run(frames))]
        workload = ("4K video chain: HSV mask (4 ref ranges) -> largest 8-connected component -> crop-fit, "
                    "fused, structured frames (blob + 0.5% specks)")
    else:
        import random
        rng = random.Random(args.seed)
        draws = [(rng.uniform(1.0, 359.0), rng.sample(["o", "h", "v", "hv"], 1)[0]) for _ in range(stop)][start:]
        angles = [a for a, _ in draws]
        flips = [D.SYM_FLIP[s_] for _, s_ in draws]
        gplan = D.plan_rotate_flip([(S, S, 3)] * B, angles, flips, src_offsets=[i * S * S * 3 for i in range(B)])
        descs = D._to_dev(gplan.descs, dev)
        out = torch.empty(gplan.total_bytes, dtype=torch.uint8, device=dev)
        flat = src.reshape(-1)
        a_out = sum(h * w * 4 for h, w in gplan.shapes)
        algo = {"ipp_rotate_flip_nearest": 3 * S * S * B + a_out}
        launches = [("ipp_rotate_flip_nearest", lambda: D.rotate_flip_nearest(flat, gplan, out, descs))]
        workload = "rotations+symmetry fused gather (NEAREST rotate, expand, bbox crop, flip)"
    plan_ms = (time.perf_counter() - t_plan) * 1e3

    stream = torch.cuda.current_stream(dev)

    def step(events=None):
        for j, (_, fn) in enumerate(launches):
            if events is not None:
                events[j][0].record(stream)
            fn()
            if events is not None:
                events[j][1].record(stream)

    for _ in range(args.warmup):
        step()
    barrier(world)
    evs = [[[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in launches]
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    barrier(world)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per kernel: time per step summed over its launches (chunked pipe: one
    # hpass/vblend pair per chunk)
    per_kernel_ms = {}
    for j, (name, _) in enumerate(launches):
        per_kernel_ms[name] = per_kernel_ms.get(name, 0.0) + float(np.mean([e[j][0].elapsed_time(e[j][1]) for e in evs]))
    n_launch = {name: sum(1 for nm, _ in launches if nm == name) for name in per_kernel_ms}
    dominant = max(per_kernel_ms, key=per_kernel_ms.get)
    ms_step = elapsed / args.steps * 1e3
    mpix = world * B * (FH * FW if args.workload == "video4k" else S * S) / 1e6
    value = mpix * args.steps / elapsed
    achieved = algo[dominant] / (per_kernel_ms[dominant] * 1e-3) / 1e9
    step_algo = sum(algo.values())
    result = {
        "metric": METRICS[args.workload],
        "value": round(value, 1),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": workload, "global_batch": world * B, "batch_per_gpu": B,
                   "image": "3840x2160x3 uint8" if args.workload == "video4k" else f"{S}x{S}x3 uint8",
                   "backgrounds": K if args.workload == "pipe5" else 0,
                   "parallelism": (f"dp{world} (item sharding, RCCL broadcast of backgrounds)"
                                   if args.workload == "pipe5" else f"dp{world} (replicas, item sharding)")},
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": load_pmc_traffic(args.workload, dominant, B),
                     "algo_bytes_per_launch": int(algo[dominant] / n_launch[dominant]),
                     "avg_launch_ms": round(per_kernel_ms[dominant] / n_launch[dominant], 4),
                     "launches_per_step": n_launch[dominant]},
        "step_hbm_gbps_algorithmic": round(step_algo / (ms_step * 1e-3) / 1e9, 1),
        "kernels_ms": {k: round(v, 4) for k, v in per_kernel_ms.items()},
        "kernels_algo_bytes": {k: int(v) for k, v in algo.items()},
        "plan_ms": round(plan_ms, 1),
    }
    if scratch_bytes is not None:
        result["label_scratch_bytes_per_step"] = int(scratch_bytes)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(args)
        except Exception as e:  # reported, never fatal to the GPU number
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
