#!/usr/bin/env python3
"""Benchmark of the MI355X-native hot path (BASELINE.json metric).

Default workload = BASELINE config 3: the 5-stage pipe
(crop_from_border → process_rotations → generate_symmetries →
process_images_with_color_masks → paste_overlay_onto_background) over a batch
of B = 4096 synthetic 1024×1024×3 uint8 sources per GPU, pasted onto 16 shared
1024×1024 backgrounds.  One "step" = one pass of the pipe over the batch with
inputs resident in HBM.  Rank 0 prints ONE JSON line.

Multi-GPU (config 4): one process per GPU.  Under ``torchrun`` the ranks come
from the environment; ``python bench.py --gpus N`` without it spawns the N
rank processes itself (before this process touches any GPU) and exits with
their status.  ``--scaling weak`` (default) gives every GPU B items;
``--scaling strong`` splits one global batch of B items over the GPUs
(contiguous blocks, ``fused.shard_range``).  Items are independent, so the
only collective on the data path is the one RCCL broadcast of the shared
backgrounds; timing is the max over ranks.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
                  [--scaling weak|strong] [--workload pipe5|rotflip|video4k]
                  [--no-cpu-baseline] [--dump-digests FILE] [--dry-run]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Mpixels/sec through 5-stage pipe, 1024×1024 uint8; achieved HBM GB/s"
METRICS = {"pipe5": METRIC,
           "rotflip": "Mpixels/sec through rotations+symmetry fused gather, 1024×1024 uint8; achieved HBM GB/s",
           "video4k": "Mpixels/sec through the 4K despeckle chain (filtres_liste -> pixels_isolés), 3840×2160 uint8"}
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="items per GPU (weak scaling) or in total (strong scaling); default 4096 for pipe5 "
                         "(config 3), 1024 for rotflip (config 2)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--backgrounds", type=int, default=16)
    ap.add_argument("--workload", choices=["pipe5", "rotflip", "video4k"], default=None,
                    help="pipe5 (default; with the rotflip and video4k legs unless --no-legs), or one workload alone")
    ap.add_argument("--frames", type=int, default=256,
                    help="video4k: 3840x2160 frames per GPU (weak) or in total (strong)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--rot-row-align", type=int, default=128,
                    help="rotflip: output row pitch alignment in bytes (A/B of the store alignment)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=192)
    ap.add_argument("--no-copy-ceiling", action="store_true")
    ap.add_argument("--stream", action="store_true",
                    help="pipe5: the streaming leg (the default; kept for scripts)")
    ap.add_argument("--no-stream", action="store_true",
                    help="pipe5: skip the streaming leg (a new plan per batch, planned on a host thread while the "
                         "previous batch runs), which is otherwise timed after the resident step and reported "
                         "beside it")
    ap.add_argument("--stream-default-priority", action="store_true",
                    help="--stream: launch the pipe on the default-priority stream (not a high-priority one)")
    ap.add_argument("--stream-lookahead", type=int, default=2,
                    help="--stream: batches planned ahead of the running one (worker threads, side streams)")
    ap.add_argument("--pipe-parts", type=int, default=1,
                    help="pipe5: run the batch as N item ranges, each range's V launch on a side stream "
                         "overlapping the next range's H launch (1 = the two launches back to back)")
    ap.add_argument("--pipe-ratio", type=float, default=1.0,
                    help="pipe5 with --pipe-parts: item range k holds a share proportional to ratio**k")
    ap.add_argument("--no-legs", action="store_true",
                    help="pipe5: skip the config-2 (rotflip) and config-5 (video4k) legs that the default run "
                         "times after the headline and reports under 'workloads'")
    ap.add_argument("--frame-noise", type=int, default=0,
                    help="video4k: +-N LSB of uniform noise per channel on the synthetic frames (0 = flat frames)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="gloo: CPU rehearsal of the N-rank path (tests)")
    ap.add_argument("--dump-digests", default=None,
                    help="rank 0 writes {global item: sha1 of its output} (outputs of every rank)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: plan, shard and broadcast, no kernels (launcher tests); digests are of the "
                         "per-item inputs and parameters")
    return ap.parse_args(argv)


# --------------------------------------------------------------------------
# N-process launcher (no torchrun)
# --------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n: int, argv) -> int:
    """Start the n rank processes of this same command and wait for them.

    This process has not touched a GPU (torch is not even imported); every
    rank is a fresh child process.  If one rank fails the others are
    terminated (they would otherwise wait in a collective) and the first
    failing status is returned."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


# --------------------------------------------------------------------------
def init_dist(args):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but {world} rank(s) are running (WORLD_SIZE={world})")
    if args.dry_run:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
        return rank, world, dev
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise SystemExit("bench.py: no ROCm GPU visible (use --dry-run for a CPU rehearsal)")
    if args.dist_backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: {world} ranks need {world} GPUs for RCCL, {ndev} visible")
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return rank, world, dev


def barrier(world, dev):
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def broadcast(t, world, backend):
    """The one exchange step: shared assets from rank 0 over RCCL/xGMI (gloo:
    through the host)."""
    import torch.distributed as dist

    if world <= 1:
        return
    if backend == "gloo" and t.is_cuda:
        h = t.cpu()
        dist.broadcast(h, src=0)
        t.copy_(h)
    else:
        dist.broadcast(t, src=0)


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


def make_sources(start: int, stop: int, size: int, seed: int, dev):
    """Synthetic sources, item i drawn from its own generator (seed, i): the
    bytes of an item do not depend on how the batch is sharded."""
    import torch

    src = torch.empty((stop - start, size, size, 3), dtype=torch.uint8, device=dev)
    gen = torch.Generator(device=dev)
    for i in range(start, stop):
        gen.manual_seed(seed * 1000003 + i)
        src[i - start].random_(0, 256, generator=gen)
    return src


def copy_ceiling(dev, nbytes: int = 1 << 30, reps: int = 10) -> float:
    """HBM GB/s of ipp_stream_copy over `nbytes` (read + write counted),
    measured here with HIP events: the copy-kernel ceiling of this box."""
    import torch
    from image_processor_pipeline_amd import _native as N
    from image_processor_pipeline_amd.device import _stream

    lib = N.load()
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a.fill_(7)
    st = _stream(dev)
    for _ in range(3):
        N.check(lib.ipp_stream_copy(a.data_ptr(), b.data_ptr(), nbytes, st), "ipp_stream_copy")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream(dev)
    e0.record(stream)
    for _ in range(reps):
        N.check(lib.ipp_stream_copy(a.data_ptr(), b.data_ptr(), nbytes, st), "ipp_stream_copy")
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    del a, b
    torch.cuda.empty_cache()
    return 2 * nbytes / (ms * 1e-3) / 1e9


def cpu_baseline(args):
    from oracle import cpu_pipe
    sample = min(args.cpu_sample, 32) if args.workload == "video4k" else args.cpu_sample
    return cpu_pipe.measure(sample, size=args.size, workload=args.workload)


def _digest(*arrays) -> str:
    h = hashlib.sha1()
    for a in arrays:
        h.update(memoryview(a).cast("B"))
    return h.hexdigest()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args.gpus, argv))
    legs = args.workload is None and not args.no_legs and not args.dry_run and not args.dump_digests
    if args.workload is None:
        args.workload = "pipe5"

    import copy
    import torch
    import torch.distributed as dist

    rank, world, dev = init_dist(args)
    result = run_workload(args, rank, world, dev)
    if legs and result is not None:
        # BASELINE configs 2 and 5 on the same box in the same run, each at
        # its own default size (B = 1024 items; 256 frames per GPU)
        result["workloads"] = {}
        for wl in ("rotflip", "video4k"):
            torch.cuda.empty_cache()
            a = copy.copy(args)
            a.workload, a.batch = wl, None
            r = run_workload(a, rank, world, dev)
            if r is not None:
                result["workloads"][wl] = leg_summary(r)
    if rank == 0 and result is not None:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def leg_summary(r: dict) -> dict:
    """The compact record of a secondary workload (the driver keeps only the
    tail of the line): its metric is the headline's, on that workload."""
    rf = r["roofline"]
    out = {"value": r["value"], "unit": r["unit"], "ms_per_step": r["ms_per_step"],
           "batch": r["config"]["global_batch"], "image": r["config"]["image"],
           "roofline": {k: rf[k] for k in ("kernel", "achieved", "frac", "traffic", "traffic_frac") if k in rf}}
    out["roofline"]["step_frac"] = rf["step"]["frac"]
    for k in ("label_scratch_bytes_per_step", "crop_reread_bytes_per_step"):
        if k in r:
            out[k] = r[k]
    if "cpu_baseline" in r:
        cb = r["cpu_baseline"]
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "cores", "kind", "value_1core") if k in cb}
    return out


def run_workload(args, rank, world, dev):
    """One workload's timed run; returns its JSON record (rank 0), or None
    for --dry-run (the digests are written here)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from image_processor_pipeline_amd import fused, device as D

    S, K = args.size, args.backgrounds
    if args.batch is None:
        args.batch = 1024 if args.workload == "rotflip" else 4096
    per_gpu = args.frames if args.workload == "video4k" else args.batch
    n_global = per_gpu if args.scaling == "strong" else world * per_gpu
    start, stop = fused.shard_range(n_global, rank, world)
    B = stop - start
    FH, FW = 2160, 3840
    scratch_bytes = None
    reread_bytes = None
    launches = []
    digests = {}
    fused_bound = None
    bg_copy = None

    t_plan = time.perf_counter()
    setup = {}
    if args.workload == "pipe5":
        src = make_sources(start, stop, S, args.seed, dev)
        bgs = torch.empty((K, S, S, 3), dtype=torch.uint8, device=dev)
        if rank == 0:
            g0 = torch.Generator(device=dev)
            g0.manual_seed(1)
            bgs.copy_(torch.randint(0, 256, (K, S, S, 3), dtype=torch.uint8, device=dev, generator=g0))
        broadcast(bgs, world, args.dist_backend)
        cfg = fused.PipeConfig()
        if torch.device(dev).type == "cuda":
            torch.cuda.synchronize(dev)
        t_src = time.perf_counter()
        setup["sources_ms"] = round((t_src - t_plan) * 1e3, 1)

        def plan_batch(k):
            return fused.plan_pipe((S, S), B, (S, S), K, cfg, seed=args.seed * 7919 + k, item_range=(start, stop),
                                   n_global=n_global)
        plan = plan_batch(0)
        t_host = time.perf_counter()
        setup["plan_host_ms"] = round((t_host - t_src) * 1e3, 1)
        setup["plan_threads"] = fused.plan_threads()
        # fused lower bound: read the crop, read the background,
        # write the composite, once each
        mt, mb, ml, mr = fused.G.crop_margins(S, S, cfg.margins)
        fused_item = 3 * (S - mt - mb) * (S - ml - mr) + 2 * 3 * S * S
        fused_bound = fused_item * B
        out = torch.empty((B, S, S, 3), dtype=torch.uint8, device=dev)
        if args.dry_run:
            digests = {start + i: _digest(src[i].numpy(), np.array([p.angle, p.ratio, p.x, p.y, p.bg_index]),
                                          np.frombuffer(p.sym.encode(), np.uint8), bgs[p.bg_index].numpy())
                       for i, p in enumerate(plan.params)}
        else:
            runner = fused.PipeRunner(plan, dev)
            setup["taps_device_ms"] = round((time.perf_counter() - t_host) * 1e3, 1)
            setup["taps_host_tiles"] = runner.host_tiles
            # the H pass also copies the background rows outside the overlay bands
            algo = {"ipp_pipe_hpass_bgcopy": plan.algo_bytes_hpass_bgcopy,
                    "ipp_pipe_vblend_bands": plan.algo_bytes_vblend_bands}
            # the H launch's copy loads each background vector once per run
            # of same-background items in a copy group (the formula above
            # counts one background read per item)
            from image_processor_pipeline_amd import _native
            bg_copy = {"bg_bytes_loaded": int(plan.copy_read_bytes), "items_per_group": _native.IPP_PIPE_COPY_GROUP}
            launches = [("ipp_pipe_hpass_bgcopy", lambda: runner.hpass_bgcopy(src, bgs, out)),
                        ("ipp_pipe_vblend_bands", lambda: runner.vblend_bands(bgs, out))]
            if args.pipe_parts > 1:
                launches = [("ipp_pipe_overlapped", lambda: runner.run_overlapped(src, bgs, out, args.pipe_parts,
                                                                                     args.pipe_ratio))]
                algo = {"ipp_pipe_overlapped": sum(algo.values())}
        outputs = lambda: {start + i: _digest(out[i].cpu().numpy()) for i in range(B)}
        workload = "5-stage pipe: crop(64px)->rotate(NEAREST,expand,bbox)->flip->HSV mask(4 ref ranges)->LANCZOS+paste"
    elif args.workload == "video4k":
        from image_processor_pipeline_amd import video_chain
        frames = video_chain.synthetic_frames(B, FH, FW, args.seed + 2, dev, start=start, noise=args.frame_noise)
        if args.dry_run:
            digests = {start + i: _digest(frames[i].numpy()) for i in range(B)}
        else:
            chain = video_chain.VideoChain(B, FH, FW, dev)
            chain.run(frames)
            torch.cuda.synchronize(dev)
            bb = chain.bbox.cpu().numpy().reshape(B, 4)
            a_crop = int(sum(max(0, x1 - x0) * max(0, y1 - y0) for x0, y0, x1, y1 in bb))
            hw = B * FH * FW
            # compulsory bytes: read each BGR frame once, write the BGRA crop once
            # (the per-tile mask words and edge roots, 1.5 KB per 64x64 tile at
            # most, and the per-component scratch are reported apart)
            algo = {"ipp_video_keep_largest": 3 * hw + 4 * a_crop}
            scratch_bytes = B * ((FW + 63) // 64) * ((FH + 63) // 64) * (512 + 1024)
            # second pass over the crop (k_ccl_inwords + k_ccl_crop_stream):
            # the BGR crop re-read, its mask words read (8 B per tile row), the
            # in-words pass's 512 B per tile read and written
            reread_bytes = 3 * a_crop + a_crop // 8 + a_crop // 4
            launches = [("ipp_video_keep_largest", lambda: chain.run(frames))]

            def outputs():
                res = {}
                bbs = chain.bbox.cpu().numpy().reshape(B, 4)
                for i in range(B):
                    x0, y0, x1, y1 = (int(v) for v in bbs[i])
                    crop = chain.out[i, :max(0, y1 - y0), :max(0, x1 - x0)].cpu().numpy() if x0 >= 0 else np.zeros(0)
                    res[start + i] = _digest(bbs[i], np.ascontiguousarray(crop))
                return res
        workload = ("4K video chain: HSV mask (4 ref ranges) -> largest 8-connected component -> crop-fit, "
                    "fused, structured frames (blob + 0.5% specks)")
    else:
        import random
        src = make_sources(start, stop, S, args.seed, dev)
        # rotations step over every file (rotations.py:89), then the symmetry
        # step over every file (symmetry.py:122): step-major, as a chained run
        rng = random.Random(args.seed)
        all_angles = [rng.uniform(1.0, 359.0) for _ in range(n_global)]
        all_syms = [rng.sample(["o", "h", "v", "hv"], 1)[0] for _ in range(n_global)]
        angles, syms = all_angles[start:stop], all_syms[start:stop]
        flips = [D.SYM_FLIP[s_] for s_ in syms]
        gplan = D.plan_rotate_flip([(S, S, 3)] * B, angles, flips, src_offsets=[i * S * S * 3 for i in range(B)],
                                   row_align=args.rot_row_align)
        if args.dry_run:
            digests = {start + i: _digest(src[i].numpy(), np.array([angles[i], flips[i]])) for i in range(B)}
        else:
            descs = D._to_dev(gplan.descs, dev)
            out = torch.empty(gplan.total_bytes, dtype=torch.uint8, device=dev)
            flat = src.reshape(-1)
            a_out = sum(h * w * 4 for h, w in gplan.shapes)
            algo = {"ipp_rotate_flip_nearest": 3 * S * S * B + a_out}
            launches = [("ipp_rotate_flip_nearest", lambda: D.rotate_flip_nearest(flat, gplan, out, descs))]

            def outputs():
                host = out.cpu().numpy()
                res = {}
                for i, ((oh, ow), off, pitch) in enumerate(zip(gplan.shapes, gplan.offsets, gplan.pitches)):
                    img = np.lib.stride_tricks.as_strided(host[int(off):], (oh, ow, 4), (int(pitch), 4, 1))
                    res[start + i] = _digest(np.ascontiguousarray(img))
                return res
        workload = "rotations+symmetry fused gather (NEAREST rotate, expand, bbox crop, flip)"
    plan_ms = (time.perf_counter() - t_plan) * 1e3
    if "plan_host_ms" in setup:   # planning proper, without making the synthetic sources
        plan_ms = setup["plan_host_ms"] + setup.get("taps_device_ms", 0.0)

    if args.dry_run:
        if world > 1:
            parts = [None] * world
            dist.all_gather_object(parts, digests)
            digests = {k: v for p in parts for k, v in p.items()}
        if rank == 0:
            if args.dump_digests:
                Path(args.dump_digests).write_text(json.dumps({str(k): v for k, v in sorted(digests.items())}))
            print(json.dumps({"metric": METRICS[args.workload], "dry_run": True, "n_gpus": world,
                              "scaling": args.scaling, "global_batch": n_global, "items": len(digests),
                              "plan_ms": round(plan_ms, 1)}), flush=True)
        return None

    ceiling = None
    if not args.no_copy_ceiling:
        barrier(world, dev)
        ceiling = copy_ceiling(dev)
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
    barrier(world, dev)
    evs = [[[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in launches]
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    barrier(world, dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    stream_res = None
    if not args.no_stream and args.workload == "pipe5":
        # Streaming: batch k of the timed run has its own plan (seed + k),
        # planned on a worker thread (host planner + device taps on a side
        # stream) while batch k-1 runs.  The clock starts with the pipeline
        # primed and stops when the last batch has finished.
        ps = fused.PipeStream(dev, plan_batch, priority=not args.stream_default_priority,
                              lookahead=args.stream_lookahead)
        clock = {}

        def mark():
            barrier(world, dev)
            clock["t0"] = time.perf_counter()
        mark.at = args.warmup
        ps.run(args.warmup + args.steps, src, bgs, out, mark=mark, record=True)
        barrier(world, dev)
        s_elapsed = time.perf_counter() - clock["t0"]
        if world > 1:
            t = torch.tensor([s_elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            s_elapsed = float(t.item())
        tim = ps.timing[args.warmup:]
        kms = [a.elapsed_time(b) for a, b in ps.events[args.warmup:]]
        stream_res = {"ms_per_step": round(s_elapsed / args.steps * 1e3, 3),
                      "value": round(n_global * S * S / 1e6 * args.steps / s_elapsed, 1),
                      "kernel_ms": round(float(np.mean(kms)), 4),
                      "plan_host_ms": round(float(np.mean([t[0] for t in tim])), 2),
                      "taps_device_ms": round(float(np.mean([t[1] for t in tim])), 2),
                      "taps_host_tiles": round(float(np.mean([t[2] for t in tim])), 1),
                      "lookahead": ps.lookahead}

    if args.dump_digests:
        mine = outputs()
        if world > 1:
            parts = [None] * world
            dist.all_gather_object(parts, mine)
            mine = {k: v for p in parts for k, v in p.items()}
        if rank == 0:
            Path(args.dump_digests).write_text(json.dumps({str(k): v for k, v in sorted(mine.items())}))

    # per kernel: time per step summed over its launches
    per_kernel_ms = {}
    for j, (name, _) in enumerate(launches):
        per_kernel_ms[name] = per_kernel_ms.get(name, 0.0) + float(np.mean([e[j][0].elapsed_time(e[j][1]) for e in evs]))
    n_launch = {name: sum(1 for nm, _ in launches if nm == name) for name in per_kernel_ms}
    dominant = max(per_kernel_ms, key=per_kernel_ms.get)
    ms_step = elapsed / args.steps * 1e3
    px_item = FH * FW if args.workload == "video4k" else S * S
    mpix = n_global * px_item / 1e6
    value = mpix * args.steps / elapsed
    achieved = algo[dominant] / (per_kernel_ms[dominant] * 1e-3) / 1e9
    step_algo = sum(algo.values())
    traffic = load_pmc_traffic(args.workload, dominant, B)
    roofline = {"bound": "hbm", "kernel": dominant, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "algo_bytes_per_launch": int(algo[dominant] / n_launch[dominant]),
                "avg_launch_ms": round(per_kernel_ms[dominant] / n_launch[dominant], 4),
                "launches_per_step": n_launch[dominant]}
    if traffic:
        # the launch's real HBM rate: its PMC bytes (committed profile of this
        # workload at this batch) over its HIP-event time, against the peak
        roofline["traffic_gbps"] = round(traffic / n_launch[dominant] / (roofline["avg_launch_ms"] * 1e-3) / 1e9, 1)
        roofline["traffic_frac"] = round(roofline["traffic_gbps"] / HBM_PEAK_GBPS, 4)
    if ceiling:
        roofline["copy_ceiling"] = round(ceiling, 1)
        roofline["frac_of_copy_ceiling"] = round(achieved / ceiling, 4)
    # The whole step against the same peak: every launch's algorithmic bytes
    # over the driver-clocked step time, so moving work (or bytes) from one
    # launch to another cannot move it; with pipe5 also the fixed fused lower
    # bound (read the crop, read the background, write the composite).
    step_gbps = step_algo / (ms_step * 1e-3) / 1e9
    roofline["step"] = {"algo_bytes": int(step_algo), "ms": round(ms_step, 3), "achieved": round(step_gbps, 1),
                        "frac": round(step_gbps / HBM_PEAK_GBPS, 4)}
    if fused_bound is not None:
        roofline["step"]["fused_bound_bytes"] = int(fused_bound)
        roofline["step"]["fused_bound_frac"] = round(fused_bound / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    result = {
        "metric": METRICS[args.workload],
        "value": round(value, 1),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": workload, "global_batch": n_global, "batch_per_gpu": B,
                   "image": "3840x2160x3 uint8" if args.workload == "video4k" else f"{S}x{S}x3 uint8",
                   "backgrounds": K if args.workload == "pipe5" else 0,
                   "parallelism": (f"dp{world} (item sharding, RCCL broadcast of backgrounds)"
                                   if args.workload == "pipe5" else f"dp{world} (replicas, item sharding)")},
        "roofline": roofline,
        "step_hbm_gbps_algorithmic": round(step_algo / (ms_step * 1e-3) / 1e9, 1),
        "kernels_ms": {k: round(v, 4) for k, v in per_kernel_ms.items()},
        "kernels_algo_bytes": {k: int(v) for k, v in algo.items()},
        "plan_ms": round(plan_ms, 1),
    }
    if setup:
        result["setup_ms"] = setup
    if stream_res is not None:
        stream_res["vs_resident"] = round(stream_res["value"] / result["value"], 4)
        result["stream"] = stream_res
    if fused_bound is not None:
        gbps = fused_bound / (ms_step * 1e-3) / 1e9
        result["fused_bound"] = {"bytes_per_item": fused_item, "bytes_per_step": int(fused_bound),
                                 "gbps": round(gbps, 1), "frac": round(gbps / HBM_PEAK_GBPS, 4)}
        if ceiling:
            result["fused_bound"]["frac_of_copy_ceiling"] = round(gbps / ceiling, 4)
    if scratch_bytes is not None:
        result["label_scratch_bytes_per_step"] = int(scratch_bytes)
    if reread_bytes is not None:
        result["crop_reread_bytes_per_step"] = int(reread_bytes)
    if bg_copy is not None:
        result["bg_copy"] = bg_copy
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(args)
        except Exception as e:  # reported, never fatal to the GPU number
            result["cpu_baseline"] = {"error": repr(e)}
    if args.workload == "video4k" and args.frame_noise:
        result["config"]["frame_noise_lsb"] = args.frame_noise
    return result


if __name__ == "__main__":
    main()
