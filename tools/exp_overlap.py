"""Experiment: hpass/vblend overlap across item chunks on two HIP streams."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch
from image_processor_pipeline_amd import fused, _native as N
from image_processor_pipeline_amd.device import _stream

dev = torch.device("cuda", 0)
B, S, K = 4096, 1024, 16
src = torch.empty((B, S, S, 3), dtype=torch.uint8, device=dev).random_(0, 256)
bgs = torch.empty((K, S, S, 3), dtype=torch.uint8, device=dev).random_(0, 256)
out = torch.empty((B, S, S, 3), dtype=torch.uint8, device=dev)
plan = fused.plan_pipe((S, S), B, (S, S), K, fused.PipeConfig(), seed=0)
r = fused.PipeRunner(plan, dev)
lib, p = r.lib, plan
dsz = p.descs.dtype.itemsize
s1 = torch.cuda.current_stream(dev)
s2 = torch.cuda.Stream(dev)

def hp(c0, c1, st):
    N.check(lib.ipp_pipe_hpass(src.data_ptr(), r.tmp.data_ptr(), r.coefs.data_ptr(), r.descs.data_ptr() + c0 * dsz,
                               c1 - c0, p.max_out_w, p.max_rows, 3, N.np_ptr(p.hsv), p.tap_format, st.cuda_stream), "h")

def vb(c0, c1, st):
    N.check(lib.ipp_pipe_vblend(r.tmp.data_ptr(), bgs.data_ptr(), out.data_ptr(), r.coefs.data_ptr(),
                                r.descs.data_ptr() + c0 * dsz, c1 - c0, p.bg_w, p.bg_h, p.max_ov_w, p.tap_format,
                                st.cuda_stream), "v")

def run(chunks, two):
    bounds = [int(v) for v in np.linspace(0, B, chunks + 1).astype(int)]
    for c in range(chunks):
        hp(bounds[c], bounds[c + 1], s1)
        if two:
            e = torch.cuda.Event(); e.record(s1); s2.wait_event(e)
            vb(bounds[c], bounds[c + 1], s2)
        else:
            vb(bounds[c], bounds[c + 1], s1)
    if two:
        e = torch.cuda.Event(); e.record(s2); s1.wait_event(e)

for chunks, two in [(1, False), (4, False), (4, True), (8, True), (16, True), (32, True), (64, True)]:
    for _ in range(2): run(chunks, two)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5): run(chunks, two)
    torch.cuda.synchronize()
    print(f"chunks={chunks} two_streams={two}: {(time.perf_counter() - t) / 5 * 1e3:.2f} ms/step", flush=True)
