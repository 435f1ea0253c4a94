"""Does overlapping batch k's V pass with batch k+1's H pass pay?  The
config-3 pipe (B=4096) run as the bench's resident step (H then V on one
stream) against a two-stream schedule with double-buffered T and outputs:
H(k) on stream A after V(k-2) (same buffers) finished, V(k) on stream B
after H(k).  Prints ms per step of each.  Usage: python tools/probes/overlap_probe.py [steps]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from image_processor_pipeline_amd import _native as N, fused  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    S, B, K = 1024, 4096, 16
    cfg = fused.PipeConfig()
    plan = fused.plan_pipe((S, S), B, (S, S), K, cfg, seed=1, item_range=(0, B), n_global=B)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    src = torch.randint(0, 256, (B, S, S, 3), dtype=torch.uint8, device=dev, generator=g)
    bgs = torch.randint(0, 256, (K, S, S, 3), dtype=torch.uint8, device=dev, generator=g)
    runner = fused.PipeRunner(plan, dev)
    lib = N.load()
    outs = [torch.empty((B, S, S, 3), dtype=torch.uint8, device=dev) for _ in range(2)]
    tmps = [runner.tmp, torch.empty_like(runner.tmp)]
    p = plan

    def H(tmp, out, st):
        N.check(lib.ipp_pipe_hpass_bgcopy(src.data_ptr(), tmp.data_ptr(), runner.coefs.data_ptr(),
                                          runner.descs.data_ptr(), len(p.descs), p.max_out_w, p.max_rows, 3,
                                          N.np_ptr(p.hsv), p.tap_format, bgs.data_ptr(), out.data_ptr(),
                                          st.cuda_stream), "hpass")

    def V(tmp, out, st):
        N.check(lib.ipp_pipe_vblend_bands(tmp.data_ptr(), bgs.data_ptr(), out.data_ptr(), runner.coefs.data_ptr(),
                                          runner.descs.data_ptr(), len(p.descs), p.bg_w, p.bg_h, p.max_ov_w,
                                          p.max_ov_h, p.tap_format, st.cuda_stream), "vblend")

    def seq(n):
        st = torch.cuda.current_stream(dev)
        for _ in range(n):
            H(tmps[0], outs[0], st)
            V(tmps[0], outs[0], st)

    def ovl(n, sa, sb):
        vdone = [None, None]
        for k in range(n):
            j = k & 1
            if vdone[j] is not None:
                sa.wait_event(vdone[j])
            H(tmps[j], outs[j], sa)
            e = torch.cuda.Event()
            e.record(sa)
            sb.wait_event(e)
            V(tmps[j], outs[j], sb)
            vdone[j] = torch.cuda.Event()
            vdone[j].record(sb)
        torch.cuda.current_stream(dev).wait_stream(sa)
        torch.cuda.current_stream(dev).wait_stream(sb)

    def timed(fn):
        fn(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(steps)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    res = {}
    for rep in range(2):
        res.setdefault("sequential", []).append(timed(seq))
        sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        res.setdefault("overlap", []).append(timed(lambda n: ovl(n, sa, sb)))
        sa, sb = torch.cuda.Stream(dev, priority=0), torch.cuda.Stream(dev, priority=-1)
        res.setdefault("overlap, V high priority", []).append(timed(lambda n: ovl(n, sa, sb)))
        sa, sb = torch.cuda.Stream(dev, priority=-1), torch.cuda.Stream(dev, priority=0)
        res.setdefault("overlap, H high priority", []).append(timed(lambda n: ovl(n, sa, sb)))
    for k, v in res.items():
        print(f"{k:28s} " + " ".join(f"{x:.3f}" for x in v) + " ms/step")
    # the two schedules give the same composite
    seq(1)
    torch.cuda.synchronize()
    a = outs[0].clone()
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    outs[0].zero_()
    outs[1].zero_()
    ovl(2, sa, sb)
    torch.cuda.synchronize()
    print("overlap output equal:", bool(torch.equal(a, outs[0])), bool(torch.equal(a, outs[1])))


if __name__ == "__main__":
    main()
