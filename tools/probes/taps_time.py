"""Time ipp_pipe_plan_taps (device taps of one pipe5 batch) on its own:
HIP events on the side stream around the call, wall clock beside them.
A/B through IPP_LIB_PATH (make variant).  Usage: python tools/probes/taps_time.py [reps]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from image_processor_pipeline_amd import _native as N, fused  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    lib = N.load()
    cfg = fused.PipeConfig()
    plan = fused.plan_pipe((1024, 1024), 4096, (1024, 1024), 16, cfg, seed=1, item_range=(0, 4096), n_global=4096)
    dev = torch.device("cuda:0")
    coefs = torch.empty(4 * (plan.coef_words + 4096), dtype=torch.uint8, device=dev)
    scratch = torch.empty(lib.ipp_pipe_taps_scratch_bytes(len(plan.axes)), dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(dev)
    stats = np.zeros(2, np.int64)
    ev, wall = [], []
    for r in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(st)
        N.check(lib.ipp_pipe_plan_taps(N.np_ptr(plan.axes), len(plan.axes), coefs.data_ptr(), scratch.data_ptr(),
                                       N.np_ptr(stats), st.cuda_stream), "ipp_pipe_plan_taps")
        e1.record(st)
        st.synchronize()
        if r >= 2:
            wall.append((time.perf_counter() - t0) * 1e3)
            ev.append(e0.elapsed_time(e1))
    print(f"taps: event {np.median(ev):.3f} ms  wall {np.median(wall):.3f} ms  host tiles {int(stats[0])}  "
          f"coef MB {plan.coef_words * 4 / 1e6:.1f}")


if __name__ == "__main__":
    main()
