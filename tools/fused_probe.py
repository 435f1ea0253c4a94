"""How many V bands the fused launch queues at bench scale (tools only)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
from image_processor_pipeline_amd import fused  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda:0")
src = bench.make_sources(0, B, 1024, 0, dev)
g0 = torch.Generator(device=dev)
g0.manual_seed(1)
bgs = torch.randint(0, 256, (16, 1024, 1024, 3), dtype=torch.uint8, device=dev, generator=g0)
plan = fused.plan_pipe((1024, 1024), B, (1024, 1024), 16, fused.PipeConfig(), seed=0)
r = fused.PipeRunner(plan, dev)
out = torch.empty((B, 1024, 1024, 3), dtype=torch.uint8, device=dev)
for _ in range(3):
    r.fused(src, bgs, out)
q = r.queued_bands()
import numpy as np  # noqa: E402
tyv = (plan.max_ov_h + 15 + 15) // 16
vb = sum(((p.y + h + 15) // 16 - p.y // 16) for p, (h, w) in zip(plan.params, plan.ov_dims))
print(f"items {B} bands {vb} queued {q} ({100.0 * q / max(vb, 1):.1f} %)")
