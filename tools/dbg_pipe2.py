"""Run the window-dump / no-dot4 debug variants (IPP_LIB_PATH) — debug only."""
import os, sys; sys.path.insert(0, '.')
import numpy as np, torch
from image_processor_pipeline_amd import fused
from oracle import ops, pipe as opipe
from tools.dbg_pipe import decode_T
mode = sys.argv[1]
cfg = fused.PipeConfig(margins=(0.05, 9, 0.1, 3))
n, H, W, K, bh, bw = 4, 150, 170, 3, 128, 160
rng = np.random.default_rng(7)
src = rng.integers(0, 256, (n, H, W, 3), np.uint8)
bgs = rng.integers(0, 256, (K, bh, bw, 3), np.uint8)
plan = fused.plan_pipe((H, W), n, (bh, bw), K, cfg, seed=7)
r = fused.PipeRunner(plan, 'cuda')
out = torch.empty((n, bh, bw, 3), dtype=torch.uint8, device='cuda')
r.run(torch.from_numpy(src).cuda(), torch.from_numpy(bgs).cuda(), out)
tmp = r.tmp.cpu().numpy()
for i in range(n):
    m = opipe.cut_out(src[i], plan.params[i], cfg)
    pm = ops.premultiply(m)
    h = plan.descs[i]['h']
    T = decode_T(tmp, plan.descs[i])
    y0, rows, nw_ = int(h['line0']), int(h['lines']), int(h['out_len'])
    if mode == 'win':
        hdr = plan.coefs[int(h['coef_off']): int(h['coef_off']) + 4 * nw_].reshape(nw_, 4)
        ref = pm[y0:y0 + rows][:, hdr[:, 0]]
    else:
        _, bh_, kh = ops.precompute_coeffs(m.shape[1], 0.0, float(m.shape[1]), nw_)
        ref = ops.resample_h(pm, nw_, bh_, kh, y0, rows)
    bad = np.argwhere((T != ref).any(-1))
    print(mode, i, 'bad', len(bad), 'rows', np.unique(bad[:, 0])[:8] if len(bad) else '', (T[tuple(bad[0])], ref[tuple(bad[0])]) if len(bad) else '')
