"""Stage-by-stage comparison of the fused pipe against the oracle (debug)."""
import sys; sys.path.insert(0, '.')
import numpy as np, torch
from image_processor_pipeline_amd import fused
from oracle import ops, pipe as opipe

def decode_T(tmp, desc):
    h = desc['h']
    rows, W = int(h['lines']), int(h['out_len'])
    groups = (rows + 3) // 4
    raw = tmp[int(h['dst_off']): int(h['dst_off']) + groups * W * 16].reshape(groups, W, 4, 4) ^ 0x80
    # [g][x][c][rr] -> [g*4+rr][x][c]
    return raw.transpose(0, 3, 1, 2).reshape(groups * 4, W, 4)[:rows]

def run(n, H, W, K, bh, bw, cfg, seed):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, 256, (n, H, W, 3), np.uint8)
    bgs = rng.integers(0, 256, (K, bh, bw, 3), np.uint8)
    plan = fused.plan_pipe((H, W), n, (bh, bw), K, cfg, seed=seed)
    r = fused.PipeRunner(plan, 'cuda')
    out = torch.empty((n, bh, bw, 3), dtype=torch.uint8, device='cuda')
    r.run(torch.from_numpy(src).cuda(), torch.from_numpy(bgs).cuda(), out)
    tmp = r.tmp.cpu().numpy()
    got = out.cpu().numpy()
    for i in range(n):
        m = opipe.cut_out(src[i], plan.params[i], cfg)
        pm = ops.premultiply(m)
        nh_, nw_ = plan.ov_dims[i]
        h = plan.descs[i]['h']
        _, bh_, kh = ops.precompute_coeffs(m.shape[1], 0.0, float(m.shape[1]), nw_)
        y0, rows = int(h['line0']), int(h['lines'])
        if nw_ != m.shape[1] or nh_ != m.shape[0]:
            Tref = ops.resample_h(pm, nw_, bh_, kh, y0, rows) if nw_ != m.shape[1] else pm[y0:y0+rows]
        else:
            Tref = pm[y0:y0+rows]
        T = decode_T(tmp, plan.descs[i])
        exp = opipe.pipe_item(src[i], bgs, plan.params[i], cfg)
        badT = np.argwhere((T != Tref).any(-1))
        badC = np.argwhere((got[i] != exp).any(-1))
        print(f"item {i}: M {m.shape} ov {(nh_, nw_)} rows {rows} y0 {y0} ngs {int(h['ksize'])} "
              f"T mismatches {len(badT)} comp mismatches {len(badC)} params {plan.params[i]}")
        if len(badT):
            y, x = badT[0]
            print('   first T bad', (y, x), T[y, x], Tref[y, x], 'rows bad', np.unique(badT[:, 0])[:10], 'cols bad', np.unique(badT[:, 1])[:10])
        elif len(badC):
            y, x = badC[0]
            print('   first comp bad', (y, x), got[i][y, x], exp[y, x])

if __name__ == '__main__':
    run(10, 150, 170, 3, 128, 160, fused.PipeConfig(margins=(0.05, 9, 0.1, 3)), 7)
    run(2, 1024, 1024, 2, 1024, 1024, fused.PipeConfig(), 11)
