import sys; sys.path.insert(0, '.')
import numpy as np, torch
from image_processor_pipeline_amd import device as D, geometry as G
from oracle import ops
rng = np.random.default_rng(5)
img = rng.integers(0, 256, (123, 77, 3), np.uint8)
p = G.hsv_params(G.REFERENCE_HSV_RANGES, None, False, bgr=True)
print(p)
out = torch.full((123, 77, 4), 7, dtype=torch.uint8, device='cuda')
got = D.hsv_mask(torch.from_numpy(img).cuda(), p).cpu().numpy()
exp = ops.color_mask_bgra(img, G.REFERENCE_HSV_RANGES)
bad = np.argwhere((got != exp).any(-1))
print('mismatch px', len(bad), bad[:5], bad[-5:])
print('rgb equal', np.array_equal(got[..., :3], exp[..., :3]), 'alpha got uniq', np.unique(got[...,3]), 'exp uniq', np.unique(exp[...,3]))
for (y, x) in bad[:5]:
    print(y, x, img[y, x], got[y, x], exp[y, x], ops.bgr_to_hsv(img[y:y+1, x:x+1]))
