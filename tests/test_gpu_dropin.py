"""GPU: the batched device mode is a drop-in for the reference's file-mode
pipeline, and the bench's multi-rank path computes what one process computes.

* The five reference steps chained through files (ProcessingPipeline, the
  plugins in image_processor_pipeline_amd.transforms) and ``fused.plan_pipe``
  + ``PipeRunner`` under the same seed produce byte-identical composites and
  the same YOLO labels (draw order + pixels).
* ``bench.py --gpus 2`` (its own launcher, gloo, both ranks on this GPU)
  writes per-item outputs identical to ``--gpus 1``.
* The pipe kernels flag a plan that breaks the LDS ring limit (ipp.h), and
  the product library ignores the diagnostic environment variables.
* Config-2 geometry: the standalone rotate+flip gather at 1024² vs the oracle.
* crop_square on non-square images with several boxes vs a NumPy restatement
  of crop_square.py:167-217.
"""
import json
import os
import random
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
from PIL import Image

torch = pytest.importorskip("torch")

from oracle import ops

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
DEV = "cuda:0"


@pytest.fixture(autouse=True, scope="module")
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def test_file_pipeline_equals_batched_pipe(tmp_path):
    from image_processor_pipeline_amd import fused, geometry as G
    from image_processor_pipeline_amd.labels_math import xyxy2xywhn
    from image_processor_pipeline_amd.pipeline import ProcessingPipeline, ProcessingStep
    from image_processor_pipeline_amd.transforms import filtres_liste, overlays, rotations, symmetry

    n, H, W, K, bh, bw, seed = 6, 150, 170, 3, 200, 240, 77
    rng = np.random.default_rng(seed)
    src = rng.integers(0, 256, (n, H, W, 3), np.uint8)
    src[:, :, :50] = (20, 20, 20)          # excluded by the first reference range
    src[:, :40, 50:] = (230, 200, 40)      # kept
    bgs = rng.integers(0, 256, (K, bh, bw, 3), np.uint8)
    (tmp_path / "src").mkdir()
    (tmp_path / "bg").mkdir()
    for i in range(n):
        Image.fromarray(src[i], "RGB").save(tmp_path / "src" / f"s{i:04d}.png")
    for k in range(K):
        Image.fromarray(bgs[k], "RGB").save(tmp_path / "bg" / f"b{k:02d}.png")
    pipe = ProcessingPipeline(root_dir=tmp_path)
    pipe.add_step(ProcessingStep("rot", rotations.process_rotations, "src", "r",
                                 options={"num_rotations": 1, "include_original": False}))
    pipe.add_step(ProcessingStep("sym", symmetry.generate_symmetries, output_dirs="s",
                                 options={"choose_random": 1, "include_original": False}))
    pipe.add_step(ProcessingStep("mask", filtres_liste.process_images_with_color_masks, output_dirs="m",
                                 options={"color_ranges_to_exclude_hsv": G.REFERENCE_HSV_RANGES}))
    pipe.add_step(ProcessingStep("ovl", overlays.paste_overlay_onto_background, ["m", "bg"], ["oi", "ol"],
                                 pairing_method="modulo", fixed_input=True))
    random.seed(seed)
    pipe.run()

    cfg = fused.PipeConfig(margins=(0, 0, 0, 0))
    plan = fused.plan_pipe((H, W), n, (bh, bw), K, cfg, seed=seed)
    runner = fused.PipeRunner(plan, DEV)
    out = torch.empty((n, bh, bw, 3), dtype=torch.uint8, device=DEV)
    runner.run(_t(src), _t(bgs), out)
    got = out.cpu().numpy()
    comps = sorted((tmp_path / "oi").iterdir())
    labels = sorted((tmp_path / "ol").iterdir())
    assert len(comps) == n and len(labels) == n
    for i in range(n):
        p = plan.params[i]
        assert comps[i].name == f"s{i:04d}_r001_{p.sym}.png"
        assert np.array_equal(np.asarray(Image.open(comps[i]).convert("RGB")), got[i]), i
        oh, ow = plan.ov_dims[i]
        box = np.array([[p.x, p.y, p.x + ow, p.y + oh]])
        cx, cy, w_, h_ = xyxy2xywhn(box, bw, bh)[0]
        assert labels[i].read_text() == f"0 {cx:.6f} {cy:.6f} {w_:.6f} {h_:.6f}"


def _bench(tmp_path, name, args):
    f = tmp_path / f"{name}.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--dist-backend", "gloo", "--size", "256",
                        "--backgrounds", "3", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
                        "--no-copy-ceiling", "--dump-digests", str(f)] + args,
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    return line, json.loads(f.read_text())


@pytest.mark.parametrize("workload", ["pipe5", "rotflip"])
def test_bench_two_ranks_equal_one(tmp_path, workload):
    one, d1 = _bench(tmp_path, "one", ["--gpus", "1", "--batch", "6", "--workload", workload])
    two, d2 = _bench(tmp_path, "two", ["--gpus", "2", "--batch", "6", "--scaling", "strong", "--workload", workload])
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["config"]["global_batch"] == 6
    assert len(d1) == 6 and d1 == d2


def test_ring_limit_is_flagged(monkeypatch):
    from image_processor_pipeline_amd import fused
    rng = np.random.default_rng(3)
    src = _t(rng.integers(0, 256, (1, 1024, 1024, 3), np.uint8))
    bgs = _t(rng.integers(0, 256, (1, 1024, 1024, 3), np.uint8))
    out = torch.empty((1, 1024, 1024, 3), dtype=torch.uint8, device=DEV)
    good = fused.PipeRunner(fused.plan_pipe((1024, 1024), 1, (1024, 1024), 1, fused.PipeConfig(), seed=0), DEV)
    good.status()
    good.run(src, bgs, out)
    assert good.status() == 0
    monkeypatch.setattr(fused, "H_RING_COLUMNS", 1 << 30)   # let the planner pass a 100x downscale
    bad = fused.plan_pipe((1024, 1024), 1, (1024, 1024), 1, fused.PipeConfig(scale_min=0.01, scale_max=0.012),
                          seed=0)
    runner = fused.PipeRunner(bad, DEV)
    runner.run(src, bgs, out)
    assert runner.status() & 1
    assert runner.status() == 0      # read-and-clear


_ENV_SCRIPT = r"""
import hashlib, sys
import numpy as np, torch
sys.path.insert(0, sys.argv[1])
from image_processor_pipeline_amd import fused, device as D
rng = np.random.default_rng(5)
n, H, W, K, bh, bw = 4, 160, 180, 2, 150, 170
src = torch.from_numpy(rng.integers(0, 256, (n, H, W, 3), np.uint8)).cuda()
bgs = torch.from_numpy(rng.integers(0, 256, (K, bh, bw, 3), np.uint8)).cuda()
cfg = fused.PipeConfig(margins=(9, 9, 9, 9))
r = fused.PipeRunner(fused.plan_pipe((H, W), n, (bh, bw), K, cfg, seed=3), "cuda:0")
out = torch.empty((n, bh, bw, 3), dtype=torch.uint8, device="cuda:0")
r.run(src, bgs, out)
out2 = torch.full_like(out, 3)
r.run(src, bgs, out2)
g = D.plan_rotate_flip([(H, W, 3)], [33.0], [1])
rot = D.rotate_flip_nearest(src[0].reshape(-1), g)
torch.cuda.synchronize()
print(hashlib.sha1(out.cpu().numpy().tobytes() + out2.cpu().numpy().tobytes() + rot.cpu().numpy().tobytes()).hexdigest())
"""


def test_diagnostic_env_vars_do_not_change_outputs(tmp_path):
    script = tmp_path / "run.py"
    script.write_text(_ENV_SCRIPT)
    base = {k: v for k, v in os.environ.items() if not k.startswith("IPP_")}
    digests = []
    for extra in ({}, {"IPP_DBG_HPASS": "11", "IPP_VB_STORE": "9", "IPP_COPY_BLOCKS": "1",
                       "IPP_GATHER_MAP": "0", "IPP_HPASS": "1", "IPP_HP_PAD": "60000"}):
        p = subprocess.run([sys.executable, str(script), str(ROOT)], capture_output=True, text=True, timeout=180,
                           env=dict(base, **extra))
        assert p.returncode == 0, p.stderr[-2000:]
        digests.append(p.stdout.strip().splitlines()[-1])
    assert digests[0] == digests[1]


def test_rotate_flip_config2_geometry_vs_oracle():
    """BASELINE config 2: 1024² RGB sources, canvases up to ≈1450² at 45°
    (the dense 8×8 tile path of ipp_gather.hip), every flip."""
    from image_processor_pipeline_amd import device as D
    rng = np.random.default_rng(12)
    angles = [45.0, 135.0, 30.5, 301.7]
    syms = ["o", "h", "v", "hv"]
    n = len(angles)
    src = rng.integers(0, 256, (n, 1024, 1024, 3), np.uint8)
    plan = D.plan_rotate_flip([(1024, 1024, 3)] * n, angles, [D.SYM_FLIP[s] for s in syms],
                              src_offsets=[i * 1024 * 1024 * 3 for i in range(n)])
    got = [v.cpu().numpy() for v in D.unpack(D.rotate_flip_nearest(_t(src).reshape(-1), plan), plan)]
    for i in range(n):
        exp = ops.flip(ops.rotate_and_crop(ops.to_rgba(src[i]), angles[i]), syms[i])
        assert got[i].shape == exp.shape and np.array_equal(got[i], exp), (angles[i], syms[i])
    assert max(g.shape[0] for g in got) >= 1440


def _crop_square_restated(img, lines, rnd):
    """crop_square.py:163-217 in NumPy (intended semantics: element-wise `&`)."""
    from image_processor_pipeline_amd.labels_math import xywhn2xyxy, xyxy2xywhn
    data = np.array([[float(v) for v in l.split()] for l in lines], np.float64)
    cls, boxes = data[:, 0].astype(int), data[:, 1:5]
    h, w = img.shape[:2]
    ab = xywhn2xyxy(boxes, w, h)
    cs = min(h, w)
    x_min, y_min = ab[:, :2].min(0)
    x_max, y_max = ab[:, 2:].max(0)
    lx, ux = max(0, int(x_max - cs)), min(int(x_min), w - cs)
    ly, uy = max(0, int(y_max - cs)), min(int(y_min), h - cs)
    x0, y0 = rnd.randint(lx, ux), rnd.randint(ly, uy)
    crop = img[y0:y0 + cs, x0:x0 + cs]
    c = np.clip(ab - np.array([[x0, y0, x0, y0]]), 0, cs)
    valid = (c[:, 0] < c[:, 2]) & (c[:, 1] < c[:, 3])
    nb = xyxy2xywhn(c[valid], cs, cs)
    text = "".join(f"{k} {a:.6f} {b:.6f} {d:.6f} {e:.6f}\n" for k, (a, b, d, e) in zip(cls[valid], nb))
    return crop, text


@pytest.mark.parametrize("hw,lines", [
    ((180, 300), ["0 0.5 0.5 0.1 0.2", "2 0.45 0.40 0.05 0.3", "1 0.52 0.6 0.0 0.1"]),   # zero-width box dropped
    ((320, 200), ["3 0.3 0.55 0.2 0.1", "0 0.6 0.5 0.3 0.2"]),
    ((241, 97), ["5 0.5 0.5 1.0 0.2"]),
])
def test_crop_square_non_square_vs_restatement(tmp_path, hw, lines):
    from image_processor_pipeline_amd import io as ipp_io
    from image_processor_pipeline_amd.transforms import crop_square
    h, w = hw
    img = np.random.default_rng(h * w).integers(0, 256, (h, w, 3), np.uint8)
    (tmp_path / "in").mkdir()
    (tmp_path / "lbl").mkdir()
    ipp_io.imwrite(tmp_path / "in" / "a.png", img)
    (tmp_path / "lbl" / "a.txt").write_text("\n".join(lines) + "\n")
    for d in ("ci", "cl"):
        (tmp_path / d).mkdir()
    for seed in range(4):
        random.seed(seed)
        res = crop_square.process_square_crop_around_bbox(tmp_path / "in" / "a.png", tmp_path / "lbl" / "a.txt",
                                                          [tmp_path / "ci", tmp_path / "cl"])
        exp_img, exp_txt = _crop_square_restated(img, lines, random.Random(seed))
        assert np.array_equal(ipp_io.imread(res[0]), exp_img), seed
        assert res[1].read_text() == exp_txt, seed


@pytest.mark.parametrize("parts,ratio", [(3, 1.0), (2, 0.3), (5, 1.0)])
def test_overlapped_item_ranges_equal_sequential(parts, ratio):
    """PipeRunner.run_overlapped (bench.py --pipe-parts): V launches of item
    range k on a side stream beside range k+1's H launch give the same bytes
    as the two whole-batch launches, including ranges that end mid-batch and
    empty ranges (more parts than copy groups)."""
    from image_processor_pipeline_amd import fused
    n, S, K = 21, 256, 3
    g = torch.Generator().manual_seed(5)
    src = torch.randint(0, 256, (n, S, S, 3), dtype=torch.uint8, generator=g).to(DEV)
    bgs = torch.randint(0, 256, (K, S, S, 3), dtype=torch.uint8, generator=g).to(DEV)
    plan = fused.plan_pipe((S, S), n, (S, S), K, fused.PipeConfig(), seed=11)
    runner = fused.PipeRunner(plan, DEV)
    ref = torch.zeros((n, S, S, 3), dtype=torch.uint8, device=DEV)
    runner.run(src, bgs, ref)
    out = torch.full((n, S, S, 3), 7, dtype=torch.uint8, device=DEV)
    runner.run_overlapped(src, bgs, out, parts, ratio)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
