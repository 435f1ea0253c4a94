"""Draw-recording stand-ins for the five reference steps of the benchmark pipe
(tests only).  Each makes exactly the ``random`` calls its reference plugin
makes, in the same place, and carries the image *geometry* (not pixels) in
small text files, so a file-mode ``ProcessingPipeline`` run records the
parameter stream a real run consumes:

* crop_from_border   — no draw (recadrages.py:13-61);
* process_rotations  — ``uniform(angle_min, angle_max)`` per rotation
  (rotations.py:88-89), output ``{stem}_r001``;
* generate_symmetries — ``sample(pool, choose_random)`` (symmetry.py:122),
  output ``{stem}_{sym}``;
* process_images_with_color_masks — no draw (filtres_liste.py:41-149);
* paste_overlay_onto_background — ``uniform(scale_min, scale_max)``
  (overlays.py:108) then ``randint`` × 2 (:133-134).

The 'modulo' shuffle of the backgrounds is made by ProcessingStep itself.
Geometry comes from the product's host planner (CPU), as the real plugins'
pixel sizes would."""
import json
import random
from pathlib import Path

from image_processor_pipeline_amd import geometry as G

LOG = []


def _dims(p: Path):
    return json.loads(Path(p).read_text())


def crop(path, output_dirs, crop_margins=(0, 0, 0, 0)):
    h, w = _dims(path)
    t, b, l, r = G.crop_margins(h, w, crop_margins)
    out = Path(output_dirs[0]) / path.name
    out.write_text(json.dumps([h - t - b, w - l - r]))
    return out


def rotate(path, output_dirs, num_rotations=1, include_original=False, angle_min=1.0, angle_max=359.0):
    h, w = _dims(path)
    outs = []
    for i in range(num_rotations):
        angle = random.uniform(angle_min, angle_max)
        LOG.append(("angle", path.stem, angle))
        plan = G.rotation_plan(w, h, angle)
        bb = G.rotated_bbox(w, h, plan)
        rw, rh = (bb[2] - bb[0], bb[3] - bb[1]) if bb else (plan.nw, plan.nh)
        out = Path(output_dirs[0]) / f"{path.stem}_r{i + 1:03d}.txt"
        out.write_text(json.dumps([rh, rw]))
        outs.append(out)
    return outs


def symmetries(path, output_dirs, pool=None, choose_random=1, include_original=False):
    pool = pool or ["o", "h", "v", "hv"]
    keys = random.sample(pool, choose_random)
    outs = []
    for k in keys:
        LOG.append(("sym", path.stem, k))
        out = Path(output_dirs[0]) / f"{path.stem}_{k}.txt"
        out.write_text(path.read_text())
        outs.append(out)
    return outs


def mask(path, output_dirs):
    out = Path(output_dirs[0]) / path.name
    out.write_text(path.read_text())
    return out


def overlay(ov_path, bg_path, output_dirs, scale_min=0.15, scale_max=0.30):
    oh, ow = _dims(ov_path)
    bh, bw = _dims(bg_path)
    ratio = random.uniform(scale_min, scale_max)
    nw, nh = G.overlay_size(ow, oh, bw, bh, ratio)
    x = random.randint(0, bw - nw)
    y = random.randint(0, bh - nh)
    LOG.append(("paste", ov_path.stem, bg_path.stem, ratio, x, y))
    out = Path(output_dirs[0]) / f"{ov_path.stem}.txt"
    out.write_text("x")
    return out
