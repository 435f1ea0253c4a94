#!/usr/bin/env python3
"""Generate golden vectors for the hot path from the reference + Pillow 12.2.0.

Runs ONLY in the build container (it imports /root/reference, which does not
exist on the GPU box).  It writes small .npz fixtures to tests/golden/; no
reference source, bytecode or derived module is copied into the repo.

What is pinned:
  * rotate_pillow.npz   — Pillow ``convert('RGBA').rotate(a, expand=True)``
                          canvases + ``getbbox()`` for fast-path and generic
                          angles (the library call at rotations.py:96-99).
  * rotations_ref.npz   — the reference's own ``process_rotations``
                          (transforms/rotations.py) run under ``random.seed``,
                          outputs read back from its PNGs, plus the angle
                          stream it drew (rotations.py:89).
  * resize_pillow.npz   — Pillow ``resize((w,h), LANCZOS)`` on RGBA with
                          arbitrary alpha (overlays.py:129), incl. one-axis and
                          identity resizes.
  * overlays_ref.npz    — the reference's ``paste_overlay_onto_background``
                          (transforms/overlays.py) under ``random.seed``:
                          composite, YOLO label, and the random stream.
  * paste_pillow.npz    — Pillow ``paste(ov, (x,y), ov)`` onto RGB.

Stubs: ``cv2`` / ``ultralytics`` / ``deprecated`` / ``icecream`` are absent
from this image; overlays.py only uses ``xyxy2xywhn`` from them on its pixel
path (label math), restated in the stub below.  None of the stubs carries
pixel arithmetic.
"""
from __future__ import annotations

import importlib.util
import io
import random
import sys
import tempfile
import types
from pathlib import Path

import numpy as np
from PIL import Image

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parents[1] / "tests" / "golden"


def _install_stubs():
    cv2 = types.ModuleType("cv2")
    sys.modules.setdefault("cv2", cv2)
    ul = types.ModuleType("ultralytics")
    ul_utils = types.ModuleType("ultralytics.utils")
    ul_ops = types.ModuleType("ultralytics.utils.ops")

    def xyxy2xywhn(x, w=640, h=640, clip=False, eps=0.0):
        x = np.asarray(x, dtype=np.float64)
        y = np.empty_like(x)
        y[..., 0] = ((x[..., 0] + x[..., 2]) / 2) / w
        y[..., 1] = ((x[..., 1] + x[..., 3]) / 2) / h
        y[..., 2] = (x[..., 2] - x[..., 0]) / w
        y[..., 3] = (x[..., 3] - x[..., 1]) / h
        return y

    ul_ops.xyxy2xywhn = xyxy2xywhn
    sys.modules.setdefault("ultralytics", ul)
    sys.modules.setdefault("ultralytics.utils", ul_utils)
    sys.modules.setdefault("ultralytics.utils.ops", ul_ops)
    dep = types.ModuleType("deprecated")
    dep.deprecated = lambda *a, **k: (lambda f: f)
    sys.modules.setdefault("deprecated", dep)
    ice = types.ModuleType("icecream")
    ice.ic = lambda *a, **k: None
    sys.modules.setdefault("icecream", ice)
    # alias the reference root as the package name its modules import from
    pkg = types.ModuleType("image_processor_pipeline")
    pkg.__path__ = [str(REF)]
    sys.modules.setdefault("image_processor_pipeline", pkg)


def _load(modname: str, path: Path):
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _pack(arrs):
    flat = np.concatenate([a.reshape(-1) for a in arrs]) if arrs else np.zeros(0, np.uint8)
    shapes = np.array([a.shape for a in arrs], np.int64)
    return flat, shapes


def gen_rotate(rng):
    srcs = [
        rng.integers(0, 256, (37, 53, 3), np.uint8),
        rng.integers(0, 256, (48, 64, 3), np.uint8),
        rng.integers(0, 256, (2, 3, 3), np.uint8),
        rng.integers(0, 256, (9, 1, 3), np.uint8),
        rng.integers(0, 256, (31, 31, 3), np.uint8),
    ]
    rgba = rng.integers(0, 256, (40, 27, 4), np.uint8)
    rgba[..., 3] = np.where(rng.random((40, 27)) < 0.3, 0, rgba[..., 3])
    rgba[:5, :, 3] = 0          # transparent border rows → non-trivial bbox
    rgba[:, -4:, 3] = 0
    srcs.append(rgba)
    angles = [0.0, 90.0, 180.0, 270.0, 360.0, 45.0, 30.5, 1.0, 359.0, 89.9999,
              90.0001, 179.5, 13.37, -33.0, 720.25, 271.5]
    angles += [float(a) for a in rng.uniform(1, 359, 6)]
    outs, bboxes, meta = [], [], []
    for si, s in enumerate(srcs):
        im = Image.fromarray(s, "RGB" if s.shape[2] == 3 else "RGBA").convert("RGBA")
        for a in angles:
            r = im.rotate(a, expand=True)
            arr = np.asarray(r)
            outs.append(arr)
            bb = r.getbbox()
            bboxes.append(bb if bb is not None else (-1, -1, -1, -1))
            meta.append((si, a))
    flat, shapes = _pack(outs)
    sflat, sshapes = _pack(srcs)
    np.savez_compressed(OUT / "rotate_pillow.npz", src_flat=sflat, src_shapes=sshapes,
                        out_flat=flat, out_shapes=shapes, bboxes=np.array(bboxes, np.int64),
                        src_index=np.array([m[0] for m in meta], np.int64),
                        angles=np.array([m[1] for m in meta], np.float64))


def gen_rotations_ref(rng, tmp: Path):
    rot = _load("ref_rotations", REF / "transforms" / "rotations.py")
    src = rng.integers(0, 256, (45, 61, 3), np.uint8)
    p = tmp / "sample.png"
    Image.fromarray(src, "RGB").save(p)
    out_dir = tmp / "rot_out"
    out_dir.mkdir()
    seed, n = 1234, 5
    random.seed(seed)
    paths = rot.process_rotations(p, [out_dir], num_rotations=n)
    random.seed(seed)
    angles = [random.uniform(1.0, 359.0) for _ in range(n)]
    outs = [np.asarray(Image.open(q).convert("RGBA")) for q in paths]
    names = [q.name for q in paths]
    flat, shapes = _pack(outs)
    np.savez_compressed(OUT / "rotations_ref.npz", src=src, seed=seed, angles=np.array(angles),
                        out_flat=flat, out_shapes=shapes, names=np.array(names))


def gen_resize(rng):
    cases = [((57, 83), (20, 30)), ((83, 57), (31, 19)), ((40, 40), (40, 17)),
             ((40, 40), (13, 40)), ((30, 20), (45, 50)), ((64, 48), (64, 48)),
             ((120, 77), (23, 14)), ((1, 9), (1, 3)), ((250, 180), (51, 37))]
    srcs, outs, sizes = [], [], []
    for (w, h), (ow, oh) in cases:
        s = rng.integers(0, 256, (h, w, 4), np.uint8)
        sel = rng.random((h, w))
        s[..., 3] = np.where(sel < 0.25, 0, np.where(sel < 0.5, 255, s[..., 3]))
        srcs.append(s)
        outs.append(np.asarray(Image.fromarray(s, "RGBA").resize((ow, oh), Image.Resampling.LANCZOS)))
        sizes.append((ow, oh))
    sflat, sshapes = _pack(srcs)
    flat, shapes = _pack(outs)
    np.savez_compressed(OUT / "resize_pillow.npz", src_flat=sflat, src_shapes=sshapes,
                        out_flat=flat, out_shapes=shapes, sizes=np.array(sizes, np.int64))


def gen_paste(rng):
    bg = rng.integers(0, 256, (70, 90, 3), np.uint8)
    ov = rng.integers(0, 256, (21, 33, 4), np.uint8)
    ov[0, :, 3] = 0
    ov[1, :, 3] = 255
    outs, pos = [], [(0, 0), (57, 49), (10, 7)]
    for x, y in pos:
        c = Image.fromarray(bg, "RGB").copy()
        o = Image.fromarray(ov, "RGBA")
        c.paste(o, (x, y), o)
        outs.append(np.asarray(c))
    np.savez_compressed(OUT / "paste_pillow.npz", bg=bg, ov=ov, pos=np.array(pos), outs=np.stack(outs))


def gen_overlays_ref(rng, tmp: Path):
    ov_mod = _load("image_processor_pipeline.transforms.overlays", REF / "transforms" / "overlays.py")
    ovs, bgs, comps, labels, streams, names = [], [], [], [], [], []
    for k, ((ow, oh), (bw, bh)) in enumerate([((90, 70), (160, 120)), ((61, 95), (128, 128)),
                                                ((200, 45), (150, 100))]):
        ov = rng.integers(0, 256, (oh, ow, 4), np.uint8)
        ov[..., 3] = np.where(rng.random((oh, ow)) < 0.3, 0, 255)
        bg = rng.integers(0, 256, (bh, bw, 3), np.uint8)
        po, pb = tmp / f"ov{k}.png", tmp / f"bg{k}.png"
        Image.fromarray(ov, "RGBA").save(po)
        Image.fromarray(bg, "RGB").save(pb)
        d_img, d_lbl = tmp / f"img{k}", tmp / f"lbl{k}"
        d_img.mkdir()
        d_lbl.mkdir()
        seed = 100 + k
        random.seed(seed)
        res = ov_mod.paste_overlay_onto_background(po, pb, [d_img, d_lbl])
        random.seed(seed)
        ratio = random.uniform(0.15, 0.30)
        streams.append(ratio)
        comps.append(np.asarray(Image.open(res[0]).convert("RGB")))
        labels.append(res[1].read_text())
        ovs.append(ov)
        bgs.append(bg)
        names.append(res[0].name)
    of, osh = _pack(ovs)
    bf, bsh = _pack(bgs)
    cf, csh = _pack(comps)
    np.savez_compressed(OUT / "overlays_ref.npz", ov_flat=of, ov_shapes=osh, bg_flat=bf, bg_shapes=bsh,
                        comp_flat=cf, comp_shapes=csh, labels=np.array(labels), ratios=np.array(streams),
                        seeds=np.array([100, 101, 102]), names=np.array(names))


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    _install_stubs()
    rng = np.random.default_rng(20250725)
    with tempfile.TemporaryDirectory() as td:
        tmp = Path(td)
        gen_rotate(rng)
        gen_rotations_ref(rng, tmp)
        gen_resize(rng)
        gen_paste(rng)
        gen_overlays_ref(rng, tmp)
    for f in sorted(OUT.glob("*.npz")):
        print(f.name, f.stat().st_size)


if __name__ == "__main__":
    main()
