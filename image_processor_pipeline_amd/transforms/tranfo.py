"""enhance_image — reference transforms/tranfo.py:9-55.

Same signature (``(input_image, apply_blur, apply_rgb, output_dirs,
**options)``, the 'sample' pairing of pipeline.py:209-225 supplies the two
flags), same draws in the same order — ``uniform(0.7, 1.3)`` for Brightness,
Contrast, Color (:38-40), ``uniform(0.5, 3)`` for the GaussianBlur radius
(:43), then 256 ``uniform(0.75, 1.25)`` per channel for the r, g, b point()
tables (:48-50) — and the same output (``output_dirs[0] / input_image.name``).
Pixels: ipp_enhance_lsum + ipp_enhance_color (+ 6 ipp_box_pass launches for
the blur) on the GPU, bit-exact with Pillow 12.2.0's ImageEnhance / Blend.c /
BoxBlur.c / point().  ``enhance_image.batch`` runs a chunk of
(path, apply_blur, apply_rgb) tuples as one batched launch set.
"""
from __future__ import annotations

import random
from pathlib import Path
from typing import Any, List, Optional

import numpy as np
from PIL import Image

from ._common import device_transform, thread_map
from .. import _rt
from .. import device as D
from ..utils.utils import _validate_dirs


def _draw(apply_blur: bool, apply_rgb: bool) -> D.EnhanceParams:
    """tranfo.py:38-50 draw order (the point() lambda runs for p = 0..255 per
    band, r then g then b; Image.point rounds the float table)."""
    f1 = random.uniform(0.7, 1.3)
    f2 = random.uniform(0.7, 1.3)
    f3 = random.uniform(0.7, 1.3)
    radius = random.uniform(0.5, 3) if apply_blur else None
    luts = None
    if apply_rgb:
        luts = np.zeros((3, 256), np.uint8)
        for c in range(3):
            luts[c] = [round(max(0, min(255, p * random.uniform(0.75, 1.25)))) for p in range(256)]
    return D.EnhanceParams(f1, f2, f3, radius, luts)


@device_transform
def enhance_image(
    input_image: Path,
    apply_blur: bool,
    apply_rgb: bool,
    output_dirs: List[Path],
    **options: Any,
) -> Optional[Path]:
    destination_img = _validate_dirs(output_dirs, 1)
    output_path = Path(destination_img) / input_image.name
    with Image.open(input_image) as src:
        img = np.asarray(src.convert("RGB"))
    params = _draw(apply_blur, apply_rgb)
    out = D.enhance_rgb([_rt.h2d(img)], [params])[0]
    Image.fromarray(_rt.d2h(out), "RGB").save(output_path)
    return output_path


def _enhance_batch(arg_tuples, output_dirs: List[Path], threads: int = 1, **options: Any) -> List:
    """Batched enhance_image for ProcessingStep: decode on host threads, draw
    every item's parameters in the sequential order, one batched launch set,
    encode on host threads (outputs identical to per-file calls)."""
    destination_img = Path(_validate_dirs(output_dirs, 1))

    def decode(args):
        with Image.open(args[0]) as src:
            return np.asarray(src.convert("RGB"))

    decoded = thread_map(decode, arg_tuples, threads)
    ok = [i for i, d in enumerate(decoded) if not isinstance(d, Exception)]
    params = {i: _draw(bool(arg_tuples[i][1]), bool(arg_tuples[i][2])) for i in ok}
    outs = D.enhance_rgb([_rt.h2d(decoded[i]) for i in ok], [params[i] for i in ok]) if ok else []
    host = {i: _rt.d2h(o) for i, o in zip(ok, outs)}

    def encode(i):
        if isinstance(decoded[i], Exception):
            raise decoded[i]
        p = destination_img / Path(arg_tuples[i][0]).name
        Image.fromarray(host[i], "RGB").save(p)
        return p

    return thread_map(encode, range(len(arg_tuples)), threads)


enhance_image.batch = _enhance_batch
