"""process_square_crop_around_bbox — reference transforms/crop_square.py:104-224.

Intended semantics (the reference cannot run as written; the
three bugs are fixed and documented in DESIGN.md §Divergences):
  * `_validate_dirs(output_dirs)` without nb_dirs (:154)   → nb_dirs=2;
  * `Path.isfile()` (:32)                                    → `is_file()`;
  * `(a < b) and (c < d)` on arrays (:210)                   → element-wise `&`.
Square side = min(H, W); top-left (x0, y0) drawn with two random.randint
(:192-193) inside the range that keeps the union of the boxes; boxes shifted,
clipped, empties dropped, re-normalised.  The crop is an exact window copy on
the GPU.
"""
from __future__ import annotations

import random
from pathlib import Path
from typing import Any, List, Optional, Tuple
from warnings import warn

import numpy as np

from ._common import device_transform
from .. import _rt
from .. import device as D
from .. import io as _io
from ..labels_math import xywhn2xyxy, xyxy2xywhn
from ..utils import utils


def _load_image(filepath: Path) -> np.ndarray:
    if not filepath.is_file():
        raise FileNotFoundError(f"Image non trouvée: {filepath}")
    img = _io.imread(str(filepath))
    if img is None:
        raise IOError(f"Impossible de charger l'image {filepath.name} via OpenCV.")
    return img


def _read_bboxes(filepath: Path) -> Tuple[np.ndarray, np.ndarray]:
    if not filepath.is_file():
        raise FileNotFoundError(f"Fichier label non trouvé : {filepath}")
    data = np.loadtxt(filepath, ndmin=2)
    try:
        classes = data[:, 0].astype(int)
        bboxes = data[:, 1:5].astype(float)
    except Exception as e:
        raise ValueError(f"Format invalide dans {filepath.name}: {e}")
    return classes, bboxes


def _save_crop_files(img, labels, img_out: Path, label_out: Path) -> None:
    utils._save_crop_files(img, labels, img_out, label_out)


@device_transform
def process_square_crop_around_bbox(
    input_image_path: Path,
    input_label_path: Path,
    output_dirs: List[Path],
    **options: Any,
) -> Optional[List[Path]]:
    image_target_dir, label_target_dir = utils._validate_dirs(output_dirs, 2)
    if input_image_path.stem != input_label_path.stem:
        warn(f"Warning [Crop Carré]: image ({input_image_path.name}) et label ({input_label_path.name}) "
             "n'ont pas le même nom. Fichier ignoré et poursuite du traitement...")
    image = _load_image(input_image_path)
    class_ids, bboxes = _read_bboxes(input_label_path)
    height, width = image.shape[:2]
    bboxes_absolute = xywhn2xyxy(bboxes, width, height)

    crop_size = min(height, width)
    x_min, y_min = bboxes_absolute[:, :2].min(axis=0)
    x_max, y_max = bboxes_absolute[:, 2:].max(axis=0)
    lower_bound_x = max(0, int(x_max - crop_size))
    upper_bound_x = min(int(x_min), width - crop_size)
    lower_bound_y = max(0, int(y_max - crop_size))
    upper_bound_y = min(int(y_min), height - crop_size)
    if lower_bound_x > upper_bound_x or lower_bound_y > upper_bound_y:
        raise RuntimeError(
            f"Impossible de trouver une position de crop carré valide contenant entièrement la bbox "
            f"[{x_min},{y_min},{x_max},{y_max}] dans une image {width}x{height} avec crop_size={crop_size}. "
            "Crop annulé.")
    x0 = random.randint(lower_bound_x, upper_bound_x)
    y0 = random.randint(lower_bound_y, upper_bound_y)

    cropped = _rt.d2h(D.copy_window(_rt.h2d(image), (x0, y0, crop_size, crop_size)))
    if cropped.size == 0:
        raise RuntimeError("Le crop a produit une image vide.")

    shifted = bboxes_absolute - np.array([[x0, y0, x0, y0]])
    clipped = np.clip(shifted, 0, crop_size)
    valid = (clipped[:, 0] < clipped[:, 2]) & (clipped[:, 1] < clipped[:, 3])
    if not any(valid):
        raise RuntimeError("Aucune bbox résiduelle après le crop.")
    new_bboxes = xyxy2xywhn(clipped[valid], crop_size, crop_size)
    img_output_path = Path(image_target_dir) / input_image_path.name
    label_output_path = Path(label_target_dir) / input_label_path.name
    _save_crop_files(cropped, (class_ids[valid], new_bboxes), img_output_path, label_output_path)
    return [img_output_path, label_output_path]
