"""keep_largest_component — reference transforms/pixels_isolés.py:8-81.

BGRA PNG only; α > 1 is foreground (threshold :32); 8-connected components
(:35); the largest area wins, ties → lowest OpenCV label (restated, see
csrc/ipp_ccl.hip); α := 0 elsewhere (:47-55); crop to the bbox of α ≠ 0
(:74-81).  The reference's `min_component_size` loop (:50-52) has no effect
and is not reproduced (the argument is accepted).  All pixel work runs in
ipp_ccl_keep_largest on the GPU.
"""
from __future__ import annotations

from pathlib import Path
from typing import List

import numpy as np

from ._common import batch_run, device_transform
from .. import _rt
from .. import batch_ops as BO
from .. import device_ccl
from .. import io as _io
from ..utils.utils import _validate_dirs


@device_transform
def keep_largest_component(file: Path, output_dirs: List[Path], min_component_size: int = 500) -> np.ndarray:
    output_dir = _validate_dirs(output_dirs, nb_dirs=1)
    if file.suffix.lower() != ".png":
        raise ValueError(f"Le fichier {file.name} n'est pas un PNG.")
    image = _io.imread(str(file), _io.IMREAD_UNCHANGED)
    if image is None:
        raise FileNotFoundError(f"Impossible de charger l'image {file.name}.")
    if image.shape[2] != 4:   # a 2-D (grey) image raises IndexError here, as in the reference
        raise AttributeError(f"L'image {file.name} ne contient pas de canal alpha, elle sera ignorée.")
    cropped = _rt.d2h(device_ccl.keep_largest_component(_rt.h2d(image)))
    output_path = Path(output_dir) / file.name
    try:
        _io.imwrite(str(output_path), cropped)
        return output_path
    except Exception as e_save:
        print(f"Erreur [{file.name} - Symétrie]: Échec de sauvegarde pour {output_path.name}: {e_save}")
        return None


def _keep_batch(arg_tuples, output_dirs: List[Path], threads: int = 1, min_component_size: int = 500,
                **options) -> List:
    """Batched keep_largest_component: decode on host threads, one
    ipp_ccl_keep_largest + one crop launch for the chunk, encode on threads."""
    output_dir = _validate_dirs(output_dirs, nb_dirs=1)

    def load(args):
        file = args[0]
        if file.suffix.lower() != ".png":
            raise ValueError(f"Le fichier {file.name} n'est pas un PNG.")
        image = _io.imread(str(file), _io.IMREAD_UNCHANGED)
        if image is None:
            raise FileNotFoundError(f"Impossible de charger l'image {file.name}.")
        if image.shape[2] != 4:   # IndexError for a 2-D image, as the per-file path
            raise AttributeError(f"L'image {file.name} ne contient pas de canal alpha, elle sera ignorée.")
        return image

    def compute(images, _args):
        return BO.keep_largest(images)

    def save(args, _img, cropped):
        file = args[0]
        if cropped is None:
            raise ValueError("aucun pixel non transparent (cv2.boundingRect(None))")
        output_path = Path(output_dir) / file.name
        try:
            _io.imwrite(str(output_path), cropped)
            return output_path
        except Exception as e_save:
            print(f"Erreur [{file.name} - Symétrie]: Échec de sauvegarde pour {output_path.name}: {e_save}")
            return None

    return batch_run(arg_tuples, threads, load, compute, save)


keep_largest_component.batch = _keep_batch
