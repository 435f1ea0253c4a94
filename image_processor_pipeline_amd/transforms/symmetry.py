"""generate_symmetries — reference transforms/symmetry.py:11-149.

Same validation order and exceptions (ValueError / FileNotFoundError / warn),
``random.sample(pool, choose_random)`` (:122), forced 'o' (:125-126), names
``{stem}_{sym}{suffix}`` (:133).  cv2.flip codes 1/0/-1 → ipp_copy_window
with mirror flags on the GPU (exact index maps)."""
from __future__ import annotations

import random
from pathlib import Path
from typing import Any, List, Optional
from warnings import warn

import numpy as np

from ._common import device_transform
from .. import _rt
from .. import device as D
from .. import io as _io

ALL_SYMS = ("o", "h", "v", "hv")


@device_transform
def generate_symmetries(
    input_path: Path,
    output_dirs: List[Path],
    pool: Optional[List[str]] = None,
    choose_random: Optional[int] = None,
    include_original: bool = True,
    **options: Any,
) -> Optional[List[Path]]:
    if not output_dirs:
        raise ValueError(f"Erreur [{input_path.name} - Symétrie]: Aucun dossier de sortie ('output_dirs') fourni.")
    output_dir = Path(output_dirs[0])

    if input_path.suffix.lower()[1:] not in _io.IMG_FORMATS:
        raise ValueError(f"Le fichier {input_path.name} n'est pas un format accepté par Yolo.")

    pool = pool if pool else list(ALL_SYMS)
    if any(sym not in ALL_SYMS for sym in pool):
        invalid_keys = [k for k in pool if k not in ALL_SYMS]
        raise ValueError(f"`pool` contient des éléments invalides : {invalid_keys}")

    choose_random = len(pool) if choose_random is None else choose_random
    if choose_random > len(pool):
        warn(f"Choix aléatoire de plus d'éléments ({choose_random}) que possible parmi {pool} ({len(pool)}).")
    elif choose_random < 0:
        raise ValueError(f"[{input_path.name} - Symétrie] `choose_random` ({choose_random}) doit être >= 0. "
                         "Aucune symétrie aléatoire générée.")

    image = _io.imread(str(input_path), _io.IMREAD_UNCHANGED)
    if image is None:
        raise FileNotFoundError(f"[{input_path.name} - Symétrie] Impossible de charger l'image.")

    filter_ = random.sample(pool, choose_random)
    if include_original and "o" not in set(filter_):
        filter_.append("o")

    gray = image.ndim == 2
    dtype = image.dtype
    if dtype != np.uint8:
        # deep images (16-bit PNG via IMREAD_UNCHANGED): flip whole pixels as
        # byte groups (cv2.flip is dtype-agnostic)
        if image.itemsize * (1 if gray else image.shape[2]) > 4:
            raise ValueError(f"[{input_path.name} - Symétrie] format de pixel non pris en charge ({dtype}).")
        h, w = image.shape[:2]
        image = np.ascontiguousarray(image).view(np.uint8).reshape(h, w, -1)
    img_dev = _rt.h2d(image)
    saved_files: List[Path] = []
    for sym in filter_:
        out = _rt.d2h(D.flip(img_dev, sym))
        if dtype != np.uint8:
            out = np.ascontiguousarray(out).view(dtype).reshape(out.shape[0], out.shape[1], -1)
        if gray:
            out = out[..., 0]
        output_filename = input_path.with_stem(f"{input_path.stem}_{sym}")
        output_path = output_dir / output_filename.name
        try:
            if _io.imwrite(str(output_path), out):
                saved_files.append(output_path)
            else:
                warn(f"Échec de sauvegarde de la symétrie '{sym}' pour {output_path.name}. Retour False depuis `.imwrite`")
        except Exception as e_save:
            warn(f"Erreur [{input_path.name} - Symétrie '{sym}']: Échec de sauvegarde pour {output_filename} : {e_save}.")
    return saved_files
