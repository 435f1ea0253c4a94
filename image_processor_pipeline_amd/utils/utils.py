"""Path and output helpers — same names, signatures and errors as the
reference's utils/utils.py (check_path :7-37, _validate_dirs :39-65,
_save_crop_files :67-98)."""
from __future__ import annotations

from pathlib import Path
from typing import List, Tuple, Union

import numpy as np

from .. import io as _io


def check_path(folder_name, root=None) -> Path:
    """Absolute paths are returned as-is; relative ones are joined to `root`
    (or the current directory)."""
    path = Path(folder_name)
    root_path = Path(root) if root else Path(".")
    return path if path.is_absolute() else root_path / path


def _validate_dirs(output_dirs: List[Path], nb_dirs: int) -> Union[Path, Tuple[Path, ...]]:
    """IndexError when fewer than `nb_dirs` output dirs are given; one Path
    for nb_dirs == 1, else a tuple."""
    if len(output_dirs) < nb_dirs:
        raise IndexError(f"Au moins {nb_dirs} dossiers de sortie requis (images, labels). "
                         f"{len(output_dirs)} fournis.")
    paths = tuple(Path(d) for d in output_dirs)
    if nb_dirs == 1:
        return paths[0]
    return paths


def _save_crop_files(img: np.ndarray, labels: Tuple[np.ndarray, np.ndarray], img_out: Path,
                     label_out: Path) -> None:
    """Write a BGR image and its YOLO labels (`cls cx cy w h`, 6 decimals)."""
    classes, bboxes = labels
    if not _io.imwrite(str(img_out), img):
        raise IOError(f"Échec écriture de l'image : {img_out}")
    with open(label_out, "w", encoding="utf-8") as f:
        for cls_id, box in zip(classes, bboxes):
            cx, cy, w, h = box
            f.write(f"{cls_id} {cx:.6f} {cy:.6f} {w:.6f} {h:.6f}\n")
