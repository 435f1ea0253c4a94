"""process_images_with_color_masks — reference transforms/filtres_liste.py:41-149.

BGR (cv2.imread IMREAD_COLOR, input alpha dropped) → 8-bit HSV (OpenCV
RGB2HSV_b) → OR over the ranges of (inRange AND zone) → NOT → alpha; output
BGRA PNG ``{prefix}{_}{stem}.png``.  One fused pass on the GPU
(ipp_hsv_mask).  `_rescale_filter` keeps its checks, prints and GIMP scaling.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, List, Optional, Tuple

from ._common import batch_run, device_transform
from .. import _rt
from .. import batch_ops as BO
from .. import device as D
from .. import geometry as G
from .. import io as _io
from ..utils.utils import _validate_dirs


def _rescale_filter(filter_tuple, use_gimp_scale: bool = False):
    return G.rescale_filter(filter_tuple, use_gimp_scale)


@device_transform
def process_images_with_color_masks(
    image_path: Path,
    output_dirs: List[Path],
    color_ranges_to_exclude_hsv: List[Tuple[int, int, int, int, int, int]],
    zones=None,
    use_gimp_scale: bool = False,
    output_prefix: str = "",
    **options: Any,
) -> Optional[Path]:
    output_dir = _validate_dirs(output_dirs, nb_dirs=1)
    if not color_ranges_to_exclude_hsv:
        raise ValueError(f"Erreur [{image_path.name} - ColorMask] : `color_ranges_to_exclude_hsv` est requis pour "
                         "traiter les données")
    if zones and len(zones) != len(color_ranges_to_exclude_hsv):
        raise ValueError(f"Les zones d'application des filtres colorimétriques ({len(zones)}) ne correspondent pas aux "
                         f"filtres ({len(color_ranges_to_exclude_hsv)}). Les 2 paramètres doivent être de même longueur !.")
    elif not zones:
        zones = [None] * len(color_ranges_to_exclude_hsv)

    image = _io.imread(str(image_path))
    if image is None:
        raise IOError("Impossible de charger l'image.")
    params = G.hsv_params(color_ranges_to_exclude_hsv, zones, use_gimp_scale, bgr=True)
    result = _rt.d2h(D.hsv_mask(_rt.h2d(image), params))

    output_filename = f"{output_prefix}{'_' if output_prefix else ''}{image_path.stem}.png"
    output_path = Path(output_dir) / output_filename
    try:
        if _io.imwrite(str(output_path), result):
            return output_path
        raise RuntimeError(f"Échec de sauvegarde (imwrite a retrouné False) pour {output_filename}")
    except Exception as e_save:
        print(f"Erreur lors de la sauvegarde de {output_path}: {e_save}")
        return None


def _masks_batch(arg_tuples, output_dirs: List[Path], threads: int = 1, color_ranges_to_exclude_hsv=None,
                 zones=None, use_gimp_scale: bool = False, output_prefix: str = "", **options: Any) -> List:
    """Batched process_images_with_color_masks: decode on host threads, one
    ipp_hsv_mask launch for the chunk, PNG encode on host threads."""
    output_dir = _validate_dirs(output_dirs, nb_dirs=1)
    ranges = color_ranges_to_exclude_hsv

    def load(args):
        image_path = args[0]
        if not ranges:
            raise ValueError(f"Erreur [{image_path.name} - ColorMask] : `color_ranges_to_exclude_hsv` est requis "
                             "pour traiter les données")
        if zones and len(zones) != len(ranges):
            raise ValueError(f"Les zones d'application des filtres colorimétriques ({len(zones)}) ne correspondent "
                             f"pas aux filtres ({len(ranges)}). Les 2 paramètres doivent être de même longueur !.")
        image = _io.imread(str(image_path))
        if image is None:
            raise IOError("Impossible de charger l'image.")
        return image

    def compute(images, _args):
        params = G.hsv_params(ranges, zones or [None] * len(ranges), use_gimp_scale, bgr=True)
        return BO.hsv_masks(images, params)

    def save(args, _img, result):
        image_path = args[0]
        output_filename = f"{output_prefix}{'_' if output_prefix else ''}{image_path.stem}.png"
        output_path = Path(output_dir) / output_filename
        try:
            if _io.imwrite(str(output_path), result):
                return output_path
            raise RuntimeError(f"Échec de sauvegarde (imwrite a retrouné False) pour {output_filename}")
        except Exception as e_save:
            print(f"Erreur lors de la sauvegarde de {output_path}: {e_save}")
            return None

    return batch_run(arg_tuples, threads, load, compute, save)


process_images_with_color_masks.batch = _masks_batch
