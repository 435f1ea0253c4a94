"""process_images_with_color_masks — reference transforms/filtres_liste.py:41-149.

BGR (cv2.imread IMREAD_COLOR, input alpha dropped) → 8-bit HSV (OpenCV
RGB2HSV_b) → OR over the ranges of (inRange AND zone) → NOT → alpha; output
BGRA PNG ``{prefix}{_}{stem}.png``.  One fused pass on the GPU
(ipp_hsv_mask).  `_rescale_filter` keeps its checks, prints and GIMP scaling.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, List, Optional, Tuple

from ._common import device_transform
from .. import _rt
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
