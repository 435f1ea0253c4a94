"""crop_from_border / fit_crop — reference transforms/recadrages.py:13-82.

Margins: fraction of the side when < 1, pixels otherwise (`_compute_crop`,
:7-10); JPG-only input (:23-24); output keeps the input name.  The crop is an
exact window copy on the GPU (ipp_copy_window); fit_crop uses Pillow's
getbbox rule via ipp_alpha_bbox."""
from __future__ import annotations

from pathlib import Path
from typing import Any, List, Optional, Tuple

import numpy as np
from PIL import Image

from ._common import batch_run, device_transform
from .. import _rt
from .. import batch_ops as BO
from .. import device as D
from .. import geometry as G
from .. import io as _io


def _compute_crop(value, total_length):
    return G.compute_crop(value, total_length)


@device_transform
def crop_from_border(
    file: Path,
    output_dirs: List[Path],
    crop_margins: Tuple[float, float, float, float] = (0, 0, 0, 0),
    **options: Any,
) -> Optional[Path]:
    output_dir = Path(output_dirs[0])
    if file.suffix.lower() not in (".jpg", ".jpeg"):
        raise ValueError(f"Le Fichier {file.name} n'est pas du type JPG.")
    crop_top, crop_bottom, crop_left, crop_right = crop_margins
    image = _io.imread(str(file), _io.IMREAD_UNCHANGED)
    if image is None:
        raise FileNotFoundError(f"Impossible de charger l'image {file.name}.")
    height, width = image.shape[:2]
    t = _compute_crop(crop_top, height)
    b = _compute_crop(crop_bottom, height)
    l = _compute_crop(crop_left, width)
    r = _compute_crop(crop_right, width)
    if t + b >= height or l + r >= width:
        raise ValueError(f"Les marges de rognage sont trop grandes pour l'image {file.name}.")
    cropped = _rt.d2h(D.copy_window(_rt.h2d(image), (l, t, width - l - r, height - t - b)))
    if image.ndim == 2:
        cropped = cropped[..., 0]
    output_path = output_dir / file.name
    try:
        if _io.imwrite(str(output_path), cropped):
            return output_path
        print(f"Avertissement [{file.name} - Symétrie]: Échec de sauvegarde (imwrite a retourné False) "
              f"pour {output_path.name}")
        return None
    except Exception as e_save:
        print(f"Erreur [{file.name} - Symétrie]: Échec de sauvegarde pour {output_path.name}: {e_save}")
        return None


def _crop_batch(arg_tuples, output_dirs: List[Path], threads: int = 1,
                crop_margins: Tuple[float, float, float, float] = (0, 0, 0, 0), **options: Any) -> List:
    """Batched crop_from_border: decode + margin checks on host threads, one
    ipp_copy_window launch for the chunk, encode on host threads."""
    output_dir = Path(output_dirs[0])

    def load(args):
        file = args[0]
        if file.suffix.lower() not in (".jpg", ".jpeg"):
            raise ValueError(f"Le Fichier {file.name} n'est pas du type JPG.")
        image = _io.imread(str(file), _io.IMREAD_UNCHANGED)
        if image is None:
            raise FileNotFoundError(f"Impossible de charger l'image {file.name}.")
        height, width = image.shape[:2]
        t, b = _compute_crop(crop_margins[0], height), _compute_crop(crop_margins[1], height)
        l, r = _compute_crop(crop_margins[2], width), _compute_crop(crop_margins[3], width)
        if t + b >= height or l + r >= width:
            raise ValueError(f"Les marges de rognage sont trop grandes pour l'image {file.name}.")
        return image, (l, t, width - l - r, height - t - b)

    def compute(items, _args):
        return BO.copy_windows([im for im, _ in items], [(k, win, 0) for k, (_, win) in enumerate(items)])

    def save(args, _item, cropped):
        file = args[0]
        output_path = output_dir / file.name
        try:
            if _io.imwrite(str(output_path), cropped):
                return output_path
            print(f"Avertissement [{file.name} - Symétrie]: Échec de sauvegarde (imwrite a retourné False) "
                  f"pour {output_path.name}")
            return None
        except Exception as e_save:
            print(f"Erreur [{file.name} - Symétrie]: Échec de sauvegarde pour {output_path.name}: {e_save}")
            return None

    return batch_run(arg_tuples, threads, load, compute, save)


crop_from_border.batch = _crop_batch


@device_transform
def fit_crop(image_path: Path, output_dirs: List[Path], **options: Any) -> Optional[List[Path]]:
    """Crop to Pillow's getbbox() (recadrages.py:63-82)."""
    output_dir = Path(output_dirs[0])
    image = Image.open(image_path)
    image.load()
    arr = np.asarray(image)
    if arr.dtype == bool:                      # mode '1'
        arr = arr.astype(np.uint8)
    h, w = arr.shape[:2]
    px = np.ascontiguousarray(arr).view(np.uint8).reshape(h, w, -1)   # bytes per pixel
    bpp = px.shape[2]
    t = _rt.h2d(px)
    # Pillow getbbox(alpha_only=True): the alpha band when the mode has one,
    # else every band (CMYK, RGBX, RGB, L, I;16, …) — non-zero bytes of a
    # pixel are a non-zero pixel.
    if image.mode in ("RGBA", "LA", "PA", "RGBa", "La"):
        bb = D.alpha_bbox([t])[0]
    elif bpp == 2:
        # 2-byte modes (I;16, I;16B, …) are stored through Pillow's image8
        # rows, so GetBBox.c scans only the first `w` BYTES of each row and
        # reports byte columns as pixel x coordinates
        head = _rt.h2d(np.ascontiguousarray(px.reshape(h, 2 * w)[:, :w]).reshape(h, w, 1))
        bb = D.alpha_bbox([head])[0]
    else:
        bb = D.alpha_bbox([t.view(h, w * bpp, 1)])[0]
        if bb:
            bb = (bb[0] // bpp, bb[1], (bb[2] - 1) // bpp + 1, bb[3])
    if not bb:
        new_image = image.copy()
    else:
        x0, y0, x1, y1 = bb
        out = _rt.d2h(D.copy_window(t, (x0, y0, x1 - x0, y1 - y0)))
        out = np.ascontiguousarray(out).view(arr.dtype).reshape((y1 - y0, x1 - x0) + arr.shape[2:])
        if image.mode == "1":
            new_image = Image.fromarray(out.astype(bool))
        elif arr.ndim == 2 and image.mode != "P":
            new_image = Image.fromarray(out)            # L, I;16, I, F
        else:
            new_image = Image.fromarray(out, image.mode)
        if image.mode == "P":
            new_image.putpalette(image.getpalette())
        # Image.crop keeps info for every mode (Image._new): icc_profile,
        # transparency, dpi… reach the PNG writer as in the reference
        new_image.info = dict(image.info)
    output_path = output_dir / image_path.name
    new_image.save(output_path)
    return output_path
