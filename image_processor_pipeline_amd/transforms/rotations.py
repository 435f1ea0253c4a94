"""process_rotations — reference transforms/rotations.py:6-133.

Same signature, draw order (one ``random.uniform(angle_min, angle_max)`` per
rotation, rotations.py:89), file naming (``{stem}_{original_key}`` and
``{stem}_{prefix}{index:03d}``, :78, :114-116) and error style (print +
continue / return None).  Pixels: Pillow ``convert('RGBA')`` + ``rotate(angle,
expand=True)`` (NEAREST) + ``getbbox()``/``crop`` run as one fused gather on
the GPU (ipp_rotate_flip_nearest), bit-exact with Pillow 12.2.0.
"""
from __future__ import annotations

import random
from pathlib import Path
from typing import Any, List, Optional

import numpy as np
from PIL import Image, UnidentifiedImageError

from ._common import device_transform, thread_map
from .. import _rt
from .. import device as D


def _rotate(img_dev, opaque: bool, angle: float, name: str, idx: int, resample: str = "nearest") -> np.ndarray:
    """rotations.py:96-109 with its two fallbacks (None / empty bbox)."""
    h, w, _ = img_dev.shape
    if resample == "bilinear":
        canvas = D.rotate_bilinear_canvas(img_dev, angle)
        bb = D.alpha_bbox([canvas])[0]
        if bb is None:
            print(f"Avertissement [{name} - Rotation]: Impossible d'obtenir BBox après rotation {idx}. "
                  "Utilisation de l'image non recadrée.")
            return _rt.d2h(canvas)
        x0, y0, x1, y1 = bb
        if x1 - x0 <= 0 or y1 - y0 <= 0:
            print(f"Avertissement [{name} - Rotation]: Recadrage après rotation {idx} vide. "
                  "Utilisation de l'image non recadrée.")
            return _rt.d2h(canvas)
        return _rt.d2h(D.copy_window(canvas, (x0, y0, x1 - x0, y1 - y0)))
    if opaque:
        plan = D.plan_rotate_flip([(h, w, img_dev.shape[2])], [angle], [0])
        return _rt.d2h(D.unpack(D.rotate_flip_nearest(img_dev.reshape(-1), plan), plan)[0])
    plan = D.plan_rotate_flip([(h, w, 4)], [angle], [0], crop_to_bbox=False)
    canvas = D.unpack(D.rotate_flip_nearest(img_dev.reshape(-1), plan), plan)[0].contiguous()
    bb = D.alpha_bbox([canvas])[0]
    if bb is None:
        print(f"Avertissement [{name} - Rotation]: Impossible d'obtenir BBox après rotation {idx}. "
              "Utilisation de l'image non recadrée.")
        return _rt.d2h(canvas)
    x0, y0, x1, y1 = bb
    if x1 - x0 <= 0 or y1 - y0 <= 0:
        print(f"Avertissement [{name} - Rotation]: Recadrage après rotation {idx} vide. "
              "Utilisation de l'image non recadrée.")
        return _rt.d2h(canvas)
    return _rt.d2h(D.copy_window(canvas, (x0, y0, x1 - x0, y1 - y0)))


@device_transform
def process_rotations(
    input_path: Path,
    output_dirs: List[Path],
    num_rotations: int = 10,
    include_original: bool = True,
    angle_min: float = 1.0,
    angle_max: float = 359.0,
    output_format: str = "png",
    output_prefix: str = "r",
    original_key: str = "r000",
    rotation_key_format: str = "{prefix}{index:03d}",
    resample: str = "nearest",
    **options: Any,
) -> Optional[List[Path]]:
    """``resample`` (not in the reference, whose rotate is NEAREST): "nearest"
    (default, bit-exact with rotations.py:96) or "bilinear" (opt-in, bit-exact
    with Pillow ``rotate(..., resample=BILINEAR)``)."""
    if resample not in ("nearest", "bilinear"):
        raise ValueError(f"resample must be 'nearest' or 'bilinear', not {resample!r}")
    if not output_dirs:
        print(f"Erreur [{input_path.name} - Rotation]: Aucun dossier de sortie ('output_paths') fourni.")
        return None
    target_dir = Path(output_dirs[0])
    try:
        src = Image.open(input_path)
        has_alpha = src.mode in ("RGBA", "LA", "PA", "RGBa", "La") or "transparency" in src.info
        img = src.convert("RGBA")
    except FileNotFoundError:
        print(f"Erreur [{input_path.name} - Rotation]: Fichier non trouvé.")
        return None
    except UnidentifiedImageError:
        print(f"Erreur [{input_path.name} - Rotation]: Impossible d'identifier ou d'ouvrir l'image (format invalide?).")
        return None
    except Exception as e:
        print(f"Erreur [{input_path.name} - Rotation]: Échec lors de la lecture du fichier: {e}")
        return None

    saved_files: List[Path] = []
    base_name = input_path.stem
    out_suffix = f".{output_format.lower()}"
    if output_format.lower() == "jpeg":
        out_suffix = ".jpg"

    if include_original:
        name = f"{base_name}_{original_key}{out_suffix}"
        p = target_dir / name
        try:
            img.save(p, format=output_format)
            saved_files.append(p)
        except Exception as e_save:
            print(f"Erreur [{input_path.name} - Rotation]: Échec sauvegarde de l'original '{name}': {e_save}")

    arr = np.asarray(img)
    # opaque sources (no alpha band) take the analytic-bbox path: α = 255 everywhere
    img_dev = _rt.h2d(arr if has_alpha else arr[..., :3])
    for i in range(num_rotations):
        angle = random.uniform(angle_min, angle_max)
        try:
            rotated = _rotate(img_dev, not has_alpha, angle, input_path.name, i + 1, resample)
            key = rotation_key_format.format(prefix=output_prefix, index=i + 1)
            p = target_dir / f"{base_name}_{key}{out_suffix}"
            Image.fromarray(rotated, "RGBA").save(p, format=output_format)
            saved_files.append(p)
        except Exception as e_rot_save:
            print(f"Erreur [{input_path.name} - Rotation]: Échec lors de la génération/sauvegarde de la rotation "
                  f"{i + 1} (angle {angle:.1f}°): {e_rot_save}")

    if not saved_files:
        print(f"Avertissement [{input_path.name} - Rotation]: Aucune image (originale ou rotation) n'a pu être sauvegardée.")
        return None
    return saved_files


def _rotations_batch(arg_tuples, output_dirs: List[Path], threads: int = 1, num_rotations: int = 10,
                     include_original: bool = True, angle_min: float = 1.0, angle_max: float = 359.0,
                     output_format: str = "png", output_prefix: str = "r", original_key: str = "r000",
                     rotation_key_format: str = "{prefix}{index:03d}", resample: str = "nearest",
                     **options: Any) -> List:
    """Batched process_rotations for ProcessingStep (one result per input).

    Decode on `threads` host threads; draw the angles in the sequential
    order (per file, then per rotation — identical outputs to per-file
    calls); all opaque sources of the chunk go through ONE fused gather
    launch (rotate + analytic bbox crop); alpha sources use the per-file
    device path; encode on host threads."""
    if not output_dirs or resample != "nearest":
        # per-file path (the bilinear mode has no batched gather)
        return [process_rotations(*a, output_dirs=output_dirs, num_rotations=num_rotations,
                                  include_original=include_original, angle_min=angle_min, angle_max=angle_max,
                                  output_format=output_format, output_prefix=output_prefix,
                                  original_key=original_key, rotation_key_format=rotation_key_format,
                                  resample=resample, **options) for a in arg_tuples]
    target_dir = Path(output_dirs[0])
    fmt = output_format.lower()
    out_suffix = ".jpg" if fmt == "jpeg" else f".{fmt}"

    def decode(args):
        p = args[0]
        try:
            src = Image.open(p)
            has_alpha = src.mode in ("RGBA", "LA", "PA", "RGBa", "La") or "transparency" in src.info
            return src.convert("RGBA"), has_alpha
        except FileNotFoundError:
            print(f"Erreur [{p.name} - Rotation]: Fichier non trouvé.")
        except UnidentifiedImageError:
            print(f"Erreur [{p.name} - Rotation]: Impossible d'identifier ou d'ouvrir l'image (format invalide?).")
        except Exception as e:
            print(f"Erreur [{p.name} - Rotation]: Échec lors de la lecture du fichier: {e}")
        return None

    decoded = thread_map(decode, arg_tuples, threads)
    angles = [[random.uniform(angle_min, angle_max) for _ in range(num_rotations)]
              if isinstance(d, tuple) else None for d in decoded]

    # one gather launch for every rotation of every opaque source
    opaque = [i for i, d in enumerate(decoded) if isinstance(d, tuple) and not d[1]]
    rotated: dict = {}
    if opaque:
        arrays = [np.asarray(decoded[i][0])[..., :3] for i in opaque]
        sizes = [a.size for a in arrays]
        flat = np.concatenate([a.reshape(-1) for a in arrays])
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
        dims, angs, src_offs, keys = [], [], [], []
        for j, i in enumerate(opaque):
            for r, a in enumerate(angles[i]):
                dims.append(arrays[j].shape)
                angs.append(a)
                src_offs.append(int(offs[j]))
                keys.append((i, r))
        if dims:
            plan = D.plan_rotate_flip(dims, angs, [0] * len(dims), src_offsets=src_offs)
            out = _rt.d2h(D.rotate_flip_nearest(_rt.h2d(flat).reshape(-1), plan))
            for k, (oh, ow), off, pitch in zip(keys, plan.shapes, plan.offsets, plan.pitches):
                rotated[k] = np.lib.stride_tricks.as_strided(
                    out[off:], (oh, ow, 4), (int(pitch), 4, 1)).copy()

    def finish(i):
        d = decoded[i]
        if not isinstance(d, tuple):
            return None
        img, has_alpha = d
        name = arg_tuples[i][0].name
        base = arg_tuples[i][0].stem
        saved: List[Path] = []
        if include_original:
            p = target_dir / f"{base}_{original_key}{out_suffix}"
            try:
                img.save(p, format=output_format)
                saved.append(p)
            except Exception as e_save:
                print(f"Erreur [{name} - Rotation]: Échec sauvegarde de l'original '{p.name}': {e_save}")
        dev = None if not has_alpha else _rt.h2d(np.asarray(img))
        for r, angle in enumerate(angles[i]):
            try:
                arr = rotated[(i, r)] if not has_alpha else _rotate(dev, False, angle, name, r + 1)
                key = rotation_key_format.format(prefix=output_prefix, index=r + 1)
                p = target_dir / f"{base}_{key}{out_suffix}"
                Image.fromarray(arr, "RGBA").save(p, format=output_format)
                saved.append(p)
            except Exception as e_rot_save:
                print(f"Erreur [{name} - Rotation]: Échec lors de la génération/sauvegarde de la rotation "
                      f"{r + 1} (angle {angle:.1f}°): {e_rot_save}")
        if not saved:
            print(f"Avertissement [{name} - Rotation]: Aucune image (originale ou rotation) n'a pu être sauvegardée.")
            return None
        return saved

    return thread_map(finish, range(len(arg_tuples)), threads)


process_rotations.batch = _rotations_batch
