"""paste_overlay_onto_background — reference transforms/overlays.py:24-187.

Diagonal-ratio sizing with one ``random.uniform(scale_min, scale_max)``
(:108) and the fit cap (:106-126), Pillow ``resize(LANCZOS)`` of the RGBA
overlay (:129), position from two ``random.randint`` (:133-134),
``background.copy().paste(ov, (x, y), ov)`` (:138-139), YOLO label (:143-149),
outputs ``{overlay_stem}{background_suffix}`` and ``{overlay_stem}.txt``
(:165-166); errors print and return None.  Resize and paste run on the GPU
(ipp_lanczos_h/v, ipp_paste_blend), bit-exact with Pillow 12.2.0.
The deprecated ``process_overlay_pair`` (:190-354) is not provided.
"""
from __future__ import annotations

import math
import random
from pathlib import Path
from typing import Any, List, Optional, Tuple

import numpy as np
from PIL import Image, UnidentifiedImageError

from ._common import batch_run, device_transform
from .. import _rt
from .. import batch_ops as BO
from .. import device as D
from .. import geometry as G
from ..labels_math import xyxy2xywhn
from ..utils import utils


def _convert_to_yolo_bbox(img_width: int, img_height: int, box: Tuple[int, int, int, int]):
    """overlays.py:13-22."""
    if img_width <= 0 or img_height <= 0:
        raise ValueError(f"Les dimensions de l'image ({img_width}x{img_height}) doivent être positives.")
    dw = 1.0 / img_width
    dh = 1.0 / img_height
    return ((box[0] + box[2]) / 2.0 * dw, (box[1] + box[3]) / 2.0 * dh, (box[2] - box[0]) * dw,
            (box[3] - box[1]) * dh)


@device_transform
def paste_overlay_onto_background(
    overlay_path: Path,
    background_path: Path,
    output_dirs: List[Path],
    yolo_class_id: int = 0,
    scale_min: float = 0.15,
    scale_max: float = 0.30,
    **options: Any,
) -> Optional[List[Path]]:
    image_target_dir, label_target_dir = utils._validate_dirs(output_dirs, nb_dirs=2)
    names = f"[{overlay_path.name} + {background_path.name}]"
    try:
        overlay = Image.open(overlay_path)
        if overlay.mode != "RGBA":
            overlay = overlay.convert("RGBA")
        background = Image.open(background_path).convert("RGB")
    except FileNotFoundError as fnf:
        print(f"Erreur {names}: Fichier non trouvé: {fnf}")
        return None
    except UnidentifiedImageError as uie:
        print(f"Erreur {names}: Impossible d'ouvrir l'image {uie}")
        return None
    except TypeError as te:
        print(f"Erreur {names}: Type d'image invalide : {te}")
        return None
    except Exception as e:
        print(f"Erreur {names}: Échec lecture fichiers: {e}")
        return None

    try:
        bw, bh = background.size
        target_ratio = random.uniform(scale_min, scale_max)
        if overlay.height == 0:
            raise ValueError(f"dimensions de l'overlay {overlay_path.name} invalides ({overlay.width}x{overlay.height}).")
        new_w, new_h = G.overlay_size(overlay.width, overlay.height, bw, bh, target_ratio)
        ov_dev = _rt.h2d(np.asarray(overlay))
        resized = D.resize_lanczos_rgba(ov_dev, new_w, new_h)
        pos_x = random.randint(0, bw - new_w)
        pos_y = random.randint(0, bh - new_h)
        comp = D.paste_blend(_rt.h2d(np.asarray(background)), resized, pos_x, pos_y)
        composite_image = Image.fromarray(_rt.d2h(comp), "RGB")
        bbox = np.array([pos_x, pos_y, pos_x + new_w, pos_y + new_h]).reshape(1, 4)
        cx, cy, w_norm, h_norm = xyxy2xywhn(bbox, bw, bh)[0]
        yolo_label_str = f"{yolo_class_id} {cx:.6f} {cy:.6f} {w_norm:.6f} {h_norm:.6f}"
    except ValueError as ve:
        print(f"Erreur de valeur {names}: {ve}")
        return None
    except Exception as e:
        print(f"Erreur {names}: Échec pendant le processus de superposition: {e}")
        return None

    saved_paths: List[Path] = []
    img_output_path = Path(image_target_dir) / f"{overlay_path.stem}{background_path.suffix}"
    label_output_path = Path(label_target_dir) / f"{overlay_path.stem}.txt"
    try:
        composite_image.save(img_output_path)
        saved_paths.append(img_output_path)
        with open(label_output_path, "w", encoding="utf-8") as f:
            f.write(yolo_label_str)
        saved_paths.append(label_output_path)
        return saved_paths
    except Exception as e_save:
        print(f"Erreur {names}: Échec lors de la sauvegarde: {e_save}")
        for p in saved_paths:
            try:
                if p.exists():
                    p.unlink()
            except OSError:
                print(f"Avertissement: Impossible de nettoyer le fichier partiellement créé {p}")
        return None


def _overlays_batch(arg_tuples, output_dirs: List[Path], threads: int = 1, yolo_class_id: int = 0,
                    scale_min: float = 0.15, scale_max: float = 0.30, **options: Any) -> List:
    """Batched paste_overlay_onto_background ('modulo' pairs): decode on host
    threads, the per-item draws (uniform ratio, then two randint) in pair
    order, ONE batched LANCZOS H + V + paste launch set for the chunk
    (batch_ops.overlays), encode + label on host threads.  Messages and
    None results as in the per-file path."""
    image_target_dir, label_target_dir = utils._validate_dirs(output_dirs, nb_dirs=2)

    def load(args):
        overlay_path, background_path = args[0], args[1]
        names = f"[{overlay_path.name} + {background_path.name}]"
        try:
            overlay = Image.open(overlay_path)
            if overlay.mode != "RGBA":
                overlay = overlay.convert("RGBA")
            background = Image.open(background_path).convert("RGB")
            return np.asarray(overlay), np.asarray(background)
        except FileNotFoundError as fnf:
            print(f"Erreur {names}: Fichier non trouvé: {fnf}")
        except UnidentifiedImageError as uie:
            print(f"Erreur {names}: Impossible d'ouvrir l'image {uie}")
        except TypeError as te:
            print(f"Erreur {names}: Type d'image invalide : {te}")
        except Exception as e:
            print(f"Erreur {names}: Échec lecture fichiers: {e}")
        return None

    def compute(items, args):
        plans, ovs, bgs, sizes, pos = [], [], [], [], []
        for item, a in zip(items, args):
            if item is None:
                plans.append(None)
                continue
            ov, bg = item
            names = f"[{a[0].name} + {a[1].name}]"
            try:
                bh, bw = bg.shape[:2]
                target_ratio = random.uniform(scale_min, scale_max)
                if ov.shape[0] == 0:
                    raise ValueError(f"dimensions de l'overlay {a[0].name} invalides ({ov.shape[1]}x{ov.shape[0]}).")
                new_w, new_h = G.overlay_size(ov.shape[1], ov.shape[0], bw, bh, target_ratio)
                if new_w <= 0 or new_h <= 0:
                    raise ValueError("height and width must be > 0")
                pos_x = random.randint(0, bw - new_w)
                pos_y = random.randint(0, bh - new_h)
            except ValueError as ve:
                print(f"Erreur de valeur {names}: {ve}")
                plans.append(None)
                continue
            except Exception as e:
                print(f"Erreur {names}: Échec pendant le processus de superposition: {e}")
                plans.append(None)
                continue
            plans.append((len(ovs), (new_w, new_h), (pos_x, pos_y), (bw, bh)))
            ovs.append(ov)
            bgs.append(bg)
            sizes.append((new_w, new_h))
            pos.append((pos_x, pos_y))
        comps = BO.overlays(ovs, bgs, sizes, pos) if ovs else []
        return [None if p is None else (comps[p[0]], p) for p in plans]

    def save(args, _item, res):
        if res is None:
            return None
        comp, (_, (new_w, new_h), (pos_x, pos_y), (bw, bh)) = res
        overlay_path, background_path = args[0], args[1]
        names = f"[{overlay_path.name} + {background_path.name}]"
        bbox = np.array([pos_x, pos_y, pos_x + new_w, pos_y + new_h]).reshape(1, 4)
        cx, cy, w_norm, h_norm = xyxy2xywhn(bbox, bw, bh)[0]
        yolo_label_str = f"{yolo_class_id} {cx:.6f} {cy:.6f} {w_norm:.6f} {h_norm:.6f}"
        saved_paths: List[Path] = []
        img_output_path = Path(image_target_dir) / f"{overlay_path.stem}{background_path.suffix}"
        label_output_path = Path(label_target_dir) / f"{overlay_path.stem}.txt"
        try:
            Image.fromarray(comp, "RGB").save(img_output_path)
            saved_paths.append(img_output_path)
            with open(label_output_path, "w", encoding="utf-8") as f:
                f.write(yolo_label_str)
            saved_paths.append(label_output_path)
            return saved_paths
        except Exception as e_save:
            print(f"Erreur {names}: Échec lors de la sauvegarde: {e_save}")
            for p in saved_paths:
                try:
                    if p.exists():
                        p.unlink()
                except OSError:
                    print(f"Avertissement: Impossible de nettoyer le fichier partiellement créé {p}")
            return None

    return batch_run(arg_tuples, threads, load, compute, save)


paste_overlay_onto_background.batch = _overlays_batch
