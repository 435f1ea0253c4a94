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

from ._common import batch_run, device_transform
from .. import _rt
from .. import batch_ops as BO
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


def _symmetries_batch(arg_tuples, output_dirs: List[Path], threads: int = 1, pool: Optional[List[str]] = None,
                      choose_random: Optional[int] = None, include_original: bool = True, **options: Any) -> List:
    """Batched generate_symmetries: validation + decode on host threads, the
    ``random.sample`` draws in file order, ONE ipp_copy_window launch for every
    flip of every image of the chunk, encode on host threads.  Deep (16-bit)
    images take the per-file path."""
    if not output_dirs:
        return [generate_symmetries(*a, output_dirs=output_dirs, pool=pool, choose_random=choose_random,
                                    include_original=include_original, **options) for a in arg_tuples]
    output_dir = Path(output_dirs[0])

    def validate(args):
        input_path = args[0]
        if input_path.suffix.lower()[1:] not in _io.IMG_FORMATS:
            raise ValueError(f"Le fichier {input_path.name} n'est pas un format accepté par Yolo.")
        pl = pool if pool else list(ALL_SYMS)
        if any(sym not in ALL_SYMS for sym in pl):
            raise ValueError(f"`pool` contient des éléments invalides : {[k for k in pl if k not in ALL_SYMS]}")
        k = len(pl) if choose_random is None else choose_random
        if k > len(pl):
            warn(f"Choix aléatoire de plus d'éléments ({k}) que possible parmi {pl} ({len(pl)}).")
        elif k < 0:
            raise ValueError(f"[{input_path.name} - Symétrie] `choose_random` ({k}) doit être >= 0. "
                             "Aucune symétrie aléatoire générée.")
        return pl, k

    # The checks (and their warnings) run here, on this thread, in file order
    # — as the per-file calls would emit them; only decoding goes to threads.
    checked = {}
    for a in arg_tuples:
        try:
            checked[id(a)] = validate(a)
        except Exception as e:
            checked[id(a)] = e

    def load(args):
        input_path = args[0]
        c = checked[id(args)]
        if isinstance(c, Exception):
            raise c
        pl, k = c
        image = _io.imread(str(input_path), _io.IMREAD_UNCHANGED)
        if image is None:
            raise FileNotFoundError(f"[{input_path.name} - Symétrie] Impossible de charger l'image.")
        return image, pl, k

    def compute(items, args):
        keys, deep, jobs, imgs = [], [], [], []
        for (image, pl, k), a in zip(items, args):
            try:
                filter_ = random.sample(pl, k)
            except Exception as e:        # e.g. choose_random > len(pool): raised for this file only
                keys.append(e)
                deep.append(False)
                continue
            if include_original and "o" not in set(filter_):
                filter_.append("o")
            keys.append(filter_)
            deep.append(image.dtype != np.uint8)
            imgs.append(image if image.dtype == np.uint8 else np.zeros((1, 1), np.uint8))
            if image.dtype == np.uint8:
                h, w = image.shape[:2]
                jobs += [(len(imgs) - 1, (0, 0, w, h), D.SYM_FLIP[s]) for s in filter_]
        flipped = iter(BO.copy_windows(imgs, jobs))
        out = []
        for (image, _, _), ks, dp in zip(items, keys, deep):
            out.append(ks if isinstance(ks, Exception) else [(s, None if dp else next(flipped)) for s in ks])
        return out

    def save(args, item, flips):
        if isinstance(flips, Exception):
            raise flips
        input_path = args[0]
        image = item[0]
        saved_files: List[Path] = []
        for sym, arr in flips:
            if arr is None:   # deep image: per-image device flip, as the per-file path
                h, w = image.shape[:2]
                raw = np.ascontiguousarray(image).view(np.uint8).reshape(h, w, -1)
                arr = _rt.d2h(D.flip(_rt.h2d(raw), sym))
                arr = np.ascontiguousarray(arr).view(image.dtype).reshape(h, w, -1)
                if image.ndim == 2:
                    arr = arr[..., 0]
            output_filename = input_path.with_stem(f"{input_path.stem}_{sym}")
            output_path = output_dir / output_filename.name
            try:
                if _io.imwrite(str(output_path), arr):
                    saved_files.append(output_path)
                else:
                    warn(f"Échec de sauvegarde de la symétrie '{sym}' pour {output_path.name}. "
                         "Retour False depuis `.imwrite`")
            except Exception as e_save:
                warn(f"Erreur [{input_path.name} - Symétrie '{sym}']: Échec de sauvegarde pour {output_filename} : "
                     f"{e_save}.")
        return saved_files

    return batch_run(arg_tuples, threads, load, compute, save)


generate_symmetries.batch = _symmetries_batch
