"""Host-side image codecs with the semantics the reference relies on.

The reference reads/writes files with ``cv2.imread``/``cv2.imwrite`` (BGR
order; ``IMREAD_COLOR`` drops alpha, ``IMREAD_UNCHANGED`` keeps it) and with
Pillow (RGB order).  OpenCV is not installed in this image, so the cv2-style
helpers below are implemented on Pillow's codecs with the same channel
conventions.  PNG is lossless, so pixel parity holds; JPEG payloads may differ
in bytes from libjpeg-turbo as used by OpenCV (quality 95 is OpenCV's default).
Codec work is host CPU work and sits outside the device hot path.
"""
from __future__ import annotations

from pathlib import Path
from typing import Optional

import numpy as np
from PIL import Image, ImageOps

IMREAD_UNCHANGED = -1
IMREAD_GRAYSCALE = 0
IMREAD_COLOR = 1

# ultralytics.data.utils.IMG_FORMATS / VID_FORMATS (ultralytics 8.x lists),
# used by symmetry.py:92 and video.py:31 for extension checks.
IMG_FORMATS = {"bmp", "dng", "jpeg", "jpg", "mpo", "png", "tif", "tiff", "webp", "pfm", "heic"}
VID_FORMATS = {"asf", "avi", "gif", "m4v", "mkv", "mov", "mp4", "mpeg", "mpg", "ts", "wmv", "webm"}


def imread(path, flags: int = IMREAD_COLOR) -> Optional[np.ndarray]:
    """cv2.imread: None when the file is missing or not decodable.

    Like OpenCV, IMREAD_COLOR and IMREAD_GRAYSCALE apply the EXIF orientation
    tag (camera JPEGs come out upright, so crop_square's YOLO boxes land on
    the right pixels) and IMREAD_UNCHANGED does not.  IMREAD_UNCHANGED keeps
    16-bit single-channel images as uint16 (and 32-bit float ones as
    float32), as cv2 does; other deep modes are refused (None) — among them
    16-bit colour PNGs, which Pillow would silently decode to 8 bits where
    cv2.IMREAD_UNCHANGED keeps 16 (their raw mode is 'RGB;16B' /
    'RGBA;16B').  IMREAD_COLOR / IMREAD_GRAYSCALE reduce them to 8 bits (the
    high byte), as cv2 does."""
    try:
        with Image.open(str(path)) as im:
            if flags == IMREAD_UNCHANGED and not str(im.mode).startswith("I;16") and any(
                    str(t[3][0] if isinstance(t[3], tuple) else t[3]).endswith(";16B")
                    for t in getattr(im, "tile", []) or []):
                return None
            im.load()
            mode = im.mode
            if flags == IMREAD_UNCHANGED:
                if mode in ("RGBA", "LA", "PA") or (mode == "P" and "transparency" in im.info):
                    arr = np.asarray(im.convert("RGBA"))
                    return arr[..., [2, 1, 0, 3]].copy()
                if mode.startswith("I;16"):
                    return np.asarray(im).astype(np.uint16)
                if mode == "I":
                    arr = np.asarray(im)
                    if arr.size and (arr.min() < 0 or arr.max() > 65535):
                        return None
                    return arr.astype(np.uint16)
                if mode == "F":
                    return np.asarray(im).astype(np.float32)
                if mode in ("L", "1"):
                    return np.asarray(im.convert("L")).copy()
                arr = np.asarray(im.convert("RGB"))
                return arr[..., ::-1].copy()
            im = ImageOps.exif_transpose(im)
            if flags == IMREAD_GRAYSCALE:
                return np.asarray(im.convert("L")).copy()
            arr = np.asarray(im.convert("RGB"))
            return arr[..., ::-1].copy()
    except (FileNotFoundError, OSError, ValueError):
        return None


def imwrite(path, img: np.ndarray) -> bool:
    """cv2.imwrite: BGR(A)/gray array → file chosen by extension."""
    path = str(path)
    ext = Path(path).suffix.lower()
    try:
        if img.dtype == np.uint16 and img.ndim == 2:
            im = Image.fromarray(img)            # 16-bit grayscale PNG/TIFF, as cv2 writes it
        elif img.dtype != np.uint8:
            return False
        elif img.ndim == 2:
            im = Image.fromarray(img, "L")
        elif img.shape[2] == 4:
            im = Image.fromarray(np.ascontiguousarray(img[..., [2, 1, 0, 3]]), "RGBA")
        else:
            im = Image.fromarray(np.ascontiguousarray(img[..., ::-1]), "RGB")
        if ext in (".jpg", ".jpeg"):
            if im.mode == "RGBA":
                im = im.convert("RGB")
            im.save(path, quality=95)
        elif ext == ".png":
            im.save(path, compress_level=1)
        else:
            im.save(path)
        return True
    except (OSError, ValueError, KeyError):
        return False
