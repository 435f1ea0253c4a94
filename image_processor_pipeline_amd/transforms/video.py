"""frame_extraction — reference transforms/video.py:6-47 (the frame source of
the config-5 chain).

Same signature, checks and output layout: ValueError without a basename
(:12-13), ``<output_dirs[0]>/<video stem>/0-raw/`` created here (:16-19),
RuntimeError when the video cannot be opened (:25-26), ValueError for a
suffix outside ultralytics' VID_FORMATS (:30-32), frames written as
``{file_basename}-frame_{n:04d}.jpg`` from n = 1 (:36-43), returns the frame
directory.

Decoding: the reference uses ``cv2.VideoCapture`` (FFmpeg).  OpenCV, FFmpeg,
PyAV and rocDecode are absent from this image (rocDecode is also
absent on the MI355X box), so ``open_video`` takes, in order:
OpenCV when a user's environment has it (identical to the reference), then
Pillow for the animated formats it decodes (GIF among VID_FORMATS; also
multi-frame WebP/PNG/TIFF).  Anything else fails as cv2 would on a codec it
cannot open (RuntimeError).  Frames are BGR uint8, as cv2 returns them.

``iter_frame_batches`` feeds decoded frames to the device chain
(video_chain.VideoChain) in batches without the JPEG round trip.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, Iterator, List, Optional

import numpy as np
from PIL import Image

from .. import io as _io


def _cv2():
    try:
        import cv2  # noqa: F401
        return cv2
    except Exception:
        return None


def open_video(video_path: Path) -> Optional[Iterator[np.ndarray]]:
    """An iterator of BGR frames, or None when no available decoder opens the
    file (cv2.VideoCapture(...).isOpened() == False)."""
    cv2 = _cv2()
    if cv2 is not None:
        cap = cv2.VideoCapture(str(video_path))
        if not cap.isOpened():
            return None

        def gen_cv2():
            try:
                while True:
                    ok, frame = cap.read()
                    if not ok:
                        break
                    yield frame
            finally:
                cap.release()
        return gen_cv2()
    try:
        im = Image.open(str(video_path))
        im.load()
    except Exception:
        return None

    def gen_pil():
        try:
            n = getattr(im, "n_frames", 1)
            for k in range(n):
                im.seek(k)
                yield np.ascontiguousarray(np.asarray(im.convert("RGB"))[..., ::-1])
        finally:
            im.close()
    return gen_pil()


def frame_extraction(video_path: Path, output_dirs: List[Path], file_basename: str,
                     **options: Any) -> Optional[Path]:
    if not file_basename:
        raise ValueError("Aucun nom de fichier de base fournit pour les nom des frames.")
    video_path = Path(video_path)
    output_dir = Path(output_dirs[0]) / video_path.stem / "0-raw"
    output_dir.mkdir(parents=True, exist_ok=True)
    frames = open_video(video_path)
    if frames is None:
        raise RuntimeError("Erreur : Impossible d'ouvrir la vidéo")
    if video_path.suffix[1:].lower() not in _io.VID_FORMATS:
        raise ValueError(f"Fichier vidéo {video_path.suffix} non pris en charge."
                         f"Format autorisés : {_io.VID_FORMATS}")
    for n, frame in enumerate(frames, start=1):
        _io.imwrite(output_dir / f"{file_basename}-frame_{n:04d}.jpg", frame)
    return output_dir


def iter_frame_batches(video_path: Path, batch: int) -> Iterator[np.ndarray]:
    """Decoded BGR frames of one video, `batch` at a time, as (F, H, W, 3)
    arrays (the last batch may be shorter) — the host side of the config-5
    chain without writing JPEGs."""
    frames = open_video(Path(video_path))
    if frames is None:
        raise RuntimeError("Erreur : Impossible d'ouvrir la vidéo")
    buf: List[np.ndarray] = []
    for f in frames:
        buf.append(f)
        if len(buf) == batch:
            yield np.stack(buf)
            buf = []
    if buf:
        yield np.stack(buf)
