"""Oracle for the 5-stage pipe item (TEST INFRASTRUCTURE ONLY).

Restates, per item, what the reference's five chained steps compute on the
pixels (files between steps are lossless PNG except the crop step's JPG,
which the in-memory pipe skips): crop_from_border (recadrages.py:37-46) →
process_rotations (rotations.py:55, 96-109) → generate_symmetries
(symmetry.py:114-119) → process_images_with_color_masks (filtres_liste.py:84-134,
cv2.imread drops the alpha written by the previous steps) →
paste_overlay_onto_background (overlays.py:83-139).
"""
import numpy as np

from oracle import ops


def cut_out(src_rgb: np.ndarray, params, cfg) -> np.ndarray:
    """Stages 1-4: returns the RGBA cut-out M (Pillow channel order)."""
    crop = ops.crop_from_border(src_rgb, cfg.margins)
    rot = ops.rotate_and_crop(ops.to_rgba(crop), params.angle)
    fl = ops.flip(rot, params.sym)
    bgr = fl[..., [2, 1, 0]]                       # cv2.imread(IMREAD_COLOR) of the PNG
    alpha = ops.hsv_alpha_mask(bgr, cfg.hsv_ranges, cfg.zones, cfg.use_gimp_scale)
    return np.concatenate([fl[..., :3], alpha[..., None]], axis=-1)


def pipe_item(src_rgb: np.ndarray, bgs: np.ndarray, params, cfg) -> np.ndarray:
    m = cut_out(src_rgb, params, cfg)
    bg = bgs[params.bg_index]
    bh, bw = bg.shape[:2]
    nw, nh = ops.overlay_geometry(m.shape[1], m.shape[0], bw, bh, params.ratio)
    ov = ops.resize_lanczos_rgba(m, nw, nh)
    return ops.paste_rgba_onto_rgb(bg, ov, params.x, params.y)
