"""ctypes binding of the gfx950 C-ABI library ``libipp.so`` (include/ipp.h).

The library is built in-tree (``make`` / ``__graft_entry__.build()``).  There
is NO CPU fallback: if the library or a GPU is missing, the device ops raise
``NativeUnavailable`` loudly instead of computing anything elsewhere.

NumPy structured dtypes below mirror the C structs field for field (offsets
are checked against the C compiler in tests/test_abi.py).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

LIB_PATH = Path(os.environ.get("IPP_LIB_PATH", str(Path(__file__).resolve().parent / "libipp.so")))
# A/B runs of an experiment build of an older tree (tools/ab.sh, gpu_ab.sh)
# may predate an entry point; only they opt in to skipping (and logging) the
# missing names.  IPP_LIB_PATH alone still requires every ipp.h entry point.
_EXPERIMENT = os.environ.get("IPP_AB_EXPERIMENT") == "1"

IPP_OK = 0
IPP_E_ARG = -1
IPP_E_LAUNCH = -2
IPP_E_RANGE = -3
IPP_MAX_HSV_RANGES = 16
IPP_TAPS_MFMA = 1
IPP_RS_PREMULTIPLY = 1
IPP_RS_UNPREMULTIPLY = 2


class NativeUnavailable(RuntimeError):
    """The HIP C-ABI library could not be loaded (never silently bypassed)."""


class NativeError(RuntimeError):
    pass


_I4 = np.int32
_I8 = np.int64

GATHER_DESC = np.dtype([
    ("src_off", _I8), ("dst_off", _I8), ("src_pitch", _I4), ("src_cn", _I4),
    ("src_w", _I4), ("src_h", _I4), ("in_x0", _I4), ("in_y0", _I4), ("in_w", _I4), ("in_h", _I4),
    ("a0", _I4), ("a1", _I4), ("a2", _I4), ("a3", _I4), ("a4", _I4), ("a5", _I4),
    ("out_w", _I4), ("out_h", _I4), ("off_x", _I4), ("off_y", _I4), ("flip", _I4), ("dst_pitch", _I4),
    ("base_off", _I8), ("lim", np.uint32), ("b", _I4, (6,)), ("prepared", _I4),
], align=True)

AFFINE_DESC = np.dtype([
    ("src_off", _I8), ("dst_off", _I8), ("src_pitch", _I4), ("src_cn", _I4),
    ("in_x0", _I4), ("in_y0", _I4), ("in_w", _I4), ("in_h", _I4),
    ("out_w", _I4), ("out_h", _I4), ("dst_pitch", _I4), ("flip", _I4), ("m", np.float64, (6,)),
], align=True)

IPP_ENH_BLUR = 1
IPP_ENH_LUT = 2
ENHANCE_DESC = np.dtype([
    ("src_off", _I8), ("dst_off", _I8), ("w", _I4), ("h", _I4), ("src_pitch", _I4), ("dst_pitch", _I4),
    ("f_brightness", np.float32), ("f_contrast", np.float32), ("f_color", np.float32), ("flags", _I4),
    ("box_r", _I4), ("box_ww", np.uint32), ("box_fw", np.uint32), ("pad_", _I4), ("lut_off", _I8),
], align=True)

COPY_DESC = np.dtype([
    ("src_off", _I8), ("dst_off", _I8), ("src_pitch", _I4), ("dst_pitch", _I4),
    ("x0", _I4), ("y0", _I4), ("w", _I4), ("h", _I4), ("cn", _I4), ("flip", _I4),
], align=True)

HSV_RANGE = np.dtype([("lo", _I4, (3,)), ("hi", _I4, (3,)), ("zone", _I4, (4,))], align=True)
HSV_PARAMS = np.dtype([("n_ranges", _I4), ("bgr", _I4), ("r", HSV_RANGE, (IPP_MAX_HSV_RANGES,))], align=True)

IMAGE_DESC = np.dtype([("off", _I8), ("w", _I4), ("h", _I4), ("pitch", _I4), ("cn", _I4)], align=True)

CCL_WORK = np.dtype([("mask_off", _I8), ("edge_off", _I8), ("p_off", _I8), ("a_off", _I8), ("ent_off", _I8), ("ent_cap", _I8),
                     ("tile_off", _I8), ("img_off", _I8)], align=True)

RESAMPLE_DESC = np.dtype([
    ("src_off", _I8), ("dst_off", _I8), ("src_pitch", _I4), ("dst_pitch", _I4),
    ("in_len", _I4), ("out_len", _I4), ("lines", _I4), ("line0", _I4), ("ksize", _I4), ("pad_", _I4),
    ("coef_off", _I8),
], align=True)

PASTE_DESC = np.dtype([
    ("bg_off", _I8), ("ov_off", _I8), ("dst_off", _I8),
    ("bg_w", _I4), ("bg_h", _I4), ("bg_pitch", _I4), ("dst_pitch", _I4),
    ("ov_w", _I4), ("ov_h", _I4), ("ov_pitch", _I4), ("x", _I4), ("y", _I4), ("pad_", _I4),
], align=True)

PIPE_DESC = np.dtype([("g", GATHER_DESC), ("h", RESAMPLE_DESC), ("v", RESAMPLE_DESC), ("p", PASTE_DESC)],
                     align=True)

PIPE_PLAN_CFG = np.dtype([
    ("src_h", _I4), ("src_w", _I4), ("src_pitch", _I4), ("crop_t", _I4), ("crop_b", _I4), ("crop_l", _I4),
    ("crop_r", _I4), ("bg_h", _I4), ("bg_w", _I4), ("n_bg", _I4), ("n_sym", _I4), ("sym_flip", _I4, (4,)),
    ("n_global", _I4), ("start", _I4), ("stop", _I4), ("given", _I4), ("n_threads", _I4),
    ("ring_cols", _I4), ("pad_", _I4), ("seed", np.uint64),
    ("angle_min", np.float64), ("angle_max", np.float64), ("scale_min", np.float64), ("scale_max", np.float64),
], align=True)

PIPE_ITEM = np.dtype([
    ("angle", np.float64), ("ratio", np.float64), ("sym", _I4), ("bg_index", _I4), ("x", _I4), ("y", _I4),
    ("rot_w", _I4), ("rot_h", _I4), ("cut_x", _I4), ("cut_y", _I4), ("cut_w", _I4), ("cut_h", _I4),
    ("ov_w", _I4), ("ov_h", _I4),
], align=True)

TAP_AXIS = np.dtype([
    ("in_size", _I4), ("out_size", _I4), ("identity", _I4), ("shift", _I4), ("phase", _I4), ("nkb", _I4),
    ("compact", _I4), ("n_tiles", _I4), ("coef_off", _I8),
], align=True)

# ipp_plan_pipe_batch totals[] slots (ipp.h IPP_PT_*)
IPP_PLAN_TOTALS = 16
IPP_PIPE_COPY_GROUP = 8   # items per background-copy group of ipp_pipe_hpass_bgcopy (ipp.h)
IPP_PIPE_MAX_OV_W = 992   # widest overlay of ipp_pipe_vblend_bands (ipp.h)
PT = dict(coef_words=0, tmp_bytes=1, max_out_w=2, max_rows=3, max_ov_w=4, max_ov_h=5, algo_h=6, algo_v=7,
          copy_bytes=8, max_tiles=9, err_item=10, err_code=11, copy_reads=12)

# (symbol, restype, argtypes) — every entry point declared in include/ipp.h.
_P = ctypes.c_void_p
_I = ctypes.c_int32
_L = ctypes.c_int64
_D = ctypes.c_double
SIGNATURES = {
    "ipp_rotate_flip_nearest": (_I, [_P, _P, _P, _I, _I, _I, _P]),
    "ipp_gather_prepare": (_I, [_P, _I]),
    "ipp_rotate_bilinear": (_I, [_P, _P, _P, _I, _I, _I, _P]),
    "ipp_copy_window": (_I, [_P, _P, _P, _I, _I, _I, _P]),
    "ipp_crop_to_bbox": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "ipp_hsv_mask": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P]),
    "ipp_lanczos_h": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "ipp_lanczos_v": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "ipp_paste_blend": (_I, [_P, _P, _P, _P, _I, _I, _I, _P]),
    "ipp_pipe_hpass_bgcopy": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _I, _P, _P, _P]),
    "ipp_pipe_vblend_bands": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "ipp_ccl_keep_largest": (_I, [_P, _P, _I, _I, _I, _P, _P, _L, _P, _P, _P, _P]),
    "ipp_ccl_scratch_layout": (_L, [_I, _I, _P]),
    "ipp_video_keep_largest": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _L, _P, _P, _P, _P, _P, _P]),
    "ipp_alpha_bbox": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "ipp_plan_lanczos": (_L, [_I, _D, _D, _I, _P, _L]),
    "ipp_plan_lanczos_ksize": (_I, [_D, _D, _I]),
    "ipp_plan_lanczos_batch": (_I, [_I, _P, _P, _P, _P, _L, _I]),
    "ipp_plan_opaque_bbox": (_I, [_I, _I, _P, _I, _I, _P]),
    "ipp_plan_mfma_size": (_L, [_I, _I, _I]),
    "ipp_plan_mfma_from_taps": (_I, [_I, _I, _I, _P, _I, _I, _P]),
    "ipp_plan_mfma_nk_bound": (_I, [_I, _I, _I]),
    "ipp_plan_pipe_axes": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _P, _I]),
    "ipp_stream_copy": (_I, [_P, _P, _L, _P]),
    "ipp_enhance_lsum": (_I, [_P, _P, _I, _L, _P, _P]),
    "ipp_enhance_color": (_I, [_P, _P, _P, _I, _L, _P, _P, _P]),
    "ipp_box_pass": (_I, [_P, _P, _P, _I, _L, _P, _I, _P, _I, _P]),
    "ipp_pipe_status": (_I, [_P, _P]),
    "ipp_plan_pipe_batch": (_I, [_P, _P, _P, _P, _P]),
    "ipp_pipe_taps_scratch_bytes": (_L, [_I]),
    "ipp_pipe_plan_taps": (_I, [_P, _I, _P, _P, _P, _P]),
    "ipp_pipe_plan_taps_cap": (_I, [_P, _I, _P, _P, _P, _L, _P]),
    "ipp_plan_mfma_tile": (_I, [_P, _I, _P, _P, _P, _L]),
    "ipp_plan_opaque_bbox_fast": (_I, [_I, _I, _P, _I, _I, _P]),
    "ipp_plan_py_hypot": (_D, [_D, _D]),
    "ipp_plan_rotation": (_I, [_I, _I, _D, _P]),
    "ipp_plan_py_random": (_I, [ctypes.c_uint64, _I, _P]),
    "ipp_version": (ctypes.c_char_p, []),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load libipp.so once; raise NativeUnavailable if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise NativeUnavailable(
            f"{LIB_PATH} not found — build it with `make` or __graft_entry__.build(); "
            "there is no CPU fallback for the hot path")
    try:
        lib = ctypes.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | getattr(os, "RTLD_LOCAL", 0))
    except OSError as e:  # pragma: no cover - environment dependent
        raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    skipped = []
    for name, (res, args) in SIGNATURES.items():
        if _EXPERIMENT and not hasattr(lib, name):
            skipped.append(name)
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if skipped:
        import sys
        print(f"_native: IPP_AB_EXPERIMENT: {LIB_PATH} lacks {', '.join(skipped)}", file=sys.stderr)
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != IPP_OK:
        raise NativeError(f"{what} failed with code {rc}")


def np_ptr(a: np.ndarray) -> int:
    return a.ctypes.data
