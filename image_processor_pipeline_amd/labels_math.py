"""YOLO box conversions used by the reference through ultralytics
(ultralytics.utils.ops.xywhn2xyxy / xyxy2xywhn, restated: ultralytics is not
installed here).  Call sites: crop_square.py:167, :217; overlays.py:146."""
import numpy as np


def xywhn2xyxy(x, w=640, h=640, padw=0, padh=0):
    x = np.asarray(x, dtype=np.float64)
    y = np.empty_like(x)
    y[..., 0] = w * (x[..., 0] - x[..., 2] / 2) + padw
    y[..., 1] = h * (x[..., 1] - x[..., 3] / 2) + padh
    y[..., 2] = w * (x[..., 0] + x[..., 2] / 2) + padw
    y[..., 3] = h * (x[..., 1] + x[..., 3] / 2) + padh
    return y


def xyxy2xywhn(x, w=640, h=640, clip=False, eps=0.0):
    x = np.asarray(x, dtype=np.float64)
    if clip:
        x = x.copy()
        x[..., [0, 2]] = x[..., [0, 2]].clip(0, w - eps)
        x[..., [1, 3]] = x[..., [1, 3]].clip(0, h - eps)
    y = np.empty_like(x)
    y[..., 0] = ((x[..., 0] + x[..., 2]) / 2) / w
    y[..., 1] = ((x[..., 1] + x[..., 3]) / 2) / h
    y[..., 2] = (x[..., 2] - x[..., 0]) / w
    y[..., 3] = (x[..., 3] - x[..., 1]) / h
    return y
