#!/usr/bin/env python3
"""Print the OpenCV RGB2HSV_b division tables embedded in csrc/ipp_hsv.h:
sdiv[i] = cvRound((255 << 12) / i), hdiv180[i] = cvRound((180 << 12) / (6 i));
cvRound = round-half-even (lrint)."""
import numpy as np

i = np.arange(256, dtype=np.float64)
with np.errstate(divide="ignore"):
    s = np.rint((255 << 12) / i)
    h = np.rint((180 << 12) / (6.0 * i))
s[0] = h[0] = 0
print("sdiv", [int(v) for v in s])
print("hdiv180", [int(v) for v in h])
