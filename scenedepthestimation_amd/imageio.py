"""Image I/O for the entry points (the reference uses OpenCV, absent here).

``imread_gray`` reproduces ``cv2.imread(path, cv2.IMREAD_GRAYSCALE)`` for 8-bit
images: single-channel data is returned as is; colour data is converted with
OpenCV's fixed-point BT.601 weights ``(R*4899 + G*9617 + B*1868 + 8192) >> 14``
(match_single.py:34-38).  JPEGs take OpenCV's own route for a grayscale read
(match.py:48-52 reads .jpg pairs): the decoder is asked for grayscale output,
so libjpeg emits the luma plane of a YCbCr JPEG directly (Pillow: ``draft("L")``
before ``load()``) instead of decoding colour and converting it -- the two differ
in the last bit wherever chroma upsampling and rounding meet.  Pillow bundles
libjpeg(-turbo) like OpenCV; an OpenCV build with another IDCT could still
differ (cv2 is absent here: parity unpinned for JPEG beyond the luma route).
``imwrite`` writes 8-bit grayscale PNGs like ``cv2.imwrite(..., uint8 array)``
(match_single.py:55, match.py:90).
"""
from __future__ import annotations

import os

import numpy as np


def imread_gray(path: str):
    """Grayscale u8 [H,W], or None when the file cannot be read (cv2.imread's behaviour)."""
    from PIL import Image
    if not os.path.exists(path):
        return None
    try:
        im = Image.open(path)
        if im.format == "JPEG" and im.mode in ("RGB", "YCbCr"):
            im.draft("L", im.size)          # libjpeg grayscale output: the luma plane, as cv2 reads it
        im.load()
    except Exception:
        return None
    if im.mode == "L":
        return np.asarray(im, dtype=np.uint8).copy()
    if im.mode == "LA":
        return np.asarray(im, dtype=np.uint8)[..., 0].copy()
    if im.mode in ("I;16", "I;16B", "I"):
        a = np.asarray(im).astype(np.uint32)
        return (a >> 8).astype(np.uint8) if a.max() > 255 else a.astype(np.uint8)
    rgb = np.asarray(im.convert("RGB"), dtype=np.uint32)
    r, g, b = rgb[..., 0], rgb[..., 1], rgb[..., 2]
    return ((r * 4899 + g * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8)


def imwrite(path: str, img_u8) -> bool:
    from PIL import Image
    a = np.asarray(img_u8)
    if a.dtype != np.uint8:
        raise TypeError("imwrite expects a uint8 image")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    Image.fromarray(a, mode="L").save(path)
    return True
