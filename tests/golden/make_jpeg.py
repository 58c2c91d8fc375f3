"""Writes tests/golden/ycbcr_4x2.jpg: a small colour (YCbCr, 4:2:0) JPEG for the grayscale-route test
(imageio.imread_gray vs cv2.imread(..., IMREAD_GRAYSCALE), match.py:48-52).  Deterministic content:
colour gradients plus a seeded texture, so the luma plane and an RGB -> gray conversion of the
decoded colours differ in many pixels.

    python tests/golden/make_jpeg.py
"""
import os

import numpy as np
from PIL import Image

H, W = 24, 40
y, x = np.mgrid[0:H, 0:W]
rng = np.random.default_rng(2014)
rgb = np.stack([(x * 6) % 256, (y * 10 + x * 3) % 256, 255 - (y * 7) % 256], -1).astype(np.int32)
rgb = np.clip(rgb + rng.integers(-30, 31, rgb.shape), 0, 255).astype(np.uint8)
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ycbcr_4x2.jpg")
Image.fromarray(rgb, "RGB").save(out, quality=80, subsampling=2)
print(out)
