"""Commit the reference's own test images as small fixtures (data only).

  tests/golden/frames.npz:
    euroc1, euroc2 : /root/reference/data2/color/{1,2}.png  (752x480 8-bit gray, EuRoC-shaped)
    rgb1_gray      : /root/reference/data/color/1.png (640x480 RGB) -> gray with
                     cv::cvtColor RGB2GRAY fixed point (B*1868 + G*9617 + R*4899 + 8192) >> 14
                     (the fixture defines the R/B assignment).
Runs only where /root/reference exists.
"""
import pathlib
import numpy as np
from PIL import Image

REF = pathlib.Path('/root/reference')
out = pathlib.Path(__file__).resolve().parent.parent / 'tests' / 'golden' / 'frames.npz'
e1 = np.array(Image.open(REF / 'data2/color/1.png'))
e2 = np.array(Image.open(REF / 'data2/color/2.png'))
rgb = np.array(Image.open(REF / 'data/color/1.png')).astype(np.int64)
R, G, B = rgb[..., 0], rgb[..., 1], rgb[..., 2]
gray = ((B * 1868 + G * 9617 + R * 4899 + 8192) >> 14).astype(np.uint8)
assert e1.dtype == np.uint8 and e1.shape == (480, 752) and gray.shape == (480, 640)
np.savez_compressed(out, euroc1=e1, euroc2=e2, rgb1_gray=gray)
print(out, out.stat().st_size)
