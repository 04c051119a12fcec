"""Commit the reference's own test images as small fixtures (data only).

  tests/golden/frames.npz:
    euroc1..euroc5 : /root/reference/data2/color/{1..5}.png  (752x480 8-bit gray, EuRoC-shaped)
    rgb1_gray..rgb5_gray : /root/reference/data/color/{1..5}.png (640x480 RGB) -> gray with
                     cv::cvtColor RGB2GRAY fixed point (B*1868 + G*9617 + R*4899 + 8192) >> 14
                     (the fixture defines the R/B assignment).
Runs only where /root/reference exists.
"""
import pathlib
import numpy as np
from PIL import Image

REF = pathlib.Path('/root/reference')
out = pathlib.Path(__file__).resolve().parent.parent / 'tests' / 'golden' / 'frames.npz'
frames = {}
for i in range(1, 6):
    e = np.array(Image.open(REF / f'data2/color/{i}.png'))
    assert e.dtype == np.uint8 and e.shape == (480, 752)
    frames[f'euroc{i}'] = e
    rgb = np.array(Image.open(REF / f'data/color/{i}.png')).astype(np.int64)
    R, G, B = rgb[..., 0], rgb[..., 1], rgb[..., 2]
    gray = ((B * 1868 + G * 9617 + R * 4899 + 8192) >> 14).astype(np.uint8)
    assert gray.shape == (480, 640)
    frames[f'rgb{i}_gray'] = gray
np.savez_compressed(out, **frames)
print(out, out.stat().st_size)
