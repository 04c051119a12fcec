"""LBD gradient planes (binary_descriptor_custom.cpp:351-399): the streaming
blur + Sobel (octave 0) and pyrDown + Sobel (octave 1) kernels equal the
oracle's computeGaussianPyramid + Sobel int16 planes, including widths that
are not multiples of 4 (partial lanes) and image borders."""
import numpy as np
import pytest

import oracle_lib as ol
import plvi
from plvi import synth
from util import real_frames

pytestmark = pytest.mark.gpu


def _cases():
    fr = real_frames()
    big = np.concatenate([fr["euroc1"], fr["euroc1"][:, :40]], axis=1)  # 792 x 480
    return [("synth1", synth.frame(1)), ("rgb1_gray", fr["rgb1_gray"]), ("euroc1", fr["euroc1"]),
            ("crop642x482", np.ascontiguousarray(big[:482, 3:645])), ("step", synth.frame(9))]


@pytest.mark.parametrize("k", range(5))
def test_lbd_sobel_planes_match_oracle(plvi_lib, k):
    tag, img = _cases()[k]
    h, w = img.shape
    lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, w, h)
    lx(img)
    for lvl in range(2):
        gx, gy = lx.debug_sobel(lvl)
        ex, ey = ol.lbd_sobel(img, lvl)
        assert gx.shape == ex.shape, tag
        for name, a, b in (("dx", gx, ex), ("dy", gy, ey)):
            bad = np.argwhere(a != b)
            assert bad.size == 0, f"{tag} L{lvl} {name}: {len(bad)} differ, first {bad[:5].tolist()}"
