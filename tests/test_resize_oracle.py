"""The resize oracle (PIL bilinear restatement, oracle/resize_ref.py) against Pillow itself."""
import numpy as np
import pytest
from PIL import Image

from oracle import resize_ref as R


@pytest.mark.parametrize('src,dst', [((1200, 1920), (512, 512)), ((1200, 1920), (240, 384)),
                                     ((1200, 1920), (240, 240)), ((37, 53), (64, 96)), ((100, 80), (100, 33))])
def test_pil_resize_bit_exact(src, dst):
    rng = np.random.default_rng(sum(src) + sum(dst))
    g = rng.integers(0, 256, src, dtype=np.uint8)
    img = np.repeat(g[..., None], 3, axis=2)                 # grayscale replicated to RGB (utils.py:215)
    img[..., 1] ^= rng.integers(0, 4, src, dtype=np.uint8)    # make channels differ a little
    want = np.asarray(Image.fromarray(img).resize((dst[1], dst[0]), Image.BILINEAR))
    got = R.pil_resize(img, dst[0], dst[1])
    np.testing.assert_array_equal(got, want)
