"""CPU: pin the Pillow restatement (oracle/pil_restate.py) and the product's
host-side tables (ssip.augment) against Pillow itself, bit-exactly."""
import numpy as np
import pytest
from PIL import Image

from oracle import pil_restate


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("src,dst", [((512, 512), (224, 224)), ((512, 512), (256, 256)), ((300, 200), (224, 224)),
                                     ((224, 224), (224, 224)), ((100, 120), (224, 224))])
def test_resize_matches_pillow(src, dst):
    a = _img(src[0], src[1], sum(src))
    ref = np.asarray(Image.fromarray(a).resize((dst[1], dst[0]), Image.BILINEAR))
    assert np.array_equal(pil_restate.resize_bilinear(a, dst[1], dst[0]), ref)


@pytest.mark.parametrize("angle", [-10.0, -3.7, 0.25, 7.5, 10.0, 29.9, -30.0])
def test_rotate_matches_pillow(angle):
    a = _img(224, 224, 3)
    ref = np.asarray(Image.fromarray(a).rotate(angle, Image.NEAREST, expand=False, fillcolor=(0, 0, 0)))
    assert np.array_equal(pil_restate.rotate_nearest(a, angle), ref)


def test_product_tables_match_oracle():
    from ssip.augment import resize_tables, rotate_fixed_point

    for n_in, n_out in [(512, 224), (512, 256), (224, 224), (300, 224), (100, 224)]:
        b1, c1, k1 = resize_tables(n_in, n_out)
        b2, c2, k2 = pil_restate.resample_coeffs(n_in, n_out)
        assert k1 == k2 and np.array_equal(b1, b2) and np.array_equal(c1, c2)
    for ang in (-10.0, 3.3, 9.99):
        assert rotate_fixed_point(ang, 224, 224) == pil_restate.rotate_params(ang, 224, 224)
