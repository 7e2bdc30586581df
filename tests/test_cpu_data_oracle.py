"""The data-format oracle (oracle/ref_data.py) against Pillow itself: BILINEAR resize of 8-bit
grayscale and RGB images, down- and up-scaling, odd sizes — bit-exact."""
import numpy as np
import pytest
from PIL import Image

from oracle import ref_data


@pytest.mark.parametrize("hw,out,mode", [((64, 64), (256, 256), "L"), ((300, 200), (256, 256), "L"),
                                         ((1024, 1024), (256, 256), "L"), ((97, 131), (64, 40), "RGB"),
                                         ((512, 384), (256, 256), "RGB"), ((256, 256), (256, 256), "L"),
                                         ((31, 700), (256, 256), "RGB")])
def test_resize_matches_pillow(hw, out, mode):
    rng = np.random.default_rng(hash((hw, out, mode)) % 2**32)
    shape = hw + ((3,) if mode == "RGB" else ())
    a = rng.integers(0, 256, size=shape, dtype=np.uint8)
    if mode == "L":  # masks are mostly binary with soft edges
        a = np.where(a > 128, 255, 0).astype(np.uint8)
    ref = np.asarray(Image.fromarray(a, mode).resize((out[1], out[0]), Image.BILINEAR))
    got = ref_data.resize_u8(a, out[0], out[1])
    assert got.shape == ref.shape and np.array_equal(got, ref)


def test_mask_rule_and_cycling():
    g = np.arange(256, dtype=np.uint8).reshape(16, 16)
    m = ref_data.mask_rule(g)
    assert m[0, 0] == 1 and m.flatten()[127] == 1 and m.flatten()[128] == 0
    assert [ref_data.ordered_mask_index(i, 3) for i in range(7)] == [0, 1, 2, 0, 1, 2, 0]
