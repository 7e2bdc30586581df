"""Output conversion and mask convention on the HIP library, bit-exact against the reference's torch
arithmetic: toU8 (code/test_inp_ddim_50.py:33-41) and OrderedMaskDataset's mask rule
(code/data/dataset.py:278-289: ToTensor's gray/255, then (m < 0.5).float()). Edge cases: values at
and beyond +-1, the 127/128 gray boundary, empty batches, ragged sizes."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def ref_to_u8(sample):
    # code/test_inp_ddim_50.py:37-40
    s = ((sample + 1) * 127.5).clamp(0, 255).to(torch.uint8)
    return s.permute(0, 2, 3, 1).contiguous().numpy()


@pytest.mark.parametrize("shape", [(1, 3, 256, 256), (3, 3, 17, 29), (2, 1, 5, 7), (16, 3, 64, 64)])
def test_to_u8_bitexact(shape):
    from ifd.data import toU8
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.rand(shape, generator=g) * 2.4 - 1.2  # includes out-of-range values on both sides
    flat = x.view(-1)
    edges = torch.tensor([-1.0, 1.0, 0.0, -1.5, 1.5, 1 / 127.5 - 1, 0.999999, -0.999999])
    flat[: edges.numel()] = edges[: flat.numel()]
    got = toU8(x.to(DEV))
    want = ref_to_u8(x)
    assert got.dtype == np.uint8 and got.shape == want.shape
    assert np.array_equal(got, want)


@pytest.mark.parametrize("dtype", [torch.float16, torch.float64, torch.float32])
def test_to_u8_cpu_and_other_dtypes(dtype):
    """The reference's toU8 takes any device / float dtype; ours moves the tensor to the GPU as fp32
    (the conversion runs in fp32, so the expectation is the reference expression on x.float())."""
    from ifd.data import toU8
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(2, 3, 9, 11, generator=g) * 2.2 - 1.1).to(dtype)
    assert np.array_equal(toU8(x, device=DEV), ref_to_u8(x.float()))


def test_to_u8_empty_and_none():
    from ifd.data import toU8
    assert toU8(None) is None
    out = toU8(torch.zeros(0, 3, 8, 8, device=DEV))
    assert out.shape == (0, 8, 8, 3)


@pytest.mark.parametrize("shape", [(1, 1, 256, 256), (4, 1, 33, 31), (0, 1, 4, 4)])
def test_mask_from_gray_bitexact(shape):
    from ifd.data import mask_from_gray
    g = torch.Generator().manual_seed(3)
    gray = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8)
    if gray.numel() >= 256:
        gray.view(-1)[:256] = torch.arange(256, dtype=torch.uint8)  # every gray level incl. 127/128
    want = ((gray.float() / 255) < 0.5).float()  # ToTensor (div 255 in fp32), dataset.py:286
    got = mask_from_gray(gray.to(DEV)).cpu()
    assert torch.equal(got, want)
    if gray.numel() >= 256:
        assert got.view(-1)[127] == 1 and got.view(-1)[128] == 0


def test_data_rejects_cpu_tensors():
    from ifd.data import mask_from_gray, to_u8_device
    with pytest.raises(RuntimeError):
        to_u8_device(torch.zeros(1, 3, 4, 4))
    with pytest.raises(RuntimeError):
        mask_from_gray(torch.zeros(1, 1, 4, 4, dtype=torch.uint8))


# ---- input side (code/data/dataset.py:231-240, 273-286), against Pillow / the oracle ----------

@pytest.mark.parametrize("hw,out,c", [((1024, 1024), (256, 256), 1), ((300, 200), (256, 256), 1),
                                      ((64, 64), (256, 256), 1), ((97, 131), (64, 40), 3),
                                      ((512, 384), (256, 256), 3), ((256, 256), (256, 256), 3),
                                      ((31, 700), (256, 256), 3), ((256, 300), (256, 256), 1)])
def test_resize_u8_matches_pillow(hw, out, c):
    from PIL import Image
    from ifd.data import resize_u8
    rng = np.random.default_rng(sum(hw) * 7 + c)
    imgs = rng.integers(0, 256, size=(2,) + hw + ((c,) if c == 3 else ()), dtype=np.uint8)
    mode = "RGB" if c == 3 else "L"
    ref = np.stack([np.asarray(Image.fromarray(a, mode).resize((out[1], out[0]), Image.BILINEAR)) for a in imgs])
    got = resize_u8(torch.from_numpy(imgs).to(DEV), out[0], out[1]).cpu().numpy()
    assert got.shape == ref.shape and np.array_equal(got, ref)


def test_images_to_float_and_inpaint_batch():
    from oracle import ref_data
    from ifd.data import OrderedMaskBank, images_to_float
    rng = np.random.default_rng(5)
    u8 = rng.integers(0, 256, size=(5, 64, 64, 3), dtype=np.uint8)
    x = images_to_float(torch.from_numpy(u8).to(DEV))
    ref = np.stack([ref_data.to_tensor_normalize(a) for a in u8])
    assert np.array_equal(x.cpu().numpy(), ref)
    raw = [np.where(rng.random((h, w)) > 0.5, 255, 0).astype(np.uint8) for h, w in ((80, 80), (64, 64), (100, 37))]
    bank = OrderedMaskBank(raw, img_size=64, device=DEV)
    idx = [0, 1, 2, 3, 7]
    b = bank.batch(x, idx)
    for j, i in enumerate(idx):
        g = ref_data.resize_u8(raw[ref_data.ordered_mask_index(i, 3)], 64, 64)
        m = ref_data.mask_rule(g)
        assert np.array_equal(b["mask"][j, 0].cpu().numpy(), m)
        assert np.array_equal(b["masked_image"][j].cpu().numpy(), ref[j] * (1 - m)[None])
    assert b["mask_idx"].tolist() == [0, 1, 2, 0, 1]
