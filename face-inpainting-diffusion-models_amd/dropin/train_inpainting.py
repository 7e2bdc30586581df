"""Drop-in for code/train_inpainting.py's `create_model_and_diffusion` (lines 199-262):
9-channel UNet on libifd, quadratic schedule, T=1000."""
import _path  # noqa: F401
from ifd.factory import create_model_and_diffusion as _factory


def create_model_and_diffusion(checkpoint_path, device, img_size=256):
    return _factory(checkpoint_path, device, img_size, steps=1000, noise_schedule="quadratic")
