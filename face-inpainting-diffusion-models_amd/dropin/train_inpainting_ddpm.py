"""Drop-in for code/train_inpainting_ddpm.py's `create_model_and_diffusion` (lines 199-262):
9-channel UNet on libifd, linear schedule, T=500."""
import _path  # noqa: F401
from ifd.factory import create_model_and_diffusion as _factory


def create_model_and_diffusion(checkpoint_path, device, img_size=256):
    return _factory(checkpoint_path, device, img_size, steps=500, noise_schedule="linear")
