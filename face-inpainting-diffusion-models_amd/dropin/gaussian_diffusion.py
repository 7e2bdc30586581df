"""Drop-in for code/gaussian_diffusion.py."""
import _path  # noqa: F401
from ifd.diffusion import GaussianDiffusion, _extract_into_tensor  # noqa: F401
