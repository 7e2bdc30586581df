"""Drop-in for code/unet.py: `DiffusionInpaintingModel` runs on libifd (UNetModel is its base)."""
import _path  # noqa: F401
from ifd.model import DiffusionInpaintingModel  # noqa: F401
from ifd.topology import UNetConfig  # noqa: F401
