"""Drop-in for code/utils/schedules.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _path  # noqa: F401,E402
from ifd.schedules import betas_for_alpha_bar, create_gaussian_diffusion, get_named_beta_schedule  # noqa: F401,E402
