"""Drop-in for code/losses.py."""
import _path  # noqa: F401
from ifd.losses import (LossType, ModelMeanType, ModelVarType, approx_standard_normal_cdf,  # noqa: F401
                        discretized_gaussian_log_likelihood, mean_flat, normal_kl)
