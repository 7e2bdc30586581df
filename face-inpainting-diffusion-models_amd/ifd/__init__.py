"""ifd — MI355X-native masked-inpainting diffusion sampler (host side).

The reverse-diffusion inpainting loop of Sayzal28/Face-Inpainting-Diffusion-Models
(code/gaussian_diffusion.py + the scripts' InpaintingSampler loops) driving its 9-channel UNet
(code/unet.py, code/nn.py), re-built on hand-written gfx950 HIP kernels behind a C ABI
(include/ifd.h, libifd.so). This package mirrors the reference's Python API for that path.
"""
from .topology import FULL, REDUCED, UNetConfig, layer_plan, state_dict_spec, gflop_per_image  # noqa: F401
from .schedules import create_gaussian_diffusion, get_named_beta_schedule, betas_for_alpha_bar  # noqa: F401
from .losses import LossType, ModelMeanType, ModelVarType  # noqa: F401


def __getattr__(name):
    # GPU-facing modules load lazily so that CPU-only tooling (manifest, topology) imports cheaply
    if name in ("DiffusionInpaintingModel", "UNetModelHIP"):
        from . import model
        return getattr(model, name)
    if name == "InpaintingSampler":
        from .sampler import InpaintingSampler
        return InpaintingSampler
    if name == "GaussianDiffusion":
        from .diffusion import GaussianDiffusion
        return GaussianDiffusion
    if name == "create_model_and_diffusion":
        from .factory import create_model_and_diffusion
        return create_model_and_diffusion
    raise AttributeError(name)
