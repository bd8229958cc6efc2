from .base import NonlinearOperator, Operator
from .blur import GaussianBlurOperator
from .identity import IdentityOperator
from .inpainting import (
    CenterInpaintingOperator,
    CenterOutpaintingOperator,
    InpaintingOperator,
    RandomInpaintingOperator,
    SidePaintingOperator,
    get_mask_inpaint_center,
    get_mask_random,
    get_mask_side_painting,
)
from .linear import GeneralSVDOperator, LinearOperator, SVDOperator

__all__ = [
    "Operator",
    "NonlinearOperator",
    "IdentityOperator",
    "LinearOperator",
    "GeneralSVDOperator",
    "SVDOperator",
    "InpaintingOperator",
    "CenterInpaintingOperator",
    "CenterOutpaintingOperator",
    "SidePaintingOperator",
    "RandomInpaintingOperator",
    "GaussianBlurOperator",
    "get_mask_inpaint_center",
    "get_mask_side_painting",
    "get_mask_random",
]
