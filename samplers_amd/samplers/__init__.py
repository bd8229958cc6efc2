from .base import PosteriorSampler
from .dps import DPSSampler, FusedDPSStep, KernelTimer

__all__ = ["PosteriorSampler", "DPSSampler", "FusedDPSStep", "KernelTimer"]
