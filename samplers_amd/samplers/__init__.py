from .base import PosteriorSampler
from .dps import DPSSampler, FusedDPSStep, KernelTimer
from .pgdm import PGDMSampler
from .psld import FusedPSLDStep, PSLDSampler
from .resample import ReSampleSampler

__all__ = ["PosteriorSampler", "DPSSampler", "PSLDSampler", "PGDMSampler", "ReSampleSampler",
           "FusedDPSStep", "FusedPSLDStep", "KernelTimer"]
