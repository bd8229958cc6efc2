"""samplers_amd — MI355X-native diffusion posterior-sampling hot path.

Drop-in for the DPS/PSLD guided step of thomashirtz/samplers: the plugin API
(samplers, InverseProblem, operators, noise models, ε-networks) mirrors the
reference; the per-step arithmetic runs in hand-written HIP kernels
(libsamplers_hip.so, C ABI in include/samplers_hip.h).
"""

__version__ = "0.1.0"

# MIOpen's find-db seed (samplers_amd/runtime.py) is merged lazily, before the first
# convolution that falls back to MIOpen (none does in the priors' DPS / PSLD steps).
