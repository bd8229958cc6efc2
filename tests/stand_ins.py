"""Deterministic stand-in ε-networks shared by the golden-vector generator
(which drives the REFERENCE samplers in the survey container) and the tests
(which drive this package on the GPU).

The real priors (diffusers checkpoints) are unavailable offline, so parity of
the hot path is pinned with priors whose Jacobian is either known in closed
form (``linear``: eps = c * x) or small enough to differentiate exactly on any
device (``conv``: a fixed-seed two-layer conv net).  The schedule is the DDPM
linear-beta schedule with diffusers' ``leading`` spacing, restated in
``samplers_amd.networks.ddpm.DDPMSchedule``.
"""

from __future__ import annotations

import math

import numpy as np
import torch
from torch import nn


def ddpm_alphas_cumprod(num_train_timesteps: int = 1000) -> torch.Tensor:
    betas = torch.linspace(1e-4, 0.02, num_train_timesteps, dtype=torch.float32)
    return torch.cumprod(1.0 - betas, dim=0)


def leading_timesteps_ascending(n: int, num_train_timesteps: int = 1000) -> torch.Tensor:
    ratio = num_train_timesteps // n
    ts = (np.arange(0, n) * ratio).round().astype(np.int64)
    return torch.from_numpy(ts)


class EpsCore(nn.Module):
    """eps(x, t) for the stand-in priors."""

    def __init__(self, kind: str, channels: int, coef: float = 0.1, seed: int = 1234) -> None:
        super().__init__()
        self.kind = kind
        self.coef = coef
        if kind == "conv":
            gen = torch.Generator().manual_seed(seed)
            hidden = 8
            self.w1 = nn.Parameter(torch.randn(hidden, channels, 3, 3, generator=gen) * 0.15,
                                   requires_grad=False)
            self.b1 = nn.Parameter(torch.randn(hidden, generator=gen) * 0.05, requires_grad=False)
            self.w2 = nn.Parameter(torch.randn(channels, hidden, 3, 3, generator=gen) * 0.15,
                                   requires_grad=False)
        elif kind != "linear":
            raise ValueError(kind)

    def forward(self, x: torch.Tensor, t) -> torch.Tensor:
        if self.kind == "linear":
            return self.coef * x
        tt = float(t) / 1000.0
        h = torch.tanh(nn.functional.conv2d(x, self.w1, self.b1, padding=1))
        return nn.functional.conv2d(h, self.w2, padding=1) * (1.0 + tt) + self.coef * x


class LatentCore(nn.Module):
    """Linear stand-in VAE: decode = nearest-upsample(f) of a 1x1 conv (4 -> C),
    encode = 1x1 conv (C -> 4) of avg_pool(f) (the posterior mean)."""

    def __init__(self, channels: int = 3, latent: int = 4, factor: int = 4, seed: int = 77) -> None:
        super().__init__()
        gen = torch.Generator().manual_seed(seed)
        self.factor, self.latent = factor, latent
        self.wd = nn.Parameter(torch.randn(channels, latent, 1, 1, generator=gen) * 0.5,
                               requires_grad=False)
        self.we = nn.Parameter(torch.randn(latent, channels, 1, 1, generator=gen) * 0.5,
                               requires_grad=False)

    def decode(self, z: torch.Tensor) -> torch.Tensor:
        x = nn.functional.conv2d(z, self.wd)
        return nn.functional.interpolate(x, scale_factor=float(self.factor), mode="nearest")

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        return nn.functional.conv2d(nn.functional.avg_pool2d(x, self.factor), self.we)

    def latent_shape(self, x_shape):
        c, h, w = x_shape
        return (self.latent, h // self.factor, w // self.factor)


def make_samplers_amd_latent_net(kind: str = "conv", coef: float = 0.1, device=None):
    """Latent stand-in implementing :class:`samplers_amd.networks.base.LatentEpsilonNetwork`."""
    from samplers_amd.networks.base import LatentEpsilonNetwork, NoCondition

    class StandInLatent(LatentEpsilonNetwork[NoCondition]):
        def __init__(self) -> None:
            acp = ddpm_alphas_cumprod()
            super().__init__(alphas_cumprod=torch.cat([acp.new_tensor([1.0]), acp]))
            self.core = EpsCore(kind, 4, coef)
            self.vae = LatentCore()

        def forward(self, x, t):
            return self.core(x, t)

        @classmethod
        def from_pretrained(cls, *a, **k):
            raise NotImplementedError

        def set_sampling_parameters(self, num_sampling_steps, batch_size=1, num_reconstructions=1):
            self._batch_size = batch_size
            self._num_sampling_steps = num_sampling_steps
            self._set_timesteps_buffer(leading_timesteps_ascending(num_sampling_steps))

        def get_latent_shape(self, x_shape):
            return self.vae.latent_shape(x_shape)

        def _decode(self, z, *, differentiable=False):
            return self.vae.decode(z)

        def _encode(self, x, *, differentiable=False):
            return self.vae.encode(x)

        @property
        def is_condition_initialized(self) -> bool:
            return True

    net = StandInLatent()
    return net.to(device) if device is not None else net


def make_samplers_amd_net(kind: str, channels: int, coef: float = 0.1, device=None):
    """Stand-in prior implementing :class:`samplers_amd.networks.base.EpsilonNetwork`."""
    from samplers_amd.networks.base import EpsilonNetwork, NoCondition

    class StandInNetwork(EpsilonNetwork[NoCondition]):
        def __init__(self) -> None:
            acp = ddpm_alphas_cumprod()
            super().__init__(alphas_cumprod=torch.cat([acp.new_tensor([1.0]), acp]))
            self.core = EpsCore(kind, channels, coef)

        def forward(self, x, t):
            if self._num_sampling_steps is None:
                raise RuntimeError("Call `set_sampling_parameters()` before sampling.")
            return self.core(x, t)

        @classmethod
        def from_pretrained(cls, *a, **k):
            raise NotImplementedError

        def set_sampling_parameters(self, num_sampling_steps, batch_size=1, num_reconstructions=1):
            self._batch_size = batch_size
            self._num_sampling_steps = num_sampling_steps
            self._num_reconstructions = num_reconstructions
            self._set_timesteps_buffer(leading_timesteps_ascending(num_sampling_steps))

        @property
        def is_condition_initialized(self) -> bool:
            return True

    net = StandInNetwork()
    return net.to(device) if device is not None else net


def fixture_x_true(batch: int, shape: tuple, seed: int = 0) -> torch.Tensor:
    gen = torch.Generator().manual_seed(seed)
    return torch.rand((batch, *shape), generator=gen) * 2 - 1


def fixture_mask(shape: tuple, kind: str, seed: int = 1) -> torch.Tensor:
    c, h, w = shape
    if kind == "random":
        gen = torch.Generator().manual_seed(seed)
        return (torch.rand(h, w, generator=gen) < 0.5).expand(c, h, w).contiguous()
    if kind == "center":
        m = torch.zeros(shape, dtype=torch.bool)
        m[..., int(h * 0.25):int(h * 0.75), int(w * 0.25):int(w * 0.75)] = True
        return m
    raise ValueError(kind)


def replay_noise(seed: int, flat_shape: tuple, num_steps: int):
    """The reference DPS RNG stream: randn(flat_shape), then one randn_like per step."""
    gen = torch.Generator().manual_seed(seed)
    init = torch.randn(flat_shape, generator=gen)
    steps = {}
    for i in range(num_steps - 1, 1, -1):
        steps[i] = torch.randn(flat_shape, generator=gen)
    return init, steps


def relative_error(a: torch.Tensor, b: torch.Tensor) -> float:
    a = a.double().reshape(-1)
    b = b.double().reshape(-1)
    return float((a - b).norm() / max(b.norm().item(), 1e-30))


def count(shape) -> int:
    return int(math.prod(shape))


# --- plugins written against the reference ABCs (no HIP descriptor, no grad_scale) -------

def make_reference_style_net(kind: str, channels: int, coef: float = 0.1, device=None,
                             latent: bool = False):
    """A network subclass written the way the reference's own adapters are
    (``/root/reference/samplers/networks/diffusers/ddpm.py:45-58``): it registers the
    ``timesteps`` buffer itself and knows nothing of ``timesteps_host``."""
    from samplers_amd.networks.base import EpsilonNetwork, LatentEpsilonNetwork

    base = LatentEpsilonNetwork if latent else EpsilonNetwork

    class RefStyle(base):
        def __init__(self):
            acp = ddpm_alphas_cumprod()
            super().__init__(alphas_cumprod=torch.cat([acp.new_tensor([1.0]), acp]))
            self.core = EpsCore(kind, 4 if latent else channels, coef)
            if latent:
                self.vae = LatentCore()

        def forward(self, x, t):
            return self.core(x, t)

        @classmethod
        def from_pretrained(cls, *a, **k):
            raise NotImplementedError

        def set_sampling_parameters(self, num_sampling_steps, batch_size=1, num_reconstructions=1):
            self._batch_size = batch_size
            self._num_sampling_steps = num_sampling_steps
            self.register_buffer("timesteps",
                                 leading_timesteps_ascending(num_sampling_steps).to(self.device))

        def get_latent_shape(self, x_shape):
            return self.vae.latent_shape(x_shape)

        def _decode(self, z, *, differentiable=False):
            return self.vae.decode(z)

        def _encode(self, x, *, differentiable=False):
            return self.vae.encode(x)

        @property
        def is_condition_initialized(self):
            return True

    net = RefStyle()
    return net.to(device) if device is not None else net


def torch_operator(shape, kept=None, device=None):
    """An ``Operator`` subclass in plain torch (no ``hip_descriptor``): identity, or the
    reference's flattened inpainting gather (``inpainting.py:49-53,132-187``)."""
    from samplers_amd.operators.base import Operator

    class TorchGather(Operator):
        def __init__(self):
            idx = None if kept is None else torch.as_tensor(kept).long()
            self.kept = idx  # plain attribute while Operator.__init__ infers y_shape
            Operator.__init__(self, shape)
            del self.__dict__["kept"]
            self.register_buffer("kept", idx)  # a buffer afterwards: moves with .to()

        def apply(self, x):
            lead = x.shape[: x.ndim - len(shape)]
            flat = x.reshape(*lead, -1)
            return x.clone() if self.kept is None else flat[..., self.kept]

        def apply_transpose(self, y):
            if self.kept is None:
                return y.clone()
            lead = y.shape[:-1]
            out = y.new_zeros(*lead, count(shape))
            out[..., self.kept] = y
            return out.reshape(*lead, *shape)

        def apply_pseudo_inverse(self, y):
            return self.apply_transpose(y)

    op = TorchGather()
    return op.to(device) if device is not None else op


def reference_style_gaussian(sigma: float):
    """A noise model defining only the reference ABC's abstract methods (``noise.py:13-79``)."""
    from samplers_amd.noise import NoiseModel

    class RefGauss(NoiseModel):
        def __init__(self):
            super().__init__()
            self.register_buffer("sigma", torch.tensor(float(sigma)))

        def log_prob(self, r):
            return -(r.square().sum(dim=tuple(range(1, r.ndim)))) / (2 * self.sigma.pow(2))

        def sample(self, shape, *, device=None, dtype=None, generator=None):
            return torch.randn(shape, generator=generator) * self.sigma

    return RefGauss()


def laplace_noise(scale: float):
    """A non-quadratic log-likelihood (smooth L1 / pseudo-Huber): no constant gradient
    factor, so the samplers must differentiate it by autograd."""
    from samplers_amd.noise import NoiseModel

    class PseudoHuber(NoiseModel):
        def __init__(self):
            super().__init__()
            self.register_buffer("scale", torch.tensor(float(scale)))

        def log_prob(self, r):
            return -(torch.sqrt(1 + (r / self.scale).square()) - 1).sum(dim=tuple(range(1, r.ndim)))

        def sample(self, shape, *, device=None, dtype=None, generator=None):
            return torch.zeros(shape)

    return PseudoHuber()
