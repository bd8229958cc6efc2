"""ε-network plugin API (mirrors ``/root/reference/samplers/networks/base.py:13-117``).

Indexing contract (identical to the reference):

* ``alphas_cumprod`` is padded: index 0 -> 1.0, index k -> alpha_bar_k, clipped
  to [1e-6, 1] (``base.py:24-25``);
* ``timesteps`` is an **ascending** buffer of indices;
* ``predict_x0(x, t) = (x - sqrt(1 - acp[t]) * forward(x, t)) / sqrt(acp[t])``.

Addition for the MI355X path: ``set_sampling_parameters`` also keeps a host
copy of the timesteps (``timesteps_host``) and of ``alphas_cumprod``
(``alphas_cumprod_host``) so samplers never read a device scalar inside the
loop (the reference's ``int(timesteps[i])`` costs two device->host syncs per
step, ``dps.py:92-93``).
"""

from __future__ import annotations

import dataclasses
from abc import ABC, abstractmethod
from typing import Generic, TypeVar

import numpy as np
import torch
from torch import Tensor

from samplers_amd.dtypes import Shape

C = TypeVar("C")


class EpsilonNetwork(torch.nn.Module, ABC, Generic[C]):
    """Variance-preserving diffusion prior wrapper."""

    def __init__(self, alphas_cumprod: Tensor):
        super().__init__()
        alphas_cumprod = alphas_cumprod.clip(1e-6, 1)
        self.register_buffer("alphas_cumprod", alphas_cumprod)
        self._acp_host: np.ndarray | None = None
        self._batch_size = None
        self._num_sampling_steps = None
        self._num_reconstructions = None
        self._ts_host: list[int] | None = None
        self._ts_src = None

    @abstractmethod
    def forward(self, x: Tensor, t: Tensor | int): ...

    def predict_noise(self, x: Tensor, t: Tensor | int):
        return self.forward(x, t)

    def predict_x0(self, x: Tensor, t: Tensor | int):
        acp_t = self.alphas_cumprod[t]
        return (x - (1 - acp_t) ** 0.5 * self.forward(x, t)) / (acp_t**0.5)

    def score(self, x: Tensor, t: Tensor):
        acp_t = self.alphas_cumprod[t]
        return -self.forward(x, t) / ((1 - acp_t) ** 0.5)

    @property
    def alphas_cumprod_host(self) -> np.ndarray:
        """fp32 host copy of ``alphas_cumprod`` (same values the device buffer holds)."""
        buf = self.alphas_cumprod
        if self._acp_host is None or getattr(self, "_acp_src", None) is not buf:
            self._acp_host = buf.detach().float().cpu().numpy().copy()
            self._acp_src = buf
        return self._acp_host

    def _set_timesteps_buffer(self, timesteps: Tensor) -> None:
        timesteps = timesteps.to(self.alphas_cumprod.device)
        self.register_buffer(name="timesteps", tensor=timesteps, persistent=True)
        self._ts_host = [int(t) for t in timesteps.cpu().tolist()]
        self._ts_src = timesteps

    @property
    def timesteps_host(self) -> list[int] | None:
        """Host copy of the ``timesteps`` buffer (``None`` before it exists).

        Subclasses written against the reference ABC register ``timesteps`` themselves in
        ``set_sampling_parameters`` (``/root/reference/samplers/networks/diffusers/ddpm.py:58``);
        the copy is then taken here, once per registered buffer (one device read per
        sampler call, none per step)."""
        buf = self._buffers.get("timesteps")
        if buf is None:
            return None
        if self._ts_src is not buf or self._ts_host is None:
            self._ts_host = [int(t) for t in buf.detach().cpu().tolist()]
            self._ts_src = buf
        return self._ts_host

    @property
    def device(self) -> torch.device:
        return self.alphas_cumprod.device

    @property
    def dtype(self) -> torch.dtype:
        return self.alphas_cumprod.dtype

    @classmethod
    @abstractmethod
    def from_pretrained(cls, *args, **kwargs): ...

    @abstractmethod
    def set_sampling_parameters(self, num_sampling_steps: int, batch_size: int = 1,
                                num_reconstructions: int = 1): ...

    @property
    def are_sampling_parameters_initialized(self) -> bool:
        return self._batch_size is not None

    def clear_sampling_parameters(self):
        self._batch_size = None
        self._num_sampling_steps = None
        self._num_reconstructions = None

    def set_condition(self, condition: C | None) -> None: ...

    @property
    @abstractmethod
    def is_condition_initialized(self) -> bool: ...

    def clear_condition(self): ...


class LatentEpsilonNetwork(EpsilonNetwork[C], ABC, Generic[C]):
    """Latent prior with a VAE: ``encode`` / ``decode`` (``base.py:88-111``)."""

    @abstractmethod
    def get_latent_shape(self, x_shape: Shape) -> Shape: ...

    def decode(self, z: Tensor, differentiable: bool = False):
        if not differentiable:
            with torch.no_grad():
                out = self._decode(z=z, differentiable=False)
            return out.detach()
        return self._decode(z=z, differentiable=True)

    @abstractmethod
    def _decode(self, z: Tensor, *, differentiable: bool = False): ...

    def encode(self, x: Tensor, differentiable: bool = False):
        if not differentiable:
            with torch.no_grad():
                out = self._encode(x=x, differentiable=False)
            return out.detach()
        return self._encode(x=x, differentiable=True)

    @abstractmethod
    def _encode(self, x: Tensor, *, differentiable: bool = False): ...


def host_timesteps(net) -> list[int]:
    """Ascending timestep indices of ``net`` on the host: ``timesteps_host`` when the network
    derives from this package's ABC, else read once from its ``timesteps`` buffer (a network
    written against the reference ABC, ``networks/base.py:13-85``, duck-typed)."""
    ts = getattr(net, "timesteps_host", None)
    if ts is None:
        buf = getattr(net, "timesteps", None)
        if buf is None:
            raise RuntimeError("Call `set_sampling_parameters()` before sampling.")
        ts = [int(t) for t in torch.as_tensor(buf).detach().cpu().tolist()]
    return list(ts)


def host_alphas_cumprod(net) -> np.ndarray:
    """fp32 host copy of ``net.alphas_cumprod`` (see ``host_timesteps``)."""
    acp = getattr(net, "alphas_cumprod_host", None)
    if acp is None:
        acp = net.alphas_cumprod.detach().float().cpu().numpy().copy()
    return acp


@dataclasses.dataclass(slots=True)
class NoCondition:
    """Placeholder type meaning "this diffusion model does NOT use any conditioning"."""
