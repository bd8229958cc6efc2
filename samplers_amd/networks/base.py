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


class Fp32Boundary:
    """A reduced-precision ε-network (bf16 / fp16) seen by the fp32 samplers.

    The reference allocates its samples in ``epsilon_net.dtype`` and runs the whole loop in
    it (``dps.py:83-87``, ``psld.py:102-106``; its scripts drive bf16 / fp16 priors,
    ``scripts/run_psld.py:14``, ``scripts/sd15.py:10``).  Here the guidance passes, the bridge
    update and the sample itself stay fp32: only the network's own calls run in its dtype —
    inputs are cast to it on the way in and outputs back to fp32 on the way out, both inside
    the autograd graph, so the input-VJP ``J^T v`` also flows through the network in its
    dtype.  Every other attribute is the wrapped network's; the samplers return their result
    in the network's dtype, as the reference's do.
    """

    def __init__(self, network) -> None:
        object.__setattr__(self, "_net", network)
        object.__setattr__(self, "_dt", network.dtype)

    def __getattr__(self, name):
        return getattr(self._net, name)

    def __setattr__(self, name, value):
        setattr(self._net, name, value)

    @property
    def dtype(self) -> torch.dtype:
        return torch.float32

    @property
    def wrapped(self):
        return self._net

    def forward(self, x: Tensor, t) -> Tensor:
        return self._net.forward(x.to(self._dt), t).to(torch.float32)

    __call__ = forward

    def predict_noise(self, x: Tensor, t) -> Tensor:
        return self.forward(x, t)

    def decode(self, z: Tensor, differentiable: bool = False) -> Tensor:
        return self._net.decode(z.to(self._dt), differentiable=differentiable).to(torch.float32)

    def encode(self, x: Tensor, differentiable: bool = False) -> Tensor:
        return self._net.encode(x.to(self._dt), differentiable=differentiable).to(torch.float32)


def fp32_view(network):
    """``network`` itself when it computes in fp32, else an ``Fp32Boundary`` around it (bf16 /
    fp16: the samples, guidance and bridge updates are fp32, wider than the network's own
    dtype).  A float64 network is refused at sampler entry: the reference runs its whole loop in
    ``epsilon_net.dtype`` (``dps.py:83-87``), and the fp32 hot path would silently return fp32
    precision in a float64 tensor.  Any other dtype is refused too (``TypeError``)."""
    dt = getattr(network, "dtype", torch.float32)
    if dt == torch.float32:
        return network
    if dt == torch.float64:
        raise TypeError("float64 ε-networks are not supported: the MI355X path samples in fp32 "
                        "(the reference would run the whole loop in float64); cast the network "
                        "with .to(torch.float32)")
    if dt not in (torch.bfloat16, torch.float16):
        raise TypeError(f"ε-network dtype {dt} is not a floating-point type the samplers accept "
                        "(float32, bfloat16, float16)")
    return Fp32Boundary(network)


def output_dtype(network) -> torch.dtype:
    """The dtype the samplers return in: the network's (``dps.py:83-87``)."""
    return getattr(network, "dtype", torch.float32)


@dataclasses.dataclass(slots=True)
class NoCondition:
    """Placeholder type meaning "this diffusion model does NOT use any conditioning"."""
