"""``InverseProblem`` (mirrors ``/root/reference/samplers/inverse_problem.py:10-67``)."""

from __future__ import annotations

from dataclasses import dataclass

import torch

from samplers_amd.dtypes import RNG, Shape, Tensor
from samplers_amd.noise import NoiseModel
from samplers_amd.operators import Operator


@dataclass
class InverseProblem:
    operator: Operator
    observation: Tensor
    noise: NoiseModel

    def residual(self, x: Tensor) -> Tensor:
        return self.observation - self.operator(x)

    def log_likelihood(self, x: Tensor) -> Tensor:
        return self.noise.log_prob(self.residual(x))

    def score(self, x: Tensor) -> Tensor:
        return self.noise.score(self.residual(x)) * (-1)

    @property
    def batch_shape(self) -> Shape:
        return self.observation.shape[: -len(self.operator.y_shape)]

    @classmethod
    def from_observation(cls, obs: Tensor, *, operator: Operator, noise: NoiseModel):
        return cls(operator=operator, observation=obs, noise=noise)

    @classmethod
    def from_clean_data(cls, x_true: Tensor, *, operator: Operator, noise: NoiseModel,
                        rng: RNG = None) -> "InverseProblem":
        """Simulate ``y = A(x_true) + ε`` with ``ε ~ noise.sample`` (``inverse_problem.py:34-67``)."""
        with torch.no_grad():
            y_clean = operator(x_true)
            eps = noise.sample(shape=y_clean.shape, device=y_clean.device, dtype=y_clean.dtype,
                               generator=rng)
            y_obs = y_clean + eps
        return cls(operator=operator, observation=y_obs, noise=noise)
