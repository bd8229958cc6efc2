"""torch-CPU restatement of ReSample — TEST INFRASTRUCTURE ONLY.

Follows ``/root/reference/samplers/samplers/resample.py:99-224`` and
``utils/resample_kernels.py:15-129`` (ε-form DDIM ``bridge_kernels.py:82-115``)
operation by operation, with prior, VAE, operator and the noise draws injected
(``draw(shape)`` returns the next standard normal tensor, in the reference's
draw order).
"""

from __future__ import annotations

from typing import Callable

import torch
from torch import Tensor


def ddim_step_eps(x: Tensor, eps_fn, acp: Tensor, t: int, t_prev: int, eta: float, draw):
    acp_t, acp_prev = acp[t], acp[t_prev]
    with torch.no_grad():
        e_t = eps_fn(x, t)
    view = (-1,) + (1,) * (x.ndim - 1)
    a_t = acp_t.to(x.dtype).view(view)
    a_prev = acp_prev.to(x.dtype).view(view)
    sqrt_oma = (1 - acp_t).sqrt().to(x.dtype).view(view)
    pred_x0 = (x - sqrt_oma * e_t) / a_t.sqrt()
    pseudo_x0 = (x - (1 - acp_t) * e_t) / a_t.sqrt()
    sigma_t = eta * ((1 - acp_prev) / (1 - acp_t) * (1 - acp_t / acp_prev)).clamp(min=0).sqrt()
    sigma = sigma_t.to(x.dtype).view(view)
    dir_xt = (1 - acp_prev - sigma_t**2).clamp(min=0).sqrt() * e_t
    noise = sigma * draw(tuple(x.shape)).to(x.dtype)
    return a_prev.sqrt() * pred_x0 + dir_xt + noise, pred_x0, pseudo_x0


def resample_reference(eps_fn, alphas_cumprod: Tensor, timesteps: list[int],
                       apply_op: Callable[[Tensor], Tensor], decode, encode,
                       observation_rows: Tensor, draw, *, latent_shape: tuple, leading: int,
                       eps: float, sigma_scale: float = 40.0, max_iters: int = 2000,
                       eta: float = 1.0, inter_timesteps: int = 5, time_travel_interval: int = 10,
                       stage_splits: int = 3, decode_output: bool = True) -> Tensor:
    acp = alphas_cumprod
    dtype = observation_rows.dtype
    z_t = draw((leading, *latent_shape)).to(dtype).requires_grad_()
    total_steps = len(timesteps) - 1
    index_split = total_steps // stage_splits
    spatial = (leading,) + (1,) * len(latent_shape)

    def pixel_optimization(x_prime):
        loss_fn = torch.nn.MSELoss()
        opt = x_prime.detach().clone().requires_grad_()
        optimizer = torch.optim.AdamW([opt], lr=1e-2)
        for _ in range(max_iters):
            optimizer.zero_grad()
            loss = loss_fn(observation_rows, apply_op(opt))
            loss.backward()
            optimizer.step()
            if loss.item() < eps**2:
                break
        return opt.detach()

    def latent_optimization(z_init):
        if not z_init.requires_grad:
            z_init = z_init.requires_grad_()
        loss_fn = torch.nn.MSELoss()
        optimizer = torch.optim.AdamW([z_init], lr=5e-3)
        losses = []
        for itr in range(max_iters):
            optimizer.zero_grad()
            out = loss_fn(observation_rows, apply_op(decode(z_init)))
            out.backward()
            optimizer.step()
            cur = out.detach().item()
            if itr >= 200:
                losses.append(cur)
                if len(losses) > 1 and losses[0] < cur:
                    break
                if len(losses) > 1:
                    losses.pop(0)
            if cur < eps**2:
                break
        return z_init.detach()

    for idx in range(len(timesteps) - 1, 1, -1):
        t, tp = int(timesteps[idx]), int(timesteps[idx - 1])
        z_t = z_t.detach().requires_grad_()
        z_next, _z0, pseudo = ddim_step_eps(z_t, eps_fn, acp, t, tp, eta, draw)
        a_t = acp[t].to(dtype).expand(spatial)
        scale = a_t * 0.5
        diff = observation_rows - apply_op(decode(pseudo))
        norm = torch.linalg.norm(diff)
        g = torch.autograd.grad(outputs=norm, inputs=z_t)[0]
        z_t = z_next - g * scale
        if idx <= (total_steps - index_split) and idx > 0 and idx % time_travel_interval == 0:
            snapshot = z_t.detach().clone()
            for k in range(idx, max(idx - inter_timesteps, 1), -1):
                if k <= 1:
                    break
                z_t, _zk, pseudo = ddim_step_eps(z_t, eps_fn, acp, int(timesteps[k]),
                                                 int(timesteps[k - 1]), eta, draw)
            a_prev = acp[tp].to(dtype).expand(spatial)
            sigma = sigma_scale * (1 - a_prev) / (1 - a_t) * (1 - a_t / a_prev)
            if idx >= index_split:
                with torch.no_grad():
                    x_pixel = decode(pseudo.detach())
                x_opt = pixel_optimization(x_pixel)
                with torch.no_grad():
                    z_opt = encode(x_opt)
            else:
                z_opt = latent_optimization(pseudo.detach())
            noise = draw(tuple(z_opt.shape)).to(dtype)
            z_t = (sigma * a_prev.sqrt() * z_opt + (1 - a_prev) * snapshot) / (sigma + 1 - a_prev) \
                + noise * torch.sqrt(1 / (1 / sigma + 1 / (1 - a_prev)))
            z_t = z_t.requires_grad_()
    final = latent_optimization(z_t.detach())
    with torch.no_grad():
        return decode(final) if decode_output else final
