"""hipGraph capture of the guided DPS/PGDM step.

At small batches (BASELINE configs[0]: B = 1) a DPS step is a few hundred short kernels —
the UNet forward, its input VJP and the two HIP passes — and host-side launch work, not
the GPU, sets the step time.  ``GraphedStepLoop`` captures one whole step into a hipGraph
(``torch.cuda.CUDAGraph``, which is hipGraph on ROCm) and replays it for every guided
iteration of ``dps.py:91-122``.  What changes between steps lives on the device:

* a schedule of ``sp_step_rec`` records (the step's fp32 scalars — computed on the host
  exactly as the by-value path computes them — its Philox step index and the prior's
  timestep), selected by a device cursor;
* the graph's first kernel writes the current timestep into the prior's timestep tensor,
  the two passes read their scalars from the schedule (``sp_dps_residual_sched`` /
  ``sp_dps_update_sched``), and the last kernel advances the cursor.

Replays run the same kernels on the same buffers as the eager loop, so the samples are
identical to ``FusedDPSStep``'s (tests/test_graph_gpu.py).  In-kernel Philox noise only
(``rng="philox"``, no ``noise_fn``), no micro-batching.
"""

from __future__ import annotations

import torch
from torch import Tensor

from samplers_amd import _hip


class GraphedStepLoop:
    """Replays one captured step of ``step`` (a ``FusedDPSStep``) over a fixed schedule."""

    def __init__(self, step, x: Tensor, schedule: list[tuple[int, int, int, int]], *, seed: int,
                 sample_offset: int = 0) -> None:
        if step.micro_batch and step.micro_batch < x.shape[0]:
            raise ValueError("graph capture runs the whole batch in one piece (no micro_batch)")
        if step.timer is not None:
            raise ValueError("graph capture and per-launch kernel timing are exclusive")
        self.step, self.x = step, x
        self.lib = step.lib
        self.seed, self.sample_offset = int(seed), int(sample_offset)
        dev = x.device
        recs = (_hip.SpStepRec * max(len(schedule), 1))()
        for r, (i, t, t_prev, s) in zip(recs, schedule):
            r.c = step.coefficients(t, t_prev, s)
            r.step, r.t = int(i), int(t)
        raw = torch.frombuffer(bytearray(bytes(recs)), dtype=torch.uint8)
        self.sched = raw.to(dev)
        self.n_steps = len(schedule)
        self.cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self.t = torch.zeros(1, dtype=torch.int64, device=dev)
        self.graph: torch.cuda.CUDAGraph | None = None

    def _body(self) -> None:
        st, lib, x = self.step, self.lib, self.x
        stream = _hip.stream_of(x)
        sched, cur = _hip.ptr(self.sched), _hip.ptr(self.cursor)
        _hip.check(lib.sp_sched_timestep(sched, cur, _hip.ptr(self.t), stream), "sp_sched_timestep")
        with torch.enable_grad():
            xr = x.detach().requires_grad_(True)
            eps = st.network.forward(xr, self.t)
        eps_c = eps.detach().contiguous()
        b = x.shape[0]
        v = torch.empty_like(x)
        part = torch.empty((b, st.partials), device=x.device, dtype=torch.float32)
        _hip.check(lib.sp_dps_residual_sched(st.desc, _hip.ptr(x), _hip.ptr(eps_c), _hip.ptr(st.y),
                                             b, st.y_div, sched, cur, _hip.ptr(v), _hip.ptr(part),
                                             stream), "sp_dps_residual_sched")
        (w,) = torch.autograd.grad(eps, xr, grad_outputs=v.view_as(eps))
        w = w.contiguous()
        _hip.check(lib.sp_dps_update_sched(st.desc, _hip.ptr(x), _hip.ptr(eps_c), _hip.ptr(st.y),
                                           _hip.ptr(v) if st.needs_v else None, _hip.ptr(w),
                                           _hip.ptr(part) if st.mode == "dps" else None,
                                           self.seed, self.sample_offset, b, st.y_div, sched, cur,
                                           _hip.ptr(x), stream), "sp_dps_update_sched")
        _hip.check(lib.sp_sched_advance(cur, stream), "sp_sched_advance")

    def capture(self) -> None:
        """Warm up on a side stream (autograd / allocator state), restore, capture."""
        self.lib.sp_timing_enable(0)  # dispatch-packet timing events cannot be captured
        keep = self.x.clone()
        side = torch.cuda.Stream(device=self.x.device)
        side.wait_stream(torch.cuda.current_stream(self.x.device))
        with torch.cuda.stream(side):
            for _ in range(min(2, self.n_steps)):
                self._body()
        torch.cuda.current_stream(self.x.device).wait_stream(side)
        self.x.copy_(keep)
        self.cursor.zero_()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._body()
        torch.cuda.current_stream(self.x.device).synchronize()
        self.cursor.zero_()

    def replay(self, count: int | None = None) -> Tensor:
        if self.n_steps == 0:
            return self.x
        if self.graph is None:
            self.capture()
        for _ in range(self.n_steps if count is None else count):
            self.graph.replay()
        return self.x


def schedule_for(timesteps: list[int]) -> list[tuple[int, int, int, int]]:
    """The guided iterations of ``dps.py:91-122``: (i, t_i, t_{i-1}, t_0), i = N-1 .. 2."""
    return [(i, int(timesteps[i]), int(timesteps[i - 1]), int(timesteps[0]))
            for i in range(len(timesteps) - 1, 1, -1)]


__all__ = ["GraphedStepLoop", "schedule_for"]
