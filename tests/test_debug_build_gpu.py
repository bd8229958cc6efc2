"""The bounds-checked debug build (``make debug`` -> samplers_amd/lib/debug/, SURVEY.md §5
"race detection / sanitizers"): every kernel's SP_DCHECK index / range invariants counted on
the device (``sp_debug_violations``).

A child process loads the debug library (``SAMPLERS_HIP_LIB``; a process holds one library)
and runs (1) the self-test launch, whose 64 threads each violate a check — the counting works
and names the site — and (2) the headline workloads on every kernel family: a DPS step of the
full ddpm-celebahq-256 UNet at 3x256² for inpainting and for blur (Winograd xi / W = 16 /
8x8-mosaic split-K tiles, stride-2 and thin convs, GroupNorm, x6 GEMMs, attention,
upsampling, both guidance passes), a PSLD step through the SD 1.5 VAE and ε-UNet at 3x256²
(fused multi-head and cross-attention, LayerNorm / GEGLU, layout GEMMs, the latent glue), and
the final predictions.  No invariant may be violated.
"""

from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]

CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from samplers_amd import _hip
lib = _hip.load_library()
assert lib.sp_debug_build() == 1, "not the debug library"
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
_hip.debug_violations()  # clear

_hip.check(lib.sp_debug_selftest(st), "sp_debug_selftest")
n, site = _hip.debug_violations()
assert n == 64 and site.startswith("1:"), (n, site)
print("selftest", n, site, flush=True)

from samplers_amd.inverse_problem import InverseProblem
from samplers_amd.networks.ddpm import DDPMNetwork
from samplers_amd.noise import GaussianNoise
from samplers_amd.operators import GaussianBlurOperator, RandomInpaintingOperator, CenterInpaintingOperator
from samplers_amd.samplers.dps import FusedDPSStep, initial_sample

shape, b = (3, 256, 256), 2
net = DDPMNetwork.from_config(seed=0, device=dev)
net.set_sampling_parameters(1000, batch_size=b)
ts = net.timesteps_host
for op in (RandomInpaintingOperator(shape, 0.5, seed=1).to(dev),
           GaussianBlurOperator(shape, kernel_size=9, sigma=3.0).to(dev)):
    y = op.apply(torch.rand((b, *shape), device=dev) * 2 - 1)
    prob = InverseProblem(op, y, GaussianNoise(0.05).to(dev))
    step = FusedDPSStep(net, prob, y, 1, gamma=1.0, eta=1.0)
    x = initial_sample((b, *shape), dev, rng="philox", seed=5, sample_offset=0, noise_fn=None)
    i = len(ts) - 1
    step(x, i, ts[i], ts[i - 1], ts[0], seed=5)
    step.predict_x0(x, ts[1])
    n, site = _hip.debug_violations()
    print(type(op).__name__, "violations", n, site, flush=True)
    assert n == 0, (type(op).__name__, n, site)
del net, step

from samplers_amd.networks.latent import LatentDiffusionNetwork, StableDiffusionCondition
from samplers_amd.samplers.psld import FusedPSLDStep
lnet = LatentDiffusionNetwork.from_config(seed=0, device=dev)
lnet.set_sampling_parameters(4, batch_size=1)
# CFG on (distinct prompt embeddings): the doubled batch, cross-attention to real contexts
lnet.set_condition(StableDiffusionCondition(prompt=None, prompt_embeds=torch.randn(1, 77, 768),
                                            guidance_scale=7.5))
op = CenterInpaintingOperator(shape, 0.5).to(dev)
y = op.apply(torch.rand((1, *shape), device=dev) * 2 - 1)
prob = InverseProblem(op, y, GaussianNoise(0.05).to(dev))
lts = lnet.timesteps_host
step = FusedPSLDStep(lnet, prob, y, 1, (4, 32, 32))
z = torch.randn(1, 4, 32, 32, device=dev)
i = len(lts) - 1
step(z, i, lts[i], lts[i - 1], lts[0], xi=torch.randn_like(z))
n, site = _hip.debug_violations()
print("PSLD violations", n, site, flush=True)
assert n == 0, ("PSLD", n, site)
print("debug build: clean", flush=True)
"""


@pytest.mark.timeout(600)
def test_debug_build_counts_violations_and_the_workloads_have_none(cuda):
    from samplers_amd import _hip

    if not _hip.DEBUG_LIB_PATH.exists():
        pytest.fail(f"{_hip.DEBUG_LIB_PATH} missing: run `make` (builds the debug library too)")
    env = dict(os.environ, SAMPLERS_HIP_LIB=str(_hip.DEBUG_LIB_PATH))
    out = subprocess.run([sys.executable, "-c", CHILD, str(ROOT)], env=env, capture_output=True,
                         text=True, timeout=540)
    print(out.stdout[-4000:], out.stderr[-4000:])
    assert out.returncode == 0, out.stderr[-2000:]
    assert "debug build: clean" in out.stdout


def test_release_build_reports_no_checks(cuda):
    from samplers_amd import _hip

    lib = _hip.load_library()
    if lib.sp_debug_build():
        pytest.skip("running under the debug library")
    assert _hip.debug_violations() == (0, None)
    assert lib.sp_debug_selftest(None) != 0  # SP_EINVAL: nothing to test in the release build
