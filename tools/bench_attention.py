"""Self-attention forward + input VJP at the SD 1.5 UNet's shapes (32 latents x 8 heads; 64x64,
32x32, 16x16 tokens; head dims 40, 80, 160), through ``networks.attention.attention``:

    python tools/bench_attention.py        (one JSON line per shape)

useful FLOP = 4 * BH * N^2 * d forward (q k^T and P v), 2.5x that for the VJP (recomputed
scores, dP, dq, dk, dv)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from samplers_amd.networks.attention import attention  # noqa: E402

SHAPES = [(256, 4096, 40), (256, 1024, 80), (256, 256, 160)]


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    from samplers_amd import _hip

    dev = torch.device("cuda:0")
    lib = _hip.load_library()
    modes = sys.argv[1:] or ["x6", "fp32"]  # the forward's kernel: split-bf16 (pre-split K / V) or exact fp32
    for (bh, n, d), mode in [(sh, md) for sh in SHAPES for md in modes]:
        lib.sp_attention_bf16x6(1 if mode == "x6" else 0)
        g = torch.Generator(device=dev).manual_seed(0)
        q, k, v = (torch.randn(bh, n, d, device=dev, generator=g).requires_grad_() for _ in range(3))
        do = torch.randn(bh, n, d, device=dev, generator=g)

        def fwd():
            with torch.no_grad():
                attention(q, k, v)

        def fwd_bwd():
            out = attention(q, k, v)
            torch.autograd.grad(out, (q, k, v), do)

        tf, tb = timed(fwd), timed(fwd_bwd)
        flop = 4.0 * bh * n * n * d
        print(json.dumps({"bh": bh, "n": n, "d": d, "fwd_kernel": mode, "fwd_ms": round(tf, 3),
                          "fwd_bwd_ms": round(tb, 3), "fwd_tflops": round(flop / tf / 1e9, 1),
                          "fwd_bwd_tflops": round(3.5 * flop / tb / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
