"""The d = 512 single-head attention's score GEMMs (DDPM UNet 16² level, SD VAE mid block) at
small batch: hipBLASLt's choice for q kᵀ (n x n, K = 512) at b = 1 is one 256x256 macro tile
on one CU.  Times the plain batched GEMM against query-chunked forms (the rows cut into
chunks, k repeated per chunk) for b in BATCHES:
    python tools/bench_score_gemm.py   -> one JSON line per (b, n, chunks)"""
import json
import os

import torch


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda")
    for b in [int(v) for v in os.environ.get("BATCHES", "1,2,4,8,64").split(",")]:
        for n, c in ((256, 512), (4096, 512)):
            if b * n * n * 4 > 8 * 2**30:
                continue
            qkv = torch.randn(b, n, 3 * c, device=dev)
            q, k, v = qkv.split(c, dim=-1)
            ref = torch.baddbmm(torch.empty(b, n, n, device=dev), q, k.transpose(1, 2), beta=0.0, alpha=0.05)
            for ch in (1, 2, 4, 8, 16, 32):
                if n % ch or n // ch < 8:
                    continue
                r = n // ch
                qc = q.reshape(b * ch, r, c)  # a view: q's row stride is 3c
                kc = k.unsqueeze(1).expand(b, ch, n, c).reshape(b * ch, n, c)
                p = torch.empty(b, n, n, device=dev)

                def run():
                    kk = k.unsqueeze(1).expand(b, ch, n, c).reshape(b * ch, n, c) if ch > 1 else k
                    torch.baddbmm(p.view(b * ch, r, n), qc if ch > 1 else q, kk.transpose(1, 2), beta=0.0,
                                  alpha=0.05, out=p.view(b * ch, r, n))
                us = timeit(run)
                err = float((p - ref).abs().max())
                print(json.dumps({"b": b, "n": n, "d": c, "chunks": ch, "us": round(us, 2),
                                  "tflops": round(2 * b * n * n * c / us / 1e6, 2), "max_abs_diff": err}),
                      flush=True)
                del kc


if __name__ == "__main__":
    main()
