"""Per-step kernel time of one DPS step from a rocprofv3 kernel trace (the last complete step
between two dps_update launches), split at the residual pass into the prior's forward and its
VJP, grouped by kind:  python tools/step_breakdown.py <run_kernel_trace.csv>"""
import collections
import csv
import sys


def kind(n: str) -> str:
    if "k_wino" in n:
        return "HIP Winograd conv tile"
    if "k_conv3x3_s2" in n:
        return "HIP stride-2 conv tile (downsampling, fwd + VJP)"
    if "k_conv3x3_thin" in n:
        return "HIP thin conv (conv_in / conv_out)"
    if "k_upsample2x" in n:
        return "HIP nearest upsampling (fwd + VJP)"
    if "k_conv3x3" in n:
        return "HIP direct conv tile"
    if "k_gn" in n:
        return "HIP GroupNorm(+SiLU) fwd / VJP"
    if "k_dps" in n or "k_blur" in n:
        return "HIP guidance passes"
    if "miopen" in n or "igemm" in n or "naive_conv" in n or "transpose" in n:
        return "MIOpen convs (16x16 / 8x8 stride-2) + layout transposes"
    if "k_gemm_x6" in n:
        return "HIP 1x1 shortcut GEMM (bf16x6, fwd + VJP)"
    if "Cijk" in n:
        return "hipBLASLt GEMMs (attention, time embedding)"
    if "CUDAFunctor_add" in n:
        return "torch adds"
    if "k_softmax" in n or "k_layernorm" in n or "k_geglu" in n or "k_conv1x1_small" in n:
        return "HIP softmax / LayerNorm / GEGLU / small 1x1"
    if "k_attn" in n:
        return "HIP fused attention"
    if "softmax" in n.lower():
        return "softmax"
    if "upsample" in n:
        return "torch nearest upsampling"
    return "other torch elementwise / copies"


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "k_dps_update" in r["Kernel_Name"]]
step = rows[ends[-2] + 1:ends[-1] + 1]
mid = next(i for i, r in enumerate(step) if "k_dps_residual" in r["Kernel_Name"] or "k_blur_dps" in r["Kernel_Name"])
tot = collections.defaultdict(float)
for name, part in (("prior forward", step[:mid]), ("prior VJP + update", step[mid:])):
    c = collections.defaultdict(lambda: [0, 0.0])
    for r in part:
        k = kind(r["Kernel_Name"])
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        c[k][0] += 1
        c[k][1] += dt
        tot[k] += dt
    print(f"{name}: {sum(v[1] for v in c.values()):.1f} ms")
    for k, v in sorted(c.items(), key=lambda kv: -kv[1][1]):
        print(f"   {k:72s} {v[0]:4d} launches {v[1]:8.2f} ms")
s = sum(tot.values())
print(f"step: {s:.1f} ms of kernel time")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"   {k:72s} {v:8.2f} ms  {100 * v / s:5.1f} %")
