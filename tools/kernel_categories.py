"""Group a rocprofv3 kernel_stats.csv into prior categories: python tools/kernel_categories.py <csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
cats = {}
for r in rows:
    n, t = r["Name"], float(r["TotalDurationNs"])
    if "Conv" in n or "igemm" in n or "conv" in n.lower() or "k_wino" in n:
        c = "conv"
    elif "k_gn_" in n:
        c = "sp groupnorm (HIP)"
    elif "Cijk" in n:
        c = "gemm"
    elif "transpose" in n:
        c = "layout transpose"
    elif "GroupNorm" in n or "RowwiseMoments" in n or "ComputeInternalGradients" in n:
        c = "torch groupnorm"
    elif "silu" in n:
        c = "torch silu"
    elif "add" in n.lower() and "Functor" in n:
        c = "torch add"
    elif "bwd_kernel" in n or "attn" in n.lower() or "fwd_kernel" in n:
        c = "attention"
    elif "sp::" in n:
        c = "sp guidance (HIP)"
    elif "Cat" in n or "copy" in n:
        c = "copy/cat"
    else:
        c = "other"
    cats[c] = cats.get(c, 0) + t
for c, t in sorted(cats.items(), key=lambda x: -x[1]):
    print(f"{c:20s} {t / tot * 100:6.2f}%  {t / 1e6:9.1f} ms")
print("total ms", round(tot / 1e6, 1))
