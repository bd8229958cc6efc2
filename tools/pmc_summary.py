"""Per-kernel HBM traffic from rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE in
separate runs, as MI355X_MICROARCH.md §rocprofv3 PMC slots requires).

    python tools/pmc_summary.py FETCH_CSV WRITE_CSV [--key KEY --json profiles/pmc_traffic.json]

Counters are KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE reports half of the bytes of a wide (16 B/lane) coalesced stream, so
fetched bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for 16-B stores.
"""
import argparse
import collections
import csv
import json
import re
from pathlib import Path


def load(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def short(name):
    m = re.search(r"sp::(k_\w+<[^>]*>)", name)
    return m.group(1) if m else name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--key", action="append", default=[],
                    help="NAME=KERNEL_SUBSTRING: record that kernel's traffic under NAME")
    ap.add_argument("--json")
    a = ap.parse_args()
    f, w = load(a.fetch), load(a.write)
    rows = {}
    for name in f:
        if name not in w:
            continue
        fb = 2 * 1024 * sum(f[name]) / len(f[name])
        wb = 1024 * sum(w[name]) / len(w[name])
        rows[name] = (len(f[name]), fb, wb)
        if "sp::" in name:
            print(f"{short(name):45s} n={len(f[name]):4d} fetch={fb/1e6:9.2f} MB "
                  f"write={wb/1e6:8.2f} MB total={(fb + wb)/1e6:9.2f} MB")
    if a.json:
        out = json.loads(Path(a.json).read_text()) if Path(a.json).exists() else {}
        for kv in a.key:
            # NAME=SUB1|SUB2: every dispatch of every kernel whose name holds one of the
            # substrings, so the per-launch figure covers the same launch set as the bench's
            # per-launch FLOPs / bytes (all variants, not the first match)
            key, subs = kv.split("=", 1)
            hits = [(k, v) for k, v in rows.items() if any(s in k for s in subs.split("|"))]
            if hits:
                n = sum(v[0] for _, v in hits)
                fb = sum(v[0] * v[1] for _, v in hits) / n
                wb = sum(v[0] * v[2] for _, v in hits) / n
                out[key] = {"hbm_bytes_per_launch": round(fb + wb), "fetch_bytes": round(fb),
                            "write_bytes": round(wb), "dispatches": n,
                            "kernels": sorted(short(k) for k, _ in hits),
                            "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                                      "KiB*1024, FETCH doubled (gfx950 wide-stream correction); "
                                      "mean over all dispatches of the listed kernels"}
        Path(a.json).write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
