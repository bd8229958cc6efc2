"""Per-kernel statistics from a rocprofv3 kernel trace (``*_kernel_trace.csv``, or the
``out_kernel_trace.csv`` that ``rocpd2csv`` writes from a ``results.db``), in the columns of
rocprofv3's ``kernel_stats.csv``:

    python tools/trace_stats.py TRACE_CSV [--out kernel_stats.csv] [--skip-dispatches N]

``--skip-dispatches`` drops the first N dispatches (warm-up)."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    ap.add_argument("--skip-dispatches", type=int, default=0)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[a.skip_dispatches:]
    dur = collections.defaultdict(list)
    for r in rows:
        dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in dur.values())
    out = []
    for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        out.append({"Name": name, "Calls": len(v), "TotalDurationNs": sum(v),
                    "AverageNs": sum(v) / len(v), "Percentage": 100.0 * sum(v) / total,
                    "MinNs": min(v), "MaxNs": max(v)})
    if a.out:
        with open(a.out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0]), quoting=csv.QUOTE_NONNUMERIC)
            w.writeheader()
            w.writerows(out)
    for r in out[:25]:
        print(f"{r['Percentage']:6.2f}%  {r['Calls']:5d}  {r['AverageNs'] / 1e3:9.1f} us  "
              f"{r['Name'][:90]}")
    print(f"total kernel time {total / 1e6:.1f} ms over {len(rows)} dispatches")


if __name__ == "__main__":
    main()
