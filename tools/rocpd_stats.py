"""rocprofv3 (ROCm 7) writes a rocpd SQLite database by default; turn its kernel dispatches
into the kernel_stats.csv layout of `--stats --output-format csv`:

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/.../kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
durs = defaultdict(list)
for name, dur in db.execute("select name, duration from kernels"):
    durs[name].append(int(dur))
total = sum(sum(v) for v in durs.values())
w = csv.writer(sys.stdout, quoting=csv.QUOTE_ALL)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
            "StdDev"])
for name, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
    s = sum(v)
    w.writerow([name, len(v), s, f"{s / len(v):.6f}", f"{100.0 * s / total:.2f}", min(v), max(v),
                f"{statistics.pstdev(v):.6f}"])
