"""Kernels of the last auction call in a rocprofv3 kernel trace (calls start at k_auc_count):
span, busy time, gaps, per-kernel totals, and the fused rounds' per-launch durations.
Usage: python tools/auction_trace.py TRACE.csv"""
import csv
import re
import sys
from collections import defaultdict

import numpy as np

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_auc_count" in r["Kernel_Name"]]
c = rows[starts[-1]:]
span = (int(c[-1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"])) / 1e3
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in c) / 1e3
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(c, c[1:])]
print(f"last call: {len(c)} kernels, span {span:.0f} us, busy {busy:.0f} us, gaps {sum(gaps):.0f} us")
agg = defaultdict(list)
for r in c:
    m = re.search(r"k_\w+", r["Kernel_Name"])
    agg[m.group(0) if m else r["Kernel_Name"][:40]].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    v = np.array(v)
    print(f"  {len(v):5d} x {v.mean():7.2f} us (p50 {np.median(v):6.2f}) = {v.sum():8.0f} us  {k}")
