"""Kernels of the last election call in a rocprofv3 kernel trace (calls end with k_state): span,
busy time, gaps, and per-kernel-name counts / total / mean durations.
Usage: python tools/call_gaps.py TRACE.csv"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
calls, cur = [], []
for r in rows:
    cur.append(r)
    if "k_state" in r["Kernel_Name"]:
        calls.append(cur)
        cur = []
c = calls[-1]
span = (int(c[-1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"])) / 1e3
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in c) / 1e3
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(c, c[1:])]
print(f"{len(calls)} calls; last: {len(c)} kernels, span {span:.1f} us, busy {busy:.1f} us, gaps {sum(gaps):.1f} us "
      f"(largest {sorted(gaps)[-5:]})")
agg = defaultdict(list)
for r in c:
    agg[r["Kernel_Name"].split("(")[0][-60:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {len(v):5d} x {sum(v) / len(v):7.2f} us = {sum(v):8.1f} us  {k}")
