"""Per-launch durations of k_tail_xcd from a rocprofv3 kernel trace, matched in order with the
SWARM_XCD_LOG lines (first round, last round, last read change count) of the same run.
Usage: python tools/xcd_trace.py TRACE.csv RUN.log"""
import csv
import re
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_tail_xcd" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
launches = [tuple(int(x) for x in m.groups()) for m in
            re.finditer(r"xcd_launch (\d+) (\d+) last_read_changes (-?\d+)", open(sys.argv[2]).read())]
print(f"{len(rows)} dispatches, {len(launches)} logged launches")
per_call = {}
for r, (a, b, c) in zip(rows, launches):
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    per_call.setdefault(a, []).append((b, c, us))
for a in sorted(per_call):
    v = per_call[a]
    b, c, _ = v[-1]
    us = sorted(x[2] for x in v)
    med = us[len(us) // 2]
    print(f"rounds {a:5d}-{b:5d} ({b - a + 1:4d}) read_changes {c:7d}: median {med:8.1f} us, "
          f"{med / (b - a + 1):6.2f} us/round (launch incl. census)")
