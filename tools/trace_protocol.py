"""Per-tick durations of the protocol kernels from a rocprofv3 kernel trace (CSV).

python tools/trace_protocol.py DIR [N] [per-tick]  -> k_tick / k_mail (and k_tick_pull) of the last N
ticks of the last run of tools/protocol_probe.py: medians, means, extremes, and the share of the
total in ticks above 2x the median (storms); per-tick lines with a third argument.
"""
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
series = {}
for r in rows:
    for k in ("k_tick", "k_mail", "k_tick_pull"):
        if k + "(" in r["Kernel_Name"]:
            series.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
for k, v in series.items():
    tail = v[-n:]
    med = statistics.median(tail)
    heavy = sum(x for x in tail if x > 2 * med)
    print(f"{k:12s} calls={len(v):5d} last{n}: median {med:7.1f} us  mean {statistics.mean(tail):7.1f}"
          f"  min {min(tail):6.1f}  max {max(tail):6.1f}  sum {sum(tail) / 1e3:6.2f} ms"
          f"  (ticks > 2x median: {sum(1 for x in tail if x > 2 * med)}, {heavy / 1e3:.2f} ms)")
if "k_tick" in series and len(sys.argv) > 3:
    for t in range(n):
        print(t + 1, *(round(series[k][-n + t], 1) for k in ("k_tick", "k_mail") if k in series))
