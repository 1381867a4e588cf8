"""Per-tick durations of the protocol kernels from a rocprofv3 kernel trace (CSV).

python tools/trace_protocol.py gpurun_out/pprof  -> k_compact / k_receive / k_sweep per tick of the
last chunked run of tools/protocol_probe.py, plus steady-state medians.
"""
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(f)))
series = {}
for r in rows:
    for k in ("k_compact", "k_receive", "k_sweep", "k_tick_pull"):
        if k + "(" in r["Kernel_Name"]:
            series.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
for k, v in series.items():
    tail = v[-n:]
    print(f"{k:12s} calls={len(v):5d} last{n}: median {statistics.median(tail):7.1f} us  mean {statistics.mean(tail):7.1f}"
          f"  min {min(tail):6.1f}  max {max(tail):6.1f}")
if "k_sweep" in series and len(sys.argv) > 3:
    for t in range(n):
        print(t + 1, *(round(series[k][-n + t], 1) for k in ("k_compact", "k_receive", "k_sweep")))
