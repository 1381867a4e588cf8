"""Per-round-range kernel durations of the longest election in a rocprofv3 kernel trace
(tools/trace_ab.sh): rounds are the k_elect_dense / k_sparse_block / k_list_round dispatches in order.
Usage: python tools/trace_ranges.py TRACE.csv [LABEL]"""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
            if "k_elect_dense" in r["Kernel_Name"] or "k_sparse_block" in r["Kernel_Name"]
            or "k_list_round" in r["Kernel_Name"] or "k_task_round" in r["Kernel_Name"])
elections, cur, prev_sparse = [], [], False
for k in ks:
    dense = "k_elect_dense" in k[2]
    if dense and prev_sparse:
        elections.append(cur)
        cur = []
    cur.append(k)
    prev_sparse = not dense
elections.append(cur)
e = max(elections, key=len)  # the longest election (the C3 one in a bench trace)
d = np.array([b - a for a, b, _ in e]) / 1e3
span = (e[-1][1] - e[0][0]) / 1e6
label = sys.argv[2] if len(sys.argv) > 2 else ""
print(f"{label} rounds launched {len(e)}: span {span:.2f} ms, kernels {d.sum() / 1e3:.2f} ms")
for lo, hi in [(1, 8), (9, 9), (10, 30), (31, 100), (101, 200), (201, 400), (401, 700), (701, 1000), (1001, 1364),
               (1365, 100000)]:
    x = d[lo - 1:hi]
    if len(x):
        print(f"   rounds {lo}-{min(hi, len(d))}: med {np.median(x):.1f} us, p90 {np.percentile(x, 90):.1f}, "
              f"sum {x.sum() / 1e3:.2f} ms")
