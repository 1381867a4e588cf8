"""Per-round kernel time of the last election call in a rocprofv3 kernel trace, by round range:
k_sparse_block dispatches are rounds dense_rounds+1, ... in order; each k_tail_xcd dispatch covers
the rounds its SWARM_XCD_LOG line names (its time is spread evenly over them).
Usage: python tools/xcd_rounds.py TRACE.csv RUN.log [RANGES]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
calls, cur = [], []
for r in rows:
    cur.append(r)
    if "k_state" in r["Kernel_Name"]:
        calls.append(cur)
        cur = []
launches = [tuple(int(x) for x in m.groups()[:2]) for m in
            re.finditer(r"xcd_launch (\d+) (\d+) last_read_changes (-?\d+)", open(sys.argv[2]).read())]
ntail = sum(1 for r in calls[-1] if "k_tail_xcd" in r["Kernel_Name"])
mine = launches[len(launches) - ntail:] if ntail else []
t = 9
per = {}
li = 0
for r in calls[-1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "k_sparse_block" in r["Kernel_Name"]:
        t += 1
        per[t] = per.get(t, 0) + d
    elif "k_tail_xcd" in r["Kernel_Name"]:
        a, b = mine[li]
        li += 1
        for q in range(a, b + 1):
            per[q] = per.get(q, 0) + d / (b - a + 1)
        t = b
    elif "fillBuffer" in r["Kernel_Name"] and t >= 10:
        per[t + 1] = per.get(t + 1, 0) + d  # memsets before a round: charged to it
edges = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "10,400,700,1000,1100,1200,1240,1300,1365,1400").split(",")]
for lo, hi in zip(edges[:-1], edges[1:]):
    v = [per[q] for q in range(lo, hi) if q in per]
    if v:
        print(f"rounds {lo:5d}-{hi - 1:5d}: {len(v):4d} rounds, {sum(v):8.1f} us, {sum(v) / len(v):6.2f} us/round")
