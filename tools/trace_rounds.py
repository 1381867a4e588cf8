"""Per-round durations of k_frontier_round from a rocprofv3 kernel trace (analysis helper)."""
import csv
import sys

import numpy as np

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "k_frontier_round"
rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
st = np.array([int(r["Start_Timestamp"]) for r in rows])
en = np.array([int(r["End_Timestamp"]) for r in rows])
d = en - st
# split into elections: a gap > 1 ms between consecutive launches starts a new one
cut = np.nonzero(st[1:] - en[:-1] > 1_000_000)[0] + 1
segs = np.split(np.arange(len(d)), cut)
print("launches", len(d), "elections", len(segs), [len(s) for s in segs])
seg = max(segs, key=len)  # the first full election
dd = d[seg]
print("longest election: sum kernel ms %.3f  wall ms %.3f" % (dd.sum() / 1e6, (en[seg[-1]] - st[seg[0]]) / 1e6))
edges = [0, 1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096]
for a, b in zip(edges[:-1], edges[1:]):
    s = dd[a:b]
    if len(s):
        print("rounds %5d-%5d: sum %.3f ms  mean %.2f us  min %.2f  max %.2f" % (
            a + 1, min(b, len(dd)), s.sum() / 1e6, s.mean() / 1e3, s.min() / 1e3, s.max() / 1e3))
gaps = st[seg][1:] - en[seg][:-1]
print("gaps: median %.2f us, sum %.3f ms" % (np.median(gaps) / 1e3, gaps.sum() / 1e6))
