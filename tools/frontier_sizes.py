"""Debug aid: how big the election frontier is, per round range, at C3 (10M agents, bench seed):
per-round changes and agents gathered (marked), from max_rounds cuts.
Usage: python tools/frontier_sizes.py [N]"""
import sys

import numpy as np

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = gen.swarm_inputs(n, 2026, t=0)
s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
r = s.elect()
ch = np.asarray(r.changes)
R = r.rounds_exec
print(f"n={n} rounds {R}")
cuts = [c for c in (1, 8, 9, 30, 60, 99, 150, 200, 300, 399, 500, 600, 700, 800, 906, 1000, 1100, 1200, 1300, R)
        if c <= R]
act = {c: s.elect(max_rounds=c).active_total for c in cuts}
prev = 0
for c in cuts:
    if prev:
        a = (act[c] - act[prev]) / (c - prev)
        seg = ch[prev:c]
        print(f"rounds {prev + 1:5d}-{c:5d}: marked/round {a:10.0f}  changes/round med {np.median(seg):8.0f} "
              f"max {seg.max():8d} min {seg.min():6d}")
    prev = c
