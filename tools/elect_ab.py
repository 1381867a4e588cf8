"""A/B timing aid: untimed wall time of swarm_elect(FRONTIER) at N agents for one libswarm build.
Usage: python tools/elect_ab.py LIBNAME [N]   (LIBNAME under swarm_amd/, e.g. libswarm.so)"""
import os
import sys
import time

sys.path.insert(0, "distributed-swarm-algorithm_amd")
import torch  # noqa: E402
from swarm_amd import _lib  # noqa: E402

_lib.load(os.path.join(_lib.HERE, sys.argv[1]))
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
d = gen.swarm_inputs(n, 2026, t=0)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
r = sw.elect()
torch.cuda.synchronize()
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    r = sw.elect()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"{sys.argv[1]}: n={n} rounds={r.rounds_exec} launched={r.rounds_launched} "
      f"elect ms min {min(ts) * 1e3:.2f} med {sorted(ts)[2] * 1e3:.2f} "
      f"leader_sum {int(r.leader.to(torch.int64).sum())} changes_sum {int(sum(r.changes))}")
