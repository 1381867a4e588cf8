"""Per-round election log (SWARM_ROUND_LOG: round, changes, marked, edges, kind, kernel us) for one
libswarm build, then a summary of kernel time by round range.
Usage: python tools/round_log.py [N] [LIBNAME] [OUT]"""
import os
import sys

sys.path.insert(0, "distributed-swarm-algorithm_amd")
sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from swarm_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
lib = sys.argv[2] if len(sys.argv) > 2 else "libswarm.so"
out = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/rounds.log"
_lib.load(os.path.join(_lib.HERE, lib))
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

d = gen.swarm_inputs(n, 2026, t=0)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
sw.elect()
os.environ["SWARM_ROUND_LOG"] = out
r = sw.elect(timed=True)
torch.cuda.synchronize()
print(lib, "n", n, "rounds", r.rounds_exec, "kernel ms", r.gather_ms)
a = np.loadtxt(out)
edges = [1, 9, 100, 400, 907, 1e9]
for lo, hi in zip(edges[:-1], edges[1:]):
    m = (a[:, 0] >= lo) & (a[:, 0] < hi)
    if m.any():
        us = a[m, 5]
        print(f"  rounds {int(lo)}-{int(min(hi, a[-1, 0] + 1)) - 1}: {m.sum()} launches, {us.sum() / 1e3:.2f} ms, "
              f"median {np.median(us):.1f} us, marked/round {a[m, 2].mean():.0f}")
