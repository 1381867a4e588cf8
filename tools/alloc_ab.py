"""A/B timing of Swarm.allocate at C3 (10M agents, 10k tasks) for one libswarm build: median HIP-event
time of the call and of k_alloc_binned's launch sequence, plus a checksum of the results (winners,
won counts, claims) so variants can be compared.  Usage: python tools/alloc_ab.py LIBNAME [N]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import _lib  # noqa: E402

_lib.load(os.path.join(_lib.HERE, sys.argv[1]))
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
d = gen.swarm_inputs(n, 2026, t=10_000)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
tx, ty, tq = (torch.as_tensor(d[k], device="cuda:0") for k in ("tx", "ty", "treq"))
sw.elect()
for _ in range(3):
    a = sw.allocate(tx, ty, tq)
torch.cuda.synchronize()
ts = []
for _ in range(40):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    a = sw.allocate(tx, ty, tq)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ck = (int(a.winner.to(torch.int64).sum()), int(a.won.to(torch.int64).sum()), int(a.nclaim.sum()),
      int(a.nmsg.sum()), round(float(a.util.sum()), 6))
print(f"{sys.argv[1]}: allocate ms med {np.median(ts):.4f} min {min(ts):.4f} check {ck} stats {a.stats}", flush=True)
