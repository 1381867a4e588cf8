"""The one-workgroup tail experiment (SWARM_TAIL_WG, elect.hip k_tail_wg): election wall time
of C2 (100k agents, bench's seed) and C3 (10M) with the tail at the given cap against without, exactness against
the first run of the process, and -- SWARM_TAIL_LOG=1 -- the per-round microseconds by marked-agent count.
The env is read once per process: run one process per setting.  Usage: python tools/tail_probe.py N [SEED]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[1])
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 2027
d = gen.swarm_inputs(n, seed)
sw = Swarm(d["ids"], d["x"], d["y"], device="cuda:0").build_graph(1.0)
r = sw.elect()
torch.cuda.synchronize()
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    r = sw.elect()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"n={n} seed={seed} SWARM_TAIL_WG={os.environ.get('SWARM_TAIL_WG', '0')}: rounds={r.rounds_exec} "
      f"elect ms med {np.median(ts) * 1e3:.3f} min {min(ts) * 1e3:.3f} leader_sum "
      f"{int(r.leader.to(torch.int64).sum())} changes_sum {int(sum(r.changes))}", flush=True)
