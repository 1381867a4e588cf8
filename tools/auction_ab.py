"""A/B timing of the C4 auction (100k agents x 100k tasks, bench.py's seed) under different
SWARM_AUCTION_FUSED / SWARM_AUCTION_TAIL settings, read per call.
Usage: python tools/auction_ab.py FUSED[:TAIL] ..."""
import os
import sys
import time

import torch

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

d = gen.swarm_inputs(100_000, 2026 + 2, t=100_000)
s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0")
tx, ty, tr = (torch.as_tensor(d[k]).cuda() for k in ("tx", "ty", "treq"))
ref = None
for spec in sys.argv[1:]:
    fused, tail = (spec.split(":") + [""])[:2]
    os.environ["SWARM_AUCTION_FUSED"] = fused
    if tail:
        os.environ["SWARM_AUCTION_TAIL"] = tail
    ts = []
    for _ in range(7):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = s.auction(tx, ty, tr)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    a = r.assigned.cpu()
    same = "ref" if ref is None else ("same" if torch.equal(a, ref) else "DIFFERENT")
    ref = a if ref is None else ref
    ts.sort()
    print(f"fused={fused} tail={os.environ.get('SWARM_AUCTION_TAIL', '-')}: rounds {r.rounds_exec} "
          f"ms min {ts[0]:.2f} med {ts[3]:.2f}  assigned {same}", flush=True)
