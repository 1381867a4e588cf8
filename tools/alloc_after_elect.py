"""The bench's election/allocation split at C3, taken apart: HIP-event time of Swarm.allocate right after an
election (as bench.py's breakdown_ms.alloc) against back-to-back allocations, with the host time of the
call beside each.  Usage: python tools/alloc_after_elect.py [LIBNAME]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import _lib, gen  # noqa: E402

_lib.load(os.path.join(_lib.HERE, sys.argv[1] if len(sys.argv) > 1 else "libswarm.so"))
from swarm_amd.swarm import Swarm  # noqa: E402

d = gen.swarm_inputs(10_000_000, 2026, t=10_000)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
tx, ty, tq = (torch.as_tensor(d[k], device="cuda:0") for k in ("tx", "ty", "treq"))
sw.elect()
sw.allocate(tx, ty, tq)
torch.cuda.synchronize()


def one(after_elect):
    if after_elect:
        sw.elect()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    h0 = time.perf_counter()
    sw.allocate(tx, ty, tq)
    h1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3, (h1 - h0) * 1e6


for label, ae, reps in (("after elect", True, 10), ("back to back", False, 40)):
    xs = np.array([one(ae) for _ in range(reps)])
    print(f"{sys.argv[1] if len(sys.argv) > 1 else 'libswarm.so'} {label:13s} events med {np.median(xs[:, 0]):6.1f} us "
          f"(min {xs[:, 0].min():6.1f})  host call med {np.median(xs[:, 1]):6.1f} us", flush=True)
