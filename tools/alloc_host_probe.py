"""Host-side cost of Swarm.allocate at C3 (10M agents, 10k tasks): wall time of each step of the
call, averaged over repetitions (the C call includes its stats sync, i.e. the device work)."""
import os
import sys
import time

sys.path.insert(0, "distributed-swarm-algorithm_amd")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from swarm_amd import _lib, gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

d = gen.swarm_inputs(int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000, 2026, t=10_000)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda").build_graph(1.0)
tx, ty, tq = (torch.as_tensor(d[k], device="cuda") for k in ("tx", "ty", "treq"))
sw.elect()
for _ in range(3):
    sw.allocate(tx, ty, tq)
torch.cuda.synchronize()
reps = 30
t0 = time.perf_counter()
for _ in range(reps):
    sw.allocate(tx, ty, tq)
torch.cuda.synchronize()
print(f"allocate() wall {1e3 * (time.perf_counter() - t0) / reps:.3f} ms/call")
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ts = []
for _ in range(reps):
    ev[0].record()
    sw.allocate(tx, ty, tq)
    ev[1].record()
    torch.cuda.synchronize()
    ts.append(ev[0].elapsed_time(ev[1]))
print(f"allocate() event span {np.median(ts):.3f} ms (median)")
# elect + allocate as in bench.py's breakdown
ts = []
for _ in range(5):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    sw.elect()
    e[1].record()
    sw.allocate(tx, ty, tq)
    e[2].record()
    torch.cuda.synchronize()
    ts.append((e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2])))
print("elect / alloc ms (bench breakdown):", [f"{a:.2f}/{b:.3f}" for a, b in ts])
# after an election, with the device drained first / host wall time of the call
for drain in (False, True):
    ts = []
    for _ in range(5):
        sw.elect()
        if drain:
            torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        t0 = time.perf_counter()
        e[0].record()
        sw.allocate(tx, ty, tq)
        e[1].record()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        ts.append((e[0].elapsed_time(e[1]), th * 1e3))
    print(f"after elect (drain={drain}): alloc event / host ms", [f"{a:.3f}/{b:.3f}" for a, b in ts])
