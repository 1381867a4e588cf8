"""Host-side cost of Swarm.allocate at C3 (10M agents, 10k tasks): wall time per call (synchronised),
the same with the GPU work alone (HIP events), and a cProfile of 50 calls.
Usage: python tools/alloc_host_probe.py [N]"""
import cProfile
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = gen.swarm_inputs(n, 2026, t=10_000)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
tx = torch.as_tensor(d["tx"], device="cuda:0")
ty = torch.as_tensor(d["ty"], device="cuda:0")
tq = torch.as_tensor(d["treq"], device="cuda:0")
sw.elect()
for _ in range(3):
    sw.allocate(tx, ty, tq)
torch.cuda.synchronize()
wall, gpu, enq = [], [], []
for _ in range(20):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    a = sw.allocate(tx, ty, tq)
    e1.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    wall.append((t2 - t0) * 1e3)
    enq.append((t1 - t0) * 1e3)
    gpu.append(e0.elapsed_time(e1))
print(f"allocate: wall {np.median(wall):.3f} ms, returned after {np.median(enq):.3f} ms, "
      f"events {np.median(gpu):.3f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    sw.allocate(tx, ty, tq)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
