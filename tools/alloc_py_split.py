"""Host cost of each piece of Swarm.allocate's Python prelude at C3 (median us over 200 reps):
what runs between the caller and libswarm's first launch.  Usage: python tools/alloc_py_split.py"""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import _lib, gen  # noqa: E402
from swarm_amd.swarm import Swarm, _fast_ptr  # noqa: E402

d = gen.swarm_inputs(10_000_000, 2026, t=10_000)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
tx, ty, tq = (torch.as_tensor(d[k], device="cuda:0") for k in ("tx", "ty", "treq"))
sw.allocate(tx, ty, tq)
torch.cuda.synchronize()
dev = sw.device
t = 10_000


def tm(name, fn, reps=200):
    xs = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        xs.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    print(f"{name:28s} {np.median(xs) * 1e6:7.1f} us", flush=True)


tm("_task_pos", lambda: sw._task_pos(tx, ty))
tm("torch.full(t, -1)", lambda: torch.full((t,), -1, dtype=torch.int32, device=dev))
tm("torch.zeros(t) f64", lambda: torch.zeros(t, dtype=torch.float64, device=dev))
tm("torch.empty(n) i32", lambda: torch.empty(sw.n, dtype=torch.int32, device=dev))
tm("torch.empty((2,t)) i64", lambda: torch.empty((2, t), dtype=torch.int64, device=dev))
tm("id_index()", sw.id_index)
tm("_indexable", lambda: sw._indexable("auto", 20.0, 100.0))
tm("_cell_index()", sw._cell_index)
tm("AllocStats()", _lib.AllocStats)
tm("with torch.cuda.device", lambda: torch.cuda.device(dev).__enter__())
tm("_lib.ctx()", _lib.ctx)
tm("_lib.stream()", _lib.stream)
tm("_fast_ptr x13", lambda: [_fast_ptr(sw.ids) for _ in range(13)])
tm("allocate() total", lambda: sw.allocate(tx, ty, tq), reps=50)


def slow():
    sw._again = None  # the full prelude every call
    return sw.allocate(tx, ty, tq)


tm("allocate() slow path", slow, reps=50)
sw.allocate(tx, ty, tq)
tm("allocate() repeat (fast path)", lambda: sw.allocate(tx, ty, tq), reps=50)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
xs = []
for _ in range(50):
    torch.cuda.synchronize()
    ev[0].record()
    sw.allocate(tx, ty, tq)
    ev[1].record()
    torch.cuda.synchronize()
    xs.append(ev[0].elapsed_time(ev[1]))
print(f"{'bench split (events)':28s} {np.median(xs) * 1e3:7.1f} us", flush=True)
