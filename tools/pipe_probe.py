"""A/B aid for the pipelined election tail (k_pipe_rounds): wall time of Swarm.elect with the tail
pipelined (default), pipelined from the first sparse round ("early") and off, on the bench's RGG
inputs at the given sizes; checks the three runs agree (leaders, per-round changes).
Usage: python tools/pipe_probe.py [N ...]   (default 100000 1000000 10000000)"""
import sys
import time

sys.path.insert(0, "distributed-swarm-algorithm_amd")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from swarm_amd import _lib, gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

_lib.load()
sizes = [int(a) for a in sys.argv[1:]] or [100_000, 1_000_000, 10_000_000]
for n in sizes:
    d = gen.swarm_inputs(n, 2026, t=0)
    sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
    ref = None
    for pipe in (False, True, "early", False, True):
        r = sw.elect(pipe=pipe)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            r = sw.elect(pipe=pipe)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        lead = r.leader.cpu().numpy()
        if ref is None:
            ref = (lead, r.changes, r.rounds_exec)
        same = np.array_equal(lead, ref[0]) and np.array_equal(r.changes, ref[1]) and r.rounds_exec == ref[2]
        rt = sw.elect(pipe=pipe, timed=True)
        print(f"n={n} pipe={pipe!s:5} rounds={r.rounds_exec} launched={r.rounds_launched} "
              f"ms min {min(ts) * 1e3:.3f} med {sorted(ts)[2] * 1e3:.3f} same={same} "
              f"pipe_from={r.pipe_from} launches={r.pipe_launches} grid={r.pipe_grid} reach={r.pipe_reach} "
              f"timed: sparse {rt.sparse_ms:.3f} ms / {rt.sparse_launches} pipe {rt.pipe_ms:.3f} ms / "
              f"{rt.pipe_rounds} rounds", flush=True)
        if not same:
            sys.exit(1)
    del sw
    torch.cuda.empty_cache()
