"""A/B of the election with and without the tiled tail rounds (swarm_elect_tiled) on the C3 swarm:
elect ms (median of 5, HIP events on the current stream), tiled rounds / launches, and a check that
all three give the same rounds and per-round changes.  Usage: python tools/tiles_ab.py [N]"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = gen.swarm_inputs(n, 2026, deg=16.0)
s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
torch.cuda.synchronize()
ti = s.tile_index()
out = {"n": n, "tile_index": ti is not None}
ref = None
for tiles in (False, True, "early"):
    s.elect(tiles=tiles)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        r = s.elect(tiles=tiles)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    if ref is None:
        ref = r
    same = r.rounds_exec == ref.rounds_exec and np.array_equal(r.changes, ref.changes) and \
        torch.equal(r.leader, ref.leader)
    rt = s.elect(tiles=tiles, timed=True)
    out[str(tiles)] = {"ms": float(np.median(ts)), "min_ms": float(min(ts)), "rounds": r.rounds_exec,
                       "tile_from": int(rt.tile_from), "tile_rounds": int(rt.tile_rounds),
                       "tile_launches": int(rt.tile_launches), "tile_ms": rt.tile_ms,
                       "sparse_ms": rt.sparse_ms, "gather_ms": rt.gather_ms, "same": bool(same)}
    print(json.dumps(out), flush=True)
