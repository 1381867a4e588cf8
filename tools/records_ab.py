"""A/B of the election with and without the record tail (swarm_elect_records) on the C3 swarm:
elect ms (median of 5, HIP events on the current stream), where the tail started, its launches /
activations / recomputes, and a check that every variant gives the same rounds, per-round changes and
leaders.  Usage: python tools/records_ab.py [N] [variants: 0,1,early]   (env SWARM_REC_* tunes)"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
variants = [{"0": False, "1": True, "early": "early"}[v] for v in (sys.argv[2] if len(sys.argv) > 2 else "0,1").split(",")]
d = gen.swarm_inputs(n, 2026, deg=16.0)
s = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
torch.cuda.synchronize()
t0 = time.time()
ri = s.record_index()
torch.cuda.synchronize()
out = {"n": n, "record_index": ri is not None, "index_s": round(time.time() - t0, 3),
       "env": {k: v for k, v in os.environ.items() if k.startswith("SWARM_REC")}}
ref = None
for rec in variants:
    s.elect(records=rec)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        r = s.elect(records=rec)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    if ref is None:
        ref = r
    same = r.rounds_exec == ref.rounds_exec and np.array_equal(r.changes, ref.changes) and \
        torch.equal(r.leader, ref.leader)
    rt = s.elect(records=rec, timed=True)
    out[str(rec)] = {"ms": round(float(np.median(ts)), 3), "min_ms": round(float(min(ts)), 3),
                     "rounds": r.rounds_exec, "record_from": int(rt.record_from),
                     "record_launches": int(rt.record_launches), "record_activations": int(rt.record_activations),
                     "record_recomputes": int(rt.record_recomputes), "record_levels": int(rt.record_levels),
                     "record_ms": round(rt.record_ms, 3),
                     "record_fallback": int(rt.record_fallback), "sparse_ms": round(rt.sparse_ms, 3),
                     "gather_ms": round(rt.gather_ms, 3), "same": bool(same)}
    print(json.dumps(out), flush=True)
