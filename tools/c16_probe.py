import sys, time, json
import numpy as np, torch
sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import gen
from swarm_amd.swarm import Swarm
W, n_per = 8, 2_500_000
ds = [gen.shard_inputs(n_per, 2026, W, q, deg=16.0, layout="blocks") for q in range(W)]
x = np.concatenate([e["x"] for e in ds]); y = np.concatenate([e["y"] for e in ds]); ids = np.concatenate([e["ids"] for e in ds]).astype(np.int32)
s = Swarm(ids, x, y, device="cuda:0").build_graph(1.0)
def t(**kw):
    r = s.elect(**kw); ts = []
    for _ in range(3):
        torch.cuda.synchronize(); a = time.perf_counter(); r = s.elect(**kw); torch.cuda.synchronize(); ts.append((time.perf_counter() - a) * 1e3)
    return r, min(ts)
r16, m16 = t(compact=True); r32, m32 = t(compact=False)
print(json.dumps({"agents": s.n, "edges": s.n_edges, "rounds": r16.rounds_exec, "ms_col16": m16, "ms_col32": m32,
                  "same": bool(np.array_equal(r16.changes, r32.changes)), "compact": r16.compact}), flush=True)
