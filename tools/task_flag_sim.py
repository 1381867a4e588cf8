"""CPU design probe: how many 64-agent tasks (the dense round's unit) hold a marked agent in each
sparse round, against the marked agents themselves -- the work of a task-granular dense round
against the frontier's per-agent gathers.  Spatial (cell-row-major) storage order as Swarm's.
Usage: python tools/task_flag_sim.py [N]"""
import sys
import time

import numpy as np

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import gen  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
t0 = time.time()
d = gen.swarm_inputs(n, 2026, deg=16.0)
perm = gen.cell_order(d["x"], d["y"], 1.0)
x, y, ids = d["x"][perm], d["y"][perm], d["ids"][perm].astype(np.int64)
rp, col = gen.rgg_csr(x, y, 1.0)
rp = rp.astype(np.int64)
deg = np.diff(rp)
E = int(rp[-1])
print(f"graph {n} agents {E} edges {time.time() - t0:.1f}s", flush=True)
nz = deg > 0
starts = rp[:-1][nz]
src = np.repeat(np.arange(n), deg)  # row of each edge
L = ids.copy()
rounds = []
marked = None  # marked for the next round (None: dense)
t = 0
while True:
    t += 1
    m = L.copy()
    m[nz] = np.maximum(m[nz], np.maximum.reduceat(L[col], starts))
    ris = m != L
    nr = int(ris.sum())
    if marked is not None:
        nm = int(marked.sum())
        tasks = np.unique(np.nonzero(marked)[0] >> 6)
        tedges = int((rp[np.minimum((tasks + 1) * 64, n)] - rp[tasks * 64]).sum())
        medges = int(deg[marked].sum())
        rounds.append((t, nr, nm, len(tasks), medges, tedges))
    L = m
    if nr == 0:
        break
    # marks for round t+1: risers and their neighbours
    nxt = ris.copy()
    nxt[col[ris[src]]] = True
    marked = nxt
ntask = (n + 63) // 64
print(f"rounds {t}; tasks {ntask}", flush=True)
for lo, hi in [(2, 9), (10, 30), (31, 100), (101, 200), (201, 400), (401, 700), (701, 1000), (1001, 100000)]:
    sel = [r for r in rounds if lo <= r[0] <= hi]
    if not sel:
        continue
    a = np.array(sel, dtype=np.float64)
    print(f"rounds {lo}-{int(a[-1, 0])}: changes {a[:, 1].mean():10.0f}  marked {a[:, 2].mean():10.0f} "
          f"({100 * a[:, 2].mean() / n:5.2f} %)  flagged tasks {a[:, 3].mean():8.0f} ({100 * a[:, 3].mean() / ntask:5.2f} %)"
          f"  edges marked {a[:, 4].mean() / 1e6:6.2f}M  task edges {a[:, 5].mean() / 1e6:6.2f}M"
          f"  ratio {a[:, 5].sum() / max(1, a[:, 4].sum()):4.1f}", flush=True)
