"""Price static chunk -> workgroup rebalancing of the sparse election rounds on the C3 swarm (CPU replay,
tools/balance_sim.c).  Usage: python tools/balance_sim.py [N]  -> per round-range listed maxima and the
modelled round times of today's grid-stride schedule against the static one."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-swarm-algorithm_amd"))
sys.path.insert(0, ROOT)
from swarm_amd import gen  # noqa: E402
from oracle import oracle  # noqa: E402  (its RGG builder; the replay itself is tools/balance_sim.c)

so = os.path.join(ROOT, "tools", "libbalance_sim.so")
subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tools", "balance_sim.c")])
lib = ctypes.CDLL(so)
lib.balance_sim.restype = ctypes.c_long
P = ctypes.c_void_p
lib.balance_sim.argtypes = [ctypes.c_long, P, P, P, ctypes.c_long, ctypes.c_long, ctypes.c_long, P]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = gen.swarm_inputs(n, 2026)
perm = gen.cell_order(d["x"], d["y"], 1.0)
x, y, ids = d["x"][perm], d["y"][perm], d["ids"][perm].astype(np.int32)
rp, col = oracle.rgg_csr(x, y, 1.0)
R = 1 << 13
out = np.zeros(R * 4, np.int64)
p = lambda a: a.ctypes.data_as(P)  # noqa: E731
rounds = lib.balance_sim(n, p(rp), p(col), p(ids), 2048, max(1, int(8e-4 * n)), R, p(out))
o = out[: rounds * 4].reshape(-1, 4)
# per-workgroup round time (DESIGN §4 per-workgroup clocks at 10M): ~3.2 us of stamp scan + list, ~3.9 us per
# 64-agent gather pass; the static schedule pays one more dependent load (~2 us) on every round it runs
A, B, EXTRA = 3.2, 3.9, 2.0
tg = A + B * np.ceil(o[:, 1] / 64.0)
ts = A + B * np.ceil(o[:, 2] / 64.0) + EXTRA
ti = A + B * np.ceil(o[:, 3] / 64.0)
res = {"rounds": int(rounds), "ranges": []}
for lo, hi in ((10, 100), (101, 400), (401, 1000), (1001, rounds)):
    sl = slice(lo - 1, min(hi, rounds))
    res["ranges"].append({"rounds": f"{lo}-{hi}", "grid_ms": float(tg[sl].sum() / 1e3), "static_ms": float(ts[sl].sum() / 1e3),
                          "ideal_ms": float(ti[sl].sum() / 1e3),
                          "listed_max_grid_mean": float(o[sl, 1].mean()), "listed_max_static_mean": float(o[sl, 2].mean()),
                          "listed_mean": float(o[sl, 3].mean())})
best = np.minimum(tg, ts)
res["static_where_better_ms_saved"] = float((tg - best)[9:].sum() / 1e3)
print(json.dumps(res, indent=1))
