"""Design probe for a record-list election tail (see tools/record_tail_sim.c).  CPU only.

python tools/record_tail_sim.py --agents 1000000 --t0 300 --tile 16
"""
import argparse
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-swarm-algorithm_amd"))
from oracle import oracle  # noqa: E402  (design probe: the Jacobi rounds are the check)
from swarm_amd import gen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=1_000_000)
    ap.add_argument("--t0", type=int, nargs="+", default=[300])
    ap.add_argument("--tile", type=int, nargs="+", default=[16])
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--delta", type=int, nargs="+", default=[0])
    a = ap.parse_args()
    so = f"/tmp/librecord_sim_{os.getpid()}.so"
    subprocess.check_call(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-o", so,
                           os.path.join(ROOT, "tools", "record_tail_sim.c")])
    lib = ctypes.CDLL(so)
    lib.rec_sim.restype = ctypes.c_long
    n = a.agents
    t_0 = time.time()
    d = gen.swarm_inputs(n, a.seed)
    perm = gen.cell_order(d["x"], d["y"])
    x, y, ids = d["x"][perm], d["y"][perm], d["ids"][perm]
    rp, col = gen.rgg_csr(x, y)
    print(f"graph {n} agents {len(col)} edges {time.time() - t_0:.1f}s", flush=True)
    lead, st, rounds, ch = oracle.elect_frontier(rp, col, ids)[:4]
    print(f"jacobi rounds_exec {rounds}", flush=True)
    cx = np.floor(x).astype(np.int64)
    cy = np.floor(y).astype(np.int64)
    P = lambda z: z.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    for t0 in a.t0:
        L1 = oracle.elect_frontier(rp, col, ids, max_rounds=t0 - 1)[0]
        L = oracle.elect_frontier(rp, col, ids, max_rounds=t0)[0]
        rise = (L != L1)
        mark = rise.copy()
        src = np.repeat(np.arange(n), np.diff(rp))
        mark[col[rise[src]]] = True
        mark = mark.astype(np.uint8)
        for ts, delta in [(ts, dl) for ts in a.tile for dl in a.delta]:
            tx, ty = cx // ts, cy // ts
            ntx = int(tx.max()) + 1
            tile_of = (ty * ntx + tx).astype(np.int32)
            ntiles = int(tile_of.max()) + 1
            order = np.argsort(tile_of, kind="stable").astype(np.int32)
            toff = np.zeros(ntiles + 1, np.int64)
            np.add.at(toff, tile_of + 1, 1)
            toff = np.cumsum(toff)
            hist = np.zeros(1 << 16, np.int64)
            fin = np.empty(n, np.int32)
            stats = np.zeros(10, np.int64)
            t_1 = time.time()
            dmax = lib.rec_sim(ctypes.c_long(n), P(rp), P(col), P(L), P(mark), P(tile_of),
                               ctypes.c_long(ntiles), P(toff), P(order), P(hist), ctypes.c_long(len(hist)),
                               P(fin), P(stats), ctypes.c_long(100000), ctypes.c_long(delta))
            ok_lead = bool(np.array_equal(fin, lead))
            tail = np.asarray(ch[t0:rounds - 1])
            ok_ch = bool(np.array_equal(hist[1:dmax + 1], tail)) and t0 + dmax + 1 == rounds
            agents_per_tile = n / ntiles
            print(f"T0 {t0} delta {delta} tile {ts}x{ts} cells (~{agents_per_tile:.0f} agents, {ntiles} tiles): "
                  f"launches {stats[0]} activations {stats[1]} levels/act {stats[2] / max(1, stats[1]):.1f} "
                  f"critical levels {stats[3]} (256 WGs: {stats[8]} levels, {stats[9]} tiles in sequence) (jacobi tail rounds {rounds - t0}) maxlen {stats[4]} ovf {stats[5]} "
                  f"recomputes {stats[6] / 1e6:.1f}M edges {stats[7] / 1e6:.1f}M | leaders {ok_lead} changes {ok_ch} "
                  f"sum tail changes {int(tail.sum())} ({time.time() - t_1:.1f}s)", flush=True)


if __name__ == "__main__":
    main()
