"""Debug aid: how much of each sparse round is workgroup imbalance (libswarm_phases.so, built with
-DSWARM_PHASES: make -C distributed-swarm-algorithm_amd/csrc phases).  For each round R: the span
(first workgroup start -> last workgroup end), the median and mean workgroup end, and the marked
agents per workgroup (median / max).  Usage: python tools/balance_sweep.py N R [R ...]"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, "distributed-swarm-algorithm_amd")
from swarm_amd import _lib  # noqa: E402

_lib.load(os.path.join(_lib.HERE, "libswarm_phases.so"))
from swarm_amd import gen  # noqa: E402
from swarm_amd.swarm import Swarm  # noqa: E402

n = int(sys.argv[1])
d = gen.swarm_inputs(n, 2026, t=0)
sw = Swarm(d["ids"], d["x"], d["y"], d["caps"], device="cuda:0").build_graph(1.0)
sw.elect()
L = _lib.lib()
L.swarm_debug_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
for R in map(int, sys.argv[2:]):
    out = np.zeros(8192 * 8, np.uint64)
    sw.elect(max_rounds=R)
    L.swarm_debug_phases(out.ctypes.data_as(ctypes.c_void_p), out.size)
    ph = out.reshape(8192, 8).astype(np.int64)
    ph = ph[ph[:, 0] > 0]
    t0 = ph[:, 0].min()
    end = (ph[:, 1] - t0) * 0.01
    dur = (ph[:, 1] - ph[:, 0]) * 0.01
    gathered = (ph[:, 6] - t0) * 0.01
    listed = (ph[:, 5] - t0) * 0.01
    print(json.dumps({"round": R, "wgs": int(len(ph)), "span": round(float(end.max()), 2),
                      "end_med": round(float(np.median(end)), 2), "end_mean": round(float(end.mean()), 2),
                      "end_p99": round(float(np.percentile(end, 99)), 2),
                      "listed_med": round(float(np.median(listed)), 2), "dur_med": round(float(np.median(dur)), 2),
                      "marked_med": int(np.median(ph[:, 2])), "marked_max": int(ph[:, 2].max()),
                      "marked_mean": round(float(ph[:, 2].mean()), 1)}), flush=True)
